"""Multi-GPU inside the C ABI (SURVEY.md §8(b) n_gpus/device_ids, §8(e)): a
handle over device_ids shards each batch contiguously over its GPUs and
all-gathers the f32 masks over RCCL (ncclAllGather in a group, one
communicator per device and slot); one-GPU-per-process callers join a clique
(vss_comm_unique_id / vss_comm_init_rank / vss_segment_gather_device).

On the one-GPU test box the RCCL paths run with one rank: the same calls
(group all-gather, communicators per slot, the gather buffers, the D2H from
the gathered masks) must give bitwise the masks of the plain handle.  The
shards and the all-gather over 2..8 GPUs run only on a multi-GPU node
(bench.py --gpus N at round end); DESIGN.md says so."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _frames(syn, n, h=480, w=640, c=3, start=0):
    return np.stack([syn.make_frame(start + i, h, w, c) for i in range(n)])


def test_device_ids_one_gpu_rccl_path_bitwise(pkg, synthetic, torch_cuda):
    f = _frames(synthetic, 8, start=40)
    with pkg.Session(dtype="bf16x2", max_batch=8, max_frame_h=480, max_frame_w=640) as plain:
        ref, _, _ = plain.segment_frames(f)
        ref_frame, _, _ = plain.segment_frames(f[:3], output_size="frame")
    with pkg.Session(dtype="bf16x2", max_batch=8, max_frame_h=480, max_frame_w=640, device_ids=[0]) as s:
        assert s.rccl and s.n_gpus == 1
        m, _, _ = s.segment_frames(f)
        assert np.array_equal(m, ref)
        for n in (1, 5):  # ragged batch sizes
            part, _, _ = s.segment_frames(f[:n])
            assert np.array_equal(part, ref[:n]), n
        fm, _, _ = s.segment_frames(f[:3], output_size="frame")
        assert np.array_equal(fm, ref_frame)
        ts = [s.submit(f), s.submit(f[:5]), s.submit(f)]  # queued through the RCCL path
        outs = [s.wait(t)[0] for t in ts]
        assert np.array_equal(outs[0], ref) and np.array_equal(outs[1], ref[:5]) and np.array_equal(outs[2], ref)


def test_device_ids_rejected(pkg, torch_cuda):
    ndev = torch_cuda.cuda.device_count()
    for ids in ([0, 0], [-1], [ndev], [0, ndev + 3]):
        with pytest.raises(pkg.VssError) as e:
            pkg.Session(max_batch=8, device_ids=ids)
        assert e.value.code == pkg.VSS_E_INVALID_ARG, ids
    with pytest.raises(pkg.VssError) as e:
        pkg.Session(max_batch=8, device_ids=[])
    assert e.value.code == pkg.VSS_E_INVALID_ARG


@pytest.mark.parametrize("form", ["ordered", "concurrent"])
def test_clique_one_rank_gather_bitwise(pkg, synthetic, torch_cuda, form):
    """Both all-gather forms (VSS_OPT_GATHER_FORM) at one rank:
    bitwise the plain handle's masks; the ordered form (the default) creates
    slot 0's communicator alone, and the form is fixed once the clique exists;
    vss_comm_status reports every slot -1 until then."""
    torch = torch_cuda
    f = _frames(synthetic, 8, start=60)
    with pkg.Session(dtype="bf16x2", max_batch=8, max_frame_h=480, max_frame_w=640, queue_depth=2) as s:
        ref, _, _ = s.segment_frames(f)
        assert s.gather_form == "ordered"
        assert s.comm_status()["async_errors"] == [-1, -1]
        s.gather_form = form
        ids = s.comm_unique_id()
        assert len(ids) == 2 * 128
        with pytest.raises(pkg.VssError):
            s.comm_init_rank(1, 0, ids[:128])  # one id per slot is required
        s.comm_init_rank(1, 0, ids)
        assert s.gather_form == form
        other = "concurrent" if form == "ordered" else "ordered"
        with pytest.raises(pkg.VssError):
            s.gather_form = other  # fixed by comm_init_rank
        st = s.comm_status()["async_errors"]
        assert st[0] in (0, 7) and (st[1] == -1 if form == "ordered" else st[1] in (0, 7)), st
        d = torch.from_numpy(f).cuda()
        outs = [torch.zeros((8, 144 * 256), dtype=torch.float32, device="cuda") for _ in range(3)]
        streams = [torch.cuda.Stream() for _ in range(2)]
        for i in range(3):
            s.segment_gather_device(d.data_ptr(), 8, 480, 640, 3, 640 * 3, 480 * 640 * 3, outs[i].data_ptr(),
                                    streams[i % 2].cuda_stream)
        torch.cuda.synchronize()
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), ref)


def test_gather_slot_order_independent_of_other_device_calls(pkg, synthetic, torch_cuda):
    """Each rank's i-th vss_segment_gather_device runs on slot (and that slot's
    communicator) i % queue_depth, counted apart from vss_segment_device calls:
    ranks that interleave different plain device calls still issue every
    collective on the same communicator (RCCL's ordering requirement).  At one
    rank: the gather counter moves only with gathers, and interleaved calls of
    both kinds on several streams keep every result bitwise."""
    torch = torch_cuda
    f = _frames(synthetic, 4, start=70)
    with pkg.Session(dtype="bf16x2", max_batch=4, max_frame_h=480, max_frame_w=640, queue_depth=3) as s:
        ref, _, _ = s.segment_frames(f)
        s.comm_init_rank(1, 0, s.comm_unique_id())
        assert s.get_option(pkg.VSS_OPT_GATHER_CALLS) == 0
        with pytest.raises(pkg.VssError):
            s.set_option(pkg.VSS_OPT_GATHER_CALLS, 0)  # read-only
        d = torch.from_numpy(f).cuda()
        outs = [torch.zeros((4, 144 * 256), dtype=torch.float32, device="cuda") for _ in range(10)]
        streams = [torch.cuda.Stream() for _ in range(3)]
        gathers = 0
        for i, kind in enumerate("gddgdgggdd"):
            st = streams[i % 3].cuda_stream
            if kind == "g":
                s.segment_gather_device(d.data_ptr(), 4, 480, 640, 3, 640 * 3, 480 * 640 * 3, outs[i].data_ptr(), st)
                gathers += 1
            else:
                s.segment_device(d.data_ptr(), 4, 480, 640, 3, 640 * 3, 480 * 640 * 3, outs[i].data_ptr(), st)
            assert s.get_option(pkg.VSS_OPT_GATHER_CALLS) == gathers
        torch.cuda.synchronize()
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), ref)
