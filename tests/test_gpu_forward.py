"""The persistent forward (k_forward: the whole network in ONE launch, tasks =
(layer, frame, tile) from a ticket counter, per-frame dependency counters
instead of kernel boundaries) against the per-layer launches of the same plan
and against the CPU oracle.

Bars: bitwise identical to the layer launches (masks and every layer's
activations; the bodies are the same code), mask <= 1e-3 vs the oracle, no
dependency wait ever gives up (VSS_OPT_FORWARD_FAULTS == 0), and the
counters re-arm across launches of different batch sizes.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MASK_TOL = 1e-3


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(autouse=True)
def persistent_plan():
    # sessions created inside these tests plan for the persistent forward
    os.environ["VSS_FORWARD"] = "1"
    yield
    os.environ.pop("VSS_FORWARD", None)


def _frames(syn, n, h=480, w=640, c=3, start=0):
    return np.stack([syn.make_frame(start + i, h, w, c) for i in range(n)])


def _both_modes(pkg, s, f):
    s.set_option(pkg.VSS_OPT_FORWARD, 1)
    a, _, _ = s.segment_frames(f)
    assert s.forward_faults() == 0
    s.set_option(pkg.VSS_OPT_FORWARD, 0)
    b, _, _ = s.segment_frames(f)
    s.set_option(pkg.VSS_OPT_FORWARD, 1)
    return a, b


@pytest.mark.parametrize("dtype", ["bf16x2", "f32"])
def test_forward_default_bitwise_vs_layer_launches(pkg, oracle, blob, synthetic, torch_cuda, dtype):
    with pkg.Session(dtype=dtype, max_batch=8) as s:
        assert s.persistent, "144x256 must run as one persistent launch"
        assert s.forward_kernel() == f"void vss::k_forward<{1 if dtype == 'bf16x2' else 0}>(vss::FwdParams)"
        f = _frames(synthetic, 8, start=900)
        for n in (8, 3, 1):
            a, b = _both_modes(pkg, s, f[:n])
            assert np.array_equal(a, b), (dtype, n, float(np.abs(a - b).max()))
        ref = oracle.forward(blob, f, 144, 256, mode=0).reshape(8, -1)
        err = float(np.abs(s.segment_frames(f)[0] - ref).max())
        print(f"{dtype}: persistent forward mask err vs oracle {err:.3e}")
        assert err <= MASK_TOL


def test_forward_every_layer_bitwise(pkg, synthetic, torch_cuda):
    with pkg.Session(dtype="bf16x2", max_batch=4) as s:
        f = _frames(synthetic, 4, start=950)
        s.set_option(pkg.VSS_OPT_KEEP_STEM, 1)
        s.set_option(pkg.VSS_OPT_FORWARD, 0)
        s.segment_frames(f)
        want = [s.read_layer(li, 4) for li in range(s.n_layers - 1)]
        s.set_option(pkg.VSS_OPT_FORWARD, 1)
        s.segment_frames(f)
        assert s.forward_faults() == 0
        for li in range(s.n_layers - 1):
            assert np.array_equal(s.read_layer(li, 4), want[li]), li


def test_forward_rearms_across_batch_sizes(pkg, synthetic, torch_cuda):
    torch = torch_cuda
    with pkg.Session(dtype="bf16x2", max_batch=8) as s:
        f = _frames(synthetic, 8, start=1000)
        ref, _, _ = s.segment_frames(f)
        d = torch.from_numpy(f).cuda()
        outs = {n: torch.empty((n, 144 * 256), dtype=torch.float32, device="cuda") for n in (8, 5, 2)}
        stream = torch.cuda.Stream()
        # graph replays and eager launches, interleaved batch sizes: each launch
        # must start from re-armed counters
        for use_graph in (1, 0):
            s.set_option(pkg.VSS_OPT_USE_GRAPH, use_graph)
            for k in range(30):
                n = (8, 5, 2)[k % 3]
                s.segment_device(d.data_ptr(), n, 480, 640, 3, 640 * 3, 480 * 640 * 3, outs[n].data_ptr(),
                                 stream.cuda_stream)
            stream.synchronize()
            for n, o in outs.items():
                assert np.array_equal(o.cpu().numpy(), ref[:n]), (use_graph, n)
        s.set_option(pkg.VSS_OPT_USE_GRAPH, 1)
        assert s.forward_faults() == 0


def test_forward_matches_autotuned_layer_plan(pkg, synthetic, torch_cuda):
    # the default plan (no VSS_FORWARD): the planner + autotuner pick any compiled
    # tile for layer launches; the arithmetic is tile-invariant, so results are identical
    f = _frames(synthetic, 6, start=1100)
    with pkg.Session(dtype="bf16x2", max_batch=8) as s:
        assert s.persistent
        a, _, _ = s.segment_frames(f)
    os.environ.pop("VSS_FORWARD")
    with pkg.Session(dtype="bf16x2", max_batch=8) as s:
        assert not s.persistent
        with pytest.raises(pkg.VssError):
            s.set_option(pkg.VSS_OPT_FORWARD, 1)
        b, _, _ = s.segment_frames(f)
    assert np.array_equal(a, b)


def test_forward_reference_size_288x512(pkg, oracle, blob, synthetic, torch_cuda):
    f = _frames(synthetic, 3, 720, 1280, 3, start=1200)
    with pkg.Session(model_h=288, model_w=512, dtype="bf16x2", max_batch=3, max_frame_h=720,
                     max_frame_w=1280) as s:
        assert s.persistent
        a, b = _both_modes(pkg, s, f)
    assert np.array_equal(a, b)
    ref = oracle.forward(blob, f, 288, 512, mode=0).reshape(3, -1)
    assert float(np.abs(a - ref).max()) <= MASK_TOL


def test_unsupported_plan_falls_back_to_layer_launches(pkg, oracle, blob, synthetic, torch_cuda):
    # at 64x64 the /8 expand layer splits its hidden channels (<= 256 pixels), a
    # shape outside the persistent forward's table: layer launches, same bars
    f = _frames(synthetic, 2, 120, 160, 3, start=1300)
    with pkg.Session(model_h=64, model_w=64, dtype="bf16x2", max_batch=2, max_frame_h=120,
                     max_frame_w=160) as s:
        assert not s.persistent
        assert s.forward_kernel() is None
        with pytest.raises(pkg.VssError) as e:
            s.set_option(pkg.VSS_OPT_FORWARD, 1)
        assert e.value.code == pkg.VSS_E_UNSUPPORTED
        m, _, _ = s.segment_frames(f)
    ref = oracle.forward(blob, f, 64, 64, mode=0).reshape(2, -1)
    assert float(np.abs(m - ref).max()) <= MASK_TOL


def test_forward_profile_events(pkg, synthetic, torch_cuda):
    with pkg.Session(dtype="bf16x2", max_batch=8) as s:
        f = _frames(synthetic, 8, start=1400)
        ref, _, _ = s.segment_frames(f)
        s.set_option(pkg.VSS_OPT_PROFILE, 1)
        for _ in range(3):
            got, _, _ = s.segment_frames(f)
            assert np.array_equal(got, ref)
        s.set_option(pkg.VSS_OPT_PROFILE, 0)
        ms, cnt = s.profile_read_forward()
        print(f"k_forward mean {ms * 1e3:.1f} us over {cnt}")
        assert cnt == 3 and ms > 0
