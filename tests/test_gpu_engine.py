"""GPU tests of the queued engine's round-3 behaviour (include/vss.h):

  * graphs are built once per (slot, batch shape) — a caller rotating output
    buffers patches the graph's pointer parameters instead of rebuilding, and
    vss_prepare_device builds them ahead of the first call;
  * host tickets are tracked per host batch: device calls on the same handle
    (which take slots round-robin and order themselves on the device only)
    never make vss_wait / vss_query report an unfinished host batch done;
  * completions (copies out of the slot's pinned buffer, callbacks) run on the
    handle's completion thread, in ticket order, without any lock held: a
    callback may call back into the handle;
  * config 5's whole batch (64 x 1080p) in one vss_submit against the oracle.
Masks are compared bitwise with the device path (same kernels) or at the 1e-3
mask bar against the oracle.
"""
import threading

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


def _frames(syn, n, h=480, w=640, c=3, start=0):
    return np.stack([syn.make_frame(start + i, h, w, c) for i in range(n)])


def test_rotating_buffers_build_once_per_slot(pkg, synthetic, torch_cuda):
    torch = torch_cuda
    B, h, w = 4, 480, 640
    f = _frames(synthetic, B, h, w)
    d = torch.from_numpy(f).cuda()
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=4) as s:
        assert s.graph_builds == 0
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(3)]  # 3 buffers over 4 slots
        st = torch.cuda.current_stream().cuda_stream
        ref = None
        for i in range(24):
            s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i % 3].data_ptr(), st)
            if i == 0:
                torch.cuda.synchronize()
                ref = outs[0].cpu().numpy().copy()
        torch.cuda.synchronize()
        # every slot sees all 3 buffers: one executable per (slot, buffer pair), never a patch
        # (the single executable per slot waited on every call of this pattern)
        assert s.graph_builds == 12, s.graph_builds
        assert s.graph_patches == 0, s.graph_patches
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), ref)
        # another frame buffer (a new pair: slot 0's fourth executable) computes the same masks
        d2 = d.clone()
        o2 = torch.empty_like(outs[0])
        s.segment_device(d2.data_ptr(), B, h, w, 3, w * 3, h * w * 3, o2.data_ptr(), st)
        torch.cuda.synchronize()
        assert np.array_equal(o2.cpu().numpy(), ref)
        assert s.graph_builds == 13
        # a new batch shape builds again
        s.segment_device(d.data_ptr(), 2, h, w, 3, w * 3, h * w * 3, o2.data_ptr(), st)
        torch.cuda.synchronize()
        assert s.graph_builds == 14
        assert np.array_equal(o2.cpu().numpy()[:2], ref[:2])


def test_graph_lru_patches_beyond_four_buffer_pairs(pkg, synthetic, torch_cuda):
    """One slot, five buffer pairs in rotation: four executables are built, and
    each later call with a pair no executable holds patches the least recently
    used one (after its own last launch) — masks bitwise equal throughout."""
    torch = torch_cuda
    B, h, w = 2, 240, 320
    f = _frames(synthetic, B, h, w, start=7)
    d = torch.from_numpy(f).cuda()
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=1) as s:
        want, _, _ = s.segment_frames(f)
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(5)]
        st = torch.cuda.Stream()
        for i in range(20):
            outs[i % 5].zero_()
            s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i % 5].data_ptr(), st.cuda_stream)
            st.synchronize()
            assert np.array_equal(outs[i % 5].cpu().numpy(), want), i
        # the host call above built the first executable of this shape (its slot
        # buffers); pairs 0-2 build the other three, and from pair 3 on five
        # pairs cycle through four executables: every call re-binds the LRU one
        assert s.graph_builds == 4, s.graph_builds
        assert s.graph_patches == 17, s.graph_patches
        # four pairs in rotation: no patch once each has its executable
        before = s.graph_patches
        for i in range(12):
            s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i % 4].data_ptr(), st.cuda_stream)
        st.synchronize()
        assert s.graph_patches - before <= 4
        for o in outs[:4]:
            assert np.array_equal(o.cpu().numpy(), want)


def test_caller_stream_destroyed_and_recreated(pkg, synthetic, torch_cuda):
    """a caller stream may be destroyed with the handle's work
    queued on it and a new stream (often at the same address) used at once:
    calls on caller streams always wait for their slot's previous work."""
    import ctypes
    torch = torch_cuda
    hip = ctypes.CDLL("libamdhip64.so")
    B, h, w = 8, 480, 640
    f = _frames(synthetic, B, h, w, start=11)
    d = torch.from_numpy(f).cuda()
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=4) as s:
        want, _, _ = s.segment_frames(f)
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(8)]
        addrs = []
        for rep in range(4):
            stp = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(stp)) == 0
            addrs.append(stp.value)
            for i in range(8):
                s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i].data_ptr(), stp.value)
            assert hip.hipStreamDestroy(stp) == 0  # work still queued on it
        torch.cuda.synchronize()
        s.synchronize()
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), want)


def test_destroy_with_callbacks_pending(pkg, synthetic, torch_cuda):
    """vss_destroy drains the completion thread before any
    engine is torn down, so every queued batch's callback fires with its masks
    before close() returns — on the plain handle and the RCCL (device_ids) one."""
    B, h, w = 2, 240, 320
    batches = [_frames(synthetic, B, h, w, start=20 + 3 * i) for i in range(4)]
    for ids in (None, [0]):
        s = pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=4, device_ids=ids)
        want = [s.segment_frames(b)[0] for b in batches]
        fired = []
        for i, b in enumerate(batches):
            s.segment_frames_async(b, lambda m, mw, mh, st, i=i: fired.append((i, st, m.copy())))
        s.close()  # immediately: the four batches are still queued or running
        assert [x[0] for x in fired] == [0, 1, 2, 3], (ids, fired)
        for i, st, m in fired:
            assert st == 0
            assert np.array_equal(m, want[i]), (ids, i)


def test_blocking_calls_from_callback_return_busy(pkg, synthetic, torch_cuda):
    """a callback runs on the completion thread, the only thread that
    completes host batches; a blocking call that would wait for a later batch's
    completion returns VSS_E_BUSY instead of deadlocking."""
    B, h, w = 2, 240, 320
    f0 = _frames(synthetic, B, h, w, start=1)
    f1 = _frames(synthetic, B, h, w, start=2)
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=2) as s:
        want1, _, _ = s.segment_frames(f1)
        submitted = threading.Event()
        box = {}
        done = threading.Event()

        def cb(_m, _mw, _mh, _st):
            submitted.wait(10)
            for name, fn in (("wait", lambda: s.wait(box["t1"])), ("synchronize", s.synchronize)):
                try:
                    fn()
                    box[name] = "returned"
                except pkg.VssError as e:
                    box[name] = e.code
            done.set()

        s.segment_frames_async(f0, cb)
        box["t1"] = s.submit(f1)  # a copy-out batch: its completion is queued behind the callback
        submitted.set()
        assert done.wait(30), "callback deadlocked"
        assert box["wait"] == pkg.VSS_E_BUSY, box
        assert box["synchronize"] == pkg.VSS_E_BUSY, box
        got, _, _ = s.wait(box["t1"])
        assert np.array_equal(got, want1)


def test_prepare_device_builds_ahead(pkg, synthetic, torch_cuda):
    torch = torch_cuda
    B, h, w = 8, 480, 640
    f = _frames(synthetic, B, h, w)
    d = torch.from_numpy(f).cuda()
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=4) as s:
        s.prepare_device(B, h, w, 3, w * 3, h * w * 3)
        assert s.graph_builds == 4
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(4)]
        streams = [torch.cuda.Stream() for _ in range(4)]
        for i in range(16):
            s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i % 4].data_ptr(),
                             streams[i % 4].cuda_stream)
        torch.cuda.synchronize()
        assert s.graph_builds == 4
        assert s.graph_patches == 4  # each slot's first call binds its buffers
        masks, _, _ = s.segment_frames(f)
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), masks)


def test_mixed_submit_and_device_calls(pkg, synthetic, torch_cuda):
    """device calls after a vss_submit reuse its slot on the device;
    the host ticket must still complete only once its masks are written."""
    torch = torch_cuda
    B, h, w = 8, 480, 640
    f = _frames(synthetic, B, h, w, start=3)
    d = torch.from_numpy(f).cuda()
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=4) as s:
        want, _, _ = s.segment_frames(f)
        outs = [torch.empty((B, s.mask_h * s.mask_w), device="cuda") for _ in range(8)]
        st = torch.cuda.Stream()
        for rep in range(3):
            t = s.submit(f)
            for i in range(8):  # 2 x queue_depth device calls: every slot reused
                s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i].data_ptr(), st.cuda_stream)
            got, _, _ = s.wait(t)
            assert np.array_equal(got, want), rep
            pinned = pkg.host_empty((B, s.mask_h * s.mask_w))
            t2 = s.submit(f, out=pinned)
            for i in range(8):
                s.segment_device(d.data_ptr(), B, h, w, 3, w * 3, h * w * 3, outs[i].data_ptr(), st.cuda_stream)
            got2, _, _ = s.wait(t2)
            assert np.array_equal(got2, want), rep
            assert s.query(t2)
        torch.cuda.synchronize()
        for o in outs:
            assert np.array_equal(o.cpu().numpy(), want)


def test_callbacks_in_order_and_reentrant(pkg, synthetic, torch_cuda):
    B, h, w = 2, 240, 320
    batches = [_frames(synthetic, B, h, w, start=10 * i) for i in range(6)]
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=4) as s:
        want = [s.segment_frames(b)[0] for b in batches]
        order, errors = [], []
        done = threading.Event()

        def cb(masks, mw, mh, status, i):
            try:
                order.append(i)
                assert status == 0
                assert np.array_equal(masks, want[i])
                # re-entrant: the completion thread holds no lock
                s.get_option(pkg.VSS_OPT_GRAPH_BUILDS)
            except Exception as e:  # noqa: BLE001
                errors.append(e)
            if len(order) == len(batches):
                done.set()

        for i, b in enumerate(batches):
            while True:
                try:
                    s.segment_frames_async(b, lambda m, mw, mh, st, i=i: cb(m, mw, mh, st, i))
                    break
                except pkg.VssError as e:
                    assert e.code == pkg.VSS_E_BUSY
                    threading.Event().wait(0.001)
        assert done.wait(30)
        s.synchronize()
        assert not errors, errors
        assert order == list(range(len(batches)))


def test_sync_calls_from_threads(pkg, synthetic, torch_cuda):
    """Synchronous vss_segment from several threads: no thread holds the handle's
    lock while it waits for the GPU, and each gets its own masks."""
    B, h, w = 2, 240, 320
    batches = [_frames(synthetic, B, h, w, start=5 * i) for i in range(4)]
    with pkg.Session(max_batch=B, max_frame_h=h, max_frame_w=w, queue_depth=2) as s:
        want = [s.segment_frames(b)[0] for b in batches]
        errs = []

        def run(i):
            try:
                for _ in range(10):
                    got, _, _ = s.segment_frames(batches[i])
                    assert np.array_equal(got, want[i])
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        ts = [threading.Thread(target=run, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert not errs, errs


def test_config5_whole_batch_64x1080p(pkg, oracle, blob, synthetic, torch_cuda):
    """BASELINE config 5's whole batch (64 x 1920x1080) as one vss_submit."""
    n, h, w = 64, 1080, 1920
    f = _frames(synthetic, n, h, w, start=100)
    with pkg.Session(max_batch=n, max_frame_h=h, max_frame_w=w, queue_depth=2) as s:
        t = s.submit(f)
        got, _, _ = s.wait(t)
    ref = oracle.forward(blob, f, 144, 256, mode=0).reshape(n, -1)
    err = float(np.abs(got - ref).max())
    print(f"64x1080p max |gpu - oracle| = {err:.3e}")
    assert err <= MASK_TOL
