"""BASELINE.json's configs through the HIP path, each against the CPU oracle
(oracle/vss_oracle.c; bars as in test_gpu_parity.py: masks <= 1e-3 max-abs,
f32 and bf16x2) — SURVEY.md §8(d)'s table:

  1: 1 x 144x256 RGB (model resolution: the resize is a ratio-1 copy)
  2: 1 x 640x480, f32
  3: 8 x 640x480, bf16x2 (the headline; also test_gpu_parity.py)
  4: 32 x 1280x720 over 8 GPUs = 4 per GPU: the per-GPU shard (4) and the
     whole batch on one GPU (32)
  5: 64 x 1920x1080 over 8 GPUs = 8 per GPU: the per-GPU shard, through the
     pipelined host path (vss_submit, several batches in flight)

plus a model resolution whose every level is odd-sized and not a power of two
(112x208: /16 = 7x13), the decoders' exact-2x upsample taps included."""
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


def _frames(syn, n, h, w, c=3, start=0):
    return np.stack([syn.make_frame(start + i, h, w, c) for i in range(n)])


def _check(masks, frames, oracle, blob, hm=144, wm=256, what=""):
    ref = oracle.forward(blob, frames, hm, wm, mode=0).reshape(len(frames), -1)
    err = float(np.abs(masks.reshape(len(frames), -1) - ref).max())
    print(f"{what}: mask max abs err vs oracle {err:.3e}")
    assert err <= MASK_TOL, (what, err)


@pytest.mark.parametrize("dtype", ["f32", "bf16x2"])
def test_config1_model_resolution_frame(pkg, oracle, blob, synthetic, torch_cuda, dtype):
    f = _frames(synthetic, 1, 144, 256, start=11)
    with pkg.Session(dtype=dtype, max_batch=1, max_frame_h=144, max_frame_w=256) as s:
        m, mw, mh = s.segment_frames(f)
        assert (mw, mh) == (256, 144)
        _check(m, f, oracle, blob, what=f"config 1 ({dtype})")


def test_config2_f32_single_vga(pkg, oracle, blob, synthetic, torch_cuda):
    f = _frames(synthetic, 1, 480, 640, start=21)
    with pkg.Session(dtype="f32", max_batch=1, max_frame_h=480, max_frame_w=640) as s:
        m, _, _ = s.segment_frames(f)
        _check(m, f, oracle, blob, what="config 2 (f32, b=1)")
        alpha, mw, mh = s.segment_frame(f[0])  # the seam triple
        assert alpha.shape == (mh * mw,) and np.array_equal(alpha, m[0])


@pytest.mark.parametrize("n", [4, 32])
def test_config4_720p_batches(pkg, oracle, blob, synthetic, torch_cuda, n):
    f = _frames(synthetic, n, 720, 1280, start=300)
    with pkg.Session(dtype="bf16x2", max_batch=n, max_frame_h=720, max_frame_w=1280) as s:
        m, _, _ = s.segment_frames(f)
        _check(m, f, oracle, blob, what=f"config 4 ({n} x 720p)")


def test_config5_1080p_pipelined(pkg, oracle, blob, synthetic, torch_cuda):
    f = _frames(synthetic, 8, 1080, 1920, start=500)
    g = _frames(synthetic, 8, 1080, 1920, start=600)
    with pkg.Session(dtype="bf16x2", max_batch=8, max_frame_h=1080, max_frame_w=1920, queue_depth=3) as s:
        sync, _, _ = s.segment_frames(f)
        _check(sync, f, oracle, blob, what="config 5 (8 x 1080p)")
        ref_g, _, _ = s.segment_frames(g)
        ts = [s.submit(x) for x in (f, g, f)]  # three in flight
        outs = [s.wait(t)[0] for t in ts]
        assert np.array_equal(outs[0], sync) and np.array_equal(outs[1], ref_g) and np.array_equal(outs[2], sync)


@pytest.mark.parametrize("dtype", ["f32", "bf16x2"])
def test_odd_model_resolution(pkg, oracle, blob, synthetic, torch_cuda, dtype):
    f = _frames(synthetic, 2, 480, 640, start=700)
    with pkg.Session(model_h=112, model_w=208, dtype=dtype, max_batch=2, max_frame_h=480, max_frame_w=640) as s:
        assert s.layer_shape(7)[1:] == (7, 13)
        m, mw, mh = s.segment_frames(f)
        assert (mw, mh) == (208, 112)
        _check(m, f, oracle, blob, hm=112, wm=208, what=f"112x208 ({dtype})")


def test_unsupported_model_resolution_refused(pkg, torch_cuda):
    with pytest.raises(pkg.VssError) as e:
        pkg.Session(model_h=144, model_w=250)
    assert e.value.code == pkg.VSS_E_INVALID_ARG


@pytest.mark.parametrize("h,w,c", [(480, 640, 3), (1080, 1920, 3), (721, 1283, 4), (300, 200, 3), (144, 256, 3)])
def test_row_fetch_bitwise(pkg, synthetic, torch_cuda, h, w, c):
    """VSS_OPT_ROW_FETCH: the queued host path moving only the rows the resize
    reads (pinned -> HBM by k_fetch_rows) gives bitwise the masks of whole
    frames by DMA and of the device path — 16-B and byte-granular rows, RGBA,
    and sizes where no row can be skipped (the DMA path then)."""
    torch = torch_cuda
    f = _frames(synthetic, 3, h, w, c, start=900)
    with pkg.Session(dtype="bf16x2", max_batch=3, max_frame_h=h, max_frame_w=w, queue_depth=2) as s:
        d = torch.from_numpy(f).cuda()
        dev = torch.empty((3, 144 * 256), dtype=torch.float32, device="cuda")
        s.segment_device(d.data_ptr(), 3, h, w, c, w * c, h * w * c, dev.data_ptr(), 0)
        s.synchronize()
        ref = dev.cpu().numpy()
        assert s.get_option(pkg.VSS_OPT_ROW_FETCH) == 1
        a = s.wait(s.submit(f))[0]
        b, _, _ = s.segment_frames(f)
        s.set_option(pkg.VSS_OPT_ROW_FETCH, 0)
        c_, _, _ = s.segment_frames(f)
        assert np.array_equal(a, ref) and np.array_equal(b, ref) and np.array_equal(c_, ref)


def test_pinned_masks_out(pkg, synthetic, torch_cuda):
    """masks_out inside a vss_host_alloc block takes the D2H directly (no
    completion copy): bitwise the masks of the copying path, model and frame
    outputs, queued with several in flight, and the zero-copy lease path."""
    import ctypes
    f = _frames(synthetic, 8, 480, 640, start=700)
    g = _frames(synthetic, 8, 480, 640, start=710)
    with pkg.Session(dtype="bf16x2", max_batch=8, max_frame_h=480, max_frame_w=640, queue_depth=3) as s:
        ref_f, _, _ = s.segment_frames(f)
        ref_g, _, _ = s.segment_frames(g)
        ref_ff, _, _ = s.segment_frames(f, output_size="frame")
        outs = [pkg.host_empty((8, s.mask_h * s.mask_w)) for _ in range(3)]
        for o in outs:
            o.fill(np.nan)
        ts = [s.submit(x, out=o) for x, o in zip((f, g, f), outs)]
        got = [s.wait(t)[0] for t in ts]
        assert all(a is o for a, o in zip(got, outs))
        assert np.array_equal(outs[0], ref_f) and np.array_equal(outs[1], ref_g) and np.array_equal(outs[2], ref_f)
        fo = pkg.host_empty((8, 480 * 640))
        fo.fill(np.nan)
        s.wait(s.submit(f, output_size="frame", out=fo))
        assert np.array_equal(fo, ref_ff)
        slot, buf = s.staging_acquire()
        buf[:g.size] = g.reshape(-1)
        zo = pkg.host_empty((8, s.mask_h * s.mask_w))
        zo.fill(np.nan)
        s.wait(s.submit_staged(slot, 8, 480, 640, 3, zo))
        assert np.array_equal(zo, ref_g)
        # a block too small for the batch is not taken for the direct D2H
        small = pkg.host_empty((4, s.mask_h * s.mask_w))
        with pytest.raises(pkg.VssError):
            s.submit(f, out=small)
    L = pkg.lib()
    assert L.vss_host_free(ctypes.c_void_p(0x1000)) == pkg.VSS_E_INVALID_ARG
    assert L.vss_host_free(None) == pkg.VSS_OK
