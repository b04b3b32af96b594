"""GPU parity of the post-processing chain (§8(f) row 1, csrc/vss_post.hip)
through the C ABI, against the CPU oracle (vsso_post) and against the
reference's own JS run under Node (tests/golden/post_chain.npz).

Bar: u8 alpha bytes BIT-EXACT; f32 refinedAlpha max |gpu - oracle| <= 1e-6
(the only non-exact operation is pow(), whose last-ulp double result may
differ between the device math library and glibc before the f32 store;
measured differences are printed).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ALPHA_TOL = 1e-6


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def post_golden():
    return np.load(os.path.join(GOLDEN, "post_chain.npz"), allow_pickle=False)


def _frames(syn, seeds, h, w, c=3):
    return np.stack([syn.make_frame(int(s), h, w, c) for s in seeds])


def _run_device(torch, chain, frames, masks, out_alpha=True, out_u8=True):
    n, fh, fw, c = frames.shape
    _, H, W = masks.shape
    df = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    dm = torch.from_numpy(np.ascontiguousarray(masks, np.float32)).cuda()
    da = torch.full((n, H, W), -1.0, dtype=torch.float32, device="cuda")
    du = torch.zeros((n, H, W), dtype=torch.uint8, device="cuda")
    chain.process_device(df.data_ptr(), n, fh, fw, c, fw * c, fh * fw * c, dm.data_ptr(),
                         da.data_ptr() if out_alpha else 0, du.data_ptr() if out_u8 else 0,
                         torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return da.cpu().numpy(), du.cpu().numpy()


def _cmp(tag, a, u, want_a, want_u):
    err = float(np.abs(a - want_a).max())
    mism = int((u != want_u).sum())
    print(f"{tag}: alpha max|d|={err:.3g} u8 mismatches={mism}")
    assert err <= ALPHA_TOL
    assert mism == 0


def test_post_vs_reference_js_golden(pkg, torch_cuda, synthetic, post_golden):
    g = post_golden
    n, H, W = g["masks"].shape
    fh, fw = (int(v) for v in g["frame_hw"])
    frames = _frames(synthetic, g["seeds"], fh, fw)
    with pkg.Session(model_h=H, model_w=W, dtype="f32", max_batch=8, autotune=False) as s:
        chain = pkg.PostChain(s)
        a, u = _run_device(torch_cuda, chain, frames, g["masks"])
        _cmp("golden", a, u, g["alpha"], g["alpha_u8"])


def test_post_state_across_calls_and_reset(pkg, torch_cuda, synthetic, post_golden):
    g = post_golden
    n, H, W = g["masks"].shape
    fh, fw = (int(v) for v in g["frame_hw"])
    frames = _frames(synthetic, g["seeds"], fh, fw)
    with pkg.Session(model_h=H, model_w=W, dtype="f32", max_batch=8, autotune=False) as s:
        chain = pkg.PostChain(s)
        parts = [_run_device(torch_cuda, chain, frames[t:t + 2], g["masks"][t:t + 2]) for t in (0, 2)]
        a = np.concatenate([p[0] for p in parts])
        u = np.concatenate([p[1] for p in parts])
        _cmp("split", a, u, g["alpha"], g["alpha_u8"])
        chain.reset()
        a2, u2 = _run_device(torch_cuda, chain, frames, g["masks"])
        assert np.array_equal(a2, a) and np.array_equal(u2, u)
        # alpha-only / u8-only outputs
        chain.reset()
        a3, u3 = _run_device(torch_cuda, chain, frames, g["masks"], out_u8=False)
        assert np.array_equal(a3, a) and not u3.any()
        chain.reset()
        a4, u4 = _run_device(torch_cuda, chain, frames, g["masks"], out_alpha=False)
        assert np.array_equal(u4, u) and np.all(a4 == -1.0)


@pytest.mark.parametrize("dtype", ["bf16x2", "f32"])
def test_segment_post_vs_oracle_full_size(pkg, torch_cuda, synthetic, oracle, dtype):
    """VGA frames, 144x256 masks: seam + chain in one call vs the oracle chain on
    the GPU's own masks (isolates the post stage), 3 calls of one stream."""
    with pkg.Session(dtype=dtype, max_batch=8) as s:
        chain = pkg.PostChain(s)
        st = oracle.PostState(s.mask_h, s.mask_w)
        for call in range(3):
            frames = _frames(synthetic, range(40 + 8 * call, 48 + 8 * call), 480, 640)
            masks, mw, mh = s.segment_frames(frames)
            masks = masks.reshape(-1, mh, mw)
            a, u, mw2, mh2 = chain.segment(frames)
            assert (mw2, mh2) == (mw, mh)
            want_a, want_u = oracle.post(masks, frames, st)
            _cmp(f"{dtype} call {call}", a.reshape(want_a.shape), u.reshape(want_u.shape), want_a, want_u)


@pytest.mark.parametrize("cfg", [dict(USE_BILATERAL=0), dict(BILATERAL_SIGMA_RANGE=30.0, BILATERAL_SIGMA_SPATIAL=2.0),
                                 dict(EMA=0.0, GAMMA=1.0), dict(NOISE_CUTOFF=0.2, HIGH_THRESHOLD=0.7, EMA=0.9)])
def test_post_config_variants_rgba_strided(pkg, torch_cuda, synthetic, oracle, cfg):
    """The settings knobs (script.ts:16-25), RGBA frames with padded rows, set live."""
    torch = torch_cuda
    H, W, fh, fw = 96, 128, 200, 300
    frames = _frames(synthetic, range(60, 63), fh, fw, 4)
    stride = fw * 4 + 64
    padded = np.zeros((3, fh, stride), np.uint8)
    padded[:, :, :fw * 4] = frames.reshape(3, fh, fw * 4)
    with pkg.Session(model_h=H, model_w=W, dtype="f32", max_batch=4, autotune=False) as s:
        masks = s.segment_frames(frames)[0].reshape(3, H, W)
        chain = pkg.PostChain(s)
        chain.set_config(**cfg)
        ocfg = oracle.PostConfig.default()
        for f, _ in ocfg._fields_:
            setattr(ocfg, f, getattr(chain.config, f))
        want_a, want_u = oracle.post(masks, frames, oracle.PostState(H, W), ocfg)
        df = torch.from_numpy(padded).cuda()
        dm = torch.from_numpy(masks).cuda()
        da = torch.empty((3, H, W), dtype=torch.float32, device="cuda")
        du = torch.empty((3, H, W), dtype=torch.uint8, device="cuda")
        chain.process_device(df.data_ptr(), 3, fh, fw, 4, stride, fh * stride, dm.data_ptr(), da.data_ptr(),
                             du.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        _cmp(f"cfg {cfg}", da.cpu().numpy(), du.cpu().numpy(), want_a, want_u)


def test_post_errors(pkg, torch_cuda):
    with pkg.Session(model_h=48, model_w=64, dtype="f32", max_batch=2, autotune=False) as s1, \
            pkg.Session(model_h=48, model_w=64, dtype="f32", max_batch=2, autotune=False) as s2:
        chain = pkg.PostChain(s1)
        f = np.zeros((1, 32, 32, 3), np.uint8)
        rc = pkg.lib().vss_segment_post(s2._h, chain._st, f.ctypes.data, 1, 32, 32, 3, 96,
                                        np.empty(48 * 64, np.float32).ctypes.data, None)
        assert rc == pkg.VSS_E_INVALID_ARG  # state of another handle
        rc = pkg.lib().vss_segment_post(s1._h, chain._st, f.ctypes.data, 1, 32, 32, 3, 96, None, None)
        assert rc == pkg.VSS_E_INVALID_ARG  # no output requested
        with pytest.raises(pkg.VssError):  # batch above max_batch
            chain.segment(np.zeros((3, 32, 32, 3), np.uint8))
        with pytest.raises(pkg.VssError):
            chain.set_config(BILATERAL_SIGMA_RANGE=0.0)


@pytest.mark.parametrize("geom", [(2, 480, 640, 3, 144, 256, 0, 0), (3, 100, 150, 4, 48, 64, 40, 24),
                                  (1, 1080, 1920, 3, 144, 256, 0, 0), (2, 7, 5, 3, 48, 64, 0, 8)])
def test_composite_bitexact_vs_oracle(pkg, torch_cuda, synthetic, oracle, geom):
    """§8(f) row 3: the RGBA output canvas, bit-exact with the oracle, incl. padded
    input rows, padded output rows, tiny frames (mask larger than the frame)."""
    torch = torch_cuda
    n, fh, fw, c, H, W, pad_in, pad_out = geom
    frames = _frames(synthetic, range(80, 80 + n), fh, fw, c)
    rng = np.random.default_rng(fh)
    alpha = rng.integers(0, 256, (n, H, W), dtype=np.uint8)
    alpha[:, : H // 4] = 0
    alpha[:, -H // 4:] = 255
    want = oracle.composite(frames, alpha)
    rs = fw * c + pad_in
    padded = np.zeros((n, fh, rs), np.uint8)
    padded[:, :, :fw * c] = frames.reshape(n, fh, fw * c)
    ors = fw * 4 + pad_out
    with pkg.Session(model_h=H, model_w=W, dtype="f32", max_batch=4, autotune=False) as s:
        df = torch.from_numpy(padded).cuda()
        da = torch.from_numpy(alpha).cuda()
        do = torch.full((n, fh, ors), 0xAB, dtype=torch.uint8, device="cuda")
        pkg.composite_device(s, df.data_ptr(), n, fh, fw, c, rs, fh * rs, da.data_ptr(), do.data_ptr(), ors, fh * ors,
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = do.cpu().numpy()
    assert np.array_equal(got[:, :, :fw * 4].reshape(want.shape), want)
    assert np.all(got[:, :, fw * 4:] == 0xAB)  # row padding untouched


def test_segment_composite_end_to_end(pkg, torch_cuda, synthetic, oracle):
    """processFrame :78-178 in one call == oracle(post(GPU masks)) composited, across
    two calls of one stream."""
    with pkg.Session(dtype="bf16x2", max_batch=4, max_frame_h=480, max_frame_w=640) as s:
        chain = pkg.PostChain(s)
        st = oracle.PostState(s.mask_h, s.mask_w)
        for call in range(2):
            frames = _frames(synthetic, range(90 + 4 * call, 94 + 4 * call), 480, 640, 4)
            masks = s.segment_frames(frames)[0].reshape(4, s.mask_h, s.mask_w)
            got = chain.composite(frames)
            _, want_u = oracle.post(masks, frames, st)
            want = oracle.composite(frames, want_u)
            assert np.array_equal(got, want), f"call {call}: {(got != want).sum()} bytes differ"
        with pytest.raises(pkg.VssError):  # more output than the handle holds
            chain.composite(np.zeros((4, 1080, 1920, 3), np.uint8))


def test_face_chain_vs_reference_js_golden(pkg, torch_cuda, synthetic):
    """§8(f) row 4 on the GPU: the stabilised EMA (warp of prevAlpha + blend),
    the face prior, the closing inside it and the clamped refine against the
    reference's own JS (tests/golden/post_face.npz); faces given from the host
    and from device memory; a call with no faces after them is the plain chain."""
    g = np.load(os.path.join(GOLDEN, "post_face.npz"), allow_pickle=False)
    import json
    n, H, W = g["masks"].shape
    fh, fw = (int(v) for v in g["frame_hw"])
    frames = _frames(synthetic, g["seeds"], fh, fw)
    faces = [pkg.FaceFrame.make(affine=f["affine"], box=f["box"], video_wh=(fw, fh))
             for f in json.loads(str(g["faces"]))]
    with pkg.Session(model_h=H, model_w=W, dtype="f32", max_batch=8, autotune=False) as s:
        chain = pkg.PostChain(s)
        chain.set_faces(faces)
        a, u = _run_device(torch_cuda, chain, frames, g["masks"])
        _cmp("face golden", a, u, g["alpha"], g["alpha_u8"])
        # the same from device memory, frame by frame (state carried across calls)
        chain.reset()
        raw = bytes((pkg.FaceFrame * n)(*faces))
        dfaces = torch_cuda.frombuffer(bytearray(raw), dtype=torch_cuda.uint8).cuda()
        size = len(raw) // n
        parts = []
        for t in range(n):
            chain.set_faces_device(dfaces.data_ptr() + t * size, 1)
            parts.append(_run_device(torch_cuda, chain, frames[t:t + 1], g["masks"][t:t + 1]))
        _cmp("face golden, per frame, device faces", np.concatenate([p[0] for p in parts]),
             np.concatenate([p[1] for p in parts]), g["alpha"], g["alpha_u8"])
        # faces are consumed by one call: the next call is the plain chain (no prior, no warp)
        chain.reset()
        a2, u2 = _run_device(torch_cuda, chain, frames, g["masks"])
        plain = np.load(os.path.join(GOLDEN, "post_chain.npz"), allow_pickle=False)
        _cmp("plain after faces", a2, u2, plain["alpha"], plain["alpha_u8"])
        with pytest.raises(pkg.VssError):  # face count must match the call's frames
            chain.set_faces(faces[:2])
            _run_device(torch_cuda, chain, frames, g["masks"])
