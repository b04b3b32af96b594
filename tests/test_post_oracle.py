"""CPU tests of the post-processing oracle (oracle/vss_oracle.c vsso_post),
pinned by tests/golden/post_chain.npz — vectors produced by the reference's own
temporalEMA / morphologicalOpening / jointBilateral3x3 / refineAlphaOnce /
alphaToImageData (frameProcessorTest.ts:204-313, :644-685) run under Node
(tests/golden/make_post_golden.py).  Bar: bit-exact (f32 alpha and u8 bytes).
"""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def post_golden():
    return np.load(os.path.join(GOLDEN, "post_chain.npz"), allow_pickle=False)


def _golden_frames(synthetic, g):
    fh, fw = (int(v) for v in g["frame_hw"])
    return np.stack([synthetic.make_frame(int(s), fh, fw, 3) for s in g["seeds"]])


def test_golden_config_is_reference_default(oracle, post_golden):
    cfg = json.loads(str(post_golden["config"]))
    d = oracle.PostConfig.default()
    assert cfg["EMA"] == d.ema and cfg["NOISE_CUTOFF"] == d.noise_cutoff
    assert cfg["HIGH_THRESHOLD"] == d.high_threshold and cfg["GAMMA"] == d.gamma
    assert cfg["BILATERAL_SIGMA_SPATIAL"] == d.sigma_spatial and cfg["BILATERAL_SIGMA_RANGE"] == d.sigma_range
    assert bool(cfg["USE_BILATERAL"]) == bool(d.use_bilateral)


def test_guide_matches_golden(oracle, synthetic, post_golden):
    g = post_golden
    frames = _golden_frames(synthetic, g)
    n, H, W = g["masks"].shape
    assert np.array_equal(oracle.post_guide(frames, H, W), g["guide"])


def test_post_chain_bitexact_vs_reference_js(oracle, synthetic, post_golden):
    g = post_golden
    frames = _golden_frames(synthetic, g)
    n, H, W = g["masks"].shape
    st = oracle.PostState(H, W)
    a, u = oracle.post(g["masks"], frames, st)
    assert np.array_equal(a, g["alpha"]), np.abs(a - g["alpha"]).max()
    assert np.array_equal(u, g["alpha_u8"])
    # the chain actually does something on this input
    assert 0.05 < float(g["alpha"].mean()) < 0.95
    assert not np.array_equal(g["alpha"][0], g["alpha"][1])


def test_post_state_carries_across_calls(oracle, synthetic, post_golden):
    g = post_golden
    frames = _golden_frames(synthetic, g)
    n, H, W = g["masks"].shape
    st = oracle.PostState(H, W)
    parts = [oracle.post(g["masks"][t:t + 1], frames[t:t + 1], st) for t in range(n)]
    assert np.array_equal(np.concatenate([p[0] for p in parts]), g["alpha"])
    assert np.array_equal(np.concatenate([p[1] for p in parts]), g["alpha_u8"])


def test_post_refine_edges(oracle, synthetic):
    """Constant masks: the opening zeroes the 1-px border (frameProcessorTest.ts
    :650-681); refine clamps below NOISE_CUTOFF and above HIGH_THRESHOLD (:280-291)."""
    H, W = 16, 24
    frames = np.stack([synthetic.make_frame(3, 40, 60, 3)])
    for v, want in [(0.03, 0.0), (0.99, 1.0)]:
        for bil in (0, 1):
            cfg = oracle.PostConfig.default()
            cfg.use_bilateral = bil
            st = oracle.PostState(H, W)
            a, u = oracle.post(np.full((1, H, W), v, np.float32), frames, st, cfg)
            assert np.all(a[0, 2:-2, 2:-2] == want)
            assert np.all(u[0, 2:-2, 2:-2] == int(want * 255))
            if not bil:  # without the bilateral the border stays exactly 0
                assert np.all(a[0, 0, :] == 0) and np.all(a[0, :, 0] == 0)
                assert np.all(a[0, 1:-1, 1:-1] == want)


def test_composite_oracle_identity_and_transparency(oracle):
    """Compositing (frameProcessorTest.ts:170-178 as defined in vss_oracle.c): at
    equal resolution the alpha passes through; alpha 0 reads back colour 0."""
    rng = np.random.default_rng(5)
    frames = rng.integers(0, 256, (2, 12, 20, 3), dtype=np.uint8)
    alpha = rng.integers(0, 256, (2, 12, 20), dtype=np.uint8)
    alpha[0, :3] = 0
    out = oracle.composite(frames, alpha)
    assert np.array_equal(out[..., 3], alpha)
    vis = alpha > 0
    assert np.array_equal(out[..., :3][vis], frames[vis])
    assert not out[..., :3][~vis].any()
    # upscaling a constant alpha keeps it constant; RGBA input drops its own alpha
    rgba = np.concatenate([frames, np.full((2, 12, 20, 1), 7, np.uint8)], -1)
    out2 = oracle.composite(np.ascontiguousarray(np.repeat(np.repeat(rgba, 3, 1), 2, 2)),
                            np.full((2, 12, 20), 200, np.uint8))
    assert np.all(out2[..., 3] == 200)


def test_face_chain_bitexact_vs_reference_js(oracle, synthetic):
    """§8(f) row 4: warp + blend of prevAlpha, the elliptical face prior, the
    closing inside it and refine's prior clamp — vsso_post_face against the
    reference's own functions run under Node (tests/golden/post_face.npz)."""
    g = np.load(os.path.join(GOLDEN, "post_face.npz"), allow_pickle=False)
    frames = _golden_frames(synthetic, g)
    n, H, W = g["masks"].shape
    fh, fw = (int(v) for v in g["frame_hw"])
    faces = [oracle.Face.make(affine=f["affine"], box=f["box"], video_wh=(fw, fh))
             for f in json.loads(str(g["faces"]))]
    st = oracle.PostState(H, W)
    a, u = oracle.post(g["masks"], frames, st, faces=faces)
    assert np.array_equal(a, g["alpha"]), np.abs(a - g["alpha"]).max()
    assert np.array_equal(u, g["alpha_u8"])
    # the face inputs change every frame of the fixture (the last through the EMA state)
    plain, _ = oracle.post(g["masks"], frames, oracle.PostState(H, W))
    assert all((plain[t] != a[t]).sum() > 100 for t in range(n))
