"""CPU tests: pin the C oracle (oracle/vss_oracle.c) before trusting it.

* Preprocessing (frameProcessorTest.ts:79-85): hand-derived known answers of
  tfjs 4.22 resizeBilinear(alignCorners=false, halfPixelCenters=false), the
  tfjs CPU-backend algorithm in float64, and the committed golden x0.
* Network: the independent PyTorch functional restatement (oracle/torch_ref.py)
  and the committed golden masks (tests/golden/, generated from torch_ref).
"""
import hashlib
import os

import numpy as np
import pytest

import torch_ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _img(ch0):
    a = np.asarray(ch0, np.uint8)
    return np.stack([a, 255 - a, a // 2], axis=2)[None]


def test_resize_known_answers_upscale(oracle):
    # 2x2 -> 4x4: ratio 0.5, srcFrac = 0, .5, 1, 1.5; ceil clamps to the last row/col
    x = _img([[0, 100], [200, 50]])
    got = oracle.preprocess(x, 4, 4)[0, 0] * 255.0
    want = np.array([[0, 50, 100, 100],
                     [100, 87.5, 75, 75],
                     [200, 125, 50, 50],
                     [200, 125, 50, 50]], np.float64)
    np.testing.assert_allclose(got, want, atol=2e-4)
    # channel order RGB kept, alpha (if any) dropped
    np.testing.assert_allclose(oracle.preprocess(x, 4, 4)[0, 1] * 255.0, 255.0 - want, atol=2e-4)


def test_resize_known_answers_downscale(oracle):
    # 4x4 -> 2x2: ratio 2, samples exactly pixels (0,0), (0,2), (2,0), (2,2)  (no half-pixel shift)
    a = np.arange(16, dtype=np.uint8).reshape(4, 4) * 10
    got = oracle.preprocess(_img(a), 2, 2)[0, 0] * 255.0
    np.testing.assert_allclose(got, [[0, 20], [80, 100]], atol=2e-4)
    # 3 -> 2 rows: srcFrac 0, 1.5 -> second output row = mean of rows 1 and 2
    b = np.array([[0, 0], [100, 100], [200, 200]], np.uint8)
    got = oracle.preprocess(_img(b), 2, 2)[0, 0] * 255.0
    np.testing.assert_allclose(got, [[0, 0], [150, 150]], atol=2e-4)


def test_rgba_alpha_dropped(oracle, synthetic):
    f3 = synthetic.make_frame(3, 60, 80, 3)
    f4 = synthetic.make_frame(3, 60, 80, 4)
    np.testing.assert_array_equal(oracle.preprocess(f3[None], 32, 48), oracle.preprocess(f4[None], 32, 48))


@pytest.mark.parametrize("fh,fw,hm,wm", [(480, 640, 144, 256), (720, 1280, 288, 512), (97, 131, 48, 64)])
def test_preprocess_vs_tfjs_cpu_f64(oracle, synthetic, fh, fw, hm, wm):
    # the WebGL (f32) and CPU (f64) tfjs backends differ only by float32 rounding
    # of the ratio and the lerps: |diff| <= 2e-5 on /255 values.
    f = synthetic.make_frame(11, fh, fw, 3)
    got = oracle.preprocess(f[None], hm, wm)[0]
    want = torch_ref.resize_legacy_f64(f, hm, wm).transpose(2, 0, 1) / 255.0
    assert np.abs(got - want).max() <= 2e-5


def test_preprocess_vs_torch_form(oracle, synthetic):
    f = np.stack([synthetic.make_frame(i, 480, 640) for i in range(2)])
    a = oracle.preprocess(f, 144, 256)
    b = torch_ref.preprocess(f, 144, 256).numpy()
    assert np.abs(a - b).max() <= 1e-6


@pytest.mark.parametrize("fh,fw,hm,wm", [(120, 160, 48, 64), (480, 640, 144, 256)])
def test_oracle_vs_torch_f32(oracle, blob, synthetic, fh, fw, hm, wm):
    f = np.stack([synthetic.make_frame(20 + i, fh, fw) for i in range(2)])
    m, taps = oracle.forward(blob, f, hm, wm, mode=0, want_taps=True)
    t_taps = []
    mt = torch_ref.forward(blob, f, hm, wm, mode=0, taps=t_taps).numpy()
    assert np.abs(m - mt).max() <= 2e-5
    for li, tt in enumerate(t_taps):
        c = np.stack([taps[i][li] for i in range(len(f))])
        tt = tt.numpy()
        assert c.shape == tt.shape
        scale = max(1.0, float(np.abs(tt).max()))
        assert np.abs(c - tt).max() <= 2e-5 * scale, f"layer {li}"


def _golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", ["vga_2f_144x256", "odd_rgba_1f_32x48"])
def test_oracle_vs_golden(oracle, blob, synthetic, name):
    g = _golden(name)
    h, w, c, hm, wm = (int(v) for v in g["shape"])
    frames = np.stack([synthetic.make_frame(int(s), h, w, c) for s in g["seeds"]])
    assert hashlib.sha256(frames.tobytes()).hexdigest() == str(g["frames_sha256"])
    assert hashlib.sha256(blob).hexdigest() == str(g["weights_sha256"])
    x0 = oracle.preprocess(frames, hm, wm)
    if "x0" in g:
        assert np.abs(x0 - g["x0"]).max() <= 1e-6
    else:
        np.testing.assert_allclose(x0.astype(np.float64).sum(axis=(2, 3)), g["x0_plane_sums"], rtol=1e-6)
    m = oracle.forward(blob, frames, hm, wm, mode=0)
    assert np.abs(m - g["masks"]).max() <= 2e-5


def test_golden_masks_not_degenerate():
    # a saturated or flat mask would make parity vacuous
    m = _golden("vga_2f_144x256")["masks"]
    assert 0.2 < m.mean() < 0.8 and m.std() > 0.15
    assert ((m > 0.05) & (m < 0.95)).mean() > 0.5


def test_bf16_round(oracle):
    assert oracle.bf16_round(1.0) == 1.0
    assert oracle.bf16_round(1.0 + 2 ** -9) == 1.0           # tie -> even
    assert oracle.bf16_round(1.0 + 3 * 2 ** -9) == 1.0 + 2 ** -7
    assert oracle.bf16_round(-3.140625) == -3.140625
