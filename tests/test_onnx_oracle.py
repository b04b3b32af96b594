"""CPU tests of the ONNX oracle (oracle/onnx_ref.py) — the checker of the GPU
ONNX sessions: its operator implementations pinned against PyTorch's
functional ops, the writer/reader round trip, and the real-weight fixtures
(tests/golden/mediapipe_*.npz) reproducing from their stored graphs (and
from the reference's own model files when /root/reference is present)."""
import os

import numpy as np
import pytest

import onnx_models as M
import onnx_ref as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ASSETS = "/root/reference/client/src/assets"


def _torch():
    import torch
    return torch


@pytest.mark.parametrize("k,s,pads,g,d", [(5, 2, [1, 1, 2, 2], 1, 1), (3, 1, [1, 1, 1, 1], 8, 1),
                                            (3, 2, [0, 0, 2, 2], 8, 1), (1, 1, [0, 0, 0, 0], 1, 1),
                                            (3, 1, [2, 2, 2, 2], 2, 2), (3, 2, [0, 1, 1, 0], 4, 1)])
def test_conv_matches_torch(k, s, pads, g, d):
    torch = _torch()
    F = torch.nn.functional
    rng = np.random.default_rng(k * 100 + s * 10 + g)
    x = rng.standard_normal((2, 8, 13, 17)).astype(np.float32)
    w = rng.standard_normal((16, 8 // g, k, k)).astype(np.float32)
    b = rng.standard_normal(16).astype(np.float32)
    got = R.conv2d(x, w, b, {"strides": [s, s], "pads": pads, "group": g, "dilations": [d, d]})
    xt = F.pad(torch.from_numpy(x).double(), (pads[1], pads[3], pads[0], pads[2]))
    want = F.conv2d(xt, torch.from_numpy(w).double(), torch.from_numpy(b).double(), stride=s, groups=g,
                    dilation=d).float().numpy()
    assert got.shape == want.shape
    assert np.abs(got - want).max() <= 1e-5 * max(1.0, np.abs(want).max())


def test_pool_resize_norm_match_torch():
    torch = _torch()
    F = torch.nn.functional
    rng = np.random.default_rng(5)
    x = rng.standard_normal((2, 3, 12, 15)).astype(np.float32)
    xt = torch.from_numpy(x).double()
    got = R._pool(x, {"kernel_shape": [2, 2], "strides": [2, 2]}, "max")
    assert np.array_equal(got, F.max_pool2d(xt, 2, 2).float().numpy())
    got = R._pool(x, {"kernel_shape": [3, 3], "strides": [2, 2], "pads": [1, 1, 1, 1], "count_include_pad": 1}, "avg")
    want = F.avg_pool2d(xt, 3, 2, padding=1, count_include_pad=True).float().numpy()
    assert np.abs(got - want).max() < 1e-6
    got = R._pool(x, {"kernel_shape": [3, 3], "strides": [2, 2], "pads": [1, 1, 1, 1]}, "avg")
    want = F.avg_pool2d(xt, 3, 2, padding=1, count_include_pad=False).float().numpy()
    assert np.abs(got - want).max() < 1e-6
    got = R._resize(x, [1, 1, 2, 2], None, {"mode": "linear", "coordinate_transformation_mode": "half_pixel"})
    want = F.interpolate(xt, scale_factor=2, mode="bilinear", align_corners=False).float().numpy()
    assert np.abs(got - want).max() < 1e-6
    got = R._resize(x, None, [2, 3, 24, 30], {"mode": "linear", "coordinate_transformation_mode": "align_corners"})
    want = F.interpolate(xt, size=(24, 30), mode="bilinear", align_corners=True).float().numpy()
    assert np.abs(got - want).max() < 1e-6
    got = R._resize(x, [1, 1, 2, 2], None, {"mode": "nearest", "coordinate_transformation_mode": "asymmetric",
                                            "nearest_mode": "floor"})
    want = F.interpolate(xt, scale_factor=2, mode="nearest").float().numpy()
    assert np.array_equal(got, want)
    m = R.load(R.make_model([R.make_node("InstanceNormalization", ["x", "s", "b"], ["y"], epsilon=1e-5)],
                            {"s": np.linspace(0.5, 2, 3, dtype=np.float32), "b": np.arange(3, dtype=np.float32)},
                            [("x", [2, 3, 12, 15])], [("y", [2, 3, 12, 15])]))
    got = R.run(m, {"x": x})["y"]
    want = F.instance_norm(xt, weight=torch.linspace(0.5, 2, 3).double(), bias=torch.arange(3).double(),
                           eps=1e-5).float().numpy()
    assert np.abs(got - want).max() < 1e-5


def test_writer_reader_round_trip():
    for name, (fn, _) in M.MODELS.items():
        data = fn()
        m = R.load(data)
        assert m.nodes and m.inputs and m.outputs, name
        # re-encode what was read: the same bytes come back
        re = R.make_model([R.make_node(n["op"], n["inputs"], n["outputs"], **n["attrs"]) for n in m.nodes],
                          m.inits, [(a, d, e) for a, e, d in m.inputs], [(a, d, e) for a, e, d in m.outputs],
                          opset=m.opset)
        assert re == data, name


@pytest.mark.parametrize("name", list(M.MODELS))
def test_synthetic_models_evaluate(name):
    fn, _ = M.MODELS[name]
    m = R.load(fn())
    out = R.run(m, M.feeds_for(name))
    for k, v in out.items():
        assert v.dtype == np.float32 and np.isfinite(v).all(), (name, k)
        assert np.abs(v).max() > 0, (name, k)


@pytest.mark.parametrize("key", ["mediapipe_face_detector", "mediapipe_face_landmarks"])
def test_golden_fixture_reproduces(key):
    model, feeds, want, meta = M.load_golden(os.path.join(GOLDEN, key + ".npz"))
    got = R.run(R.load(model), feeds)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    src = os.path.join("/root/reference", meta["source"])
    if os.path.exists(src):  # the build container: the fixture is the reference's own model
        import hashlib
        data = open(src, "rb").read()
        assert hashlib.sha256(data).hexdigest() == meta["sha256"]
        orig = R.run(R.load(data), feeds)
        for k in want:
            assert np.array_equal(orig[k], want[k]), k
