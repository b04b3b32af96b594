"""GPU ONNX sessions (include/vso.h) against the ONNX oracle
(oracle/onnx_ref.py, float64 per op) — synthetic models covering every
supported operator and fusion, a MODNet-shaped matting net, and the
reference's two real MediaPipe models (tests/golden/mediapipe_*.npz,
re-encoded from client/src/assets/*.onnx, real weights).

Bar (float32 arithmetic, f32 MFMA accumulation, vs the f64-per-op oracle):
max |gpu - oracle| <= 1e-4 * max(1, max |oracle|) per output.
"""
import os
import re

import numpy as np
import pytest

import onnx_models as M
import onnx_ref as R

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-4


@pytest.fixture(scope="module")
def ort(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vss_amd.ort as o
    return o


def _check(got, want, label):
    for k, w in want.items():
        g = got[k]
        assert g.shape == w.shape, (label, k, g.shape, w.shape)
        err = float(np.abs(g - w).max())
        scale = max(1.0, float(np.abs(w).max()))
        print(f"{label} {k}: max abs err {err:.3e} (scale {scale:.2f})")
        assert err <= TOL * scale, (label, k, err)


@pytest.mark.parametrize("name", list(M.MODELS))
def test_synthetic_models(ort, name):
    data = M.MODELS[name][0]()
    feeds = M.feeds_for(name)
    want = R.run(R.load(data), feeds)
    with ort.InferenceSession(data) as s:
        got = s.run(feeds)
        _check(got, want, name)
        again = s.run(feeds)  # graph replay: bitwise the same
        for k in got:
            assert np.array_equal(got[k], again[k])
        launches = s.launches()
        print(name, len(launches), "launches")


def test_conv_epilogue_fusions(ort):
    # BatchNormalization folded, residual Add and the activations fused: no
    # standalone launch for any of them in conv_zoo
    with ort.InferenceSession(M.conv_zoo()) as s:
        names = s.launches()
    assert all("k_unary" not in n and "k_binary" not in n and "k_affine" not in n for n in names), names
    assert sum("k_conv" in n for n in names) == len(names)


@pytest.mark.parametrize("key", ["mediapipe_face_detector", "mediapipe_face_landmarks"])
def test_reference_mediapipe_models(ort, key):
    model, feeds, want, meta = M.load_golden(os.path.join(GOLDEN, key + ".npz"))
    with ort.InferenceSession(model) as s:
        assert s.input_names == list(feeds)
        got = s.run(feeds)
        print(key, len(s.launches()), "launches")
    _check(got, want, key)


@pytest.mark.parametrize("precision", ["f32", "bf16", "f16"])
def test_conv_tile_forms(ort, precision):
    """k_conv_tile against the oracle with the same operand rounding
    (onnx_ref.run(conv_operands=...)): every convolution reads a graph input,
    so the only difference left is f32 (GPU) vs f64 (oracle) accumulation.
    Run twice: the split-K arrival counters reset themselves (bitwise equal)."""
    data = M.conv_tiles()
    rng = np.random.default_rng(5)
    feeds = {"x": rng.standard_normal((2, 40, 37, 70)).astype(np.float32),
             "x2": rng.standard_normal((2, 200, 9, 16)).astype(np.float32)}
    want = R.run(R.load(data), feeds, conv_operands=None if precision == "f32" else precision)
    with ort.InferenceSession(data, precision=precision) as s:
        got = s.run(feeds)
        again = s.run(feeds)
        for k in got:
            assert np.array_equal(got[k], again[k])
        names = s.launches()
        print(precision, s.tile_convs(), "tiled:", [n for n in names if "conv" in n])
        assert s.tile_convs() == 6  # the 1x1 stays on k_conv_small
        # x2 (9x16, batch 2) runs on 4x16 tiles with its 7 chunks split over 7
        # workgroups (the last to arrive adds the partials): conv_tile_shape
        assert any("k_conv_tile" in n and ", 4, 16, 64>" in n for n in names)
    _check(got, want, f"conv_tiles {precision}")


def test_conv_thin(ort):
    """k_conv_thin's instances (2 / 3 / 4 outputs), scalar and float4 pixel
    paths, Sigmoid and residual epilogues, against the oracle (f32: 1e-4)."""
    data = M.conv_thin()
    rng = np.random.default_rng(19)
    feeds = {"x": rng.standard_normal((2, 24, 37, 70)).astype(np.float32),
             "x2": rng.standard_normal((2, 16, 36, 64)).astype(np.float32),
             "r": rng.standard_normal((2, 4, 36, 64)).astype(np.float32)}
    want = R.run(R.load(data), feeds)
    with ort.InferenceSession(data) as s:
        got = s.run(feeds)
        names = s.launches()
    print(names)
    assert sorted(n.split("(")[0] for n in names) == ["void vso::k_conv_thin<2>", "void vso::k_conv_thin<3>",
                                                     "void vso::k_conv_thin<4>"], names
    _check(got, want, "conv_thin")


def test_se_forms(ort):
    """The SE chain's kernel forms against the oracle (f32: 1e-4 of the output
    scale): the wave-per-plane and per-workgroup pools, Gemm activations in
    the epilogue (PRelu not), the per-plane and general broadcast Mul."""
    data = M.se_forms()
    rng = np.random.default_rng(29)
    feeds = {"a": rng.standard_normal((2, 6, 4, 6)).astype(np.float32),
             "c": rng.standard_normal((2, 6, 5, 7)).astype(np.float32),
             "l": rng.standard_normal((2, 3, 40, 40)).astype(np.float32)}
    want = R.run(R.load(data), feeds)
    with ort.InferenceSession(data) as s:
        got = s.run(feeds)
        names = [n.split("(")[0] for n in s.launches()]
    print(names)
    assert names.count("void vso::k_gap_wave") == 2 and names.count("void vso::k_gap") == 1, names
    assert names.count("void vso::k_binary_planes") == 1 and names.count("vso::k_binary") >= 1, names
    assert sum("k_unary" in n for n in names) == 0, names  # Relu / Sigmoid / LeakyRelu in the GEMM epilogues
    _check(got, want, "se_forms")


def test_norm_planes(ort):
    """k_norm_plane's three forms and the two-launch path beyond it against the
    oracle (f32: 1e-4 of the output scale)."""
    data = M.norm_planes()
    rng = np.random.default_rng(17)
    feeds = {k: (rng.standard_normal(s) * 3 + 1).astype(np.float32)
             for k, s in (("a", (2, 3, 37, 70)), ("b", (2, 4, 72, 128)), ("c", (1, 2, 150, 245)), ("d", (1, 2, 200, 200)))}
    want = R.run(R.load(data), feeds)
    with ort.InferenceSession(data) as s:
        got = s.run(feeds)
        names = s.launches()
    print(names)
    assert sum("k_norm_plane<" in n for n in names) == 3, names
    assert sum("k_norm_stats" in n for n in names) == 1, names
    _check(got, want, "norm_planes")


@pytest.mark.parametrize("precision", ["bf16", "f16"])
def test_conv_upsample_fusion(ort, precision):
    """A 2x linear Resize inside its consumer convolution (k_conv_tile_up)
    against the oracle with the same operand rounding.  The interpolated
    values are rounded to the operand type in the kernel, the oracle's are
    its f64 Resize rounded: an operand may land one 16-bit step apart, so the
    bound is 1e-3 of the output scale (measured 4e-5 bf16, 1.3e-4 f16; a wrong
    tap or weight is O(1))."""
    data = M.conv_up()
    rng = np.random.default_rng(11)
    feeds = {"lo": rng.standard_normal((2, 64, 9, 17)).astype(np.float32),
             "skip": rng.standard_normal((2, 5, 18, 34)).astype(np.float32),
             "lo2": rng.standard_normal((2, 32, 11, 13)).astype(np.float32)}
    want = R.run(R.load(data), feeds, conv_operands=precision)
    with ort.InferenceSession(data, precision=precision) as s:
        got = s.run(feeds)
        again = s.run(feeds)
        names = s.launches()
    print(precision, names)
    assert sum("k_conv_tile_up<" in n for n in names) == 2, names
    assert sum("k_resize" in n for n in names) == 1, names  # the 70-channel consumer's
    for k, w in want.items():
        err = float(np.abs(got[k] - w).max())
        scale = max(1.0, float(np.abs(w).max()))
        print(f"conv_up {precision} {k}: max abs err {err:.3e} (scale {scale:.2f})")
        assert err <= 1e-3 * scale, (k, err)
        assert np.array_equal(got[k], again[k])


@pytest.mark.parametrize("precision", ["f32", "bf16", "f16"])
def test_inverted_residuals_fused(ort, precision):
    """Every MobileNetV2 inverted residual of ir_chain as one launch
    (vso_ir.hip) — k_ir (exact f32 products) in f32 sessions, k_ir_b16 (the
    1x1 products as hi + lo bf16 splits, ~2^-16 relative) in bf16 / f16 ones —
    against the f64 oracle at the f32 bar (1e-4 of the output scale): the
    1x1 / depthwise convolutions are not k_conv_tile ones, and the oracle
    rounds none of them; and bitwise the same on a second run (the
    hidden-channel slices are summed in a fixed order)."""
    data = M.ir_chain()
    feeds = {"x": np.random.default_rng(14).standard_normal((2, 16, 38, 67)).astype(np.float32)}
    want = R.run(R.load(data), feeds, conv_operands=None if precision == "f32" else precision)
    with ort.InferenceSession(data, precision=precision) as s:
        got = s.run(feeds)
        again = s.run(feeds)
        names = s.launches()
        assert s.ir_blocks() == 11, names
    if precision == "f32":
        assert sum("k_ir<" in n for n in names) == 11, names
    else:
        assert sum("k_ir_b16<" in n for n in names) == 11, names
    assert not any("k_conv_dw" in n or "k_conv_small" in n for n in names), names
    for k, w in want.items():
        err = float(np.abs(got[k] - w).max())
        scale = max(1.0, float(np.abs(w).max()))
        print(f"ir_chain {precision} {k}: max abs err {err:.3e} (scale {scale:.2f})")
        assert err <= TOL * scale, (k, err)
        assert np.array_equal(got[k], again[k])


def test_inverted_residuals_unfused_knob(ort):
    """VSO_IR=0 (read at the first plan of a process) is exercised in a child
    process: the same graph as three launches per block, equal within the f32
    bar to the fused plan."""
    import subprocess
    import sys
    code = ("import numpy as np, sys; sys.path.insert(0, 'tests'); import onnx_models as M; "
            "import importlib.util, os; spec = importlib.util.spec_from_file_location('vss_amd', "
            "'video-stream-segmenetation_amd/__init__.py', submodule_search_locations=['video-stream-segmenetation_amd']); "
            "m = importlib.util.module_from_spec(spec); sys.modules['vss_amd'] = m; spec.loader.exec_module(m); "
            "import vss_amd.ort as o; d = M.ir_chain(); "
            "x = np.random.default_rng(14).standard_normal((2, 16, 38, 67)).astype(np.float32); "
            "s = o.InferenceSession(d); r = s.run({'x': x}); "
            "print(s.ir_blocks(), sum('k_ir<' in n for n in s.launches())); "
            "np.save('gpurun_out/ir_unfused.npy', np.concatenate([v.ravel() for v in r.values()]))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, VSO_IR="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-2:] == ["0", "0"], r.stdout
    data = M.ir_chain()
    x = np.random.default_rng(14).standard_normal((2, 16, 38, 67)).astype(np.float32)
    with ort.InferenceSession(data) as s:
        fused = np.concatenate([v.ravel() for v in s.run({"x": x}).values()])
    unfused = np.load(os.path.join(root, "gpurun_out", "ir_unfused.npy"))
    scale = max(1.0, float(np.abs(unfused).max()))
    assert float(np.abs(fused - unfused).max()) <= TOL * scale


@pytest.mark.parametrize("knob,value", [("VSO_IR_B16", "0"), ("VSO_IR_WAVE", "1")])
def test_inverted_residuals_16bit_knobs(ort, knob, value):
    """The 16-bit forms' knobs (read at the first plan of a process, so in a
    child process), on a bf16 session of ir_chain: VSO_IR_B16=0 runs every
    block on the f32 form (k_ir), equal within the f32 bar to the bf16x3 form
    of this process; VSO_IR_WAVE=1 runs the 7 blocks of <= 64 input channels
    on the wave-private form (k_ir_b16w, measured slower on MODNet: opt-in) —
    the same operands, products and sums as k_ir_b16, so bitwise equal."""
    import subprocess
    import sys
    code = ("import numpy as np, sys; sys.path.insert(0, 'tests'); import onnx_models as M; "
            "import importlib.util, os; spec = importlib.util.spec_from_file_location('vss_amd', "
            "'video-stream-segmenetation_amd/__init__.py', submodule_search_locations=['video-stream-segmenetation_amd']); "
            "m = importlib.util.module_from_spec(spec); sys.modules['vss_amd'] = m; spec.loader.exec_module(m); "
            "import vss_amd.ort as o; d = M.ir_chain(); "
            "x = np.random.default_rng(14).standard_normal((2, 16, 38, 67)).astype(np.float32); "
            "s = o.InferenceSession(d, precision='bf16'); r = s.run({'x': x}); L = s.launches(); "
            "print(sum('k_ir<' in n for n in L), sum('k_ir_b16<' in n for n in L), sum('k_ir_b16w<' in n for n in L)); "
            f"np.save('gpurun_out/ir_{knob}.npy', np.concatenate([v.ravel() for v in r.values()]))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, **{knob: value}),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    want_counts = ["11", "0", "0"] if knob == "VSO_IR_B16" else ["0", "4", "7"]
    assert r.stdout.split()[-3:] == want_counts, r.stdout
    data = M.ir_chain()
    x = np.random.default_rng(14).standard_normal((2, 16, 38, 67)).astype(np.float32)
    with ort.InferenceSession(data, precision="bf16") as s:
        here = np.concatenate([v.ravel() for v in s.run({"x": x}).values()])
    other = np.load(os.path.join(root, "gpurun_out", f"ir_{knob}.npy"))
    scale = max(1.0, float(np.abs(other).max()))
    err = float(np.abs(here - other).max())
    print(f"ir_chain bf16 default vs {knob}={value}: max abs err {err:.3e} (scale {scale:.2f})")
    if knob == "VSO_IR_B16":
        assert err <= TOL * scale
    else:
        assert np.array_equal(here, other)


@pytest.mark.parametrize("model", ["conv_tiles", "conv_up"])
def test_conv_tile_xcd_order_bitwise(ort, model):
    """k_conv_tile's XCD-contiguous item order (xcd_item, vso_device.h) is a
    bijection on the grid: every tile computed by some workgroup with the same
    arithmetic.  Every k_conv_tile form of conv_tiles (3x3 / 5x5, stride 2,
    the K split that keeps the dispatcher's order, partial chunks) and the
    fused-upsample forms of conv_up, f16, in a child process with the order
    off (VSO_CONV_XCD=0, read at the first plan of a process) and in this
    process with it on: bitwise equal."""
    import subprocess
    import sys
    feeds = {"conv_tiles": ("{'x': r.standard_normal((2, 40, 37, 70)).astype(np.float32), "
                            "'x2': r.standard_normal((2, 200, 9, 16)).astype(np.float32)}"),
             "conv_up": ("{'lo': r.standard_normal((2, 64, 9, 17)).astype(np.float32), "
                         "'skip': r.standard_normal((2, 5, 18, 34)).astype(np.float32), "
                         "'lo2': r.standard_normal((2, 32, 11, 13)).astype(np.float32)}")}[model]
    code = ("import numpy as np, sys; sys.path.insert(0, 'tests'); import onnx_models as M; "
            "import importlib.util, os; spec = importlib.util.spec_from_file_location('vss_amd', "
            "'video-stream-segmenetation_amd/__init__.py', submodule_search_locations=['video-stream-segmenetation_amd']); "
            "m = importlib.util.module_from_spec(spec); sys.modules['vss_amd'] = m; spec.loader.exec_module(m); "
            f"import vss_amd.ort as o; d = M.{model}(); r = np.random.default_rng(5); f = {feeds}; "
            "s = o.InferenceSession(d, precision='f16'); g = s.run(f); "
            f"np.savez('gpurun_out/xcd0_{model}.npz', **g)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, VSO_CONV_XCD="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rng = np.random.default_rng(5)
    f = eval(feeds, {"np": np, "r": rng})
    with ort.InferenceSession(getattr(M, model)(), precision="f16") as s:
        here = s.run(f)
        names = s.launches()
    assert any("k_conv_tile" in n for n in names), names
    other = np.load(os.path.join(root, "gpurun_out", f"xcd0_{model}.npz"))
    for k, v in here.items():
        assert np.array_equal(v, other[k]), (model, k, float(np.abs(v - other[k]).max()))


@pytest.mark.parametrize("precision", ["f32", "bf16"])
def test_depthwise_separable_chain(ort, precision):
    """dw -> Clip -> 1x1 -> Clip -> dw -> Clip -> 1x1 (MobileNetV1 blocks): the
    first depthwise is computed inside its 1x1 consumer (no launch writes its
    output), so the 1x1 -> dw -> 1x1 after it — an inverted residual's shape —
    must not be planned as a fused k_ir over that unwritten input.
    The depthwise / 1x1 forms are unrounded in the 16-bit oracle as well: both
    precisions at the f32 bar."""
    data = M.dw_separable_chain()
    feeds = {"x": np.random.default_rng(31).standard_normal((2, 32, 30, 44)).astype(np.float32)}
    want = R.run(R.load(data), feeds, conv_operands=None if precision == "f32" else precision)
    with ort.InferenceSession(data, precision=precision) as s:
        got = s.run(feeds)
        names = s.launches()
        assert s.ir_blocks() == 0, names
    print(precision, names)
    _check(got, want, f"dw_separable {precision}")


def test_small_graphs_two_lanes_bitwise(ort):
    """The two-lane schedule on small graphs (forced by VSO_LANES,
    read once per process, so one child process per setting runs every case):
    a Concat tail into a dense conv, fused Resize -> conv, a pending
    InstanceNorm, k_ir blocks and a depthwise computed in its 1x1 consumer —
    bitwise equal to the one-lane capture, bf16 and f32 sessions."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    cases = [("modnet_like", "M.modnet_like()", "{'input': r.random((1, 3, 64, 96), dtype=np.float32)}"),
             ("ir_chain", "M.ir_chain()", "{'x': r.standard_normal((2, 16, 38, 67)).astype(np.float32)}"),
             ("conv_up", "M.conv_up()", "{'lo': r.standard_normal((2, 64, 9, 17)).astype(np.float32), "
              "'skip': r.standard_normal((2, 5, 18, 34)).astype(np.float32), "
              "'lo2': r.standard_normal((2, 32, 11, 13)).astype(np.float32)}"),
             ("dw_sep", "M.dw_separable_chain()", "{'x': r.standard_normal((2, 32, 30, 44)).astype(np.float32)}")]
    outs = {}
    for lanes in ("2", "1"):
        body = "; ".join(
            f"r = np.random.default_rng(3); s = o.InferenceSession({mk}, precision=pr); a = s.run({fd}); "
            f"res['{nm}_' + pr] = (np.concatenate([v.ravel() for v in a.values()]), s.lanes()); s.close()"
            for nm, mk, fd in cases)
        code = ("import numpy as np, sys; sys.path.insert(0, 'tests'); import onnx_models as M; "
                "import importlib.util, os; spec = importlib.util.spec_from_file_location('vss_amd', "
                "'video-stream-segmenetation_amd/__init__.py', submodule_search_locations=['video-stream-segmenetation_amd']); "
                "m = importlib.util.module_from_spec(spec); sys.modules['vss_amd'] = m; spec.loader.exec_module(m); "
                "import vss_amd.ort as o; res = {}\n"
                f"for pr in ('bf16', 'f32'):\n    {body}\n"
                f"np.savez('gpurun_out/small_lanes{lanes}.npz', **{{k: v[0] for k, v in res.items()}}); "
                "print(' '.join(f'{k}:{v[1]}' for k, v in res.items()))")
        r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, VSO_LANES=lanes),
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        print(lanes, r.stdout.strip())
        used = dict(kv.split(":") for kv in r.stdout.split())
        if lanes == "2":  # the graphs with independent branches put some on the side lane
            assert any(v == "2" for v in used.values()), used
        outs[lanes] = dict(np.load(os.path.join(root, "gpurun_out", f"small_lanes{lanes}.npz")))
    for k in outs["1"]:
        assert np.array_equal(outs["2"][k], outs["1"][k]), k


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_modnet_two_lanes_bitwise(ort, precision):
    """The captured graph's two lanes (vso_lane_count; launches that share no
    activation buffer on two capture streams — by default for inputs of
    >= 2^21 elements, forced here by VSO_LANES, read once per process, so in
    child processes): MODNet's graph uses both, and its outputs are bitwise
    those of a one-lane capture — the schedule orders every pair of launches
    that touch a common buffer."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    outs = {}
    for lanes in ("2", "1"):
        code = ("import numpy as np, sys; sys.path.insert(0, 'tests'); import onnx_models as M; "
                "import importlib.util, os; spec = importlib.util.spec_from_file_location('vss_amd', "
                "'video-stream-segmenetation_amd/__init__.py', submodule_search_locations=['video-stream-segmenetation_amd']); "
                "m = importlib.util.module_from_spec(spec); sys.modules['vss_amd'] = m; spec.loader.exec_module(m); "
                "import vss_amd.ort as o; d = M.modnet(144, 256); "
                "x = np.random.default_rng(23).random((2, 3, 144, 256), dtype=np.float32); "
                f"s = o.InferenceSession(d, input_shape=(2, 3, 144, 256), precision='{precision}'); "
                "a = s.run({'input': x}); b = s.run({'input': x}); print(s.lanes()); "
                "assert all(np.array_equal(a[k], b[k]) for k in a); "
                f"np.save('gpurun_out/modnet_lanes{lanes}_{precision}.npy', np.concatenate([v.ravel() for v in a.values()]))")
        r = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, VSO_LANES=lanes),
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.split()[-1] == lanes, r.stdout
        outs[lanes] = np.load(os.path.join(root, "gpurun_out", f"modnet_lanes{lanes}_{precision}.npy"))
    assert np.array_equal(outs["2"], outs["1"])


@pytest.mark.parametrize("precision", ["bf16", "f16", "f32"])
def test_conv_up_into_thin_head(ort, precision):
    """Resize -> Concat -> 1x1 head of 3 outputs: the thin head launches the
    pending Resize in front of itself, and matches the oracle with
    the same operand rounding at the conv_up bound."""
    data = M.conv_up_thin()
    rng = np.random.default_rng(12)
    feeds = {"lo": rng.standard_normal((2, 32, 9, 17)).astype(np.float32),
             "skip": rng.standard_normal((2, 16, 18, 34)).astype(np.float32)}
    want = R.run(R.load(data), feeds, conv_operands=None if precision == "f32" else precision)
    with ort.InferenceSession(data, precision=precision) as s:
        got = s.run(feeds)
        names = s.launches()
    assert sum("k_resize" in n for n in names) == 1, names
    assert sum("k_conv_thin" in n for n in names) == 1, names
    for k, w in want.items():
        err = float(np.abs(got[k] - w).max())
        print(f"conv_up_thin {precision} {k}: max abs err {err:.3e}")
        assert err <= 1e-3, (k, err)


# MODNet's matte (a sigmoid in [0, 1]) with 16-bit convolution operands, on
# the graph as exported (InstanceNormalization epsilon 1e-5 everywhere).  Every
# InstanceNorm input channel of the seeded net has a variance far above that
# epsilon on the test frame (test_modnet_instance_norm_conditioning), so the
# norm does not blow up operand rounding.
# The same-rounding bar: an oracle run with 16-bit operands is itself chaotic
# at the 16-bit quantum — any difference before a rounding point (f32 vs f64
# accumulation, a resize's arithmetic) flips some operands by one ulp, and
# the flips grow through the 5x5 / 1280-channel LR convolutions and the
# instance norms.  So each 16-bit case also runs the oracle on the input
# scaled by (1 + 2^-22) — f32-rounding-sized noise — and the GPU is held to
# 2x that self-distance ("flip floor", max and mean) from the same-rounding
# oracle (measured: bf16 1.4e-2 against a floor of 1.0e-2, f16 2.3e-3
# against 2.2e-3 — per stage, tools/modnet_taps.py: the backbone stays within
# 6e-5 of the scale, the growth starts at the LR branch).  The q4f16 form
# (the reference's model_q4f16.onnx arithmetic, main.ts:6, model.ts:12-29)
# carries f16 weights, so f16 operands round only its activations: held to
# 2e-3 of the f32 oracle too (measured 1.76e-3; the oracle's own f16 cost
# 1.76e-3).  bf16 operands round the f32-form weights too (8-bit mantissa):
# 0.089 max from the f32 oracle in the oracle alone, bounded and reported.
MODNET_TOL = {"f32": TOL, "f16": 2e-3}       # f32: vs the f32 oracle; f16: vs the f32 oracle
MODNET_FLIP = 2.0                            # 16-bit: x the oracle's flip floor, max and mean
MODNET_FLIP_EPS = 2.0 ** -22                 # the floor's input perturbation (relative)
MODNET_BF16_COST = (0.15, 0.02)              # (max, mean) vs the f32 oracle: bf16 rounding, not parity
MODNET_IN_EPS = {"f32": 1e-5, "f16": 1e-5, "bf16": 1e-5}  # the export's own epsilon


@pytest.fixture(scope="module")
def modnet_cases():
    cases = {}
    x = np.random.default_rng(21).random((1, 3, 288, 512), dtype=np.float32)
    for q4f16, prec in ((False, "f32"), (True, "f32"), (False, "bf16"), (True, "f16")):
        data = M.modnet(q4f16=q4f16, in_eps=MODNET_IN_EPS[prec])
        m = R.load(data)
        want = {"f32": R.run(m, {"input": x})}
        if prec != "f32":
            want[prec] = R.run(m, {"input": x}, conv_operands=prec)
            xp = (x * np.float32(1 + MODNET_FLIP_EPS)).astype(np.float32)
            want["floor"] = R.run(m, {"input": xp}, conv_operands=prec)
        cases[(q4f16, prec)] = (data, x, want)
    return cases


@pytest.mark.parametrize("q4f16,precision", [(False, "f32"), (True, "f32"), (False, "bf16"), (True, "f16")])
def test_modnet_topology_288x512(ort, modnet_cases, q4f16, precision):
    """The public MODNet topology at the reference's 288x512
    (onnx_models.modnet; frameProcessorTest.ts:91), f32 and q4f16 forms, on
    k_conv_tile with f32 operands (1e-4 of the f32 oracle), f16 operands (the
    reference's q4f16 arithmetic: 2e-3 of the f32 oracle) and bf16 operands;
    both 16-bit forms within 2x the flip floor of the same-rounding oracle
    (max and mean)."""
    data, x, wants = modnet_cases[(q4f16, precision)]
    label = f"modnet {'q4f16' if q4f16 else 'f32'} {precision}"
    with ort.InferenceSession(data, precision=precision) as s:
        got = s.run({"input": x})
        again = s.run({"input": x})
        names = s.launches()
        print(label, len(names), "launches,", s.tile_convs(), "tiled convolutions")
        assert s.tile_convs() >= 12  # every 3x3 / 5x5 of >= 8 MMAC (f32), every 3x3 / 5x5 (16-bit)
        # the matte head (IBNorm -> 1x1 16 -> 1 -> Sigmoid): its InstanceNorm
        # applied inside k_conv_thin, one k_norm_apply fewer than k_norm_stats
        assert any("k_conv_thin<1>" in n for n in names), names
        assert sum("k_norm_apply" in n for n in names) + 1 == sum("k_norm_stats" in n for n in names)
    for k, w in wants["f32"].items():
        err, mean = float(np.abs(got[k] - w).max()), float(np.abs(got[k] - w).mean())
        print(f"{label}: vs the f32 oracle max abs err {err:.3e}, mean {mean:.3e}")
        if precision == "f32":
            assert err <= MODNET_TOL["f32"], (label, err)
        else:
            same, fl = wants[precision][k], wants["floor"][k]
            es, ms = float(np.abs(got[k] - same).max()), float(np.abs(got[k] - same).mean())
            fmax, fmean = float(np.abs(fl - same).max()), float(np.abs(fl - same).mean())
            print(f"{label}: vs the {precision}-operand oracle max abs err {es:.3e}, mean {ms:.3e}; flip floor "
                  f"max {fmax:.3e}, mean {fmean:.3e}; oracle {precision} vs f32 {float(np.abs(same - w).max()):.3e}")
            assert es <= MODNET_FLIP * fmax and ms <= MODNET_FLIP * fmean, (label, es, ms, fmax, fmean)
            if precision == "f16":
                assert err <= MODNET_TOL["f16"], (label, err)
            else:
                assert err <= MODNET_BF16_COST[0] and mean <= MODNET_BF16_COST[1], (label, err, mean)
        assert np.array_equal(got[k], again[k])  # split-K reduction order is fixed


def test_run_device(ort):
    import torch
    data = M.modnet_like()
    feeds = M.feeds_for("modnet_like")
    with ort.InferenceSession(data) as s:
        want = s.run(feeds)
        din = [torch.from_numpy(feeds[n]).cuda() for n in s.input_names]
        dout = [torch.empty(sh, dtype=torch.float32, device="cuda") for sh in s.output_shapes]
        st = torch.cuda.Stream()
        s.run_device([t.data_ptr() for t in din], [t.data_ptr() for t in dout], st.cuda_stream)
        st.synchronize()
        for n, t in zip(s.output_names, dout):
            assert np.array_equal(t.cpu().numpy(), want[n])


def test_input_shape_override(ort):
    # a symbolic-size model gets its shape at create (the reference's MODNet
    # export takes any H x W): MODNet-like at 96 x 128
    data = M.modnet_like()  # declares 1x3x64x96
    rng = np.random.default_rng(9)
    x = rng.random((1, 3, 96, 128), dtype=np.float32)
    want = R.run(R.load(data), {"input": x})
    with ort.InferenceSession(data, input_shape=(1, 3, 96, 128)) as s:
        _check(s.run({"input": x}), want, "modnet_like 96x128")


def test_errors(ort):
    bad = R.make_model([R.make_node("Einsum", ["x", "x"], ["y"], equation="ij,jk->ik")], {},
                       [("x", [4, 4])], [("y", [4, 4])])
    with pytest.raises(ort.VsoError) as e:
        ort.InferenceSession(bad)
    assert e.value.code == ort.VSO_E_UNSUPPORTED and "Einsum" in str(e.value)
    with pytest.raises(ort.VsoError) as e:
        ort.InferenceSession(b"\x08\x01\x12\x04nope")
    assert e.value.code == ort.VSO_E_PARSE
    with ort.InferenceSession(M.modnet_like()) as s:
        with pytest.raises(ort.VsoError) as e:
            s.run({"input": np.zeros((1, 3, 10, 10), np.float32)})
        assert e.value.code == ort.VSO_E_INVALID_ARG


def test_cast_float16_bitwise(ort):
    # the GPU's Cast to FLOAT16 rounds exactly as numpy (nearest, ties to even,
    # subnormals, overflow to inf)
    rng = np.random.default_rng(4)
    v = np.concatenate([np.array([1 + 2 ** -11, 1 + 3 * 2 ** -11, 65519.0, 65520.0, -70000.0, 2 ** -25,
                                  3 * 2 ** -25, 6.1e-5, 0.0, -0.0], np.float32),
                        (rng.standard_normal(1014) * 10.0 ** rng.integers(-7, 5, 1014)).astype(np.float32)])
    m = R.make_model([R.make_node("Cast", ["v"], ["h"], to=R.DT_FLOAT16),
                      R.make_node("Cast", ["h"], ["y"], to=R.DT_FLOAT)], {}, [("v", [1024])], [("y", [1024])])
    with ort.InferenceSession(m) as s:
        got = s.run({"v": v})["y"]
    with np.errstate(over="ignore"):
        want = v.astype(np.float16).astype(np.float32)
    assert np.array_equal(got, want)


def _standalone_dw(name):
    """A depthwise convolution launched on its own (k_conv_dw or its
    plane-mapped form k_conv_dw_plane)."""
    return re.search(r"k_conv_dw(_plane<\d>)?\(", name) is not None


def _fused_pair(name):
    """A depthwise -> 1x1 pair in one launch: k_conv_dwpw, or k_conv_pw with
    its depthwise stage (DWK 3 / 5) where that pays (pixel-rich layers)."""
    return "k_conv_dwpw" in name or re.search(r"k_conv_pw<\d, [35]>", name) is not None


def test_conv_kernel_choice(ort):
    """A depthwise conv feeding a 1x1 one runs with it in one launch
    (k_conv_dwpw, or k_conv_pw's depthwise stage on pixel-rich layers); 1x1
    convolutions run on k_conv_pw where it has the workgroups (or a shallow K),
    k_conv_small takes the other convolutions with < 1024 64x64 output tiles
    (incl. the K > 128 split-K form), k_conv_gemm the large ones (conv_zoo at
    512x512: the stem); all forms are checked against the oracle by
    test_synthetic_models."""
    with ort.InferenceSession(M.conv_zoo()) as s:
        small = s.launches()
    with ort.InferenceSession(M.conv_zoo(512, 512)) as s:
        large = s.launches()
    assert not any("k_conv_gemm" in n for n in small), small
    assert any("k_conv_small<false, 16, true>" in n for n in small)  # split-K (K = 288, 360)
    assert sum(_fused_pair(n) for n in small) == 2, small            # both depthwise -> 1x1 pairs
    assert not any(_standalone_dw(n) for n in small)
    assert sum("k_conv_gemm" in n for n in large) == 1, large          # the 5x5 stem at 256x256 outputs
    assert sum(_fused_pair(n) for n in large) == 2, large


def test_residual_source_fusion(ort):
    """MaxPool(2x2 s2) -> [channel Pad] -> Add(Conv) is read by the conv's
    epilogue (no pool / pad launch): all three of the detector's, four of the
    landmark net's five (the fifth feeds two Adds).  Values: test_reference_mediapipe_models."""
    names = {}
    for key in ("mediapipe_face_detector", "mediapipe_face_landmarks"):
        model = M.load_golden(os.path.join(GOLDEN, key + ".npz"))[0]
        with ort.InferenceSession(model) as s:
            names[key] = s.launches()
    assert sum("k_pool" in n for n in names["mediapipe_face_detector"]) == 0
    assert sum("k_pool" in n for n in names["mediapipe_face_landmarks"]) == 1
    # and every depthwise conv runs inside its 1x1 consumer (k_conv_dwpw / k_conv_pw): 32 and 20 launches fewer
    for key, dw in (("mediapipe_face_detector", 32), ("mediapipe_face_landmarks", 20)):
        assert sum(_fused_pair(n) for n in names[key]) == dw, names[key]
        assert not any(_standalone_dw(n) for n in names[key])
    assert len(names["mediapipe_face_detector"]) == 45 and len(names["mediapipe_face_landmarks"]) == 28
