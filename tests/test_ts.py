"""TypeScript host (ts/segment.ts -> segment.js) over the Node-API addon."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TS = os.path.join(ROOT, "video-stream-segmenetation_amd", "ts")
NODE = shutil.which("node")


def _strip():
    import importlib.util
    spec = importlib.util.spec_from_file_location("strip_types", os.path.join(TS, "strip_types.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_generated_js_in_sync():
    src = open(os.path.join(TS, "segment.ts")).read()
    assert _strip().strip(src) == open(os.path.join(TS, "segment.js")).read(), \
        "segment.js is stale: python strip_types.py segment.ts > segment.js"


@pytest.fixture(scope="module")
def addon_built(pkg):
    if not NODE or not os.path.isdir("/usr/include/node"):
        pytest.skip("node / node headers not available")
    pkg.build()
    subprocess.run(["make", "-s", "-C", os.path.join(TS, "addon")], check=True)


def test_node_module_loads_and_fails_loudly_without_gpu(addon_built):
    import torch
    script = ("const s=require(process.argv[1]); console.log(s.version());"
              "try { new s.Segmenter({}); console.log('created'); } catch (e) { console.log('error', e.code); }")
    out = subprocess.run([NODE, "-e", script, os.path.join(TS, "segment.js")], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.split()
    assert lines[0] == "30000"
    if not torch.cuda.is_available():
        assert lines[1:] == ["error", "-2"]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16x2", "f32"])
def test_node_segment_matches_oracle_and_python_host(addon_built, pkg, oracle, blob, synthetic, tmp_path, dtype):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    frames = np.stack([synthetic.make_frame(600 + i, 480, 640, 4) for i in range(3)])
    fp, op = tmp_path / "frames.bin", tmp_path / "masks.bin"
    frames.tofile(fp)
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "run_segment.js"), str(fp), "3", "480", "640",
                          "4", str(op), dtype], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info == {"width": 256, "height": 144, "count": 3, "singleMatchesBatch": True,
                    "oversizeRejected": True, "version": 30000, "frameDims": [640, 480, 3 * 480 * 640]}
    masks = np.fromfile(op, np.float32).reshape(3, -1)
    ref = oracle.forward(blob, frames, 144, 256, mode=0).reshape(3, -1)
    assert np.abs(masks - ref).max() <= 1e-3
    # outputSize 'frame' = the model-res masks upsampled (oracle restatement, bitwise)
    fmasks = np.fromfile(str(op) + ".frame", np.float32).reshape(3, 480, 640)
    assert np.array_equal(fmasks, oracle.upsample_mask(masks.reshape(3, 144, 256), 480, 640))
    with pkg.Session(dtype=dtype, max_batch=3, max_frame_h=480, max_frame_w=640) as s:
        py, _, _ = s.segment_frames(frames)
    assert np.array_equal(masks, py)


@pytest.mark.gpu
@pytest.mark.parametrize("ids", [None, "0"])
def test_node_queue_resolves_in_call_order(addon_built, pkg, oracle, blob, synthetic, tmp_path, ids):
    """Concurrent segmentFrames promises (more than queueDepth, so some wait in
    the JS queue) resolve in call order with oracle-equal masks — the ordering
    contract of runModnetExclusive (main.ts:18-22) with batches overlapping on
    the GPU; deviceIds=[0] runs the same calls through the RCCL path.  Config 1
    (a 144x256 frame: ratio-1 resize) goes through Node here."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 3
    for (h, w) in ((480, 640), (144, 256)):
        frames = np.stack([synthetic.make_frame(800 + i, h, w, 3) for i in range(n)])
        fp, op = tmp_path / f"q{h}.bin", tmp_path / f"q{h}"
        frames.tofile(fp)
        args = [NODE, os.path.join(ROOT, "tests", "node", "run_queue.js"), str(fp), str(n), str(h), str(w), "3",
                str(op), "2"] + ([ids] if ids else [])
        out = subprocess.run(args, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr
        info = json.loads(out.stdout.strip().splitlines()[-1])
        assert info["order"] == list(range(n + 2)) and info["empty"] == "rejected", info
        assert info["queueDepth"] == 2 and info["nGpus"] == 1
        assert info["leaseEqual"] is (None if ids else True)
        ref = oracle.forward(blob, frames, 144, 256, mode=0).reshape(n, -1)
        for i in range(n):
            m = np.fromfile(f"{op}.{i}", np.float32)
            assert np.abs(m - ref[i]).max() <= 1e-3, i
        whole = np.fromfile(f"{op}.{n}", np.float32).reshape(n, -1)
        rev = np.fromfile(f"{op}.{n + 1}", np.float32).reshape(n, -1)
        assert np.abs(whole - ref).max() <= 1e-3 and np.array_equal(rev, whole[::-1])


@pytest.mark.gpu
def test_node_post_chain_matches_oracle_and_python_host(addon_built, pkg, oracle, synthetic, tmp_path):
    """PostChain (TS) over two calls of one stream == the oracle chain on the
    GPU's masks == the Python host's PostChain, bit for bit; a live knob change
    (USE_BILATERAL off, GAMMA 1) after reset matches the oracle too."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n, h, w = 4, 240, 320
    frames = np.stack([synthetic.make_frame(700 + i, h, w, 3) for i in range(n)])
    fp, op = tmp_path / "frames.bin", tmp_path / "post"
    frames.tofile(fp)
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "run_post.js"), str(fp), str(n), str(h), str(w),
                          "3", str(op), "bf16x2"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info == {"width": 256, "height": 144, "count": n, "badConfigRejected": True}
    alpha = np.fromfile(str(op) + ".f32", np.float32).reshape(n, 144, 256)
    u8 = np.fromfile(str(op) + ".u8", np.uint8).reshape(n, 144, 256)
    nobil = np.fromfile(str(op) + "_nobil.f32", np.float32).reshape(n, 144, 256)
    with pkg.Session(dtype="bf16x2", max_batch=n, max_frame_h=h, max_frame_w=w) as s:
        masks = s.segment_frames(frames)[0].reshape(n, 144, 256)
        chain = pkg.PostChain(s)
        pa, pu, _, _ = chain.segment(frames)
    want_a, want_u = oracle.post(masks, frames, oracle.PostState(144, 256))
    assert np.array_equal(alpha, want_a) and np.array_equal(u8, want_u)
    assert np.array_equal(alpha, pa.reshape(alpha.shape)) and np.array_equal(u8, pu.reshape(u8.shape))
    cfg = oracle.PostConfig.default()
    cfg.use_bilateral, cfg.gamma = 0, 1.0
    want_nb, _ = oracle.post(masks, frames, oracle.PostState(144, 256), cfg)
    assert np.array_equal(nobil, want_nb)
    # compositing after reset + default config: the RGBA canvases of the same frames
    rgba = np.fromfile(str(op) + "_rgba.u8", np.uint8).reshape(n, h, w, 4)
    assert np.array_equal(rgba, oracle.composite(frames, want_u))


def test_node_tensor_and_session_errors(addon_built):
    """ort.Tensor validates like onnxruntime-web's (float32 only here); a
    garbage model rejects InferenceSession.create with the vso error code."""
    script = r"""
const ort = require(process.argv[1]);
const r = {};
try { new ort.Tensor('int64', new BigInt64Array(1), [1]); } catch (e) { r.int64 = e instanceof TypeError; }
try { new ort.Tensor('float32', new Float32Array(5), [2, 3]); } catch (e) { r.size = e instanceof RangeError; }
const t = new ort.Tensor('float32', new Float32Array(6), [2, 3]);
r.tensor = [t.type, t.size, t.dims];
ort.InferenceSession.create(new Uint8Array([8, 1, 18, 4, 110, 111, 112, 101]), {})
  .then(() => { r.created = true; }, (e) => { r.createCode = e.code; })
  .then(() => console.log(JSON.stringify(r)));
"""
    out = subprocess.run([NODE, "-e", script, os.path.join(TS, "segment.js")], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["int64"] and r["size"] and r["tensor"] == ["float32", 6, [2, 3]]
    assert "created" not in r and r["createCode"] in ("-3", "-2")  # VSO_E_PARSE (or VSO_E_HIP with no GPU)


@pytest.mark.gpu
@pytest.mark.parametrize("key,precision", [("modnet_like", "f32"), ("mediapipe_face_detector", "f32"),
                                           ("conv_tiles", "f16")])
def test_node_onnx_session_matches_oracle_and_python_host(addon_built, pkg, tmp_path, key, precision):
    """InferenceSession.create/run from TypeScript == the ONNX oracle (within
    the 1e-4 relative bar of tests/test_gpu_onnx.py; with { precision: 'f16' }
    the oracle rounds the tiled convolutions' operands the same way) and ==
    the Python host's session bit for bit; concurrent runs serialise, bad
    feeds reject."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import onnx_models as M
    import onnx_ref as R
    if key == "modnet_like":
        model = M.modnet_like()
        feeds = M.feeds_for(key)
        want = R.run(R.load(model), feeds)
    elif key == "conv_tiles":
        model = M.conv_tiles()
        rng = np.random.default_rng(5)
        feeds = {"x": rng.standard_normal((2, 40, 37, 70)).astype(np.float32),
                 "x2": rng.standard_normal((2, 200, 9, 16)).astype(np.float32)}
        want = R.run(R.load(model), feeds, conv_operands=precision)
    else:
        model, feeds, want, _ = M.load_golden(os.path.join(ROOT, "tests", "golden", key + ".npz"))
    bad = R.make_model([R.make_node("Einsum", ["x", "x"], ["y"], equation="ij,jk->ik")], {},
                       [("x", [4, 4])], [("y", [4, 4])])
    mp, ip, bp = tmp_path / "model.onnx", tmp_path / "inputs.bin", tmp_path / "bad.onnx"
    mp.write_bytes(model)
    bp.write_bytes(bad)
    np.concatenate([np.ascontiguousarray(v, np.float32).ravel() for v in feeds.values()]).tofile(ip)
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "run_onnx.js"), str(mp), str(ip),
                          str(tmp_path / "out"), str(bp), precision], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info["inputNames"] == list(feeds) and info["outputNames"] == list(want)
    assert info["replaySame"] and info["badDimsRejected"] and info["afterReject"] and info["releasedRejects"]
    assert info["unsupported"]["code"] == "-4" and "Einsum" in info["unsupported"]["message"]
    from vss_amd import ort as pyort
    with pyort.InferenceSession(model, precision=precision) as s:
        py = s.run(feeds)
    for k, (name, w) in enumerate(want.items()):
        assert info["outputDims"][k] == list(w.shape) and info["outputTypes"][k] == "float32"
        got = np.fromfile(tmp_path / f"out_{k}.bin", np.float32).reshape(w.shape)
        err = float(np.abs(got - w).max())
        assert err <= 1e-4 * max(1.0, float(np.abs(w).max())), (name, err)
        assert np.array_equal(got, py[name]), name


@pytest.mark.gpu
def test_node_face_inputs_match_python_host(addon_built, pkg, synthetic, tmp_path):
    """PostChain.processFrames(frames, faces) from TypeScript == the Python
    host's PostChain with the same FaceFrame inputs, bit for bit (the chain
    itself is pinned against the reference's JS in tests/test_gpu_post.py)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n, h, w = 4, 240, 320
    frames = np.stack([synthetic.make_frame(820 + i, h, w, 3) for i in range(n)])
    faces = [{"box": [90.0, 40.0, 210.0, 200.0]},
             {"affine": [0.99, 0.04, 1.5, -0.04, 0.99, -2.0], "box": [95.5, 42.25, 214.0, 205.75]},
             {"affine": [1.0, 0.0, -3.0, 0.0, 1.0, 1.0]},
             None]
    fp, jp, op = tmp_path / "frames.bin", tmp_path / "faces.json", tmp_path / "face"
    frames.tofile(fp)
    jp.write_text(json.dumps(faces))
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "run_face.js"), str(fp), str(n), str(h), str(w),
                          "3", str(jp), str(op)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info == {"count": n, "width": 256, "height": 144, "mismatchRejected": True}
    alpha = np.fromfile(str(op) + ".f32", np.float32).reshape(n, -1)
    u8 = np.fromfile(str(op) + ".u8", np.uint8).reshape(n, -1)
    with pkg.Session(dtype="bf16x2", max_batch=n, max_frame_h=h, max_frame_w=w) as s:
        chain = pkg.PostChain(s)
        chain.set_faces([pkg.FaceFrame.make(affine=f.get("affine") if f else None, box=f.get("box") if f else None)
                         for f in faces])
        pa, pu, _, _ = chain.segment(frames)
        plain = pkg.PostChain(s)
        qa, _, _, _ = plain.segment(frames)
    assert np.array_equal(alpha, pa) and np.array_equal(u8, pu)
    assert all((alpha[t] != qa[t]).any() for t in range(n))  # the faces act on every frame


@pytest.mark.gpu
def test_node_face_tracker_matches_python_host(addon_built, pkg, synthetic, tmp_path):
    """FaceTracker.track (TypeScript, over two InferenceSessions) == the Python
    host's FaceTracker, number for number, across two calls; its faces drive
    PostChain.processFrames exactly as the Python host's do."""
    import ctypes  # noqa: F401
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import onnx_models as M
    import vss_amd.face as face
    import vss_amd.ort as ort
    n, h, w = 7, 120, 160
    frames = np.stack([synthetic.make_frame(700 + i, h, w, 3) for i in range(n)])
    det_b, lmk_b = M.face_detector_like(), M.face_landmarks_like()
    dp, lp, fp, op = tmp_path / "det.onnx", tmp_path / "lmk.onnx", tmp_path / "frames.bin", tmp_path / "alpha"
    dp.write_bytes(det_b)
    lp.write_bytes(lmk_b)
    frames.tofile(fp)
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "run_face_tracker.js"), str(dp), str(lp),
                          str(fp), str(n), str(h), str(w), "3", str(op)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info["releaseBlocked"] and info["releasedRejects"]
    with ort.InferenceSession(det_b) as ds, ort.InferenceSession(lmk_b) as ls, \
            pkg.Session(model_h=48, model_w=64, dtype="f32", max_batch=8, autotune=False) as s:
        tr = face.FaceTracker(ds, ls, interval=3)
        want = tr.track(frames[:4], (s.mask_w, s.mask_h)) + tr.track(frames[4:], (s.mask_w, s.mask_h))
        tr.close()
        for f, g in zip(info["faces"], want):
            assert (f["affine"] is not None) == bool(g.has_affine) and (f["box"] is not None) == bool(g.has_box)
            if g.has_affine:
                assert f["affine"] == list(g.affine)
            if g.has_box:
                assert f["box"] == list(g.box)
            assert (f["videoW"], f["videoH"]) == (w, h)
        chain = pkg.PostChain(s)
        chain.set_faces(want)
        pa, _, _, _ = chain.segment(frames)
    assert np.array_equal(np.fromfile(str(op) + ".f32", np.float32).reshape(n, -1), pa)
    assert sum(f["box"] is not None for f in info["faces"]) == 3


@pytest.mark.gpu
def test_node_result_blocks_recycled_safely(addon_built, synthetic, tmp_path):
    """The addon's pinned result blocks return to its pool when V8 collects a
    result: a result still held keeps its masks, and recycled blocks carry the
    masks of the batch they were handed to (forced collections in between)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    frames = np.stack([synthetic.make_frame(900 + i, 480, 640, 3) for i in range(4)])
    fp = tmp_path / "frames.bin"
    frames.tofile(fp)
    out = subprocess.run([NODE, "--expose-gc", os.path.join(ROOT, "tests", "node", "run_recycle.js"), str(fp), "2",
                          "480", "640", "3", "30"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    info = json.loads(out.stdout.strip().splitlines()[-1])
    assert info == {"heldIntact": True, "allEqual": True, "iters": 30}


@pytest.mark.gpu
def test_node_natural_exit_without_guard(addon_built):
    """the 400-batch loop that once crashed Node 12 at exit, run
    to a natural exit with the default settings (no exit guard since round 4;
    VSS_NODE_EXIT_GUARD=1 opts back in): the addon's own fix (no N-API call
    from a finalizer after the environment's cleanup hook, a never-destroyed
    result pool) carries it alone."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    env.pop("VSS_NODE_EXIT_GUARD", None)
    out = subprocess.run([NODE, os.path.join(ROOT, "tests", "node", "run_exit.js"), "400"], capture_output=True,
                         text=True, timeout=200, env=env)
    assert out.returncode == 0, (out.returncode, out.stderr[-2000:])
    last = json.loads(out.stdout.strip().splitlines()[-1])
    assert last["frames"] == 8 * 550 and last["guard"] == "default"
