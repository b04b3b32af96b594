"""The GPU face stage (include/vsf.h, §8(f) row 4) against its oracle
(oracle/face_ref.py, whose geometry is pinned to the reference's own JS by
tests/test_face_oracle.py).

Per face frame the stage's own intermediates are read back (vsf_inspect) and
each kernel is checked on exactly the inputs it saw:
  * detector / landmark inputs (letterbox, ROI resample): bit-exact;
  * the two ONNX sessions: within 1e-4 * max(1, |oracle|) of onnx_ref (f64);
  * decode (argmax, mapFromSquareToSrc, clamp, cropFaceROI): bit-exact;
  * estimateAffineFromLandmarks: within 1e-12 relative (device vs host libm
    atan2 / cos / sin);
  * the lastAffine scan (frame order, WARP_GAIN blend): bit-exact given those.
End to end (models through onnx_ref) the flags match and the numbers agree to
the sessions' tolerance.  Stand-in models (tests/onnx_models.py) drive the
has-box path, which the reference's real detector does not reach on synthetic
frames; the real MediaPipe models run through the same checks.
"""
import ctypes
import os

import numpy as np
import pytest

import face_ref as F
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


@pytest.fixture(scope="module")
def face(pkg, ort):
    import vss_amd.face as f
    return f


@pytest.fixture(scope="module")
def standins():
    return M.face_detector_like(), M.face_landmarks_like()


def _close(got, want, label):
    err = float(np.abs(got - want).max()) if got.size else 0.0
    scale = max(1.0, float(np.abs(want).max()) if want.size else 1.0)
    assert err <= TOL * scale, (label, err, scale)


def _check_slot(tracker, k, frame, det_m, lmk_m, w, h, mask_wh, cfg):
    """One face frame's intermediates against the oracle; returns its record."""
    idx, r = tracker.inspect(k)
    S = int(round((r["det_in"].size // 3) ** 0.5))
    det_in = r["det_in"].reshape(1, 3, S, S)
    assert np.array_equal(det_in, F.detector_input(frame, S)), "letterbox input"
    want = R.run(det_m, {"image": det_in})
    A = want["box_scores"].shape[1]
    _close(r["box_coords"], want["box_coords"].ravel(), "box_coords")
    _close(r["box_scores"], want["box_scores"].ravel(), "box_scores")
    d = F.decode(r["box_coords"].reshape(A, -1), r["box_scores"], S, w, h, cfg.face_score_thresh, cfg.roi_pad)
    assert np.array_equal(r["decode"][:10], d[:10]), (r["decode"][:10], d[:10])
    LH = LW = int(round((r["lmk_in"].size // 3) ** 0.5))
    lmk_in = r["lmk_in"].reshape(1, 3, LH, LW)
    assert np.array_equal(lmk_in, F.roi_input(frame, d, LH, LW)), "ROI input"
    if d[8] > 0:
        lw = R.run(lmk_m, {"image": lmk_in})
        _close(r["lmk_scores"], lw["scores"].ravel(), "landmark scores")
        _close(r["landmarks"], lw["landmarks"].ravel(), "landmarks")
    e = F.estimate_affine(d, r["lmk_scores"][0], r["landmarks"].reshape(-1, 3), w, h, *mask_wh,
                          cfg.landmark_score_thresh)
    assert r["decode"][10] == e[10]
    np.testing.assert_allclose(r["decode"][11:], e[11:], rtol=1e-12, atol=1e-12)
    return idx, r["decode"]


def _faces_equal(got, want_scan, w, h, exact):
    for t, (f, (aff, box)) in enumerate(zip(got, want_scan)):
        assert f.video_w == w and f.video_h == h
        assert bool(f.has_affine) == (aff is not None), t
        assert bool(f.has_box) == (box is not None), t
        if aff is not None:
            if exact:
                np.testing.assert_allclose(list(f.affine), aff, rtol=1e-12, atol=1e-12)
            else:
                np.testing.assert_allclose(list(f.affine), aff, rtol=1e-3, atol=1e-3)
        if box is not None:
            if exact:
                assert list(f.box) == list(box), t
            else:
                np.testing.assert_allclose(list(f.box), box, atol=1e-2)


@pytest.mark.parametrize("fh,fw,fc", [(120, 160, 3), (240, 320, 4)])
def test_face_stage_standins_vs_oracle(pkg, ort, face, synthetic, standins, fh, fw, fc):
    det_b, lmk_b = standins
    det_m, lmk_m = R.load(det_b), R.load(lmk_b)
    frames = np.stack([synthetic.make_frame(700 + t, fh, fw, fc) for t in range(8)])
    mask_wh = (64, 48)
    with ort.InferenceSession(det_b) as ds, ort.InferenceSession(lmk_b) as ls:
        tr = face.FaceTracker(ds, ls, interval=3)
        cfg = tr.config
        st_exact, st_e2e = F.State(), F.State()
        n_box = n_aff = 0
        for lo, hi in ((0, 4), (4, 8)):  # state carried across calls
            faces = tr.track(frames[lo:hi], mask_wh)
            dets = {}
            for k in range(tr.last_face_count()):
                idx, rec = _check_slot(tr, k, frames[idx_frame(lo, k, 3)], det_m, lmk_m, fw, fh, mask_wh, cfg)
                dets[idx] = rec
            _faces_equal(faces, F.scan(dets, hi - lo, st_exact, fw, fh, 3, cfg.warp_gain), fw, fh, exact=True)

            def run_det(x):
                o = R.run(det_m, {"image": x})
                return o["box_coords"][0], o["box_scores"][0, :, 0]

            def run_lmk(x):
                o = R.run(lmk_m, {"image": x})
                return o["scores"][0], o["landmarks"][0]

            want, _ = F.track(frames[lo:hi], run_det, run_lmk, 256, 192, 192, *mask_wh, st_e2e, interval=3)
            _faces_equal(faces, want, fw, fh, exact=False)
            n_box += sum(f.has_box for f in faces)
            n_aff += sum(f.has_affine for f in faces)
        assert n_box == 3 and n_aff >= 4  # face frames 0, 3, 6 all detect; the matrix carries forward
        tr.close()


def idx_frame(lo, k, interval):
    """Frame (within the whole clip) of the k-th face frame of the call starting at lo."""
    first = (interval - lo % interval) % interval
    return lo + first + k * interval


def test_face_stage_reference_mediapipe_models(pkg, ort, face, synthetic):
    """The reference's own detector and landmark models (re-encoded from
    client/src/assets, tests/golden/mediapipe_*.npz) behind the stage."""
    det_b = M.load_golden(os.path.join(GOLDEN, "mediapipe_face_detector.npz"))[0]
    lmk_b = M.load_golden(os.path.join(GOLDEN, "mediapipe_face_landmarks.npz"))[0]
    det_m, lmk_m = R.load(det_b), R.load(lmk_b)
    frames = np.stack([synthetic.make_frame(900 + t, 480, 640, 3) for t in range(2)])
    with ort.InferenceSession(det_b) as ds, ort.InferenceSession(lmk_b) as ls:
        tr = face.FaceTracker(ds, ls, interval=1)
        faces = tr.track(frames, (256, 144))
        assert tr.last_face_count() == 2
        dets = {}
        for k in range(2):
            idx, rec = _check_slot(tr, k, frames[k], det_m, lmk_m, 640, 480, (256, 144), tr.config)
            dets[idx] = rec
        _faces_equal(faces, F.scan(dets, 2, F.State(), 640, 480, 1, tr.config.warp_gain), 640, 480, exact=True)
        tr.close()


def test_face_stage_device_path_into_post_chain(pkg, ort, face, synthetic, standins):
    """Faces written to HBM by the stage and handed to the post chain
    (vss_post_set_faces_device) == the host path, bit for bit."""
    import torch
    det_b, lmk_b = standins
    fh, fw, n = 120, 160, 6
    frames = np.stack([synthetic.make_frame(700 + t, fh, fw, 3) for t in range(n)])
    with ort.InferenceSession(det_b) as ds, ort.InferenceSession(lmk_b) as ls, \
            pkg.Session(model_h=48, model_w=64, dtype="f32", max_batch=8, autotune=False) as s:
        mask_wh = (s.mask_w, s.mask_h)
        tr = face.FaceTracker(ds, ls, interval=3)
        host_faces = tr.track(frames, mask_wh)
        tr.reset()
        dframes = torch.from_numpy(frames).cuda()
        size = ctypes.sizeof(pkg.FaceFrame)
        dfaces = torch.zeros(n * size, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        tr.track_device(dframes.data_ptr(), n, fh, fw, 3, fw * 3, fh * fw * 3, mask_wh, dfaces.data_ptr(), stream)
        torch.cuda.synchronize()
        assert bytes(dfaces.cpu().numpy()) == bytes((pkg.FaceFrame * n)(*host_faces))
        assert any(f.has_box for f in host_faces) and any(f.has_affine for f in host_faces)
        chain = pkg.PostChain(s)
        chain.set_faces(host_faces)
        a1, u1, _, _ = chain.segment(frames)
        chain.reset()
        chain.set_faces_device(dfaces.data_ptr(), n)
        a2, u2, _, _ = chain.segment(frames)
        assert np.array_equal(a1, a2) and np.array_equal(u1, u2)
        chain.reset()
        a3, _, _, _ = chain.segment(frames)  # without faces the chain differs (the stage acted)
        assert not np.array_equal(a1, a3)
        tr.close()


def test_face_stage_validation(pkg, ort, face, standins):
    det_b, lmk_b = standins
    with ort.InferenceSession(det_b) as ds, ort.InferenceSession(lmk_b) as ls:
        with pytest.raises(pkg.VssError, match="box_coords|input"):
            face.FaceTracker(ls, ds)  # sessions swapped
        with pytest.raises(pkg.VssError, match="interval"):
            face.FaceTracker(ds, ls, interval=0)
        with pytest.raises(TypeError):
            face.FaceTracker(ds, ls, bogus=1)
        tr = face.FaceTracker(ds, ls)
        with pytest.raises(pkg.VssError):
            tr.track(np.zeros((2, 8, 8, 2), np.uint8), (16, 16))  # 2 channels
        with pytest.raises(pkg.VssError):
            tr.track(np.zeros((2, 8, 8, 3), np.uint8), (0, 16))
        assert tr.track(np.zeros((0, 8, 8, 3), np.uint8), (16, 16)) == []
        tr.close()
