"""CPU tests of the face-stage oracle (oracle/face_ref.py, §8(f) row 4),
pinned by tests/golden/face_geom.npz — vectors produced by the reference's own
cropFaceROI / runLandmarks468 / estimateAffineFromLandmarks / toSquareLetterbox
(frameProcessorTest.ts:451-642) and main.ts's lastAffine update (:79-89) run
under Node (tests/golden/make_face_golden.py).

Bar: bit-exact for the ROI rectangles, the landmark points and scores, the
letterbox mapping and the blend; the affine within 1e-14 relative (atan2 / cos /
sin of V8 and of the C library may differ in the last ulp)."""
import json
import os

import numpy as np
import pytest

import face_ref as F

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLDEN, "face_geom.npz"), allow_pickle=False)


def _cases(g):
    return json.loads(str(g["cases"]))


def test_crop_roi_matches_reference(g):
    for c, roi in zip(_cases(g)["affine"], g["roi"]):
        assert F.crop_roi(*c["box"], *c["video"], 0.25) == tuple(roi), c


def test_landmark_points_and_affine_match_reference(g):
    cs = _cases(g)["affine"]
    lm_all = g["landmarks"]
    n_aff = 0
    for k, c in enumerate(cs):
        lm = lm_all[c["lm_off"]:c["lm_off"] + c["num"] * 3].reshape(c["num"], 3)
        assert float(np.float32(c["score"])) == g["score"][k]
        d = np.zeros(F.D_COUNT)
        d[6:10] = g["roi"][k]
        if c["num"] >= 300:  # runLandmarks468's ROI-pixel points (:494-498)
            rw, rh = g["roi"][k][2], g["roi"][k][3]
            pts = [(float(lm[i, 0]) * rw, float(lm[i, 1]) * rh) for i in F.IDXS]
            assert np.array_equal(np.array(pts), g["points"][k])
        vw, vh = c["video"]
        mw, mh = c["mask"]
        r = F.estimate_affine(d, g["score"][k], lm, vw, vh, mw, mh)
        assert bool(r[10]) == bool(g["has_affine"][k]), k
        if r[10]:
            n_aff += 1
            np.testing.assert_allclose(r[11:17], g["affine"][k], rtol=1e-14, atol=1e-12)
    # the golden set holds both outcomes: matrices, and the reference's nulls
    # (score < 0.3, < 300 points, coincident anchors)
    assert 0 < n_aff < len(cs)
    assert not g["has_affine"][5] and not g["has_affine"][7]


def test_letterbox_mapping_matches_reference(g):
    for c, want in zip(_cases(g)["letterbox"], g["letterbox"]):
        geom = F.letterbox_geometry(c["target"], *c["src"])
        got = [F.map_from_square(geom, x, y) for x, y in c["pts"]]
        assert np.array_equal(np.array(got), want), c["src"]


def test_blend_matches_reference(g):
    for c, want in zip(_cases(g)["blend"], g["blend"]):
        assert np.array_equal(np.array(F.blend(c["last"], c["m"], 0.7)), want)


def test_letterbox_geometry_shapes():
    # toSquareLetterbox keeps the aspect ratio inside the square, centred
    for w, h in [(640, 480), (480, 640), (1920, 1080), (1, 1), (3, 1000)]:
        scale, dw, dh, ox, oy = F.letterbox_geometry(256, w, h)
        assert max(dw, dh) == 256 and 1 <= min(dw, dh) <= 256
        assert ox == (256 - dw) // 2 and oy == (256 - dh) // 2


def test_decode_first_best_and_thresholds():
    A = 896
    scores = np.full(A, -5.0, np.float32)
    scores[[40, 700]] = 0.9  # a tie: the first index wins (strict >, :418)
    scores[12] = np.nan      # never wins
    coords = np.zeros((A, 16), np.float32)
    coords[40, :4] = (0.25, 0.3, 0.5, 0.6)
    coords[700, :4] = (0.6, 0.6, 0.7, 0.7)
    d = F.decode(coords, scores, 256, 640, 480)
    geom = F.letterbox_geometry(256, 640, 480)
    x0, y0 = F.map_from_square(geom, float(np.float32(0.25)) * 256, float(np.float32(0.3)) * 256)
    assert d[0] == 1 and d[2] == x0 and d[3] == y0
    assert d[8] > 0  # 0.9 >= 0.6: a ROI
    low = F.decode(coords, np.where(scores > 0, np.float32(0.5), scores), 256, 640, 480)
    assert low[0] == 1 and low[8] == 0  # detected, below FACE_SCORE_THRESH: no ROI / prior
    coords[40, :4] = (0.5, 0.3, 0.25, 0.6)  # x1 <= x0: no detection (:445)
    assert F.decode(coords, scores, 256, 640, 480)[0] == 0
    assert F.decode(coords, np.full(A, np.nan, np.float32), 256, 640, 480)[0] == 0
