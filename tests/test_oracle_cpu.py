"""CPU tests of the oracle (test infrastructure): known-answer constants of the reference
extractor, the committed golden fixtures, and matcher semantics."""
import hashlib
import math
import os

import numpy as np
import pytest

from openmavis_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_quota_and_umax_kats(oracle):
    # per-level quotas (ORBextractor.cc:380-391) at the BASELINE configs
    assert list(oracle.orb_tables(1200)["quota"]) == [261, 217, 181, 151, 126, 105, 87, 72]
    assert list(oracle.orb_tables(1000)["quota"]) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(oracle.orb_tables(2000)["quota"]) == [434, 362, 302, 251, 209, 175, 145, 122]
    assert list(oracle.orb_tables(500)["quota"]) == [109, 90, 75, 63, 52, 44, 36, 31]
    # circular patch rows (ORBextractor.cc:399-413)
    assert list(oracle.orb_tables(1200)["umax"]) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    sc = oracle.orb_tables(1200)["scale"]
    assert sc[0] == 1.0 and abs(sc[7] - 1.2 ** 7) < 1e-5
    # scaled patch sizes (int)(31 * scale)
    assert [int(np.float32(31) * s) for s in sc] == [31, 37, 44, 53, 64, 77, 92, 111]


@pytest.mark.parametrize("w,h,sizes", [
    (720, 540, [(720, 540), (600, 450), (500, 375), (417, 312), (347, 260), (289, 217), (241, 181), (201, 151)]),
    (752, 480, [(752, 480), (627, 400), (522, 333), (435, 278), (363, 231), (302, 193), (252, 161), (210, 134)]),
    (1920, 1080, [(1920, 1080), (1600, 900), (1333, 750), (1111, 625), (926, 521), (772, 434), (643, 362),
                  (536, 301)]),
])
def test_level_geometry_kat(oracle, w, h, sizes):
    img = np.zeros((h, w), np.uint8)
    for l, (lw, lh) in enumerate(sizes):
        assert oracle.pyramid_level(img, l).shape == (lh, lw)


def test_fast_atan2_close_to_atan2(oracle):
    rng = np.random.default_rng(0)
    for y, x in rng.integers(-3_000_000, 3_000_000, (2000, 2)):
        ref = math.degrees(math.atan2(y, x)) % 360.0
        got = oracle.fast_atan2(float(y), float(x))
        d = abs(got - ref)
        assert min(d, 360 - d) < 0.02


def _img_sha(img):
    return hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["orb_hilti_720x540", "orb_euroc_752x480", "orb_side_320x240"])
def test_oracle_matches_golden(oracle, name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    img = synth.synth_image(int(z["seed"]), int(z["w"]), int(z["h"]))
    assert _img_sha(img) == str(z["image_sha256"]), "synthetic image generator changed"
    mono, kps, desc = oracle.orb_extract(img, int(z["nfeatures"]), 1.2, 8, int(z["ini"]), int(z["mn"]),
                                         tuple(z["lapping"]))
    assert mono == int(z["mono"])
    assert np.array_equal(kps.view(np.uint32).reshape(-1, 6), z["kps"])
    assert np.array_equal(desc, z["desc"])


def test_matcher_golden(oracle):
    z = np.load(os.path.join(GOLD, "match_hilti_frame0.npz"))
    kps = z["kps"].view(oracle.KP_DTYPE).reshape(z["kps"].shape[:2])
    desc = z["desc"]
    mono, n_kp = z["mono"], z["n_kp"]
    i2, d2 = oracle.bf_knn2(desc[0, mono[0]:n_kp[0]], desc[1, mono[1]:n_kp[1]])
    assert np.array_equal(i2, z["knn_idx"]) and np.array_equal(d2, z["knn_dist"])
    mp = {k[3:]: z[k] for k in z.files if k.startswith("mp_")}
    g = oracle.frame_geom(5, 720, 540, oracle.orb_tables(1200)["scale"])
    k2m = np.full(z["kp_to_mp"].shape, -1, np.int32)
    n = oracle.search_by_projection(g, kps, desc, n_kp, mp, 6.0, False, 50.0, 0.8, z["l2r"], z["r2l"], None, k2m)
    assert n == int(z["n_matches"]) and np.array_equal(k2m, z["kp_to_mp"])


def test_knn_ties_first_index_wins(oracle):
    a = np.zeros((1, 32), np.uint8)
    t = np.zeros((4, 32), np.uint8)
    t[0, 0] = 1          # dist 1
    t[2, 0] = 1          # dist 1 (tie, later)
    t[1, :] = 255        # dist 256
    t[3, 1] = 3          # dist 2
    i2, d2 = oracle.bf_knn2(a, t)
    assert list(i2[0]) == [0, 2] and list(d2[0]) == [1, 1]
    i2, d2 = oracle.bf_knn2(a, t[:1])
    assert list(i2[0]) == [0, -1] and d2[0, 1] == 2 ** 31 - 1


def test_grid_excludes_right_border_and_keeps_order(oracle):
    # PosInGrid rounds (x - minX) * 64 / 720: x > 714.375 lands in column 64 -> not in the grid
    kp = np.zeros((1, 4), oracle.KP_DTYPE)
    kp[0, 0] = (719.0, 10.0, 31, 0, 20, 0)
    kp[0, 1] = (5.0, 5.0, 31, 0, 20, 0)
    kp[0, 2] = (5.2, 5.1, 31, 0, 20, 1)
    kp[0, 3] = (714.0, 10.0, 31, 0, 20, 0)
    g = oracle.frame_geom(1, 720, 540, oracle.orb_tables(1200)["scale"])
    cs, idx = oracle.grid(g, kp, np.array([4], np.int32), 0)
    assert cs[-1] == 3 and 0 not in idx
    c = 0 * 48 + 0
    assert list(idx[cs[c]:cs[c + 1]]) == [1, 2]
    # window: square, strict |dx| < r, level filter [minLevel, maxLevel]
    assert list(oracle.features_in_area(g, kp, np.array([4], np.int32), 5.0, 5.0, 0.5, 0, 0, 0)) == [1]
    assert list(oracle.features_in_area(g, kp, np.array([4], np.int32), 5.0, 5.0, 0.5, -1, 1, 0)) == [1, 2]


def test_map_point_generator_is_seeded():
    imgs = synth.hilti_frame(0)
    assert imgs.shape == (5, 540, 720) and imgs.dtype == np.uint8
    kps = np.zeros((5, 10), [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                             ("response", "<f4"), ("octave", "<i4")])
    desc = np.random.default_rng(0).integers(0, 256, (5, 10, 32), dtype=np.uint8)
    a = synth.make_map_points(kps, desc, np.full(5, 10), 100, 9, 720, 540)
    b = synth.make_map_points(kps, desc, np.full(5, 10), 100, 9, 720, 540)
    for k in a:
        assert np.array_equal(a[k], b[k])
    assert (a["in_view"].sum(1) >= 1).all()


def test_frustum_oracle_kats(oracle):
    """Frame::isInFrustum restatement: a point on block 0's optical axis projects to the principal
    point; the distance-invariance window, the viewing-cosine limit, negative depth and PredictScale's
    ceil(log(ratio)/log(1.2)) behave as in src/Frame.cc:1529-1653 / src/MapPoint.cc:624-637."""
    import numpy as np
    from openmavis_amd import synth
    from openmavis_amd.matcher import make_rig
    cams, R_cl, t_cl = synth.hilti_rig(2)
    rig = make_rig(cams, R_cl, t_cl, 720, 540)
    I = np.eye(3, dtype=np.float32).reshape(-1)
    pose = np.concatenate([I, np.zeros(3), I, np.zeros(3)]).astype(np.float32)
    pos = np.array([[0, 0, 5], [0, 0, 5], [0, 0, 5], [0, 0, -5], [0, 0, 5]], np.float32)
    normal = np.array([[0, 0, 1], [0, 0, 1], [1, 0, 0], [0, 0, -1], [0, 0, 1]], np.float32)
    maxd = np.array([5 * 1.2 ** 2 * 0.9, 3.0, 10, 10, 5 * 1.2 ** 9], np.float32)   # #1: 5 > 1.2 * 3
    mind = maxd / np.float32(1.2 ** 7)
    mind[4] = 1.0
    out, n = oracle.frustum(rig, pose, pos, normal, mind, maxd, 0.5)
    assert out["in_view"][0, 0] == 1 and out["level"][0, 0] == 2
    assert abs(out["proj_x"][0, 0] - cams[0][2]) < 1e-3 and abs(out["proj_y"][0, 0] - cams[0][3]) < 1e-3
    assert out["track_depth"][0] == np.float32(5.0)
    assert out["in_view"][1, 0] == 0 and out["level"][1, 0] == -1 and out["proj_x"][1, 0] == -1   # too far
    assert out["in_view"][2, 0] == 0                                                             # viewCos 0
    assert out["in_view"][3].sum() == 0                                                          # behind
    assert out["level"][4, 0] == 7                                                               # clamped
    assert n == int((out["in_view"].sum(1) > 0).sum())


# ---- keyframe-side projection searches (ORBmatcher::Fuse / SearchByProjection(KF...) restatement) -------
def test_kf_search_oracle_recovers_true_keypoints(oracle):
    """Points derived from a keypoint of the job's block are matched back to that keypoint (or an
    equivalent one at distance <= the derived one) by Fuse; claim modes never assign a keypoint twice."""
    from openmavis_amd import synth_kfmatch as sk
    b = sk.make_kf_search(0, seed=5)
    bi, bd, nm, _ = oracle.search_kf(b, *sk.MODE_PARAMS[0])
    assert nm.sum() > 0.4 * len(bi)
    acc = (bi >= 0) & (bd <= 50)
    assert (nm == [int(acc[j["mp_start"]:j["mp_start"] + j["mp_count"]].sum()) for j in b["jobs"]]).all()
    for mode in (2, 3):
        b = sk.make_kf_search(mode, seed=5)
        bi, bd, nm, km = oracle.search_kf(b, *sk.MODE_PARAMS[mode])
        claimed = km[km != b["kp_match"]]
        assert (claimed >= 0).all() and len(claimed) == nm.sum()
        for jb in b["jobs"]:   # one keypoint per point, no keypoint twice within a keyframe
            sl = bi[jb["mp_start"]:jb["mp_start"] + jb["mp_count"]]
            sl = sl[sl >= 0]
            assert len(np.unique(sl)) == len(sl)


def test_harris_oracle_matches_numpy(oracle):
    """The oracle's OpenCV ORB HarrisResponses restatement (C, float32 at the end) against an independent numpy form of
    the published formula (Sobel-like 3x3 gradients, 7x7 sums in int64, response in float64): the integer sums agree
    exactly, so the float32 responses agree to float32 rounding of a few operations."""
    img = synth.synth_image(31, 200, 160)
    rng = np.random.default_rng(3)
    xs = rng.integers(5, 195, 300).astype(np.int32)
    ys = rng.integers(5, 155, 300).astype(np.int32)
    got = oracle.harris_responses(img, xs, ys)
    I = img.astype(np.int64)
    Ix = (I[1:-1, 2:] - I[1:-1, :-2]) * 2 + (I[:-2, 2:] - I[:-2, :-2]) + (I[2:, 2:] - I[2:, :-2])
    Iy = (I[2:, 1:-1] - I[:-2, 1:-1]) * 2 + (I[2:, :-2] - I[:-2, :-2]) + (I[2:, 2:] - I[:-2, 2:])
    ref = np.zeros(len(xs))
    scale = 1.0 / (4 * 7 * 255.0)
    for q, (x, y) in enumerate(zip(xs, ys)):
        gx = Ix[y - 4:y + 3, x - 4:x + 3]   # interior index = pixel - 1
        gy = Iy[y - 4:y + 3, x - 4:x + 3]
        a, b, c = int((gx * gx).sum()), int((gy * gy).sum()), int((gx * gy).sum())
        ref[q] = (float(a) * b - float(c) * c - 0.04 * (float(a) + b) ** 2) * scale ** 4
    assert np.allclose(got, ref, rtol=2e-6, atol=1e-12), np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-12))
    assert (np.abs(ref) > 0).mean() > 0.9
