"""CPU checks of the SearchForTriangulation restatement (oracle/tri_oracle.cpp; ORBmatcher.cc:1131-1456,
KannalaBrandt8.cpp:96-126, 219-229, 319-429, Eigen::JacobiSVD<Matrix4f>).  The reference holds no
fixtures for these (parity unpinned vs OpenCV/Eigen); these pin the restatement's behaviour, and
tools/check_tanf.c pins the std::tan(float) it depends on against glibc (exhaustive)."""
import numpy as np
import pytest

from openmavis_amd import synth_ba, synth_tri


def test_unproject_inverts_project(oracle):
    cams, _, _ = synth_ba.rig()
    rng = np.random.default_rng(0)
    for c in range(4):
        for _ in range(200):
            X = rng.normal(0, 1, 3)
            X[2] = abs(X[2]) + 0.5
            uv = synth_ba.kb8_project(cams[c].astype(np.float64), X)
            r = oracle.kb8_unproject(cams[c], np.float32(uv[0]), np.float32(uv[1]))
            assert r[2] == 1.0
            assert np.allclose(r[:2], X[:2] / X[2], rtol=2e-4, atol=2e-5)


def test_jacobi_svd_is_an_svd(oracle):
    rng = np.random.default_rng(1)
    for _ in range(200):
        A = rng.normal(0, 1, (4, 4)).astype(np.float32) * rng.choice([1e-3, 1.0, 1e3])
        V = oracle.jacobi_svd4_v(A).astype(np.float64)
        assert np.abs(V.T @ V - np.eye(4)).max() < 2e-6
        s_ref = np.linalg.svd(A.astype(np.float64), compute_uv=False)
        s = np.linalg.norm(A.astype(np.float64) @ V, axis=0)
        assert np.allclose(s, s_ref, rtol=1e-5, atol=1e-6 * s_ref[0])
        assert (np.diff(s) <= 1e-6 * s_ref[0]).all()   # descending


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_matches_are_true_correspondences(oracle, seed):
    p = synth_tri.make_tri_pair(seed=seed)
    n, m = oracle.search_for_triangulation(p)
    k1, k2 = p["kf1"], p["kf2"]
    i = np.nonzero(m >= 0)[0]
    assert n == len(i) > 100
    assert ((k1["pt"][i] == k2["pt"][m[i]]) & (k1["pt"][i] >= 0)).mean() > 0.98
    assert not k1["has_mp"][i].any() and not k2["has_mp"][m[i]].any()
    # bCoarse skips the epipolar test: a superset of candidates reaches the best-distance scan
    nc, _ = oracle.search_for_triangulation(p, coarse=True)
    assert nc >= n
    # bOnlyStereo on multi-camera keyframes: bStereo is false for every keypoint (ORBmatcher.cc:1214)
    assert oracle.search_for_triangulation(p, only_stereo=True)[0] == 0


def test_orientation_histogram_keeps_top_bins(oracle):
    p = synth_tri.make_tri_pair(seed=4)
    n, m = oracle.search_for_triangulation(p)
    no, mo = oracle.search_for_triangulation(p, check_ori=True)
    assert no <= n and ((mo < 0) | (mo == m)).all()


def test_eigen_inverse3_is_an_inverse(oracle):
    """Eigen's cofactor 3x3 inverse restated; on a camera matrix K the (2, 2) entry is (fx fy) * (1 / (fx fy)),
    not exactly 1, as Eigen computes it."""
    rng = np.random.default_rng(5)
    for _ in range(100):
        A = rng.normal(0, 1, (3, 3)).astype(np.float32) + 3 * np.eye(3, dtype=np.float32)
        Ai = oracle.eigen_inverse3(A).astype(np.float64)
        assert np.abs(Ai @ A.astype(np.float64) - np.eye(3)).max() < 1e-5
    K = np.array([[347.3, 0, 361.2], [0, 348.9, 271.7], [0, 0, 1]], np.float32)
    Ki = oracle.eigen_inverse3(K)
    fxfy = np.float32(K[0, 0] * K[1, 1])
    assert Ki[2, 2] == np.float32(fxfy * (np.float32(1) / fxfy))
    assert Ki[0, 0] == np.float32(K[1, 1] * (np.float32(1) / fxfy))


def test_pinhole_epipolar_accepts_true_pairs(oracle):
    """Pinhole::epipolarConstrain: projections of one world point pass (dsqr ~ 0 < 3.84 sigma2), a point moved off the
    epipolar line by > 2 sigma fails; a zero-length line (den == 0) is rejected."""
    rng = np.random.default_rng(6)
    k1 = np.array([350.0, 351.0, 360.0, 270.0], np.float32)
    k2 = np.array([340.0, 342.0, 355.0, 265.0], np.float32)
    a = np.deg2rad(10.0)
    R12 = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]], np.float32)
    t12 = np.array([0.3, 0.02, 0.05], np.float32)
    kp = lambda u, v: np.array([(u, v, 31.0, 0.0, 1.0, 0)], synth_tri_kp_dtype())
    n_ok = n_off = 0
    for _ in range(200):
        X2 = np.array([rng.uniform(-2, 2), rng.uniform(-2, 2), rng.uniform(3, 20)])
        X1 = R12.astype(np.float64) @ X2 + t12
        u1 = k1[0] * X1[0] / X1[2] + k1[2]
        v1 = k1[1] * X1[1] / X1[2] + k1[3]
        u2 = k2[0] * X2[0] / X2[2] + k2[2]
        v2 = k2[1] * X2[1] / X2[2] + k2[3]
        n_ok += oracle.pinhole_epipolar(k1, k2, kp(u1, v1), kp(u2, v2), R12, t12, 1.0)
        # moved 10 px across the (near-horizontal) epipolar lines of this baseline
        n_off += oracle.pinhole_epipolar(k1, k2, kp(u1, v1), kp(u2, v2 + 10.0), R12, t12, 1.0)
    assert n_ok == 200 and n_off < 10
    assert not oracle.pinhole_epipolar(k1, k2, kp(360.0, 270.0), kp(100.0, 100.0), np.eye(3, dtype=np.float32),
                                       np.zeros(3, np.float32), 1.0)   # t12 = 0: F12 = 0, den == 0


def synth_tri_kp_dtype():
    return np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])


@pytest.mark.parametrize("model", ["pinhole", ["pinhole", "kb8", "kb8", "pinhole"]])
def test_pinhole_rig_matches_are_true_correspondences(oracle, model):
    p = synth_tri.make_tri_pair(seed=7, n_pts=600, model=model)
    n, m = oracle.search_for_triangulation(p)
    k1, k2 = p["kf1"], p["kf2"]
    i = np.nonzero(m >= 0)[0]
    assert n == len(i) > 100
    assert ((k1["pt"][i] == k2["pt"][m[i]]) & (k1["pt"][i] >= 0)).mean() > 0.95
