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
