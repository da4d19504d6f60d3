"""CPU checks of the PoseInertialOptimizationLastKeyFrame restatement (oracle/ba_oracle.cpp,
Optimizer.cc:5021-5578) on seeded synthetic frames (openmavis_amd/synth_pose.py).  The reference's
tests hold no fixtures for this function (parity unpinned vs g2o/Eigen); these pin behaviour."""
import numpy as np
import pytest

from openmavis_amd import synth_ba, synth_pose


@pytest.fixture(scope="module")
def batch():
    return synth_pose.make_pose_batch(n_frames=6, n_pts=300, seed=1, outlier_frac=0.1)


def _rot_deg(Ra, Rb):
    return np.degrees(np.linalg.norm(synth_ba._log(Ra.T @ Rb)))


def test_recovers_true_state_and_flags_outliers(batch, oracle):
    st, kpo, n_good, H = oracle.pose_last_kf(batch)
    for f in range(batch["n_frames"]):
        assert _rot_deg(st["Rwb"][f], batch["true_Rwb"][f]) < 0.01
        assert np.linalg.norm(st["twb"][f] - batch["true_twb"][f]) < 2e-3
        m0, m1 = batch["mono_start"][f], batch["mono_start"][f + 1]
        truth = batch["mono_is_outlier"][m0:m1]
        flags = kpo[f, batch["mono_kp"][m0:m1]].astype(bool)
        assert (flags & truth).sum() >= 0.9 * truth.sum()       # planted outliers are found
        assert (flags & ~truth).sum() <= 0.03 * (~truth).sum()   # few inliers rejected
        assert n_good[f] == (m1 - m0) - flags.sum()
        # camera poses follow the body pose (ImuCamPose::Update)
        Rbw = st["Rwb"][f].T
        for c in range(batch["n_cams"]):
            assert np.allclose(st["Rcw"][f, c], batch["Rcb"][c] @ Rbw, atol=1e-12)


def test_marginal_hessian_is_symmetric_positive(batch, oracle):
    _, _, _, H = oracle.pose_last_kf(batch)
    for f in range(batch["n_frames"]):
        h = H[f].reshape(15, 15)
        assert np.allclose(h, h.T, rtol=1e-12, atol=1e-9)
        assert np.linalg.eigvalsh(h).min() > 0


def test_few_inliers_recover_pass(oracle):
    """With < 30 inliers the reference re-admits edges with chi2 < 18 (:5503-5526) unless bRecInit."""
    b = synth_pose.make_pose_batch(n_frames=2, n_pts=40, seed=3, outlier_frac=0.5)
    _, k_rec, n_rec, _ = oracle.pose_last_kf(b, rec_init=False)
    _, k_no, n_no, _ = oracle.pose_last_kf(b, rec_init=True)
    assert (n_rec >= n_no).all()
    assert (k_rec[:, :40].sum(1) <= k_no[:, :40].sum(1)).all()


@pytest.fixture(scope="module")
def lf_batch():
    return synth_pose.make_last_frame_batch(n_frames=6, n_pts=300, seed=1, outlier_frac=0.1)


def test_last_frame_recovers_state_and_flags_outliers(lf_batch, oracle):
    """PoseInertialOptimizationLastFrame (Optimizer.cc:5580-6170): pose / velocity pulled to the truth,
    planted outliers found, the return value nInitialCorrespondences - nBad."""
    b = lf_batch
    st, kpo, n_good, _ = oracle.pose_last_frame(b)
    for f in range(b["n_frames"]):
        assert _rot_deg(b["Rwb"][f], b["true_Rwb"][f]) > 0.4
        assert _rot_deg(st["Rwb"][f], b["true_Rwb"][f]) < 0.05
        assert np.linalg.norm(st["twb"][f] - b["true_twb"][f]) < 1e-2
        m0, m1 = b["mono_start"][f], b["mono_start"][f + 1]
        truth = b["mono_is_outlier"][m0:m1]
        flags = kpo[f, b["mono_kp"][m0:m1]].astype(bool)
        assert (flags & truth).sum() >= 0.9 * truth.sum()
        assert (flags & ~truth).sum() <= 0.05 * (~truth).sum()
        assert n_good[f] == (m1 - m0) - flags.sum()


def test_last_frame_prior_pulls_previous_frame(oracle):
    """A stiffer EdgePriorPoseImu makes the frame's estimate follow the prior more: with the prior
    information scaled up 1e4 the result moves towards what the prior implies, and the marginal
    Hessian (the next frame's prior) grows."""
    b = synth_pose.make_last_frame_batch(n_frames=3, n_pts=60, seed=8, outlier_frac=0.0)
    _, _, _, H1 = oracle.pose_last_frame(b)
    b2 = dict(b)
    b2["prior_H"] = b["prior_H"] * 1e4
    _, _, _, H2 = oracle.pose_last_frame(b2)
    for f in range(3):
        assert np.trace(H2[f].reshape(15, 15)) > np.trace(H1[f].reshape(15, 15))


def test_marginalised_hessian_and_constraint(lf_batch, oracle):
    """Marginalize(H, 0, 14) is a Schur complement of a PSD matrix (PSD, symmetric to rounding); the
    ConstraintPoseImu ctor leaves a PSD matrix unchanged to rounding and zeroes negative eigenvalues."""
    _, _, _, H = oracle.pose_last_frame(lf_batch)
    for f in range(lf_batch["n_frames"]):
        h = H[f].reshape(15, 15)
        assert np.abs(h - h.T).max() <= 1e-7 * np.abs(h).max()
        assert np.linalg.eigvalsh((h + h.T) / 2).min() > 0
    Hc = oracle.pose_constraint(H)
    assert np.abs(Hc - H).max() <= 1e-7 * np.abs(H).max()
    rng = np.random.default_rng(3)
    M = rng.normal(0, 1, (15, 15))
    S = M + M.T
    P = oracle.pose_constraint(S.reshape(1, 225))[0].reshape(15, 15)
    w, V = np.linalg.eigh(S)
    ref = (V * np.where(w < 1e-12, 0, w)) @ V.T
    assert np.abs(P - ref).max() < 1e-10


def test_last_frame_few_edges_stop_after_first_round(oracle):
    """optimizer.edges().size() < 10 (:6069): 5 visual edges + 4 break after the first round, so the
    round-0 threshold decides (all rounds use 5.991 here; the recover pass then re-admits)."""
    b = synth_pose.make_last_frame_batch(n_frames=2, n_pts=5, seed=5, outlier_frac=0.0)
    st, kpo, n_good, _ = oracle.pose_last_frame(b)
    assert (n_good <= 5).all() and (n_good >= 0).all()


def test_stereo_edges_share_the_keypoint_flag(oracle):
    b = synth_pose.make_pose_batch(n_frames=3, n_pts=200, seed=4, outlier_frac=0.1, stereo_frac=0.5)
    assert len(b["stereo_cam"]) > 100
    st, kpo, n_good, _ = oracle.pose_last_kf(b)
    for f in range(3):
        assert _rot_deg(st["Rwb"][f], b["true_Rwb"][f]) < 0.01
        nm = b["mono_start"][f + 1] - b["mono_start"][f]
        ns = b["stereo_start"][f + 1] - b["stereo_start"][f]
        assert 0 < n_good[f] <= nm + ns


def test_edges_from_matches_oracle_recovers_edges(oracle):
    """The edge-loop restatement on a frame laid out from a synthetic batch's edges gives back exactly those edges
    (as a set: keypoint order differs from the batch's), stereo edges only where mvuRight > 0 on an assigned
    keypoint, and nothing for an empty assignment."""
    from test_pose_edges_gpu import INV_SIGMA2, _frame_from_batch
    b = synth_pose.make_pose_batch(n_frames=1, n_pts=300, seed=3, stereo_frac=0.4)
    kps, n_kp, k2m, pos, track, ur = _frame_from_batch(b, 512, np.random.default_rng(3))
    o = oracle.pose_edges_from_matches(kps, n_kp, k2m, pos, track, INV_SIGMA2, ur)

    def key(cam, obs, xw, w):
        return (int(cam), tuple(np.float32(obs).tolist()), tuple(np.float32(xw).tolist()), float(w))
    got = sorted(key(*t) for t in zip(o["mono_cam"], o["mono_obs"], o["mono_xw"], o["mono_inv_sigma2"]))
    want = sorted(key(*t) for t in zip(b["mono_cam"], b["mono_obs"], b["mono_xw"], b["mono_inv_sigma2"]))
    assert got == want
    assert len(o["stereo_cam"]) == len(b["stereo_cam"])
    assert np.all(np.diff(o["mono_kp"]) > 0) and np.all(np.diff(o["stereo_kp"]) > 0)   # slot order
    assert np.array_equal(o["mono_close"].astype(bool), track[k2m[o["mono_kp"]]] < 10)
    e = oracle.pose_edges_from_matches(kps, n_kp, np.full_like(k2m, -1), pos, track, INV_SIGMA2, ur)
    assert e["mono_start"].tolist() == [0, 0] and e["stereo_start"].tolist() == [0, 0]


def test_pose_optimization_oracle_recovers_pose(oracle):
    """oracle_pose_optimization (Optimizer::PoseOptimization restated): from a 0.5 deg / ~5 cm perturbed start the
    estimate lands within 0.05 deg / 1 cm of the true camera-0 pose, and the injected outliers (8-40 px) are exactly
    the keypoints flagged, on the rigid-body (KB8 rig) and the conventional (pinhole stereo) branches."""
    from openmavis_amd import synth_pose
    for kw in (dict(n_cams=4), dict(n_cams=1, stereo_frac=0.5)):
        b = synth_pose.make_pose_only_batch(n_frames=3, n_pts=200, seed=3, **kw)
        pq, pt, kpo, ng = oracle.pose_optimization(b)
        for f in range(3):
            Rt, p = b["true_Rwb"][f], b["true_twb"][f]
            Rc = b["Rcb"][0] @ Rt.T
            tc = b["Rcb"][0] @ (-Rt.T @ p) + b["tcb"][0]
            R = synth_pose.quat_mat(pq[f])
            ang = np.degrees(np.arccos(np.clip((np.trace(R.T @ Rc) - 1) / 2, -1, 1)))
            assert ang < 0.05 and np.linalg.norm(pt[f] - tc) < 0.01
            m0, m1 = b["mono_start"][f], b["mono_start"][f + 1]
            kp = b["mono_kp"][m0:m1]
            assert np.array_equal(kpo[f][kp].astype(bool), b["mono_is_outlier"][m0:m1])
            n_edges = (m1 - m0) + (b["stereo_start"][f + 1] - b["stereo_start"][f])
            assert ng[f] == n_edges - int(kpo[f][np.concatenate([kp, b["stereo_kp"][b["stereo_start"][f]:b["stereo_start"][f + 1]]])].sum())
