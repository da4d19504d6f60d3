"""GPU parity of the batched PoseInertialOptimizationLastFrame and the ConstraintPoseImu ctor
(openmavis_amd/csrc/pose.hip) against the CPU oracle (oracle/ba_oracle.cpp, Optimizer.cc:5580-6170,
G2oTypes.h:639-659).

Bar (floating point, north star 1e-5 relative): the final frame state within 1e-7 of the oracle's (rotation
in degrees, translation / velocity / biases in m, m/s: both restate the same Gauss-Newton with the same
per-edge arithmetic; the visual sums are reduced in a different order), the marginalised Hessian within
1e-6 relative to its largest entry, Frame::mvbOutlier and the return value identical, and the
ConstraintPoseImu projection within 1e-9 relative (Jacobi eigen-decompositions on both sides: the oracle's cyclic
rotation order, the device's parallel round-robin order, equal up to rounding).
"""
import numpy as np
import pytest

from openmavis_amd import synth_ba, synth_pose
from openmavis_amd.optimizer import PoseInertialOptimizer

pytestmark = pytest.mark.gpu


# kernel paths: one workgroup per frame; the grouped (latency) kernel with its automatic part count, 3 parts, and 8
# parts (parts with few or no edges)
MODES = [(PoseInertialOptimizer.BATCH, 0), (PoseInertialOptimizer.GROUPED, 0), (PoseInertialOptimizer.GROUPED, 3),
         (PoseInertialOptimizer.GROUPED, 8)]


def _run_gpu(b, rec_init=False, mode=(PoseInertialOptimizer.AUTO, 0)):
    import torch
    dev = "cuda:0"
    arrays = {}
    for k in synth_pose.STATE_KEYS:
        arrays[k] = torch.tensor(np.asarray(b[k], np.float64), device=dev).contiguous()
    for k in synth_pose.INPUT_KEYS + synth_pose.PRIOR_KEYS:
        arrays[k] = torch.from_numpy(np.ascontiguousarray(b[k])).to(dev)
    F, cap = int(b["n_frames"]), int(b["kp_cap"])
    kpo = torch.full((F, cap), 255, dtype=torch.uint8, device=dev)
    H = torch.zeros((F, 225), dtype=torch.float64, device=dev)
    opt = PoseInertialOptimizer(max_frames=F, max_edges=max(len(b["mono_cam"]), len(b["stereo_cam"]), 1))
    opt.set_mode(*mode)
    n_good = opt.PoseInertialOptimizationLastFrame(b, arrays, kpo, H, bRecInit=rec_init)
    torch.cuda.synchronize()
    assert opt.last_error() == 0
    st = {k: arrays[k].cpu().numpy() for k in synth_pose.STATE_KEYS}
    return st, kpo.cpu().numpy(), n_good.cpu().numpy(), H.cpu().numpy()


def _compare(b, g, o):
    st_g, k_g, n_g, H_g = g
    st_o, k_o, n_o, H_o = o
    assert np.array_equal(n_g, n_o), (n_g, n_o)
    assert np.array_equal(k_g, k_o)
    for f in range(b["n_frames"]):
        ang = np.degrees(np.linalg.norm(synth_ba._log(st_g["Rwb"][f].T @ st_o["Rwb"][f])))
        assert ang < 1e-7, (f, ang)
        for k in ("twb", "vel", "bg", "ba"):
            assert np.abs(st_g[k][f] - st_o[k][f]).max() < 1e-7, (f, k)
        assert np.abs(st_g["tcw"][f] - st_o["tcw"][f]).max() < 1e-7
        assert np.abs(H_g[f] - H_o[f]).max() <= 1e-6 * np.abs(H_o[f]).max(), f


def _check(b, o, rec_init=False):
    for mode in MODES:
        _compare(b, _run_gpu(b, rec_init, mode), o)


@pytest.mark.parametrize("seed,outliers,stereo,pinhole",
                         [(1, 0.1, 0.0, False), (2, 0.25, 0.0, False), (4, 0.1, 0.5, False), (5, 0.1, 0.0, True)])
def test_pose_inertial_last_frame_matches_oracle(oracle, seed, outliers, stereo, pinhole):
    b = synth_pose.make_last_frame_batch(n_frames=12, n_pts=300, seed=seed, outlier_frac=outliers,
                                         stereo_frac=stereo, pinhole=pinhole)
    _check(b, oracle.pose_last_frame(b))


@pytest.mark.parametrize("rec_init", [False, True])
def test_pose_last_frame_few_inliers(oracle, rec_init):
    """< 30 inliers: the recover pass (:6074-6098), or not with bRecInit."""
    b = synth_pose.make_last_frame_batch(n_frames=4, n_pts=40, seed=3, outlier_frac=0.5)
    _check(b, oracle.pose_last_frame(b, rec_init), rec_init)


def test_pose_last_frame_tiny_frame(oracle):
    """Fewer than 10 edges in the graph (5 visual + 4): the reference stops after the first round."""
    b = synth_pose.make_last_frame_batch(n_frames=3, n_pts=5, seed=5, outlier_frac=0.0)
    _check(b, oracle.pose_last_frame(b))


def test_constraint_pose_imu_matches_oracle(oracle):
    """The ConstraintPoseImu projection of marginalised Hessians and of indefinite matrices."""
    import torch
    rng = np.random.default_rng(11)
    b = synth_pose.make_last_frame_batch(n_frames=4, n_pts=200, seed=6)
    H = oracle.pose_last_frame(b)[3]
    M = rng.normal(0, 1, (4, 15, 15))
    ind = (M + np.transpose(M, (0, 2, 1))).reshape(4, 225) * 1e3   # indefinite: negative eigenvalues zeroed
    Hin = np.concatenate([H, ind])
    g = PoseInertialOptimizer.ConstraintPoseImu(torch.from_numpy(Hin).cuda())
    torch.cuda.synchronize()
    o = oracle.pose_constraint(Hin)
    g = g.cpu().numpy()
    for i in range(len(Hin)):
        # the marginalised H is symmetric up to rounding; the reference's SelfAdjointEigenSolver (and the device)
        # read its lower triangle, the oracle's Jacobi the whole matrix: they differ by up to that asymmetry
        Hm = Hin[i].reshape(15, 15)
        asym = np.abs(Hm - Hm.T).max()
        assert np.abs(g[i] - o[i]).max() <= 1e-9 * np.abs(o[i]).max() + asym, i
        Hl = np.tril(Hm) + np.tril(Hm, -1).T
        assert np.abs(g[i].reshape(15, 15) - g[i].reshape(15, 15).T).max() <= 1e-9 * np.abs(o[i]).max(), i
        if np.linalg.eigvalsh(Hl).min() > 1e-6 * np.abs(Hl).max():   # positive definite: the lower half, unchanged
            assert np.abs(g[i] - Hl.reshape(-1)).max() <= 1e-9 * np.abs(o[i]).max(), i
    # in place (H_out aliasing H_in)
    t = torch.from_numpy(Hin).cuda()
    PoseInertialOptimizer.ConstraintPoseImu(t, out=t)
    torch.cuda.synchronize()
    assert np.abs(t.cpu().numpy() - g).max() == 0


def test_pose_last_frame_single_frame(oracle):
    """Tracking's call: ONE frame (1,000 matched keypoints, 30 % with a stereo edge on the same keypoint), every path."""
    b = synth_pose.make_last_frame_batch(n_frames=1, n_pts=1000, seed=7, stereo_frac=0.3)
    _check(b, oracle.pose_last_frame(b))
