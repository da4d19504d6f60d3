"""GPU parity of the batched PoseInertialOptimizationLastKeyFrame (openmavis_amd/csrc/pose.hip) against
the CPU oracle (oracle/ba_oracle.cpp, Optimizer.cc:5021-5578).

Bar (floating point, north star 1e-5 relative): the final frame state within 1e-7 of the oracle's
(rotation in degrees, translation / velocity in m, m/s: both restate the same Gauss-Newton with the same
per-edge arithmetic; only the order of the normal-equation sums differs), the marginal Hessian within
1e-6 relative, Frame::mvbOutlier and the return value identical (a flag may only differ on an edge whose
chi2 sits within 1e-4 of its threshold — none do on these seeds, so the test demands equality).
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
    for k in synth_pose.INPUT_KEYS:
        arrays[k] = torch.from_numpy(np.ascontiguousarray(b[k])).to(dev)
    F, cap = int(b["n_frames"]), int(b["kp_cap"])
    kpo = torch.full((F, cap), 255, dtype=torch.uint8, device=dev)
    H = torch.zeros((F, 225), dtype=torch.float64, device=dev)
    opt = PoseInertialOptimizer(max_frames=F, max_edges=max(len(b["mono_cam"]), len(b["stereo_cam"]), 1))
    opt.set_mode(*mode)
    n_good = opt.PoseInertialOptimizationLastKeyFrame(b, arrays, kpo, H, bRecInit=rec_init)
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
    assert np.abs(H_g - H_o).max() <= 1e-6 * np.abs(H_o).max()


def _check(b, o, rec_init=False):
    for mode in MODES:
        _compare(b, _run_gpu(b, rec_init, mode), o)


@pytest.mark.parametrize("seed,outliers,stereo,pinhole",
                         [(1, 0.1, 0.0, False), (2, 0.25, 0.0, False), (4, 0.1, 0.5, False), (5, 0.1, 0.0, True),
                          (6, 0.1, 0.5, True)])
def test_pose_inertial_last_kf_matches_oracle(oracle, seed, outliers, stereo, pinhole):
    """pinhole: a Pinhole rig (configs[3]'s camera model, Pinhole::project / projectJac in the edges)."""
    b = synth_pose.make_pose_batch(n_frames=12, n_pts=300, seed=seed, outlier_frac=outliers, stereo_frac=stereo,
                                   pinhole=pinhole)
    _check(b, oracle.pose_last_kf(b))


@pytest.mark.parametrize("rec_init", [False, True])
def test_pose_few_inliers(oracle, rec_init):
    """< 30 inliers: the recover pass (or not, with bRecInit)."""
    b = synth_pose.make_pose_batch(n_frames=4, n_pts=40, seed=3, outlier_frac=0.5)
    _check(b, oracle.pose_last_kf(b, rec_init), rec_init)


def test_pose_tiny_frame(oracle):
    """Fewer than 10 edges in the graph: the reference stops after the first round."""
    b = synth_pose.make_pose_batch(n_frames=3, n_pts=5, seed=5, outlier_frac=0.0)
    _check(b, oracle.pose_last_kf(b))


def test_pose_single_frame(oracle):
    """Tracking's call: ONE frame (1,000 matched keypoints, 30 % with a stereo edge on the same keypoint), every path."""
    b = synth_pose.make_pose_batch(n_frames=1, n_pts=1000, seed=7, stereo_frac=0.3)
    _check(b, oracle.pose_last_kf(b))


def test_grouped_capacity_is_reported():
    """More visual edges in one workgroup's keypoint range than its LDS holds: the frame is reported (n_good -1,
    OMV_ERR_CAPACITY), never silently truncated."""
    import torch
    from openmavis_amd import _lib
    b = synth_pose.make_pose_batch(n_frames=1, n_pts=1100, seed=8)
    dev = "cuda:0"
    arrays = {k: torch.tensor(np.asarray(b[k], np.float64), device=dev).contiguous() for k in synth_pose.STATE_KEYS}
    for k in synth_pose.INPUT_KEYS:
        arrays[k] = torch.from_numpy(np.ascontiguousarray(b[k])).to(dev)
    kpo = torch.zeros((1, int(b["kp_cap"])), dtype=torch.uint8, device=dev)
    opt = PoseInertialOptimizer(max_frames=1, max_edges=len(b["mono_cam"])).set_mode(PoseInertialOptimizer.GROUPED, 1)
    n_good = opt.PoseInertialOptimizationLastKeyFrame(b, arrays, kpo)
    torch.cuda.synchronize()
    assert int(n_good.cpu()[0]) == -1
    assert opt.last_error() == _lib.OMV_ERR_CAPACITY
    assert opt.last_error() == 0   # read resets it


def test_auto_mode_heavy_frame_among_light_ones(oracle):
    """AUTO over frames of very different sizes (15 light frames and one of ~2,500 edges): the grouped kernel's part
    count is sized so that no frame overflows a part, and every frame matches the oracle."""
    from openmavis_amd.synth_pose import concat_batches
    light = synth_pose.make_pose_batch(n_frames=15, n_pts=40, seed=9)
    heavy = synth_pose.make_pose_batch(n_frames=1, n_pts=2500, seed=10)
    b = concat_batches(light, heavy)
    assert np.diff(b["mono_start"]).max() > 1024 * 2
    o = oracle.pose_last_kf(b)
    _compare(b, _run_gpu(b), o)
