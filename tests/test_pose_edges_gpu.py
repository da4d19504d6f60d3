"""GPU parity of omv_pose_edges_from_matches (openmavis_amd/csrc/pose.hip): the visual-edge creation loop of
PoseInertialOptimizationLastKeyFrame / LastFrame (src/Optimizer.cc:5079-5330) on the device, against its CPU
restatement (oracle.pose_edges_from_matches); and the device chain SearchByProjection assignment -> edge lists ->
PoseInertialOptimizationLastFrame against the oracle optimisation of the oracle's edge lists.

Bar: edge lists bit-exact (integer / copied values); the chained optimisation at the pose tests' bar (state
within 1e-7, Hessian within 1e-6 relative, mvbOutlier and the return value identical).
"""
import numpy as np
import pytest

from openmavis_amd import synth_ba, synth_pose
from openmavis_amd.optimizer import PoseInertialOptimizer

pytestmark = pytest.mark.gpu

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])
INV_SIGMA2 = np.array([1.0 / np.float32(1.2) ** (2 * o) for o in range(8)], np.float32)   # as synth_pose


def _frame_from_batch(b, cap, rng, fill=0.35):
    """One multi-camera frame whose map-point assignment reproduces the one-frame batch b's visual edges: each mono
    edge's observation becomes a keypoint of its camera at a random slot (unassigned keypoints in between), its
    world point a map point; stereo edges set mvuRight of their keypoint."""
    C = int(b["n_cams"])
    kps = np.zeros((C, cap), KP_DTYPE)
    n_kp = np.zeros(C, np.int32)
    kp_to_mp = np.full(C * cap, -1, np.int32)
    uright = np.full((C, cap), -1.0, np.float32)
    n = len(b["mono_cam"])
    mp_pos = np.asarray(b["mono_xw"], np.float32).copy()
    close = np.asarray(b["mono_close"]).astype(bool)
    track = np.where(close, rng.uniform(1, 9.9, n), rng.uniform(10, 60, n)).astype(np.float32)
    octv = np.rint(-np.log(b["mono_inv_sigma2"].astype(np.float64)) / (2 * np.log(1.2))).astype(np.int32)
    st = {int(k): j for j, k in enumerate(b["stereo_kp"])}
    for e in range(n):
        c = int(b["mono_cam"][e])
        while rng.random() < fill:   # a keypoint without a map point
            i = n_kp[c]
            kps[c, i] = (rng.uniform(0, 720), rng.uniform(0, 540), 31, 0, 1, rng.integers(0, 8))
            if rng.random() < 0.3:
                uright[c, i] = rng.uniform(1, 700)
            n_kp[c] += 1
        i = n_kp[c]
        kps[c, i] = (b["mono_obs"][e][0], b["mono_obs"][e][1], 31, 0, 1, octv[e])
        kp_to_mp[c * cap + i] = e
        j = st.get(int(b["mono_kp"][e]))
        if j is not None:
            uright[c, i] = np.float32(b["stereo_obs"][j][2])
        n_kp[c] += 1
    assert n_kp.max() <= cap
    return kps, n_kp, kp_to_mp, mp_pos, track, uright


def _device_edges(opt, kps, n_kp, kp_to_mp, mp_pos, track, uright, max_edges):
    import torch
    dev = "cuda:0"
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         dict(kps=kps.view(np.int32).reshape(kps.shape + (6,)), n_kp=n_kp, kp_to_mp=kp_to_mp, mp_pos=mp_pos,
              track=track).items()}
    ur = None if uright is None else torch.from_numpy(uright).to(dev)
    arr = PoseInertialOptimizer.edge_arrays(max_edges, dev)
    opt.EdgesFromMatches(t["kps"], t["n_kp"], t["kp_to_mp"], t["mp_pos"], t["track"], INV_SIGMA2, arr, uright=ur)
    torch.cuda.synchronize()
    return arr


def _compare_edges(arr, o):
    for kind in ("mono", "stereo"):
        n = int(o[f"{kind}_start"][1])
        assert arr[f"{kind}_start"].cpu().numpy().tolist() == [0, n], kind
        for k in ("cam", "kp", "obs", "inv_sigma2", "xw") + (("close",) if kind == "mono" else ()):
            g = arr[f"{kind}_{k}"][:n].cpu().numpy()
            assert np.array_equal(g, o[f"{kind}_{k}"]), (kind, k)


@pytest.mark.parametrize("seed,stereo,with_ur", [(1, 0.0, False), (2, 0.4, True), (3, 0.0, True)])
def test_edges_from_matches_match_oracle(oracle, seed, stereo, with_ur):
    rng = np.random.default_rng(seed)
    b = synth_pose.make_pose_batch(n_frames=1, n_pts=900, seed=seed, stereo_frac=stereo)
    frame = _frame_from_batch(b, 1024, rng)
    kps, n_kp, kp_to_mp, mp_pos, track, uright = frame
    if not with_ur:
        uright = None
    opt = PoseInertialOptimizer(max_frames=1, max_edges=4096)
    arr = _device_edges(opt, kps, n_kp, kp_to_mp, mp_pos, track, uright, 4096)
    o = oracle.pose_edges_from_matches(kps, n_kp, kp_to_mp, mp_pos, track, INV_SIGMA2, uright)
    assert int(o["mono_start"][1]) == len(b["mono_cam"])
    _compare_edges(arr, o)
    assert opt.last_error() == 0


def test_edges_from_matches_edge_cases(oracle):
    """Empty frame (no keypoints), a frame with keypoints but no assignment, and capacity overflow."""
    import torch
    C, cap = 5, 256
    kps = np.zeros((C, cap), KP_DTYPE)
    mp_pos = np.zeros((4, 3), np.float32)
    track = np.zeros(4, np.float32)
    opt = PoseInertialOptimizer(max_frames=1, max_edges=64)
    for n_kp in (np.zeros(C, np.int32), np.full(C, cap, np.int32)):
        arr = _device_edges(opt, kps, n_kp, np.full(C * cap, -1, np.int32), mp_pos, track, None, 64)
        assert arr["mono_start"].cpu().tolist() == [0, 0] and arr["stereo_start"].cpu().tolist() == [0, 0]
    assert opt.last_error() == 0
    # 100 assigned keypoints into 64-edge buffers: the first 64 in slot order, OMV_ERR_CAPACITY raised
    rng = np.random.default_rng(4)
    kps["x"], kps["y"], kps["octave"] = rng.uniform(0, 700, (C, cap)), rng.uniform(0, 500, (C, cap)), 2
    k2m = np.full(C * cap, -1, np.int32)
    k2m[rng.choice(C * cap, 100, replace=False)] = rng.integers(0, 4, 100)
    n_kp = np.full(C, cap, np.int32)
    arr = _device_edges(opt, kps, n_kp, k2m, mp_pos, track, None, 64)
    o = oracle.pose_edges_from_matches(kps, n_kp, k2m, mp_pos, track, INV_SIGMA2)
    assert arr["mono_start"].cpu().tolist() == [0, 64]
    assert np.array_equal(arr["mono_kp"].cpu().numpy(), o["mono_kp"][:64])
    assert opt.last_error() != 0
    del torch


@pytest.mark.parametrize("mode", [(PoseInertialOptimizer.BATCH, 0), (PoseInertialOptimizer.GROUPED, 0)])
def test_matches_to_last_frame_chain(oracle, mode):
    """SearchByProjection's assignment -> device edge lists -> PoseInertialOptimizationLastFrame, no host round trip,
    against the oracle optimisation on the oracle's edge lists."""
    import torch
    dev = "cuda:0"
    rng = np.random.default_rng(9)
    b = synth_pose.make_last_frame_batch(n_frames=1, n_pts=800, seed=9, stereo_frac=0.3)
    cap = 1024
    kps, n_kp, kp_to_mp, mp_pos, track, uright = _frame_from_batch(b, cap, rng)
    C = int(b["n_cams"])
    E = 4096
    opt = PoseInertialOptimizer(max_frames=1, max_edges=E)
    opt.set_mode(*mode)
    arr = _device_edges(opt, kps, n_kp, kp_to_mp, mp_pos, track, uright, E)
    oe = oracle.pose_edges_from_matches(kps, n_kp, kp_to_mp, mp_pos, track, INV_SIGMA2, uright)
    # the batch the optimisation sees: b's state / rig / prior, the frame's edge lists, kp index space C * cap
    bo = dict(b)
    bo.update(oe)
    bo["kp_cap"] = C * cap
    o = oracle.pose_last_frame(bo)
    bd = dict(bo)
    bd.update({k: np.zeros(E, np.int32) for k in ("mono_cam", "stereo_cam")})   # lengths = the device bounds
    arrays = dict(arr)
    for k in synth_pose.STATE_KEYS:
        arrays[k] = torch.tensor(np.asarray(b[k], np.float64), device=dev).contiguous()
    for k in synth_pose.INPUT_KEYS[:6] + synth_pose.PRIOR_KEYS:
        arrays[k] = torch.from_numpy(np.ascontiguousarray(b[k])).to(dev)
    kpo = torch.full((1, C * cap), 255, dtype=torch.uint8, device=dev)
    H = torch.zeros((1, 225), dtype=torch.float64, device=dev)
    n_good = opt.PoseInertialOptimizationLastFrame(bd, arrays, kpo, H)
    torch.cuda.synchronize()
    assert opt.last_error() == 0
    st_o, k_o, n_o, H_o = o
    assert int(n_good.cpu()[0]) == int(n_o[0])
    assert np.array_equal(kpo.cpu().numpy(), k_o)
    ang = np.degrees(np.linalg.norm(synth_ba._log(arrays["Rwb"].cpu().numpy()[0].T @ st_o["Rwb"][0])))
    assert ang < 1e-7
    for k in ("twb", "vel", "bg", "ba"):
        assert np.abs(arrays[k].cpu().numpy()[0] - st_o[k][0]).max() < 1e-7, k
    assert np.abs(H.cpu().numpy()[0] - H_o[0]).max() <= 1e-6 * np.abs(H_o[0]).max()
