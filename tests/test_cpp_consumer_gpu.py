"""The C++ integration path: tests/cpp/omv_consumer.cpp (g++, include/omv.h + include/omv_adapters.hpp, linked
against libomv_hip.so only — no torch, no Python binding) runs the adapters INTEGRATION.md describes on the GPU.

- ORBextractor::operator() adapter, one image per call: bit-exact vs the CPU oracle;
- MultiCameraFrame (batched extraction + AssignFeaturesToGrid + lapping knn) and the SearchByProjection
  adapter: keypoints, descriptors, stereo pairs, assignments and match count bit-exact vs the oracle;
- LocalInertialBAWindow (keyframes added in mixed fixed / optimisable order, flattened optimisable-first like
  the reference's vertex creation): identical LM trials / iterations / status to the Python path on the same
  window, state and chi2 within the LocalInertialBA parity bar of tests/test_lba_gpu.py.
The binary runs as a child process (no exec from this process)."""
import os
import subprocess

import numpy as np
import pytest

from openmavis_amd import build as omv_build, synth, synth_ba

pytestmark = pytest.mark.gpu

W, H, C = 720, 540, 5
LAP = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)


def _consumer():
    if not os.path.exists(omv_build.CONSUMER_BIN):
        pytest.fail(f"{omv_build.CONSUMER_BIN} not built (python -m openmavis_amd.build)")
    return omv_build.CONSUMER_BIN


def _run(mode, d):
    r = subprocess.run([_consumer(), mode, str(d)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]


def _meta(d, **kv):
    with open(os.path.join(d, "meta.txt"), "w") as f:
        for k, v in kv.items():
            f.write(f"{k} {v}\n")


def _w(d, name, a):
    np.ascontiguousarray(a).tofile(os.path.join(d, name + ".bin"))


def _r(d, name, dtype):
    return np.fromfile(os.path.join(d, name + ".bin"), dtype)


def test_orb_extractor_adapter(tmp_path, oracle):
    imgs = np.stack([synth.hilti_frame(40)[0], synth.hilti_frame(41)[1], synth.synth_image(77, W, H)])
    laps = np.array([[0, 720], [0, 720], [0, 0]], np.int32)
    _meta(tmp_path, n=len(imgs), W=W, H=H, nfeatures=1200, ini=15, min=7)
    _w(tmp_path, "images", imgs)
    _w(tmp_path, "lapping", laps)
    _run("orb", tmp_path)
    mono = _r(tmp_path, "mono", np.int32)
    for i, img in enumerate(imgs):
        om, ok, od = oracle.orb_extract(img, 1200, 1.2, 8, 15, 7, tuple(laps[i]))
        k = _r(tmp_path, f"kps_{i}", oracle.KP_DTYPE)
        d = _r(tmp_path, f"desc_{i}", np.uint8).reshape(-1, 32)
        assert mono[i] == om and len(k) == len(ok)
        assert np.array_equal(k.view(np.uint32), ok.view(np.uint32)), f"image {i} keypoints"
        assert np.array_equal(d, od), f"image {i} descriptors"


def test_multicamera_frame_and_search_by_projection(tmp_path, oracle):
    imgs = synth.hilti_frame(42)
    M = 3000
    # oracle first: the keypoints the map points are derived from (identical on the device, checked below)
    cap = 1200 + 64 * 8
    kps = np.zeros((C, cap), oracle.KP_DTYPE)
    desc = np.zeros((C, cap, 32), np.uint8)
    n_kp, mono = np.zeros(C, np.int32), np.zeros(C, np.int32)
    for c in range(C):
        mono[c], k, d = oracle.orb_extract(imgs[c], 1200, 1.2, 8, 15, 7, tuple(LAP[c]))
        n_kp[c] = len(k)
        kps[c, :len(k)], desc[c, :len(k)] = k, d
    mp = synth.make_map_points(kps, desc, n_kp, M, 9, W, H)
    _meta(tmp_path, C=C, W=W, H=H, nfeatures=1200, ini=15, min=7, M=M, th=6.0, far=0, th_far=20.0, nnratio=0.8)
    _w(tmp_path, "images", imgs)
    _w(tmp_path, "lapping", LAP)
    for k in ("desc", "proj_x", "proj_y", "view_cos", "level", "in_view", "track_depth", "is_bad", "has_obs"):
        _w(tmp_path, "mp_" + k, mp[k])
    _run("frame", tmp_path)
    dcap = int(open(os.path.join(tmp_path, "kp_cap.txt")).read())
    for c in range(C):
        k = _r(tmp_path, f"kps_{c}", oracle.KP_DTYPE)
        d = _r(tmp_path, f"desc_{c}", np.uint8).reshape(-1, 32)
        assert len(k) == n_kp[c] and np.array_equal(k.view(np.uint32), kps[c, :n_kp[c]].view(np.uint32)), f"cam {c}"
        assert np.array_equal(d, desc[c, :n_kp[c]]), f"cam {c} descriptors"
    l2r, r2l = _r(tmp_path, "l2r", np.int32), _r(tmp_path, "r2l", np.int32)
    # the lapping knn + Lowe pairs (Frame.cc:1461-1491)
    q, t = desc[0, mono[0]:n_kp[0]], desc[1, mono[1]:n_kp[1]]
    i2, d2 = oracle.bf_knn2(q, t)
    el2r = np.full(dcap, -1, np.int32)
    for qi in range(len(q)):
        if i2[qi, 1] >= 0 and float(d2[qi, 0]) < float(d2[qi, 1]) * 0.8:
            el2r[mono[0] + qi] = mono[1] + i2[qi, 0]
    assert np.array_equal(l2r, el2r)
    # SearchByProjection on the device frame: the oracle on the same frame (padded to the device's row capacity)
    kp_d = np.zeros((C, dcap), oracle.KP_DTYPE)
    de_d = np.zeros((C, dcap, 32), np.uint8)
    for c in range(C):
        kp_d[c, :n_kp[c]], de_d[c, :n_kp[c]] = kps[c, :n_kp[c]], desc[c, :n_kp[c]]
    sf = [1.0]
    for _ in range(7):
        sf.append(float(np.float32(sf[-1] * 1.2)))   # mvScaleFactor: (float)(previous * scaleFactor)
    g = oracle.frame_geom(C, W, H, sf)
    exp = np.full(C * dcap, -1, np.int32)
    n = oracle.search_by_projection(g, kp_d, de_d, n_kp, mp, 6.0, False, 20.0, 0.8, l2r, r2l,
                                    np.zeros(C * dcap, np.uint8), exp)
    got = _r(tmp_path, "kp_to_mp", np.int32)
    assert int(_r(tmp_path, "n_matches", np.int32)[0]) == n and n > 300
    assert np.array_equal(got, exp)


LBA_ARRAYS = ("cam", "Rcb", "tcb", "Rbc", "tbc", "kf_imu", "Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts",
              "pt_track_depth", "mono_pt", "mono_kf", "mono_cam", "mono_obs", "mono_inv_sigma2", "imu_kf1", "imu_kf2",
              "preint")
STEREO_ARRAYS = ("stereo_pt", "stereo_kf", "stereo_obs", "stereo_inv_sigma2")


def _run_lba_window(d, prob, large=True, rec_init=False, warm_small=False, rccl=False):
    K, n_opt = prob["n_kf"], prob["n_opt"]
    # window insertion order: fixed and optimisable keyframes interleaved (relative order kept in each group,
    # so the flattened vertex order equals the problem's)
    fixed, opt = list(range(n_opt, K)), list(range(n_opt))
    order = np.array([x for pair in zip(fixed, opt) for x in pair] + fixed[len(opt):] + opt[len(fixed):], np.int32)
    _meta(d, n_cams=prob["n_cams"], n_kf=K, n_opt=n_opt, n_pts=len(prob["pts"]), large=int(large),
          rec_init=int(rec_init), warm_small=int(warm_small), bf=float(prob.get("bf", 0.0)), rccl=int(rccl))
    _w(d, "kf_order", order)
    for k in LBA_ARRAYS + (STEREO_ARRAYS if prob.get("n_stereo", 0) else ()) + (("cam_model",) if "cam_model" in prob else ()):
        _w(d, k, prob[k])
    _run("lba", d)
    res = dict(line.split() for line in open(os.path.join(d, "result.txt")))
    st = {k: _r(d, "out_" + k, np.float64) for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts")}
    return res, st


def _check_against_python(d, prob, res, st, oracle, large=True):
    from test_lba_gpu import _compare_state, _solver
    opts = dict(opt_it=4, lambda_init=1e-2, max_trials=10, large=True) if large else \
        dict(opt_it=10, lambda_init=1e0, max_trials=10, large=False)
    rp, sp = _solver(prob).set_problem(prob).optimize(**opts)
    assert (int(res["iterations"]), int(res["trials"]), int(res["status"])) == (rp["iterations"], rp["trials"], rp["status"])
    for k in ("err", "err_end"):
        assert abs(float(res[k]) - rp[k]) <= 1e-5 * abs(rp[k]), (k, res[k], rp[k])
    ro, so, _ = oracle.lba_optimize(prob, **opts)
    _compare_state(prob, {k: v.reshape(so[k].shape) for k, v in st.items()}, so, oracle)
    chi2 = _r(d, "out_chi2", np.float64)
    assert np.allclose(chi2, rp["mono_chi2"], rtol=1e-6, atol=1e-3)
    if prob.get("n_stereo", 0):
        schi2 = _r(d, "out_stereo_chi2", np.float64)
        assert len(schi2) == prob["n_stereo"]
        assert np.allclose(schi2, rp["stereo_chi2"], rtol=1e-6, atol=1e-3)
        assert np.array_equal(_r(d, "out_stereo_outlier", np.uint8), rp["stereo_outlier"])


def test_local_inertial_ba_window(tmp_path, oracle):
    prob = synth_ba.make_lba_problem(n_kf=20, n_opt=10, n_pts=1500, seed=11)
    res, st = _run_lba_window(tmp_path, prob)
    _check_against_python(tmp_path, prob, res, st, oracle)


def test_local_inertial_ba_window_stereo_recinit_regrow(tmp_path, oracle):
    """EdgeStereo observations through add_stereo (Optimizer.cc:3108-3143), every inertial edge robust under bRecInit
    (:2972), and a smaller window optimised first on the same adapter (the handle is re-created for the larger one)."""
    prob = synth_ba.make_lba_problem(n_kf=20, n_opt=10, n_pts=1500, seed=12, stereo_frac=0.5)
    prob["imu_robust"] = np.ones_like(prob["imu_robust"])   # bRecInit: i == N-1 || bRecInit
    assert prob["n_stereo"] > 300
    res, st = _run_lba_window(tmp_path, prob, rec_init=True, warm_small=True)
    _check_against_python(tmp_path, prob, res, st, oracle)


def test_local_inertial_ba_window_fail_keeps_state(tmp_path):
    """The FAIL guard (Optimizer.cc:3317-3321, !bLarge): a NaN observation makes err NaN, the reference returns
    before writing anything back -- keyframes AND points keep their input values."""
    prob = synth_ba.make_lba_problem(n_kf=12, n_opt=6, n_pts=600, seed=13)
    prob["mono_obs"] = prob["mono_obs"].copy()
    prob["mono_obs"][5, 0] = np.nan
    res, st = _run_lba_window(tmp_path, prob, large=False)
    assert int(res["status"]) == 1   # OMV_LBA_FAIL
    for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts"):
        assert np.array_equal(st[k], np.asarray(prob[k], np.float64).ravel()), k


def test_local_inertial_ba_window_rccl_single_rank(tmp_path, oracle):
    """INTEGRATION.md §4b compiled: the window on a one-rank RCCL communicator (ncclGetUniqueId / ncclCommInitRank,
    omv_lba_set_comm with an ncclAllReduce callback).  The landmark-sharded call sequence runs for real -- two in-place
    all-reduces per LM step on the handle's stream, directly launched gated steps, one host wait per batch of steps --
    and the outcome meets the same bar as the unsharded window."""
    prob = synth_ba.make_lba_problem(n_kf=20, n_opt=10, n_pts=1500, seed=11)
    res, st = _run_lba_window(tmp_path, prob, rccl=True)
    _check_against_python(tmp_path, prob, res, st, oracle)
    trials, calls, syncs = int(res["trials"]), int(res["allreduce_calls"]), int(res["host_syncs"])
    assert calls >= 2 * trials, (calls, trials)   # [blocks | b | rhs] and [chi(A), chi, computeScale] per step
    assert syncs <= (trials + 3) // 4 + 1 and (trials < 2 or syncs < trials), (syncs, trials)


def _oracle_frame(oracle, imgs, cap):
    kps = np.zeros((C, cap), oracle.KP_DTYPE)
    desc = np.zeros((C, cap, 32), np.uint8)
    n_kp = np.zeros(C, np.int32)
    for c in range(C):
        _, k, d = oracle.orb_extract(imgs[c], 1200, 1.2, 8, 15, 7, tuple(LAP[c]))
        n_kp[c] = len(k)
        kps[c, :len(k)], desc[c, :len(k)] = k, d
    return kps, desc, n_kp


def test_search_by_projection_last_frame_adapter(tmp_path, oracle):
    """SearchByProjection(Frame&, const Frame& LastFrame, th, bMono) (ORBmatcher.cc:1985-2413) through the
    SearchByProjectionLastFrame adapter on a MultiCameraFrame: assignments (LastFrame slots) and count bit-exact vs the
    oracle, forward motion (level window) with the rotation-histogram filter."""
    from openmavis_amd.orb import ORBextractor
    imgs = synth.hilti_frame(44)
    cap = ORBextractor(1200, 1.2, 8, 15, 7, width=W, height=H, max_images=C).max_keypoints()
    kps, desc, n_kp = _oracle_frame(oracle, imgs, cap)
    cams, R_cl, t_cl = synth.hilti_rig(C)
    rng = np.random.default_rng(5)
    Tcw = synth.random_se3(rng)
    last = synth.make_last_frame(kps, desc, n_kp, 91, cams, Tcw)
    Tlw = Tcw.copy()
    Tlw[6] -= np.float32(0.5)
    Trl = np.concatenate([synth.quat_from_R(R_cl[1].astype(np.float64)), t_cl[1]]).astype(np.float32)
    occ = (rng.random(C * cap) < 0.03).astype(np.uint8)
    mb = 0.11
    _meta(tmp_path, C=C, W=W, H=H, nfeatures=1200, ini=15, min=7, last_cap=cap, nnratio=0.9, check_ori=1, th=7.0,
          bmono=0, mb=mb)
    _w(tmp_path, "images", imgs)
    _w(tmp_path, "lapping", LAP)
    _w(tmp_path, "cams", np.asarray(cams, np.float32))
    _w(tmp_path, "Tcw", Tcw), _w(tmp_path, "Tlw", Tlw), _w(tmp_path, "Trl", Trl), _w(tmp_path, "occ", occ)
    _w(tmp_path, "last_pos", last["pos"]), _w(tmp_path, "last_desc", last["desc"])
    _w(tmp_path, "last_valid", last["valid"]), _w(tmp_path, "last_obs", last["has_obs"])
    _w(tmp_path, "last_kps", last["kps"])
    _run("lastframe", tmp_path)
    got, n = _r(tmp_path, "kp_to_mp", np.int32), int(_r(tmp_path, "n_matches", np.int32)[0])
    g = oracle.frame_geom(C, W, H, _scale_factors())
    exp = np.full(C * cap, -1, np.int32)
    n_o = oracle.search_last_frame(g, kps, desc, n_kp, cams, Tcw, Tlw, Trl, last["pos"], last["desc"], last["valid"],
                                   last["has_obs"], last["kps"], 7.0, False, mb, True, occ, exp)
    assert n == n_o and n > 200, (n, n_o)
    assert np.array_equal(got, exp)


def _scale_factors():
    sf = [1.0]
    for _ in range(7):
        sf.append(float(np.float32(sf[-1] * 1.2)))   # mvScaleFactor: (float)(previous * scaleFactor)
    return sf


@pytest.mark.parametrize("model,check_ori,coarse", [("kb8", False, False), ("kb8", True, False), ("pinhole", False, True)])
def test_search_for_triangulation_adapter(tmp_path, oracle, model, check_ori, coarse):
    """SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse) (ORBmatcher.cc:1131-1456) through the
    adapter: KeyFrameView (keypoints in [L|R|SL|SR] order, FeatureVector CSR) -> vMatchedPairs and the count, bit-exact vs
    the oracle's vMatches12."""
    from openmavis_amd import synth_tri
    p = synth_tri.make_tri_pair(seed=21, n_pts=700, model=model)
    meta = dict(check_ori=int(check_ori), coarse=int(coarse), only_stereo=0)
    for k in ("kf1", "kf2"):
        kf = p[k]
        for f in ("n", "n_left", "n_right", "n_sideleft"):
            meta[f"{k}_{f}"] = int(kf[f])
        _w(tmp_path, f"{k}_kps", kf["kps"])
        for f in ("desc", "has_mp", "node_id", "node_start", "node_idx"):
            _w(tmp_path, f"{k}_{f}", kf[f])
    _meta(tmp_path, **meta)
    _w(tmp_path, "level_sigma2", np.asarray(p["level_sigma2"], np.float32))
    _w(tmp_path, "T", np.asarray(p["T"], np.float32))
    _w(tmp_path, "cams", np.asarray(p["cams"], np.float32))
    if "cam_model" in p:
        _w(tmp_path, "cam_model", np.asarray(p["cam_model"], np.int32))
    _run("tri", tmp_path)
    n = int(_r(tmp_path, "n_matches", np.int32)[0])
    pairs = _r(tmp_path, "pairs", np.int64).reshape(-1, 2)
    n_o, m_o = oracle.search_for_triangulation(p, coarse=coarse, check_ori=check_ori)
    exp = np.stack([np.nonzero(m_o >= 0)[0], m_o[m_o >= 0]], 1) if (m_o >= 0).any() else np.zeros((0, 2), np.int64)
    assert n == n_o and n > 20, (n, n_o)
    assert np.array_equal(pairs, exp)


POSE_KEYS = ("cam", "Rcb", "tcb", "Rbc", "tbc", "Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "kf_Rwb", "kf_twb",
             "kf_vel", "kf_bg", "kf_ba", "preint", "mono_cam", "mono_kp", "mono_obs", "mono_inv_sigma2", "mono_xw",
             "mono_close")


@pytest.mark.parametrize("lf,stereo,rec_init", [(False, 0.0, False), (False, 0.3, False), (True, 0.3, False),
                                                (True, 0.0, True)])
def test_pose_inertial_optimizer_adapter(tmp_path, oracle, lf, stereo, rec_init):
    """PoseInertialOptimizationLastKeyFrame / LastFrame (Optimizer.cc:5021, :5580) through the PoseInertialOptimizer
    adapter on ONE frame (Tracking's call; the grouped kernel): state within 1e-7, mvbOutlier and the return value
    exact, the Hessian within 1e-6 relative -- the bar of tests/test_pose_gpu.py; LastFrame also the ConstraintPoseImu
    of its marginal within 1e-9 relative."""
    from openmavis_amd import synth_pose
    mk = synth_pose.make_last_frame_batch if lf else synth_pose.make_pose_batch
    b = mk(n_frames=1, n_pts=800, seed=13, outlier_frac=0.12, stereo_frac=stereo)
    _meta(tmp_path, n_cams=int(b["n_cams"]), lf=int(lf), rec_init=int(rec_init), bf=float(b["bf"]), kp_cap=int(b["kp_cap"]))
    for k in POSE_KEYS:
        _w(tmp_path, k, np.asarray(b[k]))
    if len(b["stereo_cam"]):
        for k in ("stereo_cam", "stereo_kp", "stereo_obs", "stereo_inv_sigma2", "stereo_xw"):
            _w(tmp_path, k, np.asarray(b[k]))
    if lf:
        for k in ("prior_Rwb", "prior_twb", "prior_vel", "prior_bg", "prior_ba", "prior_H", "preint_kf"):
            _w(tmp_path, k, np.asarray(b[k]))
    _run("pose", tmp_path)
    st_o, k_o, n_o, H_o = (oracle.pose_last_frame if lf else oracle.pose_last_kf)(b, rec_init)
    assert int(_r(tmp_path, "n_good", np.int32)[0]) == int(n_o[0])
    kpo = _r(tmp_path, "out_kpo", np.uint8)
    has_edge = np.zeros(int(b["kp_cap"]), bool)
    has_edge[b["mono_kp"]] = True
    if len(b["stereo_kp"]):
        has_edge[b["stereo_kp"]] = True
    assert np.array_equal(kpo[has_edge], k_o[0][has_edge]) and (kpo[~has_edge] == 255).all()
    R = _r(tmp_path, "out_Rwb", np.float64).reshape(3, 3)
    ang = np.degrees(np.linalg.norm(synth_ba._log(R.T @ st_o["Rwb"][0])))
    assert ang < 1e-7, ang
    for k in ("twb", "vel", "bg", "ba", "tcw"):
        assert np.abs(_r(tmp_path, "out_" + k, np.float64) - st_o[k][0].ravel()).max() < 1e-7, k
    H = _r(tmp_path, "out_H", np.float64)
    assert np.abs(H - H_o[0]).max() <= 1e-6 * np.abs(H_o[0]).max()
    if lf:
        Hc = _r(tmp_path, "out_Hc", np.float64)
        o = oracle.pose_constraint(H_o[:1])[0]
        assert np.abs(Hc - o).max() <= 1e-6 * np.abs(o).max()


def test_fuse_adapter(tmp_path, oracle):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th, cameraID) (ORBmatcher.cc:1458-1647) through the Fuse adapter, one call per
    camera block of a keyframe: per map point the chosen keypoint (N-index) and distance, and nFused, bit-exact vs the
    oracle."""
    from openmavis_amd import synth_kfmatch as sk
    b = sk.make_kf_search(0, seed=5)
    th, md = sk.MODE_PARAMS[0]
    bi_o, bd_o, n_o, _ = oracle.search_kf(b, th, md)
    jobs = [(i, j) for i, j in enumerate(b["jobs"]) if j["kf"] == 0]
    K, cap = 0, int(b["kp_cap"])
    rows = np.concatenate([b["mp_list"][j["mp_start"]:j["mp_start"] + j["mp_count"]] for _, j in jobs])
    scale = _scale_factors()
    ils = [float(np.float32(1.0) / np.float32(np.float32(s) * np.float32(s))) for s in scale]
    _meta(tmp_path, C=int(b["n_cams"]), kp_cap=cap, W=int(b["width"]), H=int(b["height"]), bf=float(b["bf"]), th=th,
          n_jobs=len(jobs), max_points=len(rows))
    _w(tmp_path, "scale_factors", np.asarray(scale, np.float32))
    _w(tmp_path, "inv_level_sigma2", np.asarray(ils, np.float32))
    _w(tmp_path, "cams", np.asarray(b["cams"], np.float32))
    if b.get("cam_model") is not None:
        _w(tmp_path, "cam_model", np.asarray(b["cam_model"], np.int32))
    _w(tmp_path, "kps", b["kps"][K]), _w(tmp_path, "desc", b["desc"][K]), _w(tmp_path, "n_kp", b["n_kp"][K])
    _w(tmp_path, "uright", b["uright"][K])
    _w(tmp_path, "job_cam", np.array([j["cam"] for _, j in jobs], np.int32))
    _w(tmp_path, "job_count", np.array([j["mp_count"] for _, j in jobs], np.int32))
    _w(tmp_path, "job_Tcw", np.stack([np.asarray(j["Tcw"], np.float32) for _, j in jobs]))
    _w(tmp_path, "job_Ow", np.stack([np.asarray(j["Ow"], np.float32) for _, j in jobs]))
    for k in ("pos", "normal", "min_dist", "max_dist", "desc"):
        _w(tmp_path, "mp_" + k, b["mps"][k][rows])
    _run("fuse", tmp_path)
    bi, bd, nf = _r(tmp_path, "best_idx", np.int32), _r(tmp_path, "best_dist", np.int32), _r(tmp_path, "n_fused", np.int32)
    ent = np.concatenate([np.arange(j["mp_start"], j["mp_start"] + j["mp_count"]) for _, j in jobs])
    assert np.array_equal(bi, bi_o[ent]) and np.array_equal(bd, bd_o[ent])
    assert np.array_equal(nf, n_o[[i for i, _ in jobs]]) and nf.sum() > 30


# ---- the round-6 drop-ins: PoseOptimization, CreateNewMapPoints' loop, the map-point refresh, the fuse sequence --------
def test_pose_optimization_adapter(tmp_path, oracle):
    """Optimizer::PoseOptimization(Frame*) through the C++ adapter on one 4-camera frame: pose within the GPU parity
    bar of tests/test_pose_only_gpu.py (1e-7), mvbOutlier and nGood identical to the oracle."""
    from openmavis_amd import synth_pose
    b = synth_pose.make_pose_only_batch(n_frames=1, n_pts=400, seed=21, n_cams=4, outlier_frac=0.15)
    rq, rt, rk, rn = oracle.pose_optimization(b)
    _meta(tmp_path, n_cams=4, bf=float(b["bf"]), kp_cap=int(b["kp_cap"]))
    _w(tmp_path, "cams", np.asarray(b["cam"], np.float32))
    if "cam_model" in b:
        _w(tmp_path, "cam_model", np.asarray(b["cam_model"], np.int32))
    _w(tmp_path, "rig_q", np.asarray(b["rig_q"], np.float64)), _w(tmp_path, "rig_t", np.asarray(b["rig_t"], np.float64))
    _w(tmp_path, "pose_q", np.asarray(b["pose_q"][0], np.float64)), _w(tmp_path, "pose_t", np.asarray(b["pose_t"][0], np.float64))
    for k, dt in (("mono_cam", np.int32), ("mono_kp", np.int32), ("mono_obs", np.float64)):
        _w(tmp_path, k, np.asarray(b[k], dt))
    _w(tmp_path, "mono_w", np.asarray(b["mono_inv_sigma2"], np.float32))
    _w(tmp_path, "mono_xw", np.asarray(b["mono_xw"], np.float32))
    _run("posopt", tmp_path)
    q, t = _r(tmp_path, "q", np.float64), _r(tmp_path, "t", np.float64)
    kpo, ng = _r(tmp_path, "kpo", np.uint8), _r(tmp_path, "n_good", np.int32)
    assert ng[0] == rn[0]
    np.testing.assert_array_equal(kpo[b["mono_kp"]], rk[0][b["mono_kp"]])
    np.testing.assert_allclose(q, rq[0], rtol=0, atol=1e-7)
    np.testing.assert_allclose(t, rt[0], rtol=0, atol=1e-7)


def _cnmp_kf_files(d, k, kf, s):
    p = f"kf{k}_"
    _w(d, p + "ints", np.array([kf["n"], kf["n_left"], kf["n_right"], kf["n_sideleft"]], np.int32))
    _w(d, p + "keys", kf["kps"]), _w(d, p + "desc", kf["desc"]), _w(d, p + "has_mp", kf["has_mp"].astype(np.uint8))
    _w(d, p + "node_id", kf["node_id"].astype(np.uint32)), _w(d, p + "node_start", kf["node_start"].astype(np.int32))
    _w(d, p + "node_idx", kf["node_idx"].astype(np.int32))
    sg = np.zeros(16, np.float32)
    sg[:8] = s["sigma2"]
    _w(d, p + "sigma2", sg), _w(d, p + "Tcw", kf["Tcw"].astype(np.float32)), _w(d, p + "Ow", kf["Ow"].astype(np.float32))
    fx, fy = np.float32(s["fx"]), np.float32(s["fy"])
    geom = np.concatenate([kf["Rwc"], kf["twc"], [fx, fy, s["cx"], s["cy"], np.float32(1) / fx, np.float32(1) / fy,
                                                  np.float32(s["mb"]), np.float32(s["mbf"])]]).astype(np.float32)
    _w(d, p + "geom", geom), _w(d, p + "uright", kf["uright"]), _w(d, p + "depth", kf["depth"])
    sc = np.zeros(16, np.float32)
    sc[:8] = s["scale"]
    _w(d, p + "scale", sc)


def test_create_new_map_points_adapter(tmp_path, oracle):
    """LocalMapping::CreateNewMapPoints' neighbour loop through the C++ adapter, split over two calls (a
    CheckNewKeyFrames() boundary): the new points in the reference's creation order with their x3D bits, the search
    counts and the current keyframe's has-map-point flags, identical to the interleaved oracle."""
    from openmavis_amd import synth_cnmp
    s = synth_cnmp.make_cnmp_chain(seed=8, n_neigh=10)
    hm, nm, outs, _ = oracle.local_mapping_create_new_map_points(s)
    n_nb = len(s["nbs"])
    _meta(tmp_path, n_nb=n_nb, split=4, n_cams=4, inertial=1, monocular=0, coarse=0, far=0, th_far=50.0,
          scale_factor=s["scale_factor"])
    _w(tmp_path, "cams", s["cams"]), _w(tmp_path, "cam_model", s["cam_model"])
    _cnmp_kf_files(tmp_path, 0, s["kf1"], s)
    for j, nb in enumerate(s["nbs"]):
        _cnmp_kf_files(tmp_path, j + 1, nb["kf2"], s)
    _w(tmp_path, "T", np.stack([nb["T"] for nb in s["nbs"]]).astype(np.float32))
    _w(tmp_path, "skip", np.array([nb["skip"] for nb in s["nbs"]], np.int32))
    _run("cnmp", tmp_path)
    rec = _r(tmp_path, "points", np.int32).reshape(-1, 4)
    x = _r(tmp_path, "x3d", np.float32).reshape(-1, 3)
    exp = [(j, i, int(m12[i]), int(st[i] == 2)) for j, (m12, st, _x) in enumerate(outs) for i in np.flatnonzero(st > 0)]
    assert [tuple(r) for r in rec] == exp
    ex = np.array([outs[j][2][i] for j, i, _, _ in exp], np.float32).reshape(-1, 3)
    assert np.array_equal(x.view(np.uint32), ex.view(np.uint32))
    np.testing.assert_array_equal(_r(tmp_path, "has_mp1", np.uint8), hm)
    np.testing.assert_array_equal(_r(tmp_path, "n_matches", np.int32), nm)
    assert len(exp) > 200


def test_map_point_refresh_adapter(tmp_path, oracle):
    """MapPoint::ComputeDistinctiveDescriptors / UpdateNormalAndDepth through the C++ adapter: rows, descriptors and
    the float normal / distances bit-exact vs the oracle."""
    from openmavis_amd import synth_mappoint
    mp = synth_mappoint.make_points(n_points=600, seed=4)
    g = synth_mappoint.make_geometry(n_points=800, seed=5)
    for k in ("desc", "desc_start", "desc_row"):
        _w(tmp_path, k, mp[k])
    for k in ("obs_start", "obs_center", "pos", "ref_center", "ref_level_scale", "ref_max_scale"):
        _w(tmp_path, k, np.ascontiguousarray(g[k]))
    P = len(g["obs_start"]) - 1
    _w(tmp_path, "normal_in", np.full((P, 3), np.nan, np.float32))
    _w(tmp_path, "min_in", np.full(P, np.nan, np.float32)), _w(tmp_path, "max_in", np.full(P, np.nan, np.float32))
    _run("mprefresh", tmp_path)
    best = oracle.distinctive_descriptors(mp["desc"], mp["desc_start"], mp["desc_row"])
    np.testing.assert_array_equal(_r(tmp_path, "best", np.int32), best)
    d = _r(tmp_path, "desc_out", np.uint8).reshape(-1, 32)
    has = best >= 0
    np.testing.assert_array_equal(d[has], mp["desc"][best[has]])
    on, omin, omax = oracle.normal_depth(**g)
    for name, ref in (("normal", on), ("min_dist", omin), ("max_dist", omax)):
        got = _r(tmp_path, name, np.float32).reshape(ref.shape)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), name


def test_search_in_neighbors_fuse_adapter(tmp_path, oracle):
    """SearchInNeighbors' fuse sequence through the C++ adapter: final mvpMapPoints, isBad / mpReplaced / nObs /
    mObservations, the edit log, nFused per call and the final descriptors identical to the literal oracle."""
    from openmavis_amd import synth_fuse
    from openmavis_amd.matcher import kf_search_params
    s = synth_fuse.make_fuse_scene(seed=5, n_targets=6)
    ref = oracle.search_in_neighbors_fuse(s)
    sc = [1.0]
    for _ in range(1, s["nlevels"]):
        sc.append(float(np.float32(sc[-1] * np.float32(1.2))))
    p = kf_search_params(3.0, 50.0, s["cams"], nlevels=s["nlevels"])
    _meta(tmp_path, n_kf=s["n_kf"], n_cams=s["n_cams"], kp_cap=s["kp_cap"], width=s["width"], height=s["height"],
          bf=s["bf"], th=3.0, current=s["current"])
    _w(tmp_path, "scale", np.array(sc, np.float32)), _w(tmp_path, "cams", s["cams"])
    _w(tmp_path, "inv_sigma2", np.array([p.inv_level_sigma2[i] for i in range(16)], np.float32))
    for k in ("kps", "desc", "n_kp", "uright", "n_blocks", "Tcw", "Ow", "kf_mps", "bad", "n_obs", "obs_start", "obs_kf",
              "obs_idx", "targets"):
        _w(tmp_path, k, np.ascontiguousarray(s[k]))
    for k in ("pos", "normal", "min_dist", "max_dist"):
        _w(tmp_path, k, s["mps"][k])
    _w(tmp_path, "mp_desc", s["mps"]["desc"])
    _run("fuseseq", tmp_path)
    for k, dt in (("kf_mps", np.int32), ("bad", np.int32), ("n_obs", np.int32), ("replaced", np.int32),
                  ("obs_start", np.int32), ("obs_kf", np.int32), ("obs_idx", np.int32), ("log", np.int32),
                  ("n_fused", np.int32)):
        np.testing.assert_array_equal(_r(tmp_path, "out_" + k, dt), np.asarray(ref[k]).ravel(), err_msg=k)
    np.testing.assert_array_equal(_r(tmp_path, "out_desc", np.uint8).reshape(-1, 32), ref["desc"])
    assert (ref["log"][:, 0] == 1).sum() > 20
