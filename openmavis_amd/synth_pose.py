"""Seeded synthetic batches for Optimizer::PoseInertialOptimizationLastKeyFrame (Optimizer.cc:5021-5578).

Each frame of the batch is a tracked frame 0.05-0.2 s after its last keyframe on the smooth trajectory of
synth_ba (1 m/s arc), seen by the 5-camera Kannala-Brandt rig.  The keyframe's state is the truth (its
vertices are fixed in the reference); the frame's initial state is the truth perturbed by ~0.5 deg /
3 cm / 5 cm/s (what the IMU prediction hands the optimiser).  Matched map points: `n_pts` per frame in
random cameras at 2-25 m, observed at the true projection + N(0, 0.7 px); a fraction of them are
outliers (observation moved by 8-40 px).  stereo_frac adds an EdgeStereoOnlyPose on the same keypoint
(kp_ur > 0, :5160-5186) with u_R = u - bf / z + noise.  The preintegration is synth_ba.preintegrate of
the true motion (float32, the IMU::Preintegrated layout of include/omv.h).
"""
import numpy as np

from . import synth_ba


def make_pose_batch(n_frames=8, n_pts=300, seed=1, outlier_frac=0.1, stereo_frac=0.0, n_cams=5, bf=40.0,
                    rot_noise_deg=0.5, trans_noise=0.03, vel_noise=0.05, pinhole=False):
    rng = np.random.Generator(np.random.PCG64(seed))
    cams, Rbc, tbc = synth_ba.rig()
    cams, Rbc, tbc = cams[:n_cams], Rbc[:n_cams], tbc[:n_cams]
    Rcb = np.transpose(Rbc, (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc)

    def cam_pose(R, t):
        Rbw = R.T
        tbw = -Rbw @ t
        return np.einsum("cij,jk->cik", Rcb, Rbw), np.einsum("cij,j->ci", Rcb, tbw) + tcb

    F = n_frames
    out = {k: [] for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "kf_Rwb", "kf_twb", "kf_vel", "kf_bg",
                           "kf_ba", "preint", "true_Rwb", "true_twb", "true_vel", "t")}
    mono = {k: [] for k in ("cam", "kp", "obs", "w", "xw", "close", "outlier")}
    st = {k: [] for k in ("cam", "kp", "obs", "w", "xw")}
    m_start, s_start = [0], [0]
    kp_cap = 0
    for f in range(F):
        t_kf = 0.37 * f + float(rng.uniform(0, 0.2))
        dt = float(rng.choice([0.05, 0.1, 0.15, 0.2]))
        Rk, pk, vk = synth_ba._pose_at(t_kf)
        Rt, pt, vt = synth_ba._pose_at(t_kf + dt)
        out["kf_Rwb"].append(Rk), out["kf_twb"].append(pk), out["kf_vel"].append(vk)
        out["kf_bg"].append(np.zeros(3)), out["kf_ba"].append(np.zeros(3))
        out["preint"].append(synth_ba.preintegrate(t_kf, t_kf + dt))
        out["true_Rwb"].append(Rt), out["true_twb"].append(pt), out["true_vel"].append(vt)
        out["t"].append(t_kf + dt)
        ax = rng.normal(0, 1, 3)
        ax /= np.linalg.norm(ax)
        R0 = Rt @ synth_ba._exp(ax * np.deg2rad(rot_noise_deg))
        u, _, vh = np.linalg.svd(R0)
        R0 = u @ vh
        t0 = pt + rng.normal(0, trans_noise, 3)
        out["Rwb"].append(R0), out["twb"].append(t0)
        out["vel"].append(vt + rng.normal(0, vel_noise, 3))
        out["bg"].append(rng.normal(0, 1e-4, 3)), out["ba"].append(rng.normal(0, 1e-3, 3))
        Rc0, tc0 = cam_pose(R0, t0)
        out["Rcw"].append(Rc0), out["tcw"].append(tc0)
        Rct, tct = cam_pose(Rt, pt)
        kp = 0
        while kp < n_pts:
            c = int(rng.integers(0, n_cams))
            d = rng.normal(0, 1, 3)
            d[2] = abs(d[2]) * 1.5 + 0.6
            d /= np.linalg.norm(d)
            Xc = d * rng.uniform(2.0, 25.0)
            uv = synth_ba.cam_project(cams[c].astype(np.float64), Xc, pinhole)
            if not (5 <= uv[0] <= 715 and 5 <= uv[1] <= 535):
                continue
            Xw = (Rct[c].T @ (Xc - tct[c])).astype(np.float32)   # MapPoint::GetWorldPos is float
            obs = uv + rng.normal(0, 0.7, 2)
            bad = rng.random() < outlier_frac
            if bad:
                obs = obs + rng.uniform(8, 40, 2) * rng.choice([-1, 1], 2)
            w = np.float32(1.0 / np.float32(1.2) ** (2 * int(rng.integers(0, 8))))
            mono["cam"].append(c), mono["kp"].append(kp), mono["obs"].append(obs), mono["w"].append(w)
            mono["xw"].append(Xw), mono["close"].append(rng.random() < 0.3), mono["outlier"].append(bad)
            if stereo_frac > 0 and rng.random() < stereo_frac:
                ur = np.float32(uv[0] - bf / Xc[2] + rng.normal(0, 0.7))
                if ur > 0:
                    st["cam"].append(c), st["kp"].append(kp), st["obs"].append([obs[0], obs[1], float(ur)])
                    st["w"].append(w), st["xw"].append(Xw)
            kp += 1
        kp_cap = max(kp_cap, kp)
        m_start.append(len(mono["cam"]))
        s_start.append(len(st["cam"]))
    b = {k: np.array(v, np.float64) for k, v in out.items() if k != "preint"}
    b["preint"] = np.stack(out["preint"]).astype(np.float32)
    b.update(n_frames=F, n_cams=n_cams, cam=cams, Rcb=Rcb, tcb=tcb, Rbc=Rbc, tbc=tbc, bf=np.float32(bf),
             kp_cap=kp_cap,
             mono_start=np.array(m_start, np.int32), mono_cam=np.array(mono["cam"], np.int32),
             mono_kp=np.array(mono["kp"], np.int32), mono_obs=np.array(mono["obs"], np.float64).reshape(-1, 2),
             mono_inv_sigma2=np.array(mono["w"], np.float32), mono_xw=np.array(mono["xw"], np.float32).reshape(-1, 3),
             mono_close=np.array(mono["close"], np.uint8), mono_is_outlier=np.array(mono["outlier"], bool),
             stereo_start=np.array(s_start, np.int32), stereo_cam=np.array(st["cam"], np.int32),
             stereo_kp=np.array(st["kp"], np.int32), stereo_obs=np.array(st["obs"], np.float64).reshape(-1, 3),
             stereo_inv_sigma2=np.array(st["w"], np.float32), stereo_xw=np.array(st["xw"], np.float32).reshape(-1, 3))
    if pinhole:
        b["cam_model"] = np.full(n_cams, 1, np.int32)   # OMV_CAM_PINHOLE
    return b


PRIOR_KEYS = ("prior_Rwb", "prior_twb", "prior_vel", "prior_bg", "prior_ba", "prior_H", "preint_kf")


def make_last_frame_batch(n_frames=8, n_pts=300, seed=1, outlier_frac=0.1, stereo_frac=0.0, n_cams=5, bf=40.0,
                          frame_dt=0.05, prior_rot_deg=0.1, prior_trans=0.01, prior_vel=0.02, pinhole=False):
    """Batches for Optimizer::PoseInertialOptimizationLastFrame (Optimizer.cc:5580-6170): make_pose_batch's
    frames and edges, each with a previous frame `frame_dt` earlier.  The previous frame carries the
    ConstraintPoseImu its own optimisation left (pFp->mpcpi: the true state perturbed by ~0.1 deg / 1 cm /
    2 cm/s, and a dense SPD 15x15 information); its vertices start from that state cast to float, as
    SetImuPoseVelocity(...cast<float>()) stored it (:6103-6109).  `preint` becomes the frame-to-frame
    preintegration (mpImuPreintegratedFrame); the keyframe-to-frame one moves to `preint_kf`
    (mpImuPreintegrated, whose covariance gives EdgeGyroRW / EdgeAccRW their information)."""
    b = make_pose_batch(n_frames=n_frames, n_pts=n_pts, seed=seed, outlier_frac=outlier_frac,
                        stereo_frac=stereo_frac, n_cams=n_cams, bf=bf, pinhole=pinhole)
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    F = int(b["n_frames"])
    b["preint_kf"] = b["preint"]
    pre, pr = [], {k: [] for k in PRIOR_KEYS[:6]}
    scale = np.array([3e2] * 3 + [1e2] * 3 + [3e1] * 3 + [1e3] * 3 + [1e2] * 3)
    for f in range(F):
        t = float(b["t"][f])
        tp = t - frame_dt
        Rp, pp, vp = synth_ba._pose_at(tp)
        ax = rng.normal(0, 1, 3)
        ax /= np.linalg.norm(ax)
        Rq = Rp @ synth_ba._exp(ax * np.deg2rad(prior_rot_deg))
        u, _, vh = np.linalg.svd(Rq)
        pr["prior_Rwb"].append(u @ vh)
        pr["prior_twb"].append(pp + rng.normal(0, prior_trans, 3))
        pr["prior_vel"].append(vp + rng.normal(0, prior_vel, 3))
        pr["prior_bg"].append(rng.normal(0, 1e-4, 3))
        pr["prior_ba"].append(rng.normal(0, 1e-3, 3))
        M = rng.normal(0, 1, (15, 15))
        H = scale[:, None] * (M.T @ M / 15 + np.eye(15)) * scale[None, :]
        pr["prior_H"].append(((H + H.T) / 2).reshape(225))
        pre.append(synth_ba.preintegrate(tp, t))
    for k, v in pr.items():
        b[k] = np.array(v, np.float64)
    b["preint"] = np.stack(pre).astype(np.float32)
    # Frame::mpPrevFrame's vertices: the prior's state through the float setters
    for k in ("Rwb", "twb", "vel", "bg", "ba"):
        b["kf_" + k] = b["prior_" + k].astype(np.float32).astype(np.float64)
    return b


STATE_KEYS = ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba")
INPUT_KEYS = ("kf_Rwb", "kf_twb", "kf_vel", "kf_bg", "kf_ba", "preint", "mono_start", "mono_cam", "mono_kp",
              "mono_obs", "mono_inv_sigma2", "mono_xw", "mono_close", "stereo_start", "stereo_cam", "stereo_kp",
              "stereo_obs", "stereo_inv_sigma2", "stereo_xw")


def as_pose_struct(batch, struct_cls, arrays):
    """Fill an omv_pose_batch from `batch` (host rig arrays) and `arrays` (name -> pointer-bearing array:
    numpy for the oracle, torch device tensors for the product).  Returns (struct, keepalive)."""
    import ctypes
    keep = []

    def hptr(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    def anyptr(a):
        if hasattr(a, "data_ptr"):
            return ctypes.c_void_p(a.data_ptr()) if a.numel() else None
        return ctypes.c_void_p(a.ctypes.data) if a.size else None

    s = struct_cls()
    s.n_frames, s.n_cams = int(batch["n_frames"]), int(batch["n_cams"])
    s.cam = hptr(batch["cam"], np.float32)
    for k in ("Rcb", "tcb", "Rbc", "tbc"):
        setattr(s, k, hptr(batch[k], np.float64))
    s.bf = float(batch["bf"])
    for k in STATE_KEYS + INPUT_KEYS:   # absent keys stay NULL (the pose-only call reads only the edges)
        if k in arrays:
            setattr(s, k, anyptr(arrays[k]))
    s.kp_cap = int(batch["kp_cap"])
    s.n_mono, s.n_stereo = int(len(batch["mono_cam"])), int(len(batch["stereo_cam"]))
    if "cam_model" in batch:
        s.cam_model = hptr(batch["cam_model"], np.int32)
    return s, keep


def as_prior_struct(struct_cls, arrays):
    """Fill an omv_pose_prior from `arrays` (PRIOR_KEYS -> numpy or torch device arrays)."""
    import ctypes
    s = struct_cls()
    for k in PRIOR_KEYS:
        a = arrays[k]
        p = a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data
        setattr(s, k[6:] if k.startswith("prior_") else k, ctypes.c_void_p(p))
    return s


def tile_batch(b, F):
    """Repeat a generated batch's frames (with their edges) up to F frames (cheap large batches)."""
    n0 = int(b["n_frames"])
    out = dict(b)
    fr = [f % n0 for f in range(F)]
    for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "kf_Rwb", "kf_twb", "kf_vel", "kf_bg", "kf_ba", "preint",
              "true_Rwb", "true_twb", "true_vel", "t") + tuple(k for k in PRIOR_KEYS if k in b):
        out[k] = np.ascontiguousarray(np.asarray(b[k])[fr])
    for kind in ("mono", "stereo"):
        st = b[f"{kind}_start"]
        idx = np.concatenate([np.arange(st[f], st[f + 1]) for f in fr]).astype(np.int64)
        counts = np.array([st[f + 1] - st[f] for f in fr])
        out[f"{kind}_start"] = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        for k in [k for k in b if k.startswith(kind + "_") and k != f"{kind}_start"]:
            out[k] = np.ascontiguousarray(np.asarray(b[k])[idx])
    out["n_frames"] = F
    return out


def concat_batches(a, b):
    """Frames of batch `a` then of batch `b` (same rig) in one batch: frames of different sizes in one call."""
    out = dict(a)
    for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "kf_Rwb", "kf_twb", "kf_vel", "kf_bg", "kf_ba", "preint",
              "true_Rwb", "true_twb", "true_vel", "t") + tuple(k for k in PRIOR_KEYS if k in a):
        out[k] = np.ascontiguousarray(np.concatenate([np.asarray(a[k]), np.asarray(b[k])]))
    for kind in ("mono", "stereo"):
        sa, sb = np.asarray(a[f"{kind}_start"]), np.asarray(b[f"{kind}_start"])
        out[f"{kind}_start"] = np.concatenate([sa, sb[1:] + sa[-1]]).astype(np.int32)
        for k in [k for k in a if k.startswith(kind + "_") and k != f"{kind}_start"]:
            out[k] = np.ascontiguousarray(np.concatenate([np.asarray(a[k]), np.asarray(b[k])]))
    out["n_frames"] = int(a["n_frames"]) + int(b["n_frames"])
    out["kp_cap"] = max(int(a["kp_cap"]), int(b["kp_cap"]))
    return out


def quat_of(R):
    """Eigen's Quaternion(const Matrix3&) (quaternionbase_assign_impl), coefficients (x, y, z, w), w >= 0."""
    m = np.asarray(R, np.float64)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    q = np.zeros(4)
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0], q[1], q[2] = (m[2, 1] - m[1, 2]) * t, (m[0, 2] - m[2, 0]) * t, (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    return q if q[3] >= 0 else -q


def quat_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def make_pose_only_batch(n_frames=8, n_pts=300, seed=1, outlier_frac=0.1, n_cams=4, stereo_frac=0.0, bf=40.0,
                         rot_noise_deg=0.5, trans_noise=0.03):
    """Batches for Optimizer::PoseOptimization (Optimizer.cc:855-1278).  n_cams >= 2: the rigid-body branch
    (:981-1120, Kannala-Brandt rig, one mono edge per keypoint on camera c through T_c0 = mTrl / mTsll / mTsrl);
    n_cams == 1: the conventional branch (:911-979, pinhole camera 0) where a keypoint with a right coordinate gets
    an EdgeStereoSE3ProjectXYZOnlyPose INSTEAD of the mono edge (`stereo_frac` of them).  The frame's pose Tcw
    (camera 0) and the rig come through Sophus::SE3f (float quaternion / translation) cast to double, as the
    reference builds its SE3Quats (:871-873, :1040-1042).  Adds pose_q / pose_t [F][4] / [F][3] and rig_q / rig_t
    [n_cams][4] / [3] to make_pose_batch's dict (whose state / IMU arrays the pose-only call ignores)."""
    pin = n_cams == 1
    b = make_pose_batch(n_frames=n_frames, n_pts=n_pts, seed=seed, outlier_frac=outlier_frac,
                        stereo_frac=stereo_frac if pin else 0.0, n_cams=n_cams, bf=bf, rot_noise_deg=rot_noise_deg,
                        trans_noise=trans_noise, pinhole=pin)
    F = int(b["n_frames"])
    if pin and len(b["stereo_cam"]):   # stereo XOR mono per keypoint
        keep = np.ones(len(b["mono_cam"]), bool)
        for f in range(F):
            skp = set(b["stereo_kp"][b["stereo_start"][f]:b["stereo_start"][f + 1]].tolist())
            for e in range(b["mono_start"][f], b["mono_start"][f + 1]):
                if int(b["mono_kp"][e]) in skp:
                    keep[e] = False
        counts = [int(keep[b["mono_start"][f]:b["mono_start"][f + 1]].sum()) for f in range(F)]
        for k in [k for k in b if k.startswith("mono_") and k != "mono_start"]:
            b[k] = np.ascontiguousarray(np.asarray(b[k])[keep])
        b["mono_start"] = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)

    def se3f(R, t):
        q = quat_of(R).astype(np.float32)
        q = (q / np.linalg.norm(q.astype(np.float64))).astype(np.float32)   # Sophus keeps a unit quaternion
        return q.astype(np.float64), np.asarray(t, np.float32).astype(np.float64)

    pq, pt = [], []
    for f in range(F):
        q, t = se3f(b["Rcw"][f][0], b["tcw"][f][0])
        pq.append(q), pt.append(t)
    b["pose_q"], b["pose_t"] = np.array(pq), np.array(pt)
    rq, rt = [np.array([0, 0, 0, 1.0])], [np.zeros(3)]
    for c in range(1, n_cams):   # T_c0 = T_cb T_b0
        R = b["Rcb"][c] @ b["Rcb"][0].T
        t = b["tcb"][c] - R @ b["tcb"][0]
        q, tt = se3f(R, t)
        rq.append(q), rt.append(tt)
    b["rig_q"], b["rig_t"] = np.array(rq), np.array(rt)
    return b
