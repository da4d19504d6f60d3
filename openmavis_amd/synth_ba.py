"""Seeded synthetic LocalInertialBA problems.

50 keyframes at 10 Hz on a smooth 1 m/s trajectory; the latest `n_opt` (25) are optimisable (window
order: current keyframe first, like Optimizer::LocalInertialBA's vpOptimizableKFs), the rest fixed.
A 5-camera Kannala-Brandt rig with the Hilti-2022 intrinsics/extrinsics
(Examples/Multi-Inertial/HiltiChallenge2022.yaml; camera 5 = camera 3 rotated 20 deg so it overlaps).
20,000 points, each observed in 3 consecutive keyframes x 2 cameras (120,000 EdgeMono), observations =
projection + N(0, 0.7 px), point init = truth + N(0, 5 cm), optimisable poses perturbed by 0.5 deg /
2 cm, invSigma2 from an octave U{0..7}.  One EdgeInertial (+GyroRW, AccRW) per optimisable keyframe
from a 400 Hz preintegration of the true motion (ImuTypes.cc:160-239 formulas, float32 outputs); the
edge to the fixed keyframe is robust with information x 1e-2 (Optimizer.cc:2978-2987).
"""
import numpy as np

from .synth_ba_const import CAMS, T_B_C1, T_C1_C2, T_B_C3, T_B_C4, IMU_NOISE

PREINT_FLOATS = 292
G = np.array([0.0, 0.0, -float(np.float32(9.81))])


def _hat(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]], dtype=np.float64)


def _exp(w):
    d = np.linalg.norm(w)
    W = _hat(w)
    if d < 1e-9:
        return np.eye(3) + W
    return np.eye(3) + W * np.sin(d) / d + W @ W * (1 - np.cos(d)) / (d * d)


def _rightJ(w):
    d = np.linalg.norm(w)
    W = _hat(w)
    if d < 1e-9:
        return np.eye(3)
    return np.eye(3) - W * (1 - np.cos(d)) / d ** 2 + W @ W * (d - np.sin(d)) / d ** 3


def kb8_project(k, X):
    """KannalaBrandt8::project in double (vectorised; generation only)."""
    x, y, z = X[..., 0], X[..., 1], X[..., 2]
    r = np.sqrt(x * x + y * y)
    th = np.arctan2(r, z)
    psi = np.arctan2(y, x)
    rr = th + k[4] * th ** 3 + k[5] * th ** 5 + k[6] * th ** 7 + k[7] * th ** 9
    return np.stack([k[0] * rr * np.cos(psi) + k[2], k[1] * rr * np.sin(psi) + k[3]], -1)


def pinhole_project(k, X):
    """Pinhole::project in double (vectorised; generation only)."""
    return np.stack([k[0] * X[..., 0] / X[..., 2] + k[2], k[1] * X[..., 1] / X[..., 2] + k[3]], -1)


def cam_project(k, X, pinhole=False):
    return pinhole_project(k, X) if pinhole else kb8_project(k, X)


def rig():
    """(cam params [5][8] float32, Rbc [5][3][3], tbc [5][3]) — camera -> body."""
    Tbc = [T_B_C1, T_B_C1 @ T_C1_C2, T_B_C3, T_B_C4]
    a = np.deg2rad(20.0)
    Ry = np.array([[np.cos(a), 0, np.sin(a), 0], [0, 1, 0, 0], [-np.sin(a), 0, np.cos(a), 0], [0, 0, 0, 1]])
    Tbc.append(T_B_C3 @ Ry)
    cams = np.array(CAMS + [CAMS[2]], dtype=np.float32)
    Rbc = np.stack([T[:3, :3] for T in Tbc])
    # re-orthonormalise the YAML's 8-digit rotations so the rig is an exact rigid transform
    for i in range(len(Rbc)):
        u, _, vt = np.linalg.svd(Rbc[i])
        Rbc[i] = u @ vt
    tbc = np.stack([T[:3, 3] for T in Tbc])
    return cams, Rbc, tbc


def trajectory(n_kf, dt=0.1, speed=1.0, yaw_rate=0.15):
    """Body poses (Rwb, twb, vwb) at keyframe times on a planar arc with a gentle pitch wobble."""
    t = np.arange(n_kf) * dt
    return [_pose_at(ti, speed, yaw_rate) for ti in t]


def _pose_at(t, speed=1.0, yaw_rate=0.15):
    yaw = yaw_rate * t
    pitch = 0.03 * np.sin(0.7 * t)
    Rz = np.array([[np.cos(yaw), -np.sin(yaw), 0], [np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]])
    Ry = np.array([[np.cos(pitch), 0, np.sin(pitch)], [0, 1, 0], [-np.sin(pitch), 0, np.cos(pitch)]])
    R = Rz @ Ry
    if yaw_rate != 0:
        p = np.array([speed / yaw_rate * np.sin(yaw), speed / yaw_rate * (1 - np.cos(yaw)), 0.05 * np.sin(0.5 * t)])
    else:
        p = np.array([speed * t, 0.0, 0.05 * np.sin(0.5 * t)])
    v = np.array([speed * np.cos(yaw), speed * np.sin(yaw), 0.025 * np.cos(0.5 * t)])
    return R, p, v


def preintegrate(t0, t1, freq=400.0, speed=1.0, yaw_rate=0.15):
    """IMU::Preintegrated::IntegrateNewMeasurement over [t0, t1) from exact kinematics (zero bias)."""
    ng, na, ngw, naw = IMU_NOISE
    sf = np.sqrt(freq)
    Nga = np.diag([(ng * sf) ** 2] * 3 + [(na * sf) ** 2] * 3)
    NgaWalk = np.diag([ngw ** 2] * 3 + [naw ** 2] * 3)
    dR, dV, dP = np.eye(3), np.zeros(3), np.zeros(3)
    JRg, JVg, JVa, JPg, JPa = (np.zeros((3, 3)) for _ in range(5))
    C = np.zeros((15, 15))
    n = int(round((t1 - t0) * freq))
    h = (t1 - t0) / n
    for s in range(n):
        ta, tb = t0 + s * h, t0 + (s + 1) * h
        Ra, pa, va = _pose_at(ta, speed, yaw_rate)
        Rb, pb, vb = _pose_at(tb, speed, yaw_rate)
        w = _log(Ra.T @ Rb) / h
        acc_w = (vb - va) / h
        a = Ra.T @ (acc_w - G)
        theta = np.linalg.norm(w)
        W = _hat(w)
        if theta < 1e-9:
            J1 = h * np.eye(3) + 0.5 * h * h * W
            J2 = 0.5 * h * h * np.eye(3) + h ** 3 / 6 * W
        else:
            J1 = h * np.eye(3) + (1 - np.cos(h * theta)) / theta ** 2 * W + (h * theta - np.sin(h * theta)) / theta ** 3 * W @ W
            J2 = (0.5 * h * h * np.eye(3) + (h * theta - np.sin(h * theta)) / theta ** 3 * W
                  + (0.5 * h * h * theta ** 2 + np.cos(h * theta) - 1) / theta ** 4 * W @ W)
        dP = dP + dV * h + dR @ J2 @ a
        dV = dV + dR @ J1 @ a
        A = np.eye(9, 15)
        B = np.zeros((9, 6))
        Wa = _hat(a)
        A[3:6, 0:3] = -dR @ _hat(J1 @ a)
        A[6:9, 0:3] = -dR @ _hat(J2 @ a)
        A[6:9, 3:6] = h * np.eye(3)
        A[0:3, 9:12] = -h * np.eye(3)
        A[3:6, 12:15] = -dR @ J1
        A[6:9, 12:15] = -dR @ J2
        B[3:6, 3:6] = dR @ J1
        B[6:9, 3:6] = dR @ J2
        JPa = JPa + JVa * h - dR @ J2
        JPg = JPg + JVg * h - dR @ J2 @ Wa @ JRg
        JVa = JVa - dR @ J1
        JVg = JVg - dR @ J1 @ Wa @ JRg
        dRi = _exp(w * h)
        rJ = _rightJ(w * h)
        dR = dR @ dRi
        u, _, vt = np.linalg.svd(dR)
        dR = u @ vt
        A[0:3, 0:3] = dRi.T
        B[0:3, 0:3] = rJ * h
        C[:9, :9] = A @ C @ A.T + B @ Nga @ B.T
        C[9:, 9:] += h * h * NgaWalk
        JRg = dRi.T @ JRg - rJ * h
    out = np.concatenate([dR.ravel(), dV, dP, JRg.ravel(), JVg.ravel(), JVa.ravel(), JPg.ravel(), JPa.ravel(),
                          np.zeros(6), [t1 - t0], C.ravel()])
    assert out.size == PREINT_FLOATS
    return out.astype(np.float32)


def _log(R):
    c = np.clip((np.trace(R) - 1) / 2, -1, 1)
    th = np.arccos(c)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) / 2
    return w if th < 1e-12 else w * th / np.sin(th)


def make_lba_problem(n_kf=50, n_opt=25, n_pts=20000, seed=5, obs_noise=0.7, pt_noise=0.05, rot_noise_deg=0.5,
                     trans_noise=0.02, n_cams=5, stereo_frac=0.0, bf=40.0, pinhole=False):
    """stereo_frac > 0: that fraction of the camera-0 observations become EdgeStereo observations
    (u, v, u_R = u - bf / z + noise), as LocalInertialBA creates them for keypoints with a right
    coordinate / depth (Optimizer.cc:3108-3143); drawn from a separate stream, so the rest of the
    window is the same as with stereo_frac = 0.  pinhole: every camera a Pinhole (fx fy cx cy of the Hilti
    cameras, Pinhole.cpp), problem["cam_model"] = OMV_CAM_PINHOLE per camera."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cams, Rbc, tbc = rig()
    cams, Rbc, tbc = cams[:n_cams], Rbc[:n_cams], tbc[:n_cams]
    Rcb = np.transpose(Rbc, (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc)
    true = trajectory(n_kf)
    # keyframe array order: optimisable newest-first (ids n_kf-1 .. n_kf-n_opt), then fixed newest-first
    ids = list(range(n_kf - 1, -1, -1))
    slot = {kid: s for s, kid in enumerate(ids)}
    Rwb_t = np.stack([true[k][0] for k in ids])
    twb_t = np.stack([true[k][1] for k in ids])
    vel_t = np.stack([true[k][2] for k in ids])

    def cam_pose(R, t):
        Rbw = R.T
        tbw = -Rbw @ t
        Rcw = np.einsum("cij,jk->cik", Rcb, Rbw)
        tcw = np.einsum("cij,j->ci", Rcb, tbw) + tcb
        return Rcw, tcw

    # points: 3 consecutive keyframes (at least one optimisable) x 2 cameras
    first_opt_id = n_kf - n_opt
    pts_t, obs_pt, obs_kf, obs_cam, obs_uv = [], [], [], [], []
    while len(pts_t) < n_pts:
        s = int(rng.integers(max(0, first_opt_id - 2), n_kf - 2))
        trip = [s, s + 1, s + 2]
        c1 = int(rng.integers(0, n_cams))
        Rcw1, tcw1 = cam_pose(*true[s + 1][:2])
        # random direction within 60 deg of camera c1's axis, depth 2..20 m
        d = rng.normal(0, 1, 3)
        d[2] = abs(d[2]) * 1.5 + 0.6
        d /= np.linalg.norm(d)
        Xc = d * rng.uniform(2.0, 20.0)
        Xw = Rcw1[c1].T @ (Xc - tcw1[c1])
        others = [c for c in rng.permutation(n_cams) if c != c1]
        chosen = None
        for c2 in [c1] + list(others):
            if c2 == c1:
                continue
            ok = True
            for k in trip:
                Rcw, tcw = cam_pose(*true[k][:2])
                for c in (c1, c2):
                    X = Rcw[c] @ Xw + tcw[c]
                    if X[2] < 0.3:
                        ok = False
                        break
                    uv = cam_project(cams[c].astype(np.float64), X, pinhole)
                    if not (5 <= uv[0] <= 715 and 5 <= uv[1] <= 535):
                        ok = False
                        break
                if not ok:
                    break
            if ok:
                chosen = c2
                break
        if chosen is None:
            continue
        p = len(pts_t)
        pts_t.append(Xw)
        for k in trip:
            Rcw, tcw = cam_pose(*true[k][:2])
            for c in (c1, chosen):
                uv = cam_project(cams[c].astype(np.float64), Rcw[c] @ Xw + tcw[c], pinhole) + rng.normal(0, obs_noise, 2)
                obs_pt.append(p)
                obs_kf.append(slot[k])
                obs_cam.append(c)
                obs_uv.append(uv)
    pts_t = np.array(pts_t)
    # initial state
    Rwb = Rwb_t.copy()
    twb = twb_t.copy()
    for s in range(n_opt):
        ax = rng.normal(0, 1, 3)
        ax /= np.linalg.norm(ax)
        Rwb[s] = Rwb_t[s] @ _exp(ax * np.deg2rad(rot_noise_deg))
        u, _, vt = np.linalg.svd(Rwb[s])
        Rwb[s] = u @ vt
        twb[s] = twb_t[s] + rng.normal(0, trans_noise, 3)
    Rcw = np.zeros((n_kf, n_cams, 3, 3))
    tcw = np.zeros((n_kf, n_cams, 3))
    for s in range(n_kf):
        Rcw[s], tcw[s] = cam_pose(Rwb[s], twb[s])
    vel = vel_t + np.concatenate([rng.normal(0, 0.02, (n_opt, 3)), np.zeros((n_kf - n_opt, 3))])
    bg = np.concatenate([rng.normal(0, 1e-4, (n_opt, 3)), np.zeros((n_kf - n_opt, 3))])
    ba = np.concatenate([rng.normal(0, 1e-3, (n_opt, 3)), np.zeros((n_kf - n_opt, 3))])
    pts = pts_t + rng.normal(0, pt_noise, pts_t.shape)
    # inertial edges: window keyframe s (id ids[s]) with its previous keyframe (id - 1)
    imu_kf1, imu_kf2, pre = [], [], []
    for s in range(n_opt):
        kid = ids[s]
        imu_kf1.append(slot[kid - 1])
        imu_kf2.append(s)
        pre.append(preintegrate((kid - 1) * 0.1, kid * 0.1))
    imu_robust = np.zeros(n_opt, np.uint8)
    imu_robust[n_opt - 1] = 1
    imu_scale = np.ones(n_opt, np.float32)
    imu_scale[n_opt - 1] = 1e-2
    inv_sig = (1.0 / np.float32(1.2) ** (2 * rng.integers(0, 8, len(obs_pt)))).astype(np.float32)
    obs_pt, obs_kf, obs_cam = np.array(obs_pt, np.int32), np.array(obs_kf, np.int32), np.array(obs_cam, np.int32)
    obs_uv = np.array(obs_uv, np.float64)
    st = np.zeros(len(obs_pt), bool)
    if stereo_frac > 0:
        srng = np.random.Generator(np.random.PCG64(seed + 7919))
        st = (obs_cam == 0) & (srng.random(len(obs_pt)) < stereo_frac)
    st_obs = np.zeros((len(obs_pt), 3))
    for e in np.nonzero(st)[0]:
        k = obs_kf[e]
        Rc_t, tc_t = cam_pose(Rwb_t[k], twb_t[k])
        z = (Rc_t[0] @ pts_t[obs_pt[e]] + tc_t[0])[2]
        st_obs[e, :2] = obs_uv[e]
        st_obs[e, 2] = np.float32(obs_uv[e, 0] - bf / z + srng.normal(0, obs_noise))   # mvuRight is a float
    st &= st_obs[:, 2] >= 0   # mvuRight < 0 means "no right coordinate": an EdgeMono (:3075)
    st_obs = st_obs[st]
    extra = dict(n_stereo=int(st.sum()), stereo_pt=obs_pt[st], stereo_kf=obs_kf[st], stereo_obs=st_obs,
                 stereo_inv_sigma2=inv_sig[st], bf=np.float32(bf)) if stereo_frac > 0 else {}
    keep_m = ~st
    obs_pt, obs_kf, obs_cam, obs_uv, inv_sig = obs_pt[keep_m], obs_kf[keep_m], obs_cam[keep_m], obs_uv[keep_m], inv_sig[keep_m]
    if pinhole:
        extra["cam_model"] = np.full(n_cams, 1, np.int32)   # OMV_CAM_PINHOLE
    return dict(**extra,
        n_cams=n_cams, cam=cams, Rcb=Rcb, tcb=tcb, Rbc=Rbc, tbc=tbc, n_kf=n_kf, n_opt=n_opt,
        kf_imu=np.ones(n_kf, np.uint8), Rwb=Rwb, twb=twb, Rcw=Rcw, tcw=tcw, vel=vel, bg=bg, ba=ba,
        pts=pts, pt_track_depth=rng.uniform(1.0, 60.0, len(pts)).astype(np.float32),
        mono_pt=obs_pt, mono_kf=obs_kf, mono_cam=obs_cam, mono_obs=obs_uv, mono_inv_sigma2=inv_sig,
        imu_kf1=np.array(imu_kf1, np.int32), imu_kf2=np.array(imu_kf2, np.int32), preint=np.stack(pre),
        imu_robust=imu_robust, imu_info_scale=imu_scale,
        truth=dict(Rwb=Rwb_t, twb=twb_t, pts=pts_t),
    )


# ---- ctypes view (shared by the product binding and the oracle wrapper) -----------------------------
DOUBLE_FIELDS = ("Rcb", "tcb", "Rbc", "tbc", "Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts", "mono_obs")


def as_struct(prob, struct_cls):
    """Fill an omv_lba_problem ctypes struct from a problem dict; returns (struct, keepalive dict)."""
    import ctypes
    keep = {}

    def arr(name, dtype):
        a = np.array(prob[name], dtype=dtype, order="C", copy=True)   # never alias the caller's arrays
        keep[name] = a
        return ctypes.c_void_p(a.ctypes.data)

    s = struct_cls()
    s.n_cams = int(prob["n_cams"])
    s.cam = arr("cam", np.float32)
    for f in ("Rcb", "tcb", "Rbc", "tbc", "Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts", "mono_obs"):
        setattr(s, f, arr(f, np.float64))
    s.n_kf, s.n_opt = int(prob["n_kf"]), int(prob["n_opt"])
    s.kf_imu = arr("kf_imu", np.uint8)
    s.n_pts = int(len(prob["pts"]))
    s.pt_track_depth = arr("pt_track_depth", np.float32)
    s.n_mono = int(len(prob["mono_pt"]))
    for f in ("mono_pt", "mono_kf", "mono_cam", "imu_kf1", "imu_kf2"):
        setattr(s, f, arr(f, np.int32))
    s.mono_inv_sigma2 = arr("mono_inv_sigma2", np.float32)
    s.n_imu = int(len(prob["imu_kf1"]))
    s.preint = arr("preint", np.float32)
    s.imu_robust = arr("imu_robust", np.uint8)
    s.imu_info_scale = arr("imu_info_scale", np.float32)
    s.n_stereo = int(len(prob.get("stereo_pt", ())))
    if s.n_stereo:
        for f in ("stereo_pt", "stereo_kf"):
            setattr(s, f, arr(f, np.int32))
        s.stereo_obs = arr("stereo_obs", np.float64)
        s.stereo_inv_sigma2 = arr("stereo_inv_sigma2", np.float32)
    s.bf = float(prob.get("bf", 0.0))
    if "cam_model" in prob:
        s.cam_model = arr("cam_model", np.int32)
    return s, keep


def read_state(keep):
    """The (possibly updated) state arrays of a keepalive dict, as a dict of copies."""
    return {k: keep[k].copy() for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts")}
