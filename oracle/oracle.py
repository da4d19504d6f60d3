"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/liboracle.so, the CPU restatement of the
reference (see orb_oracle.cpp / match_oracle.cpp headers).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker / baseline, never as
the thing measured or shipped.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4")])

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", HERE])
        _lib = ctypes.CDLL(LIB)
    return _lib


def use_library(path):
    """Switch the restatement library (the contraction study loads oracle/liboracle_fma.so)."""
    global _lib
    _lib = ctypes.CDLL(path)
    return _lib


def set_contract(mode):
    """0: no contraction (parity mode); 1: GCC's contraction of the reference's own steering products."""
    lib().oracle_set_contract(int(mode))


class _Ptr(ctypes.c_void_p):
    """A c_void_p that keeps its array alive for the duration of the call it is passed to (a temporary
    like `_p(x.copy())` would otherwise be freed before the C function reads it)."""


def _p(a):
    if a is None:
        return None
    p = _Ptr(a.ctypes.data)
    p._keep = a
    return p


def std_sort_pairs(k1, k2):
    """libstdc++ std::sort of (k1, k2) pairs (compareNodes order): the sorted original indices."""
    k1 = np.ascontiguousarray(k1, np.int32)
    k2 = np.ascontiguousarray(k2, np.int32)
    perm = np.zeros(len(k1), np.int32)
    lib().oracle_std_sort_pairs(_p(k1), _p(k2), ctypes.c_int(len(k1)), _p(perm))
    return perm


def orb_tables(nfeatures=1200, scale=1.2, nlevels=8):
    sc, isc, s2, is2 = (np.zeros(nlevels, np.float32) for _ in range(4))
    q = np.zeros(nlevels, np.int32)
    um = np.zeros(16, np.int32)
    lib().oracle_orb_tables(nfeatures, ctypes.c_float(scale), nlevels, _p(sc), _p(isc), _p(s2), _p(is2), _p(q), _p(um))
    return dict(scale=sc, inv_scale=isc, sigma2=s2, inv_sigma2=is2, quota=q, umax=um)


def pyramid_level(img, level, nfeatures=1200, scale=1.2, nlevels=8):
    img = np.ascontiguousarray(img)
    h, w = img.shape
    ow, oh = ctypes.c_int(), ctypes.c_int()
    lib().oracle_orb_pyramid_level(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, level, None,
                                   ctypes.byref(ow), ctypes.byref(oh))
    out = np.zeros((oh.value, ow.value), np.uint8)
    lib().oracle_orb_pyramid_level(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, level, _p(out),
                                   ctypes.byref(ow), ctypes.byref(oh))
    return out


def harris_responses(level_img, xs, ys):
    """OpenCV ORB's HarrisResponses (blockSize 7, k 0.04) at integer level positions (an extra the reference lacks)."""
    L = np.ascontiguousarray(level_img)
    h, w = L.shape
    xs = np.ascontiguousarray(xs, dtype=np.int32)
    ys = np.ascontiguousarray(ys, dtype=np.int32)
    out = np.zeros(len(xs), np.float32)
    lib().oracle_harris_responses(_p(L), w, h, w, _p(xs), _p(ys), len(xs), _p(out))
    return out


def level_candidates(level_img, ini_th, min_th):
    L = np.ascontiguousarray(level_img)
    h, w = L.shape
    cap = 200000
    xs, ys, rs = (np.zeros(cap, np.float32) for _ in range(3))
    n = lib().oracle_orb_level_candidates(_p(L), w, h, ini_th, min_th, _p(xs), _p(ys), _p(rs), cap)
    return xs[:n].copy(), ys[:n].copy(), rs[:n].copy()


def distribute(xs, ys, resp, minX, maxX, minY, maxY, N):
    xs, ys, resp = (np.ascontiguousarray(a, dtype=np.float32) for a in (xs, ys, resp))
    cap = len(xs) + 8
    sel = np.zeros(cap, np.int32)
    n = lib().oracle_orb_distribute(_p(xs), _p(ys), _p(resp), len(xs), minX, maxX, minY, maxY, N, _p(sel), cap)
    return sel[:n].copy()


def orb_extract(img, nfeatures=1200, scale=1.2, nlevels=8, ini_th=15, min_th=7, lapping=(0, 0)):
    """ORBextractor::operator() restated: returns (monoIndex, kps[KP_DTYPE], desc (n,32) u8)."""
    img = np.ascontiguousarray(img)
    h, w = img.shape
    cap = nfeatures + 64 * nlevels
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    mono = ctypes.c_int()
    n = lib().oracle_orb_extract(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, ini_th, min_th,
                                 int(lapping[0]), int(lapping[1]), _p(kps), _p(desc), cap, ctypes.byref(mono))
    return mono.value, kps[:n].copy(), desc[:n].copy()


def orb_extract_frame(imgs, nfeatures, lapping, scale=1.2, nlevels=8, ini_th=15, min_th=7, threaded=True):
    """Multi-camera frame, one std::thread per camera like src/Frame.cc:1841-1862."""
    imgs = np.ascontiguousarray(imgs)
    nc, h, w = imgs.shape
    cap = nfeatures + 64 * nlevels
    kps = np.zeros((nc, cap), KP_DTYPE)
    desc = np.zeros((nc, cap, 32), np.uint8)
    n_out = np.zeros(nc, np.int32)
    mono = np.zeros(nc, np.int32)
    ptrs = (ctypes.c_void_p * nc)(*[imgs[c].ctypes.data for c in range(nc)])
    lap = np.ascontiguousarray(np.asarray(lapping, np.int32).reshape(nc, 2))
    lib().oracle_orb_extract_frame(nc, ptrs, w, h, w, nfeatures, ctypes.c_float(scale), nlevels, ini_th, min_th,
                                   _p(lap), _p(kps), _p(desc), cap, _p(n_out), _p(mono), int(threaded))
    return n_out, mono, kps, desc


def fast_atan2(y, x):
    f = lib().oracle_fast_atan2
    f.restype = ctypes.c_float
    return f(ctypes.c_float(y), ctypes.c_float(x))


class FrameGeom(ctypes.Structure):
    _fields_ = [("n_cams", ctypes.c_int), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float), ("nlevels", ctypes.c_int),
                ("scale_factors", ctypes.c_float * 16), ("cam_model", ctypes.c_int * 8)]


def frame_geom(n_cams, width, height, scale_factors, cam_model=None):
    """omv_frame_geom; cam_model: per block 0 (KannalaBrandt8) / 1 (Pinhole), default all KB8."""
    g = FrameGeom()
    g.n_cams, g.min_x, g.max_x, g.min_y, g.max_y = n_cams, 0.0, float(width), 0.0, float(height)
    g.nlevels = len(scale_factors)
    for i, s in enumerate(scale_factors):
        g.scale_factors[i] = float(s)
    for i, m in enumerate(cam_model if cam_model is not None else ()):
        g.cam_model[i] = int(m)
    return g


def grid(geom, kps, n_kp, cam):
    """Frame::AssignFeaturesToGrid of one camera: (cell_start[3073], idx[])."""
    kps = np.ascontiguousarray(kps)
    n_kp = np.ascontiguousarray(n_kp, np.int32)
    cap = kps.shape[1]
    cs = np.zeros(64 * 48 + 1, np.int32)
    idx = np.zeros(cap, np.int32)
    n = lib().oracle_grid(ctypes.byref(geom), _p(kps), cap, _p(n_kp), cam, _p(cs), _p(idx))
    return cs, idx[:n]


def features_in_area(geom, kps, n_kp, x, y, r, min_level, max_level, cam):
    kps = np.ascontiguousarray(kps)
    n_kp = np.ascontiguousarray(n_kp, np.int32)
    out = np.zeros(kps.shape[1], np.int32)
    n = lib().oracle_features_in_area(ctypes.byref(geom), _p(kps), kps.shape[1], _p(n_kp), ctypes.c_float(x),
                                      ctypes.c_float(y), ctypes.c_float(r), min_level, max_level, cam, _p(out),
                                      kps.shape[1])
    return out[:n]


def search_by_projection(geom, kps, desc, n_kp, mp, th, far_points, th_far, nnratio, l2r, r2l, occ_init, kp_to_mp):
    """ORBmatcher::SearchByProjection(Frame&, MPs, ...) restated; mutates kp_to_mp, returns nmatches."""
    kps = np.ascontiguousarray(kps)
    desc = np.ascontiguousarray(desc)
    n_kp = np.ascontiguousarray(n_kp, np.int32)
    cap = kps.shape[1]
    M = mp["desc"].shape[0]
    a = {k: np.ascontiguousarray(v) for k, v in mp.items()}
    l2r = np.ascontiguousarray(l2r, np.int32)
    r2l = np.ascontiguousarray(r2l, np.int32)
    occ = np.ascontiguousarray(occ_init, np.uint8) if occ_init is not None else np.zeros(kps.shape[0] * cap, np.uint8)
    assert kp_to_mp.dtype == np.int32 and kp_to_mp.flags.c_contiguous
    f = lib().oracle_search_by_projection
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + \
        [ctypes.c_void_p] * 9 + [ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_float, ctypes.c_float] + \
        [ctypes.c_void_p] * 4
    return f(ctypes.cast(ctypes.byref(geom), ctypes.c_void_p), _p(kps), _p(desc), cap, _p(n_kp), _p(a["desc"]),
             _p(a["proj_x"]), _p(a["proj_y"]), _p(a["view_cos"]), _p(a["level"]), _p(a["in_view"]),
             _p(a["track_depth"]), _p(a["is_bad"]), _p(a["has_obs"]), M, th, int(far_points), th_far, nnratio,
             _p(l2r), _p(r2l), _p(occ), _p(kp_to_mp))


def bf_knn2(q, t):
    q = np.ascontiguousarray(q, np.uint8)
    t = np.ascontiguousarray(t, np.uint8)
    nq, nt = q.shape[0], t.shape[0]
    idx2 = np.zeros((nq, 2), np.int32)
    dist2 = np.zeros((nq, 2), np.int32)
    lib().oracle_bf_knn2(_p(q), nq, _p(t), nt, _p(idx2), _p(dist2))
    return idx2, dist2


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oracle_descriptor_distance(_p(a), _p(b))


class RigF(ctypes.Structure):
    _fields_ = [("n_cams", ctypes.c_int), ("cam", (ctypes.c_float * 8) * 8), ("R_cl", (ctypes.c_float * 9) * 8),
                ("t_cl", (ctypes.c_float * 3) * 8), ("t_lc", (ctypes.c_float * 3) * 8), ("min_x", ctypes.c_float),
                ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("log_scale_factor", ctypes.c_float), ("n_levels", ctypes.c_int),
                ("model", ctypes.c_int * 8)]


def frustum(rig, pose, pos, normal, min_dist, max_dist, cos_limit=0.5, view_cos=None, track_depth=None):
    """Frame::isInFrustum restated for one frame.  rig: a ctypes struct with omv_rig's layout (copied);
    pose: float32 [24]; pos/normal [M, 3], min/max_dist [M].  view_cos / track_depth: prior values
    (left untouched where the reference leaves them).  Returns (dict, n_in_view)."""
    r = RigF.from_buffer_copy(bytes(rig))
    M, C = len(pos), r.n_cams
    pose = np.ascontiguousarray(pose, np.float32)
    pos = np.ascontiguousarray(pos, np.float32)
    normal = np.ascontiguousarray(normal, np.float32)
    mind = np.ascontiguousarray(min_dist, np.float32)
    maxd = np.ascontiguousarray(max_dist, np.float32)
    out = dict(proj_x=np.zeros((M, C), np.float32), proj_y=np.zeros((M, C), np.float32),
               view_cos=np.array(view_cos if view_cos is not None else np.zeros((M, C)), np.float32),
               level=np.zeros((M, C), np.int32), in_view=np.zeros((M, C), np.uint8),
               track_depth=np.array(track_depth if track_depth is not None else np.zeros(M), np.float32))
    n = lib().oracle_frustum(ctypes.byref(r), _p(pose), _p(pos), _p(normal), _p(mind), _p(maxd), M,
                             ctypes.c_float(cos_limit), _p(out["proj_x"]), _p(out["proj_y"]), _p(out["view_cos"]),
                             _p(out["level"]), _p(out["in_view"]), _p(out["track_depth"]))
    return out, n


class SE3F(ctypes.Structure):
    _fields_ = [("q", ctypes.c_float * 4), ("t", ctypes.c_float * 3)]


def _se3(v):
    v = np.asarray(v, np.float32).reshape(7)
    return SE3F((ctypes.c_float * 4)(*v[:4].tolist()), (ctypes.c_float * 3)(*v[4:].tolist()))


def search_last_frame(geom, kps, desc, n_kp, cams, Tcw, Tlw, Trl, last_pos, last_desc, last_valid, last_obs,
                      last_kps, th, bMono, mb, check_ori, occ_init, kp_to_mp):
    """ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) restated for one frame.
    kp_to_mp is modified in place (last-frame slots); returns nmatches."""
    C, cap = kps.shape[0], kps.shape[1]
    kps = np.ascontiguousarray(kps)
    desc = np.ascontiguousarray(desc, np.uint8)
    n_kp = np.ascontiguousarray(n_kp, np.int32)
    cams = np.ascontiguousarray(np.asarray(cams, np.float32).reshape(-1, 8))
    S = len(last_valid)
    lp = np.ascontiguousarray(last_pos, np.float32)
    ld = np.ascontiguousarray(last_desc, np.uint8)
    lv = np.ascontiguousarray(last_valid, np.uint8)
    lo = np.ascontiguousarray(last_obs, np.uint8)
    lk = np.ascontiguousarray(last_kps)
    occ = np.ascontiguousarray(occ_init if occ_init is not None else np.zeros(C * cap), np.uint8)
    t1, t2, t3 = _se3(Tcw), _se3(Tlw), _se3(Trl)
    return lib().oracle_search_last_frame(ctypes.byref(geom), _p(kps), _p(desc), cap, _p(n_kp), _p(cams),
                                          ctypes.byref(t1), ctypes.byref(t2), ctypes.byref(t3), _p(lp), _p(ld), _p(lv),
                                          _p(lo), _p(lk), S, ctypes.c_float(th), int(bMono), ctypes.c_float(mb),
                                          int(check_ori), _p(occ), _p(kp_to_mp))


# ---- LocalInertialBA ------------------------------------------------------------------------------
_VP = ctypes.c_void_p


# the omv_lba_* structs of include/omv.h (ctypes layouts shared with the product binding)
from openmavis_amd._lib import LbaOpts, LbaProblem, LbaResult  # noqa: E402


def lba_evaluate(prob):
    from openmavis_amd.synth_ba import as_struct
    s, keep = as_struct(prob, LbaProblem)
    E, I = s.n_mono, s.n_imu
    S = s.n_stereo
    me, jx, jp = np.zeros((E, 2)), np.zeros((E, 6)), np.zeros((E, 12))
    ie, ij = np.zeros((I, 9)), np.zeros((I, 9, 24))
    se, sx, sp = np.zeros((S, 3)), np.zeros((S, 9)), np.zeros((S, 18))
    lib().oracle_lba_evaluate(ctypes.byref(s), _p(me), _p(jx), _p(jp), _p(ie), _p(ij), _p(se), _p(sx), _p(sp))
    return dict(mono_err=me, mono_jx=jx, mono_jp=jp, imu_err=ie, imu_jac=ij, stereo_err=se, stereo_jx=sx,
                stereo_jp=sp)


def lba_optimize(prob, opt_it=4, lambda_init=1e-2, max_trials=10, large=True, log_cap=256):
    """LocalInertialBA optimisation restated; returns (result dict, final state dict, trial log)."""
    from openmavis_amd.synth_ba import as_struct, read_state
    s, keep = as_struct(prob, LbaProblem)
    o = LbaOpts(opt_it, lambda_init, max_trials, int(large))
    chi2 = np.zeros(s.n_mono)
    outl = np.zeros(s.n_mono, np.uint8)
    s_chi2 = np.zeros(s.n_stereo)
    s_outl = np.zeros(s.n_stereo, np.uint8)
    r = LbaResult()
    r.mono_chi2, r.mono_outlier = _p(chi2), _p(outl)
    r.stereo_chi2, r.stereo_outlier = _p(s_chi2), _p(s_outl)
    log = np.zeros((log_cap, 3))
    lib().oracle_lba_optimize(ctypes.byref(s), ctypes.byref(o), ctypes.byref(r), _p(log), log_cap)
    res = dict(err=r.err, err_end=r.err_end, status=r.status, iterations=r.iterations, trials=r.trials,
               lambda_=r.lambda_, mono_chi2=chi2, mono_outlier=outl, stereo_chi2=s_chi2, stereo_outlier=s_outl)
    return res, read_state(keep), log[:r.trials].copy()


# ---- PoseInertialOptimizationLastKeyFrame ---------------------------------------------------------
def pose_last_kf(batch, rec_init=False):
    """Restated Optimizer::PoseInertialOptimizationLastKeyFrame on every frame of a synth_pose batch.
    Returns (state dict, kp_outlier [F][kp_cap] uint8, n_good [F], H [F][225])."""
    from openmavis_amd._lib import PoseBatch
    from openmavis_amd.synth_pose import INPUT_KEYS, STATE_KEYS, as_pose_struct
    arrays = {}
    for k in STATE_KEYS:
        arrays[k] = np.array(batch[k], np.float64, copy=True, order="C")
    for k in INPUT_KEYS:
        arrays[k] = np.ascontiguousarray(batch[k])
    s, keep = as_pose_struct(batch, PoseBatch, arrays)
    F, cap = int(batch["n_frames"]), int(batch["kp_cap"])
    kpo = np.full((F, cap), 255, np.uint8)
    n_good = np.zeros(F, np.int32)
    H = np.zeros((F, 225))
    for f in range(F):
        lib().oracle_pose_inertial_last_kf(ctypes.byref(s), f, int(bool(rec_init)), _p(kpo[f]),
                                           _p(n_good[f:f + 1]), _p(H[f]))
    del keep
    return {k: arrays[k] for k in STATE_KEYS}, kpo, n_good, H


# ---- PoseInertialOptimizationLastFrame ------------------------------------------------------------
def pose_last_frame(batch, rec_init=False, frames=None):
    """Restated Optimizer::PoseInertialOptimizationLastFrame on the frames of a
    synth_pose.make_last_frame_batch batch (all, or the indices in `frames`).  Returns (state dict,
    kp_outlier [F][kp_cap] uint8, n_good [F], H [F][225]: Marginalize's frame block)."""
    from openmavis_amd._lib import PoseBatch, PosePrior
    from openmavis_amd.synth_pose import INPUT_KEYS, PRIOR_KEYS, STATE_KEYS, as_pose_struct, as_prior_struct
    arrays = {}
    for k in STATE_KEYS:
        arrays[k] = np.array(batch[k], np.float64, copy=True, order="C")
    for k in INPUT_KEYS + PRIOR_KEYS:
        arrays[k] = np.ascontiguousarray(batch[k])
    s, keep = as_pose_struct(batch, PoseBatch, arrays)
    pr = as_prior_struct(PosePrior, arrays)
    F, cap = int(batch["n_frames"]), int(batch["kp_cap"])
    kpo = np.full((F, cap), 255, np.uint8)
    n_good = np.zeros(F, np.int32)
    H = np.zeros((F, 225))
    for f in (range(F) if frames is None else frames):
        lib().oracle_pose_inertial_last_frame(ctypes.byref(s), ctypes.byref(pr), f, int(bool(rec_init)), _p(kpo[f]),
                                              _p(n_good[f:f + 1]), _p(H[f]))
    del keep
    return {k: arrays[k] for k in STATE_KEYS}, kpo, n_good, H


# ---- PoseOptimization -------------------------------------------------------------------------------
def pose_optimization(batch, frames=None):
    """Restated Optimizer::PoseOptimization on the frames of a synth_pose.make_pose_only_batch batch (all, or the
    indices in `frames`).  Returns (pose_q [F][4], pose_t [F][3], kp_outlier [F][kp_cap] uint8, n_good [F])."""
    from openmavis_amd._lib import PoseBatch
    from openmavis_amd.synth_pose import INPUT_KEYS, STATE_KEYS, as_pose_struct
    arrays = {k: np.ascontiguousarray(batch[k]) for k in STATE_KEYS + INPUT_KEYS}
    s, keep = as_pose_struct(batch, PoseBatch, arrays)
    F, cap = int(batch["n_frames"]), int(batch["kp_cap"])
    pq = np.array(batch["pose_q"], np.float64, copy=True, order="C")
    pt = np.array(batch["pose_t"], np.float64, copy=True, order="C")
    rq = np.ascontiguousarray(batch["rig_q"], np.float64)
    rt = np.ascontiguousarray(batch["rig_t"], np.float64)
    kpo = np.full((F, cap), 255, np.uint8)
    n_good = np.zeros(F, np.int32)
    for f in (range(F) if frames is None else frames):
        n_good[f] = lib().oracle_pose_optimization(ctypes.byref(s), _p(rq), _p(rt), f, _p(pq[f]), _p(pt[f]), _p(kpo[f]))
    del keep
    return pq, pt, kpo, n_good


def pose_edges_from_matches(kps, n_kp, kp_to_mp, mp_pos, mp_track_depth, inv_level_sigma2, uright=None):
    """The visual-edge creation loop of PoseInertialOptimizationLastKeyFrame / LastFrame restated for the
    multi-camera frame (bRight; src/Optimizer.cc:5079-5330 and :5640-5800): walk the keypoints in the
    concatenated [L | R | SL | SR] order (slot = cam * kp_cap + i); a keypoint with a map point gets an
    EdgeMonoOnlyPose of its block (obs = the raw keypoint, invSigma2 = mvInvLevelSigma2[octave] /
    uncertainty2 (= 1), bClose = mTrackDepth < 10) and, when mvuRight > 0, an EdgeStereoOnlyPose (obs x, y,
    u_R).  kps: structured omv_kp [C][kp_cap] (x, y, octave fields).  Returns the edge-list dict of a
    one-frame pose batch (mono_* / stereo_*, starts [0, n])."""
    C, cap = kps.shape
    lv = np.asarray(inv_level_sigma2, np.float32)
    mono = {k: [] for k in ("cam", "kp", "obs", "w", "xw", "close")}
    st = {k: [] for k in ("cam", "kp", "obs", "w", "xw")}
    for c in range(C):
        for i in range(int(n_kp[c])):
            s = c * cap + i
            mp = int(kp_to_mp[s])
            if mp < 0:
                continue
            k = kps[c, i]
            w = lv[min(int(k["octave"]) & 15, len(lv) - 1)]
            xw = np.asarray(mp_pos[mp], np.float32)
            mono["cam"].append(c), mono["kp"].append(s), mono["obs"].append([float(k["x"]), float(k["y"])])
            mono["w"].append(w), mono["xw"].append(xw), mono["close"].append(mp_track_depth[mp] < np.float32(10))
            ur = np.float32(uright[c, i]) if uright is not None else np.float32(-1)
            if ur > 0:
                st["cam"].append(c), st["kp"].append(s), st["obs"].append([float(k["x"]), float(k["y"]), float(ur)])
                st["w"].append(w), st["xw"].append(xw)
    return dict(mono_start=np.array([0, len(mono["cam"])], np.int32), mono_cam=np.array(mono["cam"], np.int32),
                mono_kp=np.array(mono["kp"], np.int32), mono_obs=np.array(mono["obs"], np.float64).reshape(-1, 2),
                mono_inv_sigma2=np.array(mono["w"], np.float32),
                mono_xw=np.array(mono["xw"], np.float32).reshape(-1, 3), mono_close=np.array(mono["close"], np.uint8),
                stereo_start=np.array([0, len(st["cam"])], np.int32), stereo_cam=np.array(st["cam"], np.int32),
                stereo_kp=np.array(st["kp"], np.int32), stereo_obs=np.array(st["obs"], np.float64).reshape(-1, 3),
                stereo_inv_sigma2=np.array(st["w"], np.float32),
                stereo_xw=np.array(st["xw"], np.float32).reshape(-1, 3))


def pose_constraint(H):
    """ConstraintPoseImu ctor restated on [n][225] matrices."""
    H = np.ascontiguousarray(H, np.float64).reshape(-1, 225)
    out = np.zeros_like(H)
    for i in range(len(H)):
        lib().oracle_pose_constraint(_p(H[i]), _p(out[i]))
    return out


# ---- SearchForTriangulation -----------------------------------------------------------------------
def search_for_triangulation(pair, only_stereo=False, coarse=False, check_ori=False):
    """Restated ORBmatcher::SearchForTriangulation on a synth_tri pair: (nmatches, match12 [kf1.n])."""
    from openmavis_amd._lib import KfView, TriPair
    from openmavis_amd.synth_tri import kf_struct
    keep = []

    def arr(_name, a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    p = TriPair()
    p.kf1 = kf_struct(pair["kf1"], KfView, pair["level_sigma2"], arr)
    p.kf2 = kf_struct(pair["kf2"], KfView, pair["level_sigma2"], arr)
    for i in range(10):
        for j in range(12):
            p.T[i][j] = float(pair["T"][i, j])
    m12 = np.full(pair["kf1"]["n"], -7, np.int32)
    p.match12 = ctypes.c_void_p(m12.ctypes.data)
    cams = np.ascontiguousarray(pair["cams"], np.float32)
    cm = pair.get("cam_model")
    cm = None if cm is None else np.ascontiguousarray(cm, np.int32)
    lib().oracle_search_for_triangulation.restype = ctypes.c_int
    n = lib().oracle_search_for_triangulation(ctypes.byref(p), _p(cams), _p(cm), int(only_stereo), int(coarse),
                                              int(check_ori))
    return n, m12


def eigen_inverse3(m):
    """Eigen Matrix3f::inverse() restated (cofactor formula), float32 [3][3]."""
    m = np.ascontiguousarray(m, np.float32).reshape(3, 3)
    r = np.zeros((3, 3), np.float32)
    lib().oracle_eigen_inverse3(_p(m), _p(r))
    return r


def pinhole_epipolar(k1, k2, kp1, kp2, R12, t12, unc):
    """Pinhole::epipolarConstrain restated: bool.  kp1 / kp2: one-element KP_DTYPE arrays."""
    f = lib().oracle_pinhole_epipolar
    f.restype = ctypes.c_int
    a = [np.ascontiguousarray(x, np.float32) for x in (k1, k2, R12, t12)]
    return bool(f(_p(a[0]), _p(a[1]), _p(np.ascontiguousarray(kp1)), _p(np.ascontiguousarray(kp2)), _p(a[2]), _p(a[3]),
                  ctypes.c_float(unc)))


def kb8_unproject(cam, x, y):
    ray = np.zeros(3, np.float32)
    lib().oracle_kb8_unproject(_p(np.ascontiguousarray(cam, np.float32)), ctypes.c_float(x), ctypes.c_float(y), _p(ray))
    return ray


def jacobi_svd4_v(A):
    A = np.ascontiguousarray(A, np.float32).reshape(4, 4)
    V = np.zeros((4, 4), np.float32)
    lib().oracle_jacobi_svd4_v(_p(A), _p(V))
    return V


def stereo_triangulate(kpsL, nL, kpsR, nR, cams, Rlr, tlr, sigma2, l2r):
    """Frame::ComputeMultiFishEyeMatches' depth check on Lowe candidates l2r [nL] (right index or -1):
    returns (l2r, r2l [nR], depth [nL], p3d [nL][3])."""
    l2r = np.ascontiguousarray(l2r[:nL], np.int32).copy()
    r2l = np.full(max(nR, 1), -1, np.int32)
    depth = np.zeros(max(nL, 1), np.float32)
    p3d = np.zeros((max(nL, 1), 3), np.float32)
    c = np.ascontiguousarray(cams, np.float32).reshape(-1, 8)
    lib().oracle_stereo_triangulate(_p(np.ascontiguousarray(kpsL)), int(nL), _p(np.ascontiguousarray(kpsR)), int(nR),
                                    _p(c[0].copy()), _p(c[1].copy()), _p(np.ascontiguousarray(Rlr, np.float32)),
                                    _p(np.ascontiguousarray(tlr, np.float32)), _p(np.ascontiguousarray(sigma2, np.float32)),
                                    _p(l2r), _p(r2l), _p(depth), _p(p3d))
    return l2r, r2l[:nR], depth[:nL], p3d[:nL]


def depth_from_undistorted(keys, depth, undist, bf):
    """GetDepthFromUndistortedPoints for one camera block: keys (KP_DTYPE [n]), depth float [h][w],
    undist an omv_fisheye_undist (openmavis_amd._lib.FisheyeUndist).  Returns (u_right [n], xy [n][2])."""
    keys = np.ascontiguousarray(keys)
    n = len(keys)
    d = np.ascontiguousarray(depth, np.float32)
    ur = np.zeros(max(n, 1), np.float32)
    xy = np.zeros((max(n, 1), 2), np.float32)
    lib().oracle_depth_from_undistorted(_p(keys) if n else None, int(n), _p(d), int(d.shape[1]), int(d.shape[0]),
                                        ctypes.byref(undist), ctypes.c_float(bf), _p(ur), _p(xy))
    return ur[:n], xy[:n]


# ---- keyframe-side projection searches -----------------------------------------------------------------
def search_kf(b, th, max_dist, check_ori=True):
    """Restated ORBmatcher::Fuse / Fuse(Sim3) / SearchByProjection(KF, Sim3) / SearchByProjection(Frame&, KF)
    on a synth_kfmatch batch (mode b["mode"]).  Returns (best_idx, best_dist, n_matches, kp_match)."""
    from openmavis_amd._lib import FrameGeom, KfSearchJob
    from openmavis_amd.matcher import kf_search_params
    g = FrameGeom()
    g.n_cams, g.min_x, g.max_x, g.min_y, g.max_y, g.nlevels = b["n_cams"], 0.0, float(b["width"]), 0.0, \
        float(b["height"]), b["nlevels"]
    s = np.float32(1.0)
    for i in range(b["nlevels"]):
        g.scale_factors[i] = float(s)
        s = np.float32(s * np.float32(1.2))
    for c, mdl in enumerate(b.get("cam_model", ())):
        g.cam_model[c] = int(mdl)
    uright = np.ascontiguousarray(b["uright"], np.float32)
    angle = np.ascontiguousarray(b["mp_angle"], np.float32)
    p = kf_search_params(th, max_dist, b["cams"], bf=float(b["bf"]), nlevels=b["nlevels"])
    p.uright, p.mp_angle = _p(uright), _p(angle)
    p.mode, p.check_ori = int(b["mode"]), int(bool(check_ori))
    jobs = (KfSearchJob * len(b["jobs"]))()
    for i, jb in enumerate(b["jobs"]):
        jobs[i].kf, jobs[i].cam = jb["kf"], jb["cam"]
        T = np.asarray(jb["Tcw"], np.float32)
        for q in range(4):
            jobs[i].Tcw.q[q] = float(T[q])
        for q in range(3):
            jobs[i].Tcw.t[q] = float(T[4 + q])
            jobs[i].Ow[q] = float(jb["Ow"][q])
        jobs[i].mp_start, jobs[i].mp_count = jb["mp_start"], jb["mp_count"]
    n_e = len(b["mp_list"])
    best_idx = np.zeros(n_e, np.int32)
    best_dist = np.zeros(n_e, np.int32)
    n_m = np.zeros(len(b["jobs"]), np.int32)
    kp_match = np.array(b["kp_match"], np.int32, copy=True)
    m = b["mps"]
    lib().oracle_search_kf(ctypes.byref(g), _p(np.ascontiguousarray(b["kps"])), _p(np.ascontiguousarray(b["desc"])),
                           int(b["kp_cap"]), _p(np.ascontiguousarray(b["n_kp"], np.int32)), int(b["n_kf"]),
                           len(b["jobs"]), jobs, _p(b["mp_list"]), _p(m["pos"]), _p(m["normal"]), _p(m["min_dist"]),
                           _p(m["max_dist"]), _p(m["desc"]), ctypes.byref(p), _p(kp_match), _p(best_idx),
                           _p(best_dist), _p(n_m))
    return best_idx, best_dist, n_m, kp_match


# ---- IMU preintegration ---------------------------------------------------------------------------------
def preintegrate(b, Nga, NgaWalk):
    """IMU::Preintegrated::IntegrateNewMeasurement restated on every record of a synth_imu batch from
    Initialize(bias).  Returns (records [n][292] float32, avg [n][6])."""
    n = len(b["start"]) - 1
    rec = np.zeros((n, 292), np.float32)
    rec[:, [0, 4, 8]] = 1.0
    rec[:, 60:66] = b["bias"]
    avg = np.zeros((n, 6), np.float32)
    Nga = np.ascontiguousarray(Nga, np.float32)
    NgaWalk = np.ascontiguousarray(NgaWalk, np.float32)
    meas = np.ascontiguousarray(b["meas"], np.float32)
    for r in range(n):
        s0, s1 = int(b["start"][r]), int(b["start"][r + 1])
        lib().oracle_preintegrate(_p(rec[r]), _p(avg[r]), _p(meas[s0:s1]), s1 - s0, _p(Nga), _p(NgaWalk))
    return rec, avg


# ---- DBoW2 vocabulary transform ---------------------------------------------------------------------------
def bow_transform(v, desc, n_desc, levelsup):
    """TemplatedVocabulary::transform(features, BowVector, FeatureVector, levelsup) restated per set of a
    synth_bow vocabulary dict.  Returns a list of dicts (word, wval, node, bow_word, bow_value, fv_node,
    fv_start, fv_idx) per set."""
    from openmavis_amd._lib import Vocab
    keep = {k: np.ascontiguousarray(v[k]) for k in ("child_start", "child_ids", "desc", "word_id", "weight")}
    voc = Vocab(len(v["weight"]), v["n_words"], v["L"], v["scoring"], v["weighting"],
                *[ctypes.c_void_p(keep[k].ctypes.data) for k in ("child_start", "child_ids", "desc", "word_id",
                                                                 "weight")])
    out = []
    for s in range(desc.shape[0]):
        n = int(n_desc[s])
        d = np.ascontiguousarray(desc[s, :n])
        word, node, bw, fvn, fvi = (np.zeros(max(n, 1), np.int32) for _ in range(5))
        wval, bv = np.zeros(max(n, 1)), np.zeros(max(n, 1))
        fvs = np.zeros(n + 1, np.int32)
        nb, nf = ctypes.c_int32(), ctypes.c_int32()
        lib().oracle_bow_transform(ctypes.byref(voc), _p(d), n, int(levelsup), _p(word), _p(wval), _p(node), _p(bw),
                                   _p(bv), ctypes.byref(nb), _p(fvn), _p(fvs), _p(fvi), ctypes.byref(nf))
        out.append(dict(word=word[:n], wval=wval[:n], node=node[:n], bow_word=bw[:nb.value], bow_value=bv[:nb.value],
                        fv_node=fvn[:nf.value], fv_start=fvs[:nf.value + 1], fv_idx=fvi[:fvs[nf.value]]))
    return out


# ---- SearchByBoW / SearchForInitialization ---------------------------------------------------------
def search_by_bow(job, kf_kf=False, nnratio=0.75, check_ori=True):
    """Restated ORBmatcher::SearchByBoW on a job {kf, other} of synth keyframe dicts (numpy):
    (nmatches, match) with match [other.n] ((KF, F)) or [kf.n] ((KF1, KF2))."""
    from openmavis_amd._lib import BowJob, KfView, OMV_BOW_KF_FRAME, OMV_BOW_KF_KF
    from openmavis_amd.synth_tri import kf_struct
    keep = []

    def arr(_name, a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    j = BowJob()
    j.kf = kf_struct(job["kf"], KfView, np.ones(16), arr)
    j.other = kf_struct(job["other"], KfView, np.ones(16), arr)
    m = np.full(job["kf"]["n"] if kf_kf else job["other"]["n"], -7, np.int32)
    j.match = ctypes.c_void_p(m.ctypes.data)
    f = lib().oracle_search_by_bow
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int]
    n = f(ctypes.cast(ctypes.byref(j), ctypes.c_void_p), OMV_BOW_KF_KF if kf_kf else OMV_BOW_KF_FRAME, nnratio,
          int(check_ori))
    return n, m


def search_for_initialization(geom, kps1, desc1, kps2, desc2, prev, window=100, nnratio=0.9, check_ori=True):
    """Restated ORBmatcher::SearchForInitialization: (nmatches, vnMatches12 [n1], vbPrevMatched [n1][2]).
    kps*: structured (KP_DTYPE) arrays of mvKeysUn; geom: F2's frame geometry."""
    kps1, kps2 = np.ascontiguousarray(kps1), np.ascontiguousarray(kps2)
    desc1, desc2 = np.ascontiguousarray(desc1, np.uint8), np.ascontiguousarray(desc2, np.uint8)
    prev = np.array(prev, np.float32, copy=True).reshape(-1, 2)
    m12 = np.full(len(kps1), -7, np.int32)
    f = lib().oracle_search_for_initialization
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    n = f(ctypes.cast(ctypes.byref(geom), ctypes.c_void_p), _p(kps1), _p(desc1), len(kps1), _p(kps2), _p(desc2),
          len(kps2), _p(prev), int(window), nnratio, int(check_ori), _p(m12))
    return n, m12, prev


# ---- SearchBySim3 ------------------------------------------------------------------------------------
def _kf_geom(b):
    from openmavis_amd._lib import FrameGeom
    g = FrameGeom()
    g.n_cams, g.min_x, g.max_x, g.min_y, g.max_y, g.nlevels = b["n_cams"], 0.0, float(b["width"]), 0.0, \
        float(b["height"]), b["nlevels"]
    s = np.float32(1.0)
    for i in range(b["nlevels"]):
        g.scale_factors[i] = float(s)
        s = np.float32(s * np.float32(1.2))
    return g


def search_by_sim3(b, th=7.5):
    """Restated ORBmatcher::SearchBySim3 on a synth_sim3 batch: (match12 [n1] per side-1 entry, n_found [jobs])."""
    from openmavis_amd.matcher import sim3_job_array
    g = _kf_geom(b)
    jobs = sim3_job_array(b["jobs"])
    m = b["mps"]
    kp1, mp1 = np.ascontiguousarray(b["kp1"], np.int32), np.ascontiguousarray(b["mp1"], np.int32)
    kp2, mp2 = np.ascontiguousarray(b["kp2"], np.int32), np.ascontiguousarray(b["mp2"], np.int32)
    match12 = np.full(max(len(kp1), 1), -7, np.int32)
    n_found = np.zeros(max(len(b["jobs"]), 1), np.int32)
    f = lib().oracle_search_by_sim3
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + \
        [ctypes.c_void_p] * 9 + [ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    f(ctypes.cast(ctypes.byref(g), ctypes.c_void_p), _p(np.ascontiguousarray(b["kps"])),
      _p(np.ascontiguousarray(b["desc"])), int(b["kp_cap"]), _p(np.ascontiguousarray(b["n_kp"], np.int32)),
      int(b["n_kf"]), len(b["jobs"]), ctypes.cast(jobs, ctypes.c_void_p), _p(kp1), _p(mp1), _p(kp2), _p(mp2),
      _p(m["pos"]), _p(m["min_dist"]), _p(m["max_dist"]), _p(m["desc"]), float(th), float(np.float32(np.log(np.float64(np.float32(1.2))))),
      int(b["nlevels"]), _p(match12), _p(n_found))
    return match12[:len(kp1)], n_found[:len(b["jobs"])]


def distinctive_descriptors(desc, desc_start, desc_row):
    """MapPoint::ComputeDistinctiveDescriptors restated (mappoint_oracle.cpp): the chosen row per point, -1 if none."""
    desc = np.ascontiguousarray(desc, np.uint8)
    start = np.ascontiguousarray(desc_start, np.int32)
    rows = np.ascontiguousarray(desc_row, np.int32)
    n = len(start) - 1
    best = np.zeros(max(n, 0), np.int32)
    lib().oracle_distinctive_descriptors(ctypes.c_int(n), _p(start), _p(rows), _p(desc), _p(best))
    return best


def normal_depth(obs_start, obs_center, pos, ref_center, ref_level_scale, ref_max_scale):
    """MapPoint::UpdateNormalAndDepth restated: (normal [P][3], min_dist [P], max_dist [P]) float32; NaN where the
    point has no entries (untouched)."""
    start = np.ascontiguousarray(obs_start, np.int32)
    cen = np.ascontiguousarray(obs_center, np.float32)
    P = np.ascontiguousarray(pos, np.float32)
    rc = np.ascontiguousarray(ref_center, np.float32)
    ls = np.ascontiguousarray(ref_level_scale, np.float32)
    ms = np.ascontiguousarray(ref_max_scale, np.float32)
    n = len(start) - 1
    normal = np.full((n, 3), np.nan, np.float32)
    dmin = np.full(n, np.nan, np.float32)
    dmax = np.full(n, np.nan, np.float32)
    lib().oracle_normal_depth(ctypes.c_int(n), _p(start), _p(cen), _p(P), _p(rc), _p(ls), _p(ms), _p(normal), _p(dmin),
                              _p(dmax))
    return normal, dmin, dmax


def create_new_map_points(d, inertial=True, far_points=False, th_far=50.0, check_baseline=False, side1_state=0):
    """omv_create_new_map_points restated (tri_oracle.cpp) on a synth_cnmp set: the jobs in order with the state chain.
    Returns per job (status [kf1.n] int32: 1 triangulated, 2 UnprojectStereo, 0 none; x3D [kf1.n][3] float32); the
    has_mp1 marks and the final side-1 state are attached as attributes of the returned list."""
    from openmavis_amd._lib import CnmpJob, CnmpKf, KfView
    from openmavis_amd.synth_cnmp import cnmp_kf_struct
    keep = []

    def arr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    k1 = cnmp_kf_struct(d["kf1"], d, CnmpKf, KfView, arr)
    jobs = (CnmpJob * len(d["jobs"]))()
    outs = []
    for j, jb in enumerate(d["jobs"]):
        jobs[j].kf2 = cnmp_kf_struct(jb["kf2"], d, CnmpKf, KfView, arr)
        jobs[j].match12 = arr(np.ascontiguousarray(jb["match12"], np.int32))
        st = np.full(d["kf1"]["n"], -9, np.int32)
        x = np.full((d["kf1"]["n"], 3), np.nan, np.float32)
        jobs[j].x3D, jobs[j].status = arr(x), arr(st)
        outs.append((st, x))
    cams = np.ascontiguousarray(d["cams"], np.float32)
    cm = np.ascontiguousarray(d["cam_model"], np.int32)
    has_mp1 = np.zeros(max(int(d["kf1"]["n"]), 1), np.uint8)
    s1 = np.array([side1_state], np.int32)
    lib().oracle_create_new_map_points(ctypes.c_int(len(d["jobs"])), ctypes.byref(k1), jobs, _p(cams), _p(cm),
                                       ctypes.c_int(d["n_cams"]), ctypes.c_int(int(inertial)),
                                       ctypes.c_int(int(far_points)), ctypes.c_float(th_far),
                                       ctypes.c_float(d["scale_factor"]), ctypes.c_int(int(check_baseline)), _p(s1),
                                       _p(has_mp1))
    outs = _Outs(outs)
    outs.has_mp1, outs.side1 = has_mp1[:int(d["kf1"]["n"])], int(s1[0])
    return outs


class _Outs(list):
    pass


def local_mapping_create_new_map_points(d, inertial=True, monocular=False, coarse=False, far_points=False,
                                        th_far=50.0, side1_state=0, has_mp1=None, nb_range=None):
    """LocalMapping::CreateNewMapPoints' whole neighbour loop restated (tri_oracle.cpp) on a synth_cnmp.make_cnmp_chain
    set: (has_mp1 [kf1.n] uint8, n_matches [n_neigh], per neighbour (match12, status, x3D), final side-1 state).
    nb_range = (lo, hi) runs only those neighbours, from `has_mp1` / `side1_state` (composition checks)."""
    from openmavis_amd._lib import CnmpJob, CnmpKf, KfView, TriPair
    from openmavis_amd.synth_cnmp import chain_kf_struct
    from openmavis_amd.synth_tri import kf_struct
    keep = []

    def arr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    nbs = d["nbs"] if nb_range is None else d["nbs"][nb_range[0]:nb_range[1]]
    n1 = int(d["kf1"]["n"])
    k1 = chain_kf_struct(d["kf1"], d, CnmpKf, KfView, arr)
    pairs = (TriPair * max(len(nbs), 1))()
    jobs = (CnmpJob * max(len(nbs), 1))()
    outs = []
    for j, nb in enumerate(nbs):
        pairs[j].kf1 = kf_struct(d["kf1"], KfView, d["sigma2"], lambda _n, a: arr(a))
        pairs[j].kf2 = kf_struct(nb["kf2"], KfView, d["sigma2"], lambda _n, a: arr(a))
        for i in range(10):
            for q in range(12):
                pairs[j].T[i][q] = float(nb["T"][i, q])
        m12 = np.full(max(n1, 1), -9, np.int32)
        st = np.full(max(n1, 1), -9, np.int32)
        x = np.full((max(n1, 1), 3), np.nan, np.float32)
        pairs[j].match12 = arr(m12)
        jobs[j].kf2 = chain_kf_struct(nb["kf2"], d, CnmpKf, KfView, arr)
        jobs[j].match12, jobs[j].x3D, jobs[j].status = pairs[j].match12, arr(x), arr(st)
        keep.extend([m12, st, x])
        outs.append((m12, st, x))
    skip = np.ascontiguousarray([int(nb.get("skip", 0)) for nb in nbs] or [0], np.int32)
    hm = np.array(d["kf1"]["has_mp"] if has_mp1 is None else has_mp1, np.uint8, copy=True)
    n_matches = np.zeros(max(len(nbs), 1), np.int32)
    s1 = np.array([side1_state], np.int32)
    cams = np.ascontiguousarray(d["cams"], np.float32)
    cm = np.ascontiguousarray(d["cam_model"], np.int32)
    lib().oracle_local_mapping_create_new_map_points(
        ctypes.byref(k1), _p(hm), ctypes.c_int(len(nbs)), pairs, jobs, _p(skip), _p(cams), _p(cm),
        ctypes.c_int(d["n_cams"]), ctypes.c_int(int(inertial)), ctypes.c_int(int(not monocular)),
        ctypes.c_int(int(coarse)), ctypes.c_int(int(far_points)), ctypes.c_float(th_far),
        ctypes.c_float(d["scale_factor"]), _p(n_matches), _p(s1))
    return hm, n_matches[:len(nbs)], [(m[:n1], s[:n1], x[:n1]) for m, s, x in outs], int(s1[0])


# ---- LocalMapping::SearchInNeighbors' fuse sequence ---------------------------------------------------------------
def search_in_neighbors_fuse(s, th=3.0, obs_cap=None, log_cap=None):
    """The reference's phase A / phase B Fuse loop restated literally (match_oracle.cpp oracle_search_in_neighbors_fuse)
    on a synth_fuse scene: returns dict(kf_mps, bad, n_obs, replaced, obs_start, obs_kf, obs_idx, log, n_fused, desc)."""
    from openmavis_amd._lib import FrameGeom, FuseGraph
    from openmavis_amd.matcher import kf_search_params
    from openmavis_amd.synth_fuse import fuse_graph_struct
    keep = []

    def arr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    obs_cap = obs_cap or 4 * len(s["obs_kf"]) + 1024
    log_cap = log_cap or 4 * int(s["n_mps"]) + 1024
    out = {}
    G = fuse_graph_struct(s, FuseGraph, arr, out, obs_cap, log_cap)
    g = FrameGeom()
    g.n_cams, g.min_x, g.max_x, g.min_y, g.max_y, g.nlevels = s["n_cams"], 0.0, float(s["width"]), 0.0, \
        float(s["height"]), s["nlevels"]
    sc = np.float32(1.0)
    for i in range(s["nlevels"]):
        g.scale_factors[i] = float(sc)
        sc = np.float32(sc * np.float32(1.2))
    uright = np.ascontiguousarray(s["uright"], np.float32)
    p = kf_search_params(th, 50.0, s["cams"], bf=float(s["bf"]), nlevels=s["nlevels"])
    p.uright = _p(uright)
    p.mode = 0
    m = {k: np.ascontiguousarray(v) for k, v in s["mps"].items()}
    mdesc = np.array(m["desc"], np.uint8, copy=True)
    C, T = int(s["n_cams"]), len(s["targets"])
    n_fused = np.zeros(T * C + C, np.int32)
    targets = np.ascontiguousarray(s["targets"], np.int32)
    f = lib().oracle_search_in_neighbors_fuse
    f.restype = ctypes.c_int
    rc = f(ctypes.byref(g), _p(np.ascontiguousarray(s["kps"])), _p(np.ascontiguousarray(s["desc"])),
           _p(np.ascontiguousarray(s["n_kp"], np.int32)), int(s["kp_cap"]), ctypes.byref(G), int(s["current"]), T,
           _p(targets), _p(m["pos"]), _p(m["normal"]), _p(m["min_dist"]), _p(m["max_dist"]), _p(mdesc),
           ctypes.byref(p), _p(n_fused))
    assert rc == 0, "oracle capacity"
    n_rows = int(out["out_obs_start"][-1])
    return dict(kf_mps=out["kf_mps"], bad=out["bad"], n_obs=out["n_obs"], replaced=out["replaced"][:s["n_mps"]],
                obs_start=out["out_obs_start"], obs_kf=out["out_obs_kf"][:n_rows], obs_idx=out["out_obs_idx"][:n_rows],
                log=out["log"][:G.n_log], n_fused=n_fused, desc=mdesc)
