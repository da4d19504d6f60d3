"""ctypes binding of libomv_hip.so (the C ABI in include/omv.h).

There is deliberately no CPU fallback: if the HIP library is missing or no GPU is visible, every
product entry point raises.  The CPU oracle under oracle/ is test infrastructure only.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libomv_hip.so")

OMV_OK = 0
OMV_ERR_ARG = 1
OMV_ERR_HIP = 2
OMV_ERR_CAPACITY = 3
OMV_ERR_NO_DEVICE = 4
CAM_KB8 = 0       # OMV_CAM_KB8
CAM_PINHOLE = 1   # OMV_CAM_PINHOLE
_ERRS = {1: "bad argument", 2: "HIP runtime error", 3: "device capacity exceeded", 4: "no HIP device"}


class OmvError(RuntimeError):
    pass


def check(status, what="omv call"):
    if status != OMV_OK:
        raise OmvError(f"{what} failed: {_ERRS.get(status, status)} ({status})")


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int),
                ("ini_th_fast", ctypes.c_int), ("min_th_fast", ctypes.c_int)]


class KeyPoint(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float),
                ("angle", ctypes.c_float), ("response", ctypes.c_float), ("octave", ctypes.c_int32)]


class FrameGeom(ctypes.Structure):
    _fields_ = [("n_cams", ctypes.c_int), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float), ("nlevels", ctypes.c_int),
                ("scale_factors", ctypes.c_float * 16), ("cam_model", ctypes.c_int * 8)]


class MpView(ctypes.Structure):
    _fields_ = [("desc", ctypes.c_void_p), ("proj_x", ctypes.c_void_p), ("proj_y", ctypes.c_void_p),
                ("view_cos", ctypes.c_void_p), ("level", ctypes.c_void_p), ("in_view", ctypes.c_void_p),
                ("track_depth", ctypes.c_void_p), ("is_bad", ctypes.c_void_p), ("has_obs", ctypes.c_void_p)]


class Rig(ctypes.Structure):
    """omv_rig (include/omv.h)."""
    _fields_ = [("n_cams", ctypes.c_int), ("cam", (ctypes.c_float * 8) * 8), ("R_cl", (ctypes.c_float * 9) * 8),
                ("t_cl", (ctypes.c_float * 3) * 8), ("t_lc", (ctypes.c_float * 3) * 8), ("min_x", ctypes.c_float),
                ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("log_scale_factor", ctypes.c_float), ("n_levels", ctypes.c_int),
                ("model", ctypes.c_int * 8)]


class SE3f(ctypes.Structure):
    """omv_se3f: Sophus::SE3f as unit quaternion (x, y, z, w) + translation."""
    _fields_ = [("q", ctypes.c_float * 4), ("t", ctypes.c_float * 3)]


class Vocab(ctypes.Structure):
    """omv_vocab (include/omv.h)."""
    _fields_ = [("n_nodes", ctypes.c_int), ("n_words", ctypes.c_int), ("L", ctypes.c_int), ("scoring", ctypes.c_int),
                ("weighting", ctypes.c_int)] + [(n, ctypes.c_void_p) for n in (
                    "child_start", "child_ids", "desc", "word_id", "weight")]


class KfSearchJob(ctypes.Structure):
    """omv_kf_search_job (include/omv.h)."""
    _fields_ = [("kf", ctypes.c_int), ("cam", ctypes.c_int), ("Tcw", SE3f), ("Ow", ctypes.c_float * 3),
                ("mp_start", ctypes.c_int), ("mp_count", ctypes.c_int)]


class Sim3f(ctypes.Structure):
    """omv_sim3f (include/omv.h)."""
    _fields_ = [("q", ctypes.c_float * 4), ("t", ctypes.c_float * 3), ("scale", ctypes.c_float)]


class Sim3Job(ctypes.Structure):
    """omv_sim3_job (include/omv.h)."""
    _fields_ = [("kf1", ctypes.c_int), ("kf2", ctypes.c_int), ("T1w", SE3f), ("T2w", SE3f), ("S12", Sim3f),
                ("S21", Sim3f), ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("start1", ctypes.c_int), ("count1", ctypes.c_int), ("start2", ctypes.c_int),
                ("count2", ctypes.c_int)]


class KfMps(ctypes.Structure):
    """omv_kf_mps (include/omv.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("pos", "normal", "min_dist", "max_dist", "desc")]


class KfSearchParams(ctypes.Structure):
    """omv_kf_search_params (include/omv.h)."""
    _fields_ = [("mode", ctypes.c_int), ("th", ctypes.c_float), ("max_dist", ctypes.c_float), ("bf", ctypes.c_float),
                ("uright", ctypes.c_void_p), ("inv_level_sigma2", ctypes.c_float * 16),
                ("log_scale_factor", ctypes.c_float), ("n_levels", ctypes.c_int), ("cams", (ctypes.c_float * 8) * 8),
                ("check_ori", ctypes.c_int), ("mp_angle", ctypes.c_void_p)]


OMV_KF_FUSE, OMV_KF_FUSE_SIM3, OMV_KF_SBP_SIM3, OMV_KF_SBP_FRAME = 0, 1, 2, 3


class LastFrame(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("valid", ctypes.c_void_p),
                ("has_obs", ctypes.c_void_p), ("kps", ctypes.c_void_p), ("S", ctypes.c_int)]


class MpWorld(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_void_p), ("normal", ctypes.c_void_p), ("min_dist", ctypes.c_void_p),
                ("max_dist", ctypes.c_void_p)]


class MpTrack(ctypes.Structure):
    _fields_ = [("proj_x", ctypes.c_void_p), ("proj_y", ctypes.c_void_p), ("view_cos", ctypes.c_void_p),
                ("level", ctypes.c_void_p), ("in_view", ctypes.c_void_p), ("track_depth", ctypes.c_void_p)]


# omv_frame_pose: Rcw[9] tcw[3] Rwc[9] Ow[3] floats = 24 floats per frame (pass a float32 [F, 24] array)
FRAME_POSE_FLOATS = 24


class LbaProblem(ctypes.Structure):
    """omv_lba_problem (include/omv.h)."""
    _fields_ = [("n_cams", ctypes.c_int), ("cam", ctypes.c_void_p), ("Rcb", ctypes.c_void_p),
                ("tcb", ctypes.c_void_p), ("Rbc", ctypes.c_void_p), ("tbc", ctypes.c_void_p),
                ("n_kf", ctypes.c_int), ("n_opt", ctypes.c_int), ("kf_imu", ctypes.c_void_p),
                ("Rwb", ctypes.c_void_p), ("twb", ctypes.c_void_p), ("Rcw", ctypes.c_void_p),
                ("tcw", ctypes.c_void_p), ("vel", ctypes.c_void_p), ("bg", ctypes.c_void_p),
                ("ba", ctypes.c_void_p), ("n_pts", ctypes.c_int), ("pts", ctypes.c_void_p),
                ("pt_track_depth", ctypes.c_void_p), ("n_mono", ctypes.c_int), ("mono_pt", ctypes.c_void_p),
                ("mono_kf", ctypes.c_void_p), ("mono_cam", ctypes.c_void_p), ("mono_obs", ctypes.c_void_p),
                ("mono_inv_sigma2", ctypes.c_void_p), ("n_imu", ctypes.c_int), ("imu_kf1", ctypes.c_void_p),
                ("imu_kf2", ctypes.c_void_p), ("preint", ctypes.c_void_p), ("imu_robust", ctypes.c_void_p),
                ("imu_info_scale", ctypes.c_void_p), ("n_stereo", ctypes.c_int), ("stereo_pt", ctypes.c_void_p),
                ("stereo_kf", ctypes.c_void_p), ("stereo_obs", ctypes.c_void_p),
                ("stereo_inv_sigma2", ctypes.c_void_p), ("bf", ctypes.c_float), ("cam_model", ctypes.c_void_p)]


class PoseBatch(ctypes.Structure):
    """omv_pose_batch (include/omv.h)."""
    _fields_ = [("n_frames", ctypes.c_int), ("n_cams", ctypes.c_int), ("cam", ctypes.c_void_p),
                ("Rcb", ctypes.c_void_p), ("tcb", ctypes.c_void_p), ("Rbc", ctypes.c_void_p), ("tbc", ctypes.c_void_p),
                ("bf", ctypes.c_float)] + [(n, ctypes.c_void_p) for n in (
                    "Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "kf_Rwb", "kf_twb", "kf_vel", "kf_bg", "kf_ba",
                    "preint", "mono_start", "mono_cam", "mono_kp", "mono_obs", "mono_inv_sigma2", "mono_xw",
                    "mono_close", "stereo_start", "stereo_cam", "stereo_kp", "stereo_obs", "stereo_inv_sigma2",
                    "stereo_xw")] + [("kp_cap", ctypes.c_int), ("n_mono", ctypes.c_int), ("n_stereo", ctypes.c_int),
                                   ("cam_model", ctypes.c_void_p)]


class PosePrior(ctypes.Structure):
    """omv_pose_prior (include/omv.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("Rwb", "twb", "vel", "bg", "ba", "H", "preint_kf")]


class KfView(ctypes.Structure):
    """omv_kf_view (include/omv.h)."""
    _fields_ = [("n", ctypes.c_int), ("n_left", ctypes.c_int), ("n_right", ctypes.c_int),
                ("n_sideleft", ctypes.c_int), ("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("has_mp", ctypes.c_void_p), ("n_nodes", ctypes.c_int), ("node_id", ctypes.c_void_p),
                ("node_start", ctypes.c_void_p), ("node_idx", ctypes.c_void_p), ("level_sigma2", ctypes.c_float * 16)]


OMV_TRI_PAIRS = 10


class CnmpKf(ctypes.Structure):
    """omv_cnmp_kf (include/omv.h)."""
    _fields_ = [("kf", KfView), ("kps_raw", ctypes.c_void_p), ("Tcw", (ctypes.c_float * 12) * 4),
                ("Ow", (ctypes.c_float * 3) * 4), ("Rwc", ctypes.c_float * 9), ("twc", ctypes.c_float * 3),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("invfx", ctypes.c_float), ("invfy", ctypes.c_float), ("mb", ctypes.c_float), ("mbf", ctypes.c_float),
                ("uright", ctypes.c_void_p), ("depth", ctypes.c_void_p), ("scale_factors", ctypes.c_float * 16)]


class CnmpJob(ctypes.Structure):
    """omv_cnmp_job (include/omv.h)."""
    _fields_ = [("kf2", CnmpKf), ("match12", ctypes.c_void_p), ("x3D", ctypes.c_void_p), ("status", ctypes.c_void_p)]


class FuseGraph(ctypes.Structure):
    """omv_fuse_graph (include/omv.h)."""
    _fields_ = [("n_kf", ctypes.c_int), ("n_blocks", ctypes.c_void_p), ("Tcw", ctypes.c_void_p), ("Ow", ctypes.c_void_p),
                ("uright", ctypes.c_void_p), ("kf_mps", ctypes.c_void_p), ("n_mps", ctypes.c_int),
                ("bad", ctypes.c_void_p), ("n_obs", ctypes.c_void_p), ("replaced", ctypes.c_void_p),
                ("obs_start", ctypes.c_void_p), ("obs_kf", ctypes.c_void_p), ("obs_idx", ctypes.c_void_p),
                ("out_obs_start", ctypes.c_void_p), ("out_obs_kf", ctypes.c_void_p), ("out_obs_idx", ctypes.c_void_p),
                ("obs_cap", ctypes.c_int), ("log", ctypes.c_void_p), ("log_cap", ctypes.c_int), ("n_log", ctypes.c_int32),
                ("n_reevaluated", ctypes.c_int32), ("n_device_calls", ctypes.c_int32)]


class CnmpNeighbour(ctypes.Structure):
    """omv_cnmp_neighbour (include/omv.h)."""
    _fields_ = [("kf2", CnmpKf), ("T", (ctypes.c_float * 12) * 10), ("skip", ctypes.c_int),
                ("match12", ctypes.c_void_p), ("x3D", ctypes.c_void_p), ("status", ctypes.c_void_p)]


class TriPair(ctypes.Structure):
    """omv_tri_pair (include/omv.h)."""
    _fields_ = [("kf1", KfView), ("kf2", KfView), ("T", (ctypes.c_float * 12) * OMV_TRI_PAIRS),
                ("match12", ctypes.c_void_p)]


class BowJob(ctypes.Structure):
    """omv_bow_job (include/omv.h)."""
    _fields_ = [("kf", KfView), ("other", KfView), ("match", ctypes.c_void_p)]


OMV_BOW_KF_FRAME, OMV_BOW_KF_KF = 0, 1


class FisheyeUndist(ctypes.Structure):
    """omv_fisheye_undist (include/omv.h)."""
    _fields_ = [("K", ctypes.c_float * 4), ("D", ctypes.c_double * 4), ("newK", ctypes.c_float * 4)]


class LbaOpts(ctypes.Structure):
    _fields_ = [("opt_it", ctypes.c_int), ("lambda_init", ctypes.c_double), ("max_trials", ctypes.c_int),
                ("large", ctypes.c_int)]


class LbaResult(ctypes.Structure):
    _fields_ = [("err", ctypes.c_float), ("err_end", ctypes.c_float), ("status", ctypes.c_int),
                ("iterations", ctypes.c_int), ("trials", ctypes.c_int), ("lambda_", ctypes.c_double),
                ("mono_chi2", ctypes.c_void_p), ("mono_outlier", ctypes.c_void_p),
                ("stereo_chi2", ctypes.c_void_p), ("stereo_outlier", ctypes.c_void_p)]


# numpy dtype with the omv_kp layout (24 bytes)
try:
    import numpy as _np

    KP_DTYPE = _np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                          ("response", "<f4"), ("octave", "<i4")])
except ImportError:  # pragma: no cover
    KP_DTYPE = None

# Every symbol include/omv.h declares: (name, restype, argtypes)
_VP, _I, _F, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
# omv_allreduce_fn: int (*)(void *ctx, double *buf, size_t count, void *stream)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
SIGNATURES = {
    "omv_orb_create": (_I, [ctypes.POINTER(OrbParams), _I, _I, _I, ctypes.POINTER(_VP)]),
    "omv_orb_destroy": (_I, [_VP]),
    "omv_selftest_node_sort": (_I, [_VP, _VP, _I, _VP, _VP]),
    "omv_orb_max_keypoints": (_I, [_VP]),
    "omv_orb_scale_tables": (_I, [_VP, _VP, _VP, _VP, _VP]),
    "omv_orb_extract_batch": (_I, [_VP, _I, _VP, _SZ, _SZ, _VP, _VP, _VP, _VP, _VP, _VP]),
    "omv_orb_extract_host": (_I, [_VP, _VP, _SZ, _I, _I, _VP, _VP, _VP, _VP]),
    "omv_orb_last_error": (_I, [_VP]),
    "omv_orb_enable_timing": (_I, [_VP, _I]),
    "omv_orb_set_harris": (_I, [_VP, _VP]),
    "omv_orb_stage_ms": (_I, [_VP, _VP, ctypes.POINTER(ctypes.c_longlong), _I]),
    "omv_orb_last_counts": (_I, [_VP, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_longlong)]),
    "omv_orb_debug_level": (_I, [_VP, _I, _I, _VP, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "omv_matcher_create": (_I, [_I, _I, _I, _I, ctypes.POINTER(_VP)]),
    "omv_matcher_destroy": (_I, [_VP]),
    "omv_matcher_assign_grid": (_I, [_VP, _I, ctypes.POINTER(FrameGeom), _VP, _VP, _VP]),
    "omv_matcher_grid_debug": (_I, [_VP, _I, _I, _VP, _VP]),
    "omv_matcher_enable_timing": (_I, [_VP, _I]),
    "omv_matcher_last_error": (_I, [_VP]),
    "omv_matcher_stage_ms": (_I, [_VP, _VP, _I]),
    "omv_matcher_search_projection": (_I, [_VP, _I, ctypes.POINTER(FrameGeom), _VP, _VP, _VP,
                                           ctypes.POINTER(MpView), _I, _F, _I, _F, _F, _VP, _VP, _VP, _VP,
                                           _VP, _VP]),
    "omv_matcher_stereo_lapping": (_I, [_VP, _I, _VP, _VP, _VP, ctypes.c_double, _VP, _VP, _VP]),
    "omv_bf_knn2": (_I, [_I, _VP, _I, _VP, _VP, _I, _VP, _VP, _VP, _VP]),
    "omv_matcher_search_last_frame": (_I, [_VP, _I, ctypes.POINTER(FrameGeom), _VP, _VP, _VP, _VP, _VP, _VP,
                                           ctypes.POINTER(SE3f), ctypes.POINTER(LastFrame), _F, _I, _F, _I, _VP, _VP,
                                           _VP, _VP]),
    "omv_frustum": (_I, [_I, _VP, ctypes.POINTER(Rig), ctypes.POINTER(MpWorld), _I, _F, ctypes.POINTER(MpTrack), _VP,
                         _VP]),
    "omv_lba_create": (_I, [_I, _I, _I, _I, _I, ctypes.POINTER(_VP)]),
    "omv_lba_destroy": (_I, [_VP]),
    "omv_lba_set_problem": (_I, [_VP, ctypes.POINTER(LbaProblem)]),
    "omv_lba_optimize": (_I, [_VP, ctypes.POINTER(LbaOpts), ctypes.POINTER(LbaProblem), ctypes.POINTER(LbaResult)]),
    "omv_lba_evaluate": (_I, [_VP, _VP, _VP, _VP, _VP]),
    "omv_lba_evaluate_stereo": (_I, [_VP, _VP, _VP, _VP]),
    "omv_lba_stage_ms": (_I, [_VP, _VP, ctypes.POINTER(_I)]),
    "omv_lba_host_syncs": (_I, [_VP, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "omv_lba_enable_timing": (_I, [_VP, _I]),
    "omv_lba_set_driver": (_I, [_VP, _I]),
    "omv_lba_reset": (_I, [_VP]),
    "omv_lba_set_comm": (_I, [_VP, _I, _I, _VP, _VP]),
    "omv_tri_debug": (_I, [_VP, _VP, _VP, _VP, _VP, _VP, _F, _F, _VP]),
    "omv_matcher_stereo_triangulate": (_I, [_VP, _I, _I, _I, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, _VP, _VP,
                                            _VP, _VP]),
    "omv_matcher_search_for_triangulation": (_I, [_VP, _I, ctypes.POINTER(TriPair), _VP, _VP, _I, _I, _I, _VP, _VP]),
    "omv_matcher_search_by_bow": (_I, [_VP, _I, ctypes.POINTER(BowJob), _I, _F, _I, _VP, _VP]),
    "omv_matcher_bow_rescans": (_I, [ctypes.POINTER(ctypes.c_int64), _I]),
    "omv_matcher_search_for_initialization": (_I, [_VP, _I, _VP, ctypes.POINTER(FrameGeom), _VP, _VP, _VP, _VP, _I,
                                                   _F, _I, _VP, _VP, _VP]),
    "omv_pose_create": (_I, [_I, _I, ctypes.POINTER(_VP)]),
    "omv_pose_destroy": (_I, [_VP]),
    "omv_pose_inertial_last_kf": (_I, [_VP, ctypes.POINTER(PoseBatch), _I, _VP, _VP, _VP, _VP]),
    "omv_pose_inertial_last_frame": (_I, [_VP, ctypes.POINTER(PoseBatch), ctypes.POINTER(PosePrior), _I, _VP, _VP,
                                          _VP, _VP]),
    "omv_pose_constraint": (_I, [_I, _VP, _VP, _VP]),
    "omv_pose_optimization": (_I, [_VP, ctypes.POINTER(PoseBatch), _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "omv_pose_set_mode": (_I, [_VP, _I, _I]),
    "omv_pose_edges_from_matches": (_I, [_VP, _I, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, _I] + [_VP] * 14),
    "omv_pose_last_error": (_I, [_VP, ctypes.POINTER(ctypes.c_int32), _VP]),
    "omv_matcher_search_kf": (_I, [_VP, _I, ctypes.POINTER(FrameGeom), _VP, _VP, _VP, _I, ctypes.POINTER(KfSearchJob),
                                   _I, _VP, ctypes.POINTER(KfMps), ctypes.POINTER(KfSearchParams), _VP, _VP, _VP, _VP,
                                   _VP]),
    "omv_search_in_neighbors_fuse": (_I, [_VP, ctypes.POINTER(FrameGeom), _VP, _VP, _VP, _I, ctypes.POINTER(FuseGraph),
                                          _I, _I, _VP, ctypes.POINTER(KfMps), ctypes.POINTER(KfSearchParams), _VP, _VP]),
    "omv_matcher_search_by_sim3": (_I, [_VP, _I, ctypes.POINTER(FrameGeom), _VP, _VP, _VP, _I, ctypes.POINTER(Sim3Job),
                                        _I, _VP, _VP, _I, _VP, _VP, ctypes.POINTER(KfMps), _F, _F, _I, _VP, _VP, _VP]),
    "omv_imu_preintegrate": (_I, [_I, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "omv_bow_transform": (_I, [ctypes.POINTER(Vocab), _I, _VP, _I, _VP, _I] + [_VP] * 10 + [_VP]),
    "omv_lba_shard": (_I, [_VP, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), _VP]),
    "omv_frame_uright": (_I, [_I, _I, _I, _I, _VP, _VP, _VP, _I, _I, ctypes.POINTER(FisheyeUndist), _F, _VP, _VP,
                              _VP]),
    "omv_frame_pack": (_I, [_I, _I, _I, _I, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "omv_mappoint_distinctive_descriptors": (_I, [_I, _VP, _VP, _VP, _VP, _VP, _VP]),
    "omv_create_new_map_points": (_I, [_I, _VP, _VP, _VP, _VP, _I, _I, _I, ctypes.c_float, ctypes.c_float, _I, _VP,
                                       _VP, _VP]),
    "omv_local_mapping_create_new_map_points": (_I, [_VP, _VP, _VP, _I, _VP, _VP, _VP, _I, _I, _I, _I, _I,
                                                     ctypes.c_float, ctypes.c_float, _VP, _VP, _VP]),
    "omv_mappoint_normal_depth": (_I, [_I, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
}

_lib = None
missing = []


def load(path=LIB_PATH):
    """Load libomv_hip.so and bind every declared symbol; raises if absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OmvError(f"{path} not built: run `python -m openmavis_amd.build` (hipcc, gfx950). "
                       "There is no CPU fallback.")
    # torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Import it first so this
    # library binds to the runtime torch uses: one HIP runtime per process, shared device pointers.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover
        pass
    lib = ctypes.CDLL(path)
    missing.clear()
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:  # a declared symbol the build does not export (tests flag this)
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class _Ptr(ctypes.c_void_p):
    """A c_void_p that keeps its tensor / array alive while the call it is passed to runs (so that
    `ptr(np.ascontiguousarray(x))` on a temporary cannot dangle)."""


def ptr(t):
    """Device/host pointer of a torch tensor or numpy array as c_void_p (keeps `t` alive)."""
    if t is None:
        return None
    p = _Ptr(t.data_ptr() if hasattr(t, "data_ptr") else t.ctypes.data)
    p._keep = t
    return p
