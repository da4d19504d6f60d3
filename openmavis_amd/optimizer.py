"""Host-side mirror of Optimizer::LocalInertialBA's optimisation (src/Optimizer.cc:2728-3385) on the
device LM of libomv_hip.so (openmavis_amd/csrc/lba.hip).

The reference builds a g2o graph from the local window (:2740-3267: VertexPose / VertexVelocity /
VertexGyroBias / VertexAccBias, EdgeInertial + EdgeGyroRW + EdgeAccRW per keyframe pair, EdgeMono per
observation) and runs `optimizer.optimize(opt_it)` with Levenberg-Marquardt (:3270-3274), then the
outlier test (:3282-3296) and the FAIL guard (:3317-3321).  Here the flattened graph is a problem dict
(see openmavis_amd.synth_ba.make_lba_problem for the field list, which is omv_lba_problem's):

    ba = LocalInertialBA(max_kf=64, max_cams=5, max_pts=40000, max_mono=300000, max_imu=64)
    ba.set_problem(prob)
    res, state = ba.optimize(opt_it=10, lambda_init=1.0, large=False)

`res` carries err / err_end (activeRobustChi2 before/after, as floats like the reference), status
(OMV_LBA_OK / OMV_LBA_FAIL), the LM iteration / trial counts and per-edge chi2 + outlier flags; `state`
the optimised Rwb, twb, Rcw, tcw, vel, bg, ba, pts.  There is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from .synth_ba import as_struct, read_state

OMV_LBA_OK = 0
OMV_LBA_FAIL = 1


def lba_options(large):
    """LocalInertialBA's LM settings: bLarge -> 4 iterations, user lambda 1e-2; else 10 and 1e0."""
    return dict(opt_it=4, lambda_init=1e-2) if large else dict(opt_it=10, lambda_init=1e0)


class LocalInertialBA:
    """`rank`, `world`, `allreduce`: landmark sharding (omv_lba_set_comm).  Every rank
    passes the same full problem; `allreduce(ptr, count, stream)` sums `count` doubles of device
    memory in place over the ranks (openmavis_amd.dist.LbaAllReduce).  After optimize() a rank's
    result holds its own landmarks / edges (`shard()` names them) and every keyframe."""

    def __init__(self, max_kf=64, max_cams=5, max_pts=40000, max_mono=400000, max_imu=64, rank=0, world=1,
                 allreduce=None):
        lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(lib.omv_lba_create(max_kf, max_cams, max_pts, max_mono, max_imu, ctypes.byref(h)),
                   "omv_lba_create")
        self._lib, self._h = lib, h
        self._s = None
        self._keep = None
        self._cb = None
        if world > 1 and allreduce is None:
            raise ValueError("LocalInertialBA: world > 1 needs an allreduce")
        if allreduce is not None:   # a collective given: the sharded call sequence, also on one rank

            def _cb(_ctx, buf, count, stream):
                try:
                    allreduce(buf, count, stream)
                    return 0
                except Exception as exc:   # reported by the failing omv_lba_optimize status
                    print(f"LocalInertialBA allreduce failed: {exc!r}")
                    return 1
            self._cb = _lib.ALLREDUCE_FN(_cb)
            _lib.check(lib.omv_lba_set_comm(h, int(rank), int(world), ctypes.cast(self._cb, ctypes.c_void_p), None),
                       "omv_lba_set_comm")

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.omv_lba_destroy(self._h)
            self._h = None

    def set_problem(self, prob):
        s, keep = as_struct(prob, _lib.LbaProblem)
        _lib.check(self._lib.omv_lba_set_problem(self._h, ctypes.byref(s)), "omv_lba_set_problem")
        self._s, self._keep = s, keep
        return self

    def optimize(self, opt_it=10, lambda_init=1e0, max_trials=10, large=False, chi2=True, state_copy=True):
        """chi2=False: only the outlier flags (what the reference's culling uses), no per-edge chi2 read-back.
        The optimised state is written back into the problem's host arrays (as the reference writes its keyframes and
        map points); state_copy=False returns those arrays themselves instead of copies (the next optimize() of this
        problem overwrites them)."""
        if self._s is None:
            raise _lib.OmvError("LocalInertialBA.optimize: no problem set")
        o = _lib.LbaOpts(int(opt_it), float(lambda_init), int(max_trials), int(bool(large)))
        E, S = self._s.n_mono, self._s.n_stereo
        want = bool(chi2)
        chi2 = np.zeros(E) if want else None
        outl = np.zeros(E, np.uint8)
        s_chi2 = np.zeros(S) if want else None
        s_outl = np.zeros(S, np.uint8)
        r = _lib.LbaResult()
        r.mono_chi2, r.mono_outlier = (_lib.ptr(chi2) if want else None), _lib.ptr(outl)
        r.stereo_chi2, r.stereo_outlier = (_lib.ptr(s_chi2) if want else None), _lib.ptr(s_outl)
        _lib.check(self._lib.omv_lba_optimize(self._h, ctypes.byref(o), ctypes.byref(self._s), ctypes.byref(r)),
                   "omv_lba_optimize")
        res = dict(err=r.err, err_end=r.err_end, status=r.status, iterations=r.iterations, trials=r.trials,
                   lambda_=r.lambda_, mono_chi2=chi2, mono_outlier=outl, stereo_chi2=s_chi2, stereo_outlier=s_outl)
        if not state_copy:
            return res, {k: self._keep[k] for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "pts")}
        return res, read_state(self._keep)

    def reset(self):
        """Restore the state uploaded by set_problem (device copy)."""
        _lib.check(self._lib.omv_lba_reset(self._h), "omv_lba_reset")
        return self

    def evaluate(self):
        """Residuals and visual Jacobians at the uploaded state (caller's edge order)."""
        E, I = self._s.n_mono, self._s.n_imu
        me, jx, jp, ie = np.zeros((E, 2)), np.zeros((E, 6)), np.zeros((E, 12)), np.zeros((I, 9))
        _lib.check(self._lib.omv_lba_evaluate(self._h, _lib.ptr(me), _lib.ptr(jx), _lib.ptr(jp), _lib.ptr(ie)),
                   "omv_lba_evaluate")
        S = self._s.n_stereo
        se, sx, sp = np.zeros((S, 3)), np.zeros((S, 9)), np.zeros((S, 18))
        _lib.check(self._lib.omv_lba_evaluate_stereo(self._h, _lib.ptr(se), _lib.ptr(sx), _lib.ptr(sp)),
                   "omv_lba_evaluate_stereo")
        return dict(mono_err=me, mono_jx=jx, mono_jp=jp, imu_err=ie, stereo_err=se, stereo_jx=sx, stereo_jp=sp)

    def shard(self):
        """(caller indices of the landmarks this rank owns, number of its visual edges)."""
        n_p, n_e = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(self._lib.omv_lba_shard(self._h, ctypes.byref(n_p), ctypes.byref(n_e), None), "omv_lba_shard")
        idx = np.zeros(n_p.value, np.int32)
        _lib.check(self._lib.omv_lba_shard(self._h, None, None, _lib.ptr(idx)), "omv_lba_shard")
        return idx, n_e.value

    def enable_timing(self, on=True):
        """Per-stage events on the next optimize() calls (direct launches instead of the captured LM step)."""
        _lib.check(self._lib.omv_lba_enable_timing(self._h, int(bool(on))), "omv_lba_enable_timing")
        return self

    def set_driver(self, host_driven):
        """True: g2o's LM decisions on the host (read-back per trial); False (default): on the device."""
        _lib.check(self._lib.omv_lba_set_driver(self._h, int(bool(host_driven))), "omv_lba_set_driver")
        return self

    def host_syncs(self):
        """(host waits of the last optimize()'s LM loop, its trials): the device driver waits once per batch."""
        n, t = ctypes.c_int(0), ctypes.c_int(0)
        _lib.check(self._lib.omv_lba_host_syncs(self._h, ctypes.byref(n), ctypes.byref(t)), "omv_lba_host_syncs")
        return n.value, t.value

    def stage_ms(self):
        """Device ms of the last optimize: build, schur, solve, update+errors; and the trial count."""
        ms = np.zeros(4)
        t = ctypes.c_int(0)
        _lib.check(self._lib.omv_lba_stage_ms(self._h, _lib.ptr(ms), ctypes.byref(t)), "omv_lba_stage_ms")
        return dict(build=ms[0], schur=ms[1], solve=ms[2], update=ms[3], trials=t.value)


class PoseInertialOptimizer:
    """Host-side mirror of Optimizer::PoseInertialOptimizationLastKeyFrame (src/Optimizer.cc:5021-5578)
    for a batch of frames on the device (openmavis_amd/csrc/pose.hip).

        opt = PoseInertialOptimizer(max_frames=256, max_edges=400000)
        n_good = opt.PoseInertialOptimizationLastKeyFrame(batch, arrays, kp_outlier, H, bRecInit=False)

    `batch` carries the rig (host numpy: cam, Rcb, tcb, Rbc, tbc, bf, n_frames, n_cams, kp_cap and the
    edge arrays' lengths); `arrays` maps every omv_pose_batch pointer field (state in/out, the last
    keyframe's fixed vertices, preintegration, frame-major edges) to a device tensor.  kp_outlier
    (uint8 [F][kp_cap]) receives Frame::mvbOutlier, H (float64 [F][225] or None) the ConstraintPoseImu
    Hessian; the int32 [F] return tensor holds the reference's return value per frame.  No CPU fallback.
    """

    def __init__(self, max_frames=256, max_edges=400000):
        lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(lib.omv_pose_create(int(max_frames), int(max_edges), ctypes.byref(h)), "omv_pose_create")
        self._lib, self._h = lib, h

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.omv_pose_destroy(self._h)
            self._h = None

    AUTO, BATCH, GROUPED = 0, 1, 2

    def set_mode(self, mode, parts=0):
        """Kernel choice (omv_pose_set_mode): AUTO (grouped kernel up to 16 frames per call, else one workgroup per
        frame), BATCH or GROUPED (`parts` workgroups per frame; 0 = one per 126 (LastFrame) / 190 (LastKeyFrame)
        visual edges of the mean frame, at least ceil(batch edges / 1022), at most 48 -- include/omv.h)."""
        _lib.check(self._lib.omv_pose_set_mode(self._h, int(mode), int(parts)), "omv_pose_set_mode")
        return self

    def last_error(self, stream=None):
        """Device error word since the last read (0, or OMV_ERR_CAPACITY / OMV_ERR_HIP from the grouped kernel)."""
        import torch
        e = ctypes.c_int32(0)
        st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(self._lib.omv_pose_last_error(self._h, ctypes.byref(e), ctypes.c_void_p(st)), "omv_pose_last_error")
        return e.value

    EDGE_KEYS = ("mono_start", "mono_cam", "mono_kp", "mono_obs", "mono_inv_sigma2", "mono_xw", "mono_close",
                 "stereo_start", "stereo_cam", "stereo_kp", "stereo_obs", "stereo_inv_sigma2", "stereo_xw")

    @staticmethod
    def edge_arrays(max_edges, device):
        """Device buffers for one frame's edge lists (the omv_pose_batch edge fields of a one-frame batch)."""
        import torch
        z = dict(device=device)
        E = int(max_edges)
        return dict(mono_start=torch.zeros(2, dtype=torch.int32, **z), mono_cam=torch.zeros(E, dtype=torch.int32, **z),
                    mono_kp=torch.zeros(E, dtype=torch.int32, **z), mono_obs=torch.zeros((E, 2), dtype=torch.float64, **z),
                    mono_inv_sigma2=torch.zeros(E, dtype=torch.float32, **z),
                    mono_xw=torch.zeros((E, 3), dtype=torch.float32, **z), mono_close=torch.zeros(E, dtype=torch.uint8, **z),
                    stereo_start=torch.zeros(2, dtype=torch.int32, **z),
                    stereo_cam=torch.zeros(E, dtype=torch.int32, **z), stereo_kp=torch.zeros(E, dtype=torch.int32, **z),
                    stereo_obs=torch.zeros((E, 3), dtype=torch.float64, **z),
                    stereo_inv_sigma2=torch.zeros(E, dtype=torch.float32, **z),
                    stereo_xw=torch.zeros((E, 3), dtype=torch.float32, **z))

    def EdgesFromMatches(self, kps, n_kp, kp_to_mp, mp_pos, mp_track_depth, inv_level_sigma2, arrays, uright=None,
                         stream=None):
        """The edge-creation loop of PoseInertialOptimizationLastKeyFrame / LastFrame (src/Optimizer.cc:5079-5330)
        for ONE multi-camera frame, on the device (omv_pose_edges_from_matches): kps int32 [C][kp_cap][6] (omv_kp
        rows), n_kp [C], kp_to_mp [C*kp_cap] (SearchByProjection's assignment), mp_pos float [M][3], mp_track_depth
        [M], inv_level_sigma2 host sequence (Frame::mvInvLevelSigma2), uright float [C][kp_cap] or None; writes the
        edge lists into `arrays` (edge_arrays' buffers; their length bounds the edge count).  Asynchronous."""
        import torch
        C, cap = int(kps.shape[-3]), int(kps.shape[-2])
        E = int(arrays["mono_cam"].shape[0])
        lv = (ctypes.c_float * 16)(*[float(x) for x in inv_level_sigma2][:16])
        st = stream if stream is not None else torch.cuda.current_stream(kps.device).cuda_stream
        a = arrays
        _lib.check(self._lib.omv_pose_edges_from_matches(
            self._h, C, cap, _lib.ptr(kps), _lib.ptr(n_kp), _lib.ptr(kp_to_mp), _lib.ptr(mp_pos),
            _lib.ptr(mp_track_depth), lv, len(inv_level_sigma2), _lib.ptr(uright), E,
            *[_lib.ptr(a[k]) for k in self.EDGE_KEYS], ctypes.c_void_p(st)), "omv_pose_edges_from_matches")
        return arrays

    def PoseInertialOptimizationLastKeyFrame(self, batch, arrays, kp_outlier, H=None, bRecInit=False, stream=None):
        import torch
        from .synth_pose import as_pose_struct
        s, keep = as_pose_struct(batch, _lib.PoseBatch, arrays)
        n_good = torch.zeros(s.n_frames, dtype=torch.int32, device=kp_outlier.device)
        st = stream if stream is not None else torch.cuda.current_stream(kp_outlier.device).cuda_stream
        _lib.check(self._lib.omv_pose_inertial_last_kf(self._h, ctypes.byref(s), int(bool(bRecInit)),
                                                       _lib.ptr(kp_outlier), _lib.ptr(n_good), _lib.ptr(H),
                                                       ctypes.c_void_p(st)),
                   "omv_pose_inertial_last_kf")
        del keep
        return n_good

    def PoseInertialOptimizationLastFrame(self, batch, arrays, kp_outlier, H=None, bRecInit=False, stream=None):
        """Optimizer::PoseInertialOptimizationLastFrame (src/Optimizer.cc:5580-6170) on every frame of the
        batch.  As PoseInertialOptimizationLastKeyFrame, but `arrays`' kf_* tensors hold the previous
        frame's vertices (free here, not written back), `preint` is mpImuPreintegratedFrame, and `arrays`
        also carries the previous frame's ConstraintPoseImu (prior_Rwb / prior_twb / prior_vel / prior_bg /
        prior_ba, prior_H [F][225]) and preint_kf (mpImuPreintegrated).  H receives Marginalize's frame
        block; ConstraintPoseImu() turns it into the next prior."""
        import torch
        from .synth_pose import as_pose_struct, as_prior_struct
        s, keep = as_pose_struct(batch, _lib.PoseBatch, arrays)
        pr = as_prior_struct(_lib.PosePrior, arrays)
        n_good = torch.zeros(s.n_frames, dtype=torch.int32, device=kp_outlier.device)
        st = stream if stream is not None else torch.cuda.current_stream(kp_outlier.device).cuda_stream
        _lib.check(self._lib.omv_pose_inertial_last_frame(self._h, ctypes.byref(s), ctypes.byref(pr),
                                                          int(bool(bRecInit)), _lib.ptr(kp_outlier), _lib.ptr(n_good),
                                                          _lib.ptr(H), ctypes.c_void_p(st)),
                   "omv_pose_inertial_last_frame")
        del keep
        return n_good

    def PoseOptimization(self, batch, arrays, pose_q, pose_t, kp_outlier, stream=None):
        """Optimizer::PoseOptimization (src/Optimizer.cc:855-1278) on every frame of the batch (omv_pose_optimization):
        `batch` as above plus rig_q / rig_t (host [n_cams][4] / [3], T_c0 = mTrl / mTsll / mTsrl); `arrays` needs only
        the edge tensors (EDGE_KEYS); pose_q / pose_t (float64 device [F][4] (x y z w) / [F][3]) hold Frame::GetPose()
        and receive the optimised Tcw; kp_outlier (uint8 [F][kp_cap]) receives mvbOutlier.  Returns the int32 [F]
        return values (nInitialCorrespondences - nBad).  Asynchronous; no CPU fallback."""
        import numpy as np
        import torch
        from .synth_pose import as_pose_struct
        s, keep = as_pose_struct(batch, _lib.PoseBatch, arrays)
        rq = np.ascontiguousarray(batch["rig_q"], np.float64)
        rt = np.ascontiguousarray(batch["rig_t"], np.float64)
        n_good = torch.zeros(s.n_frames, dtype=torch.int32, device=kp_outlier.device)
        st = stream if stream is not None else torch.cuda.current_stream(kp_outlier.device).cuda_stream
        _lib.check(self._lib.omv_pose_optimization(self._h, ctypes.byref(s), _lib.ptr(rq), _lib.ptr(rt), _lib.ptr(pose_q),
                                                   _lib.ptr(pose_t), _lib.ptr(kp_outlier), _lib.ptr(n_good),
                                                   ctypes.c_void_p(st)), "omv_pose_optimization")
        del keep
        return n_good

    @staticmethod
    def ConstraintPoseImu(H, out=None, stream=None):
        """The ConstraintPoseImu ctor's projection (include/G2oTypes.h:639-659) of device float64 [n][225]
        matrices; returns `out` (may be H itself)."""
        import torch
        lib = _lib.load()
        out = torch.empty_like(H) if out is None else out
        st = stream if stream is not None else torch.cuda.current_stream(H.device).cuda_stream
        _lib.check(lib.omv_pose_constraint(int(H.shape[0]), _lib.ptr(H), _lib.ptr(out), ctypes.c_void_p(st)),
                   "omv_pose_constraint")
        return out
