"""Host-side mirror of the reference's ORBmatcher for the multi-camera frame (include/ORBmatcher.h),
running on the HIP matchers of libomv_hip.so.

    m = ORBmatcher(nnratio=0.8, checkOri=True)
    n = m.SearchByProjection(frames, mps, th, bFarPoints, thFarPoints)

`frames` is a FrameBatch (device tensors of the extractor's batched output plus per-frame
mvLeftToRightMatch / mvRightToLeftMatch / mvpMapPoints), `mps` a MapPointBatch (the SoA the
reference reads from MapPoint after Frame::isInFrustum).  Like the reference, SearchByProjection
returns the match count and mutates the frame's map-point assignment (frames.kp_to_mp).
"""
import ctypes

import numpy as np

from . import _lib

FRAME_GRID_COLS = 64
FRAME_GRID_ROWS = 48
TH_HIGH = 100
TH_LOW = 50
HISTO_LENGTH = 30


def frame_geom(n_cams, width, height, scale_factors, cam_model=None):
    """omv_frame_geom.  cam_model: per camera block "kb8" / "pinhole" (or 0 / 1); default every block KB8."""
    g = _lib.FrameGeom()
    g.n_cams = n_cams
    g.min_x, g.max_x, g.min_y, g.max_y = 0.0, float(width), 0.0, float(height)   # image bounds (no undistortion)
    g.nlevels = len(scale_factors)
    for i, s in enumerate(scale_factors):
        g.scale_factors[i] = float(s)
    for i, m in enumerate(cam_model if cam_model is not None else ()):
        g.cam_model[i] = {"kb8": _lib.CAM_KB8, "pinhole": _lib.CAM_PINHOLE}.get(m, m) if isinstance(m, str) else int(m)
    return g


class FrameBatch:
    """n_frames multi-camera frames resident on the GPU (torch tensors, padded per camera)."""

    def __init__(self, torch, n_frames, n_cams, kp_cap, width, height, scale_factors, device="cuda", cam_model=None):
        self.torch = torch
        self.n_frames, self.n_cams, self.kp_cap = n_frames, n_cams, kp_cap
        self.geom = frame_geom(n_cams, width, height, scale_factors, cam_model)
        z = dict(device=device)
        self.kps = torch.zeros((n_frames, n_cams, kp_cap, 6), dtype=torch.int32, **z)
        self.desc = torch.zeros((n_frames, n_cams, kp_cap, 32), dtype=torch.uint8, **z)
        self.n_kp = torch.zeros((n_frames, n_cams), dtype=torch.int32, **z)
        self.mono = torch.zeros((n_frames, n_cams), dtype=torch.int32, **z)
        self.l2r = torch.full((n_frames, kp_cap), -1, dtype=torch.int32, **z)
        self.r2l = torch.full((n_frames, kp_cap), -1, dtype=torch.int32, **z)
        self.kp_to_mp = torch.full((n_frames, n_cams * kp_cap), -1, dtype=torch.int32, **z)
        self.occ_init = None
        self.n_matches = torch.zeros(n_frames, dtype=torch.int32, **z)


class MapPointBatch:
    """Local map points per frame: device SoA of the fields SearchByProjection reads."""

    FIELDS = ("desc", "proj_x", "proj_y", "view_cos", "level", "in_view", "track_depth", "is_bad", "has_obs")

    def __init__(self, **arrays):
        for k in self.FIELDS:
            setattr(self, k, arrays[k])
        self.M = arrays["desc"].shape[-2]

    def view(self):
        v = _lib.MpView()
        for k in self.FIELDS:
            setattr(v, k, _lib.ptr(getattr(self, k)))
        return v


class TriPairBatch:
    """The omv_tri_pair array of a list of keyframe pairs (see ORBmatcher.SearchForTriangulation), built
    once so repeated searches over resident keyframes pay no per-pair host marshalling."""

    def __init__(self, pairs):
        from .synth_tri import kf_struct
        self.n = len(pairs)
        self.arr = (_lib.TriPair * max(self.n, 1))()
        self._keep = []
        self.device = None

        def ptr(_name, t):
            self._keep.append(t)
            return ctypes.c_void_p(t.data_ptr())

        for i, p in enumerate(pairs):
            self.arr[i].kf1 = kf_struct(p["kf1"], _lib.KfView, p["kf1"]["level_sigma2"], ptr)
            self.arr[i].kf2 = kf_struct(p["kf2"], _lib.KfView, p["kf2"]["level_sigma2"], ptr)
            T = np.ascontiguousarray(np.asarray(p["T"], np.float32).reshape(_lib.OMV_TRI_PAIRS, 12))
            ctypes.memmove(ctypes.addressof(self.arr[i].T), T.ctypes.data, T.nbytes)
            self.arr[i].match12 = ctypes.c_void_p(p["match12"].data_ptr())
            self._keep.append(p["match12"])
            self.device = p["match12"].device


class BowJobBatch:
    """The omv_bow_job array of a list of SearchByBoW jobs (see ORBmatcher.SearchByBoW), built once."""

    def __init__(self, jobs):
        from .synth_tri import kf_struct
        self.n = len(jobs)
        self.arr = (_lib.BowJob * max(self.n, 1))()
        self._keep = []
        self.device = None

        def ptr(_name, t):
            self._keep.append(t)
            return ctypes.c_void_p(t.data_ptr())

        for i, j in enumerate(jobs):
            self.arr[i].kf = kf_struct(j["kf"], _lib.KfView, j["kf"].get("level_sigma2", np.ones(16)), ptr)
            self.arr[i].other = kf_struct(j["other"], _lib.KfView, j["other"].get("level_sigma2", np.ones(16)), ptr)
            self.arr[i].match = ctypes.c_void_p(j["match"].data_ptr())
            self._keep.append(j["match"])
            self.device = j["match"].device


class ORBmatcher:
    def __init__(self, nnratio=0.6, checkOri=True):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self._lib = _lib.load()
        self._h = None
        self._shape = None

    def _handle(self, frames, M=0):
        # one workspace per (frames, cams, kp_cap); grows (and drops the grid) only when M exceeds it
        M = max(M, self._shape[3] if self._shape else 1)
        shape = (frames.n_frames, frames.n_cams, frames.kp_cap, M)
        if self._h is None or any(a < b for a, b in zip(self._shape, shape)) or self._shape[1:3] != shape[1:3]:
            self.close()
            h = ctypes.c_void_p()
            _lib.check(self._lib.omv_matcher_create(frames.n_frames, frames.n_cams, frames.kp_cap, max(M, 1),
                                                    ctypes.byref(h)), "omv_matcher_create")
            self._h, self._shape = h, (frames.n_frames, frames.n_cams, frames.kp_cap, max(M, 1))
        return self._h

    def close(self):
        if self._h is not None:
            self._lib.omv_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _stream(stream):
        return ctypes.c_void_p(stream.cuda_stream) if stream is not None else None

    def AssignFeaturesToGrid(self, frames, stream=None):
        h = self._handle(frames)
        _lib.check(self._lib.omv_matcher_assign_grid(h, frames.n_frames, ctypes.byref(frames.geom),
                                                     _lib.ptr(frames.kps), _lib.ptr(frames.n_kp),
                                                     self._stream(stream)), "omv_matcher_assign_grid")

    STAGES = ("grid", "stereo_knn", "proj_candidates", "proj_resolve")

    def enable_timing(self, on=True):
        _lib.check(self._lib.omv_matcher_enable_timing(self._h, int(bool(on))))

    def stage_ms(self, reset=True):
        ms = np.zeros(4, np.float64)
        _lib.check(self._lib.omv_matcher_stage_ms(self._h, _lib.ptr(ms), int(bool(reset))))
        return dict(zip(self.STAGES, ms.tolist()))

    def last_error(self):
        return self._lib.omv_matcher_last_error(self._h)

    def grid(self, frame, cam):
        cs = np.zeros(FRAME_GRID_COLS * FRAME_GRID_ROWS + 1, np.int32)
        idx = np.zeros(self._shape[2], np.int32)
        _lib.check(self._lib.omv_matcher_grid_debug(self._h, frame, cam, _lib.ptr(cs), _lib.ptr(idx)))
        return cs, idx[:cs[-1]]

    def SearchByProjectionLastFrame(self, frames, last, Tcw, Tlw, cams, Trl, th, bMono=False, mb=0.0, stream=None):
        """ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, th, bMono)
        (src/ORBmatcher.cc:1985-2413): the last frames' tracked points (`last`: dict of device tensors
        pos [F, S, 3], desc [F, S, 32], valid / has_obs [F, S] uint8, kps [F, S, 6] (omv_kp rows)) are
        projected with the current poses Tcw and matched into frames.kp_to_mp (last-frame slots).
        Tcw / Tlw: device float32 [F, 7] (qx qy qz qw tx ty tz); cams: [C][8]; Trl: 7 floats.
        Returns the per-frame match counts (device tensor)."""
        h = self._handle(frames, last["pos"].shape[1])
        self.AssignFeaturesToGrid(frames, stream)
        S = last["pos"].shape[1]
        lf = _lib.LastFrame(_lib.ptr(last["pos"]), _lib.ptr(last["desc"]), _lib.ptr(last["valid"]),
                            _lib.ptr(last["has_obs"]), _lib.ptr(last["kps"]), S)
        c = np.ascontiguousarray(np.asarray(cams, np.float32).reshape(-1, 8)[:frames.n_cams])
        trl = _lib.SE3f()
        t7 = np.asarray(Trl, np.float32).reshape(7)
        for q in range(4):
            trl.q[q] = float(t7[q])
        for q in range(3):
            trl.t[q] = float(t7[4 + q])
        _lib.check(self._lib.omv_matcher_search_last_frame(
            h, frames.n_frames, ctypes.byref(frames.geom), _lib.ptr(frames.kps), _lib.ptr(frames.desc),
            _lib.ptr(frames.n_kp), _lib.ptr(c), _lib.ptr(Tcw), _lib.ptr(Tlw), ctypes.byref(trl), ctypes.byref(lf),
            ctypes.c_float(th), int(bool(bMono)), ctypes.c_float(mb), int(self.mbCheckOrientation),
            _lib.ptr(frames.occ_init), _lib.ptr(frames.kp_to_mp), _lib.ptr(frames.n_matches), self._stream(stream)),
            "omv_matcher_search_last_frame")
        return frames.n_matches

    def StereoTriangulate(self, frames, cams, Rlr, tlr, level_sigma2, stream=None):
        """The depth check of Frame::ComputeMultiFishEyeMatches (src/Frame.cc:1488-1512) on the pairs
        StereoLapping left in frames.l2r: KannalaBrandt8::TriangulateMatches with mRlr / mtlr.  Fills
        frames.depth (mvDepth of the left keypoints) and frames.p3d (mvStereo3Dpoints), clears failed
        pairs and rebuilds frames.r2l."""
        import torch
        if not hasattr(frames, "depth"):
            frames.depth = torch.full((frames.n_frames, frames.kp_cap), -1.0, dtype=torch.float32,
                                      device=frames.l2r.device)
            frames.p3d = torch.zeros((frames.n_frames, frames.kp_cap, 3), dtype=torch.float32, device=frames.l2r.device)
        h = self._handle(frames)
        c = np.ascontiguousarray(np.asarray(cams, np.float32).reshape(-1, 8)[:2])
        R = np.ascontiguousarray(np.asarray(Rlr, np.float32).reshape(9))
        t = np.ascontiguousarray(np.asarray(tlr, np.float32).reshape(3))
        sg = np.ascontiguousarray(np.asarray(level_sigma2, np.float32))
        _lib.check(self._lib.omv_matcher_stereo_triangulate(
            h, frames.n_frames, frames.n_cams, frames.kp_cap, _lib.ptr(frames.kps), _lib.ptr(frames.n_kp),
            _lib.ptr(frames.mono), _lib.ptr(c), _lib.ptr(R), _lib.ptr(t), _lib.ptr(sg), len(sg), _lib.ptr(frames.l2r),
            _lib.ptr(frames.r2l), _lib.ptr(frames.depth), _lib.ptr(frames.p3d), self._stream(stream)),
            "omv_matcher_stereo_triangulate")

    def SearchForTriangulation(self, pairs, cams, bOnlyStereo=False, bCoarse=False, stream=None, cam_model=None):
        """ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:1131-1456) for a batch of multi-camera
        keyframe pairs.  pairs: list of dicts {kf1, kf2, T, match12}: kf* hold the omv_kf_view fields
        (n, n_left, n_right, n_sideleft ints; kps / desc / has_mp / node_id / node_start / node_idx device
        tensors; level_sigma2 host floats), T the 10 camera-pair transforms (float [10][12]), match12 a
        device int32 [kf1.n] receiving vMatches12.  cams: host [4][8] KB8 parameters (L, R, SL, SR).
        `pairs` may also be a prebuilt TriPairBatch.  Returns the per-pair match counts (device int32
        tensor); synchronous.  cam_model: per camera 0 (KannalaBrandt8) / 1 (Pinhole), default all KB8."""
        import torch
        if self._h is None:
            h = ctypes.c_void_p()
            _lib.check(self._lib.omv_matcher_create(1, 1, 1, 1, ctypes.byref(h)), "omv_matcher_create")
            self._h, self._shape = h, (1, 1, 1, 1)
        batch = pairs if isinstance(pairs, TriPairBatch) else TriPairBatch(pairs)
        n, arr, dev = batch.n, batch.arr, batch.device
        out = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        c = np.ascontiguousarray(np.asarray(cams, np.float32).reshape(4, 8))
        cm = None if cam_model is None else np.ascontiguousarray(np.asarray(cam_model, np.int32).reshape(4))
        _lib.check(self._lib.omv_matcher_search_for_triangulation(
            self._h, n, arr, _lib.ptr(c), _lib.ptr(cm), int(bool(bOnlyStereo)), int(bool(bCoarse)), int(self.mbCheckOrientation),
            _lib.ptr(out), self._stream(stream)), "omv_matcher_search_for_triangulation")
        return out[:n]

    def _scratch_handle(self):
        if self._h is None:
            h = ctypes.c_void_p()
            _lib.check(self._lib.omv_matcher_create(1, 1, 1, 1, ctypes.byref(h)), "omv_matcher_create")
            self._h, self._shape = h, (1, 1, 1, 1)
        return self._h

    def SearchByBoW(self, jobs, kf_kf=False, stream=None):
        """ORBmatcher::SearchByBoW (src/ORBmatcher.cc:349-666, (KeyFrame, Frame); with kf_kf the (KeyFrame,
        KeyFrame) overload :1006-1129) for a batch of jobs.  jobs: list of dicts {kf, other, match}: kf / other
        hold the omv_kf_view fields (n, n_left, n_right, n_sideleft ints; kps / desc / has_mp / node_id /
        node_start / node_idx device tensors; n_left = -1 for a single-camera frame, n_sideleft = -1 without side
        cameras), match a device int32 tensor: (KF, F) [other.n] the keyframe keypoint whose map point each frame
        keypoint received, (KF1, KF2) [kf.n] the pKF2 keypoint of each pKF1 keypoint (-1 none).  `jobs` may be a
        prebuilt BowJobBatch.  Returns the per-job match counts (device int32 tensor); synchronous."""
        import torch
        h = self._scratch_handle()
        batch = jobs if isinstance(jobs, BowJobBatch) else BowJobBatch(jobs)
        out = torch.zeros(max(batch.n, 1), dtype=torch.int32, device=batch.device)
        _lib.check(self._lib.omv_matcher_search_by_bow(
            h, batch.n, batch.arr, _lib.OMV_BOW_KF_KF if kf_kf else _lib.OMV_BOW_KF_FRAME, ctypes.c_float(self.mfNNratio),
            int(self.mbCheckOrientation), _lib.ptr(out), self._stream(stream)), "omv_matcher_search_by_bow")
        return out[:batch.n]

    def bow_rescans(self, reset=True):
        """Diagnostic: keyframe keypoints whose SearchByBoW short list ran out (node rescanned), all calls."""
        v = ctypes.c_int64()
        _lib.check(self._lib.omv_matcher_bow_rescans(ctypes.byref(v), int(bool(reset))), "omv_matcher_bow_rescans")
        return int(v.value)

    def SearchForInitialization(self, frames, pairs, prev_matched, windowSize=100, stream=None, grid_ready=False):
        """ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
        (src/ORBmatcher.cc:895-1004) for frame pairs of a single-camera FrameBatch (block 0 = mvKeysUn).  pairs:
        [(f1, f2), ...] frame indices; prev_matched: device float32 [n_pairs, kp_cap, 2] (vbPrevMatched, updated
        in place).  Returns (vnMatches12 device int32 [n_pairs, kp_cap], per-pair counts device int32)."""
        import torch
        h = self._handle(frames)
        if not grid_ready:
            self.AssignFeaturesToGrid(frames, stream)
        pr = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
        n = len(pr)
        dev = frames.kps.device
        m12 = torch.full((max(n, 1), frames.kp_cap), -1, dtype=torch.int32, device=dev)
        cnt = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        _lib.check(self._lib.omv_matcher_search_for_initialization(
            h, n, _lib.ptr(pr), ctypes.byref(frames.geom), _lib.ptr(frames.kps), _lib.ptr(frames.desc),
            _lib.ptr(frames.n_kp), _lib.ptr(prev_matched), int(windowSize), ctypes.c_float(self.mfNNratio),
            int(self.mbCheckOrientation), _lib.ptr(m12), _lib.ptr(cnt), self._stream(stream)),
            "omv_matcher_search_for_initialization")
        return m12[:n], cnt[:n]

    def StereoLapping(self, frames, ratio=0.8, stream=None):
        """Lowe-ratio knn candidates of ComputeMultiFishEyeMatches (before triangulation)."""
        h = self._handle(frames)
        _lib.check(self._lib.omv_matcher_stereo_lapping(h, frames.n_frames, _lib.ptr(frames.desc),
                                                        _lib.ptr(frames.n_kp), _lib.ptr(frames.mono),
                                                        ctypes.c_double(ratio), _lib.ptr(frames.l2r),
                                                        _lib.ptr(frames.r2l), self._stream(stream)),
                   "omv_matcher_stereo_lapping")

    def SearchByProjection(self, frames, mps, th=3.0, bFarPoints=False, thFarPoints=50.0, stream=None,
                           grid_ready=False):
        """Returns the per-frame match counts (device tensor); mutates frames.kp_to_mp."""
        if self._h is None or mps.M > self._shape[3]:
            grid_ready = False   # a new workspace has no grid yet
        h = self._handle(frames, mps.M)
        if not grid_ready:
            self.AssignFeaturesToGrid(frames, stream)
        v = mps.view()
        _lib.check(self._lib.omv_matcher_search_projection(
            h, frames.n_frames, ctypes.byref(frames.geom), _lib.ptr(frames.kps), _lib.ptr(frames.desc),
            _lib.ptr(frames.n_kp), ctypes.byref(v), mps.M, ctypes.c_float(th), int(bool(bFarPoints)),
            ctypes.c_float(thFarPoints), ctypes.c_float(self.mfNNratio), _lib.ptr(frames.l2r),
            _lib.ptr(frames.r2l), _lib.ptr(frames.occ_init), _lib.ptr(frames.kp_to_mp),
            _lib.ptr(frames.n_matches), self._stream(stream)), "omv_matcher_search_projection")
        return frames.n_matches

    # ---- keyframe-side projection searches (omv_matcher_search_kf) -----------------------------------
    def _search_kf(self, kfs, mode, jobs, mp_list, mps, params, kp_match, stream):
        h = self._handle(kfs, max(1, -(-len(mp_list) // (kfs.n_frames * kfs.n_cams))))
        self.AssignFeaturesToGrid(kfs, stream)
        import torch
        dev = kfs.kps.device
        n_e = int(mp_list.shape[0])
        best_idx = torch.empty(max(n_e, 1), dtype=torch.int32, device=dev)
        best_dist = torch.empty(max(n_e, 1), dtype=torch.int32, device=dev)
        n_matches = torch.empty(max(len(jobs), 1), dtype=torch.int32, device=dev)
        arr = (_lib.KfSearchJob * max(len(jobs), 1))()
        for i, jb in enumerate(jobs):
            arr[i].kf, arr[i].cam = int(jb["kf"]), int(jb["cam"])
            T = np.asarray(jb["Tcw"], np.float32).reshape(7)
            for q in range(4):
                arr[i].Tcw.q[q] = float(T[q])
            for q in range(3):
                arr[i].Tcw.t[q] = float(T[4 + q])
                arr[i].Ow[q] = float(np.float32(jb["Ow"][q]))
            arr[i].mp_start, arr[i].mp_count = int(jb["mp_start"]), int(jb["mp_count"])
        m = _lib.KfMps(*[_lib.ptr(mps[k]) for k in ("pos", "normal", "min_dist", "max_dist", "desc")])
        params.mode = mode
        _lib.check(self._lib.omv_matcher_search_kf(
            h, kfs.n_frames, ctypes.byref(kfs.geom), _lib.ptr(kfs.kps), _lib.ptr(kfs.desc), _lib.ptr(kfs.n_kp),
            len(jobs), arr, n_e, _lib.ptr(mp_list), ctypes.byref(m), ctypes.byref(params), _lib.ptr(kp_match),
            _lib.ptr(best_idx), _lib.ptr(best_dist), _lib.ptr(n_matches), self._stream(stream)), "omv_matcher_search_kf")
        return best_idx[:n_e], best_dist[:n_e], n_matches[:len(jobs)]

    def Fuse(self, kfs, jobs, mp_list, mps, params, stream=None):
        """ORBmatcher::Fuse(pKF, vpMapPoints, th, cameraID) (src/ORBmatcher.cc:1458-1647) for a batch of
        jobs (keyframe, cameraID, its pose Tcw [qx qy qz qw tx ty tz] and centre Ow, a run of mp_list).
        `kfs`: a FrameBatch of the keyframes; mps: dict of device tensors pos / normal / min_dist /
        max_dist / desc (omv_kf_mps); params: kf_search_params(...).  Returns (best_idx, best_dist,
        n_fused): per entry the chosen keypoint (the keyframe's N-index, -1 none) and its distance —
        accepted when <= TH_LOW; the caller applies Replace / AddObservation in entry order — and the
        reference's return value per job."""
        return self._search_kf(kfs, _lib.OMV_KF_FUSE, jobs, mp_list, mps, params, None, stream)

    def FuseSim3(self, kfs, jobs, mp_list, mps, params, stream=None):
        """ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:1649-1769): one job per camera block,
        each with Tiw = GetRelativePose*() * SE3f(Scw.rotationMatrix(), Scw.translation() / Scw.scale())."""
        return self._search_kf(kfs, _lib.OMV_KF_FUSE_SIM3, jobs, mp_list, mps, params, None, stream)

    def SearchByProjectionSim3(self, kfs, jobs, mp_list, mps, vpMatched, params, stream=None):
        """ORBmatcher::SearchByProjection(pKF, Siw, vpPoints, vpMatched, th, ratioHamming, cameraID)
        (:668-776; the vpPointsKFs overload :778-893 matches identically).  vpMatched: device int32
        [n_kf][n_cams * kp_cap] slot claims (-1 free), updated in place with the mp_list values."""
        return self._search_kf(kfs, _lib.OMV_KF_SBP_SIM3, jobs, mp_list, mps, params, vpMatched, stream)

    def SearchByProjectionKF(self, frames, jobs, mp_list, mps, params, stream=None):
        """ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:2415-2535): each
        job projects one keyframe's map points (its mvKeysUn angles in params.mp_angle) into a frame of
        `frames` (camera block 0); claims go to frames.kp_to_mp (Frame::mvpMapPoints)."""
        params.check_ori = int(self.mbCheckOrientation)
        return self._search_kf(frames, _lib.OMV_KF_SBP_FRAME, jobs, mp_list, mps, params, frames.kp_to_mp, stream)

    def SearchBySim3(self, kfs, jobs, kp1, mp1, kp2, mp2, mps, th=7.5, stream=None):
        """ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, S12, th) (src/ORBmatcher.cc:1771-1983) for keyframe
        pairs of the FrameBatch `kfs`.  jobs: dicts (see sim3_job_array) or a prebuilt omv_sim3_job array; kp1 /
        mp1: device int32, per pair in job order, the pKF1 keypoints (N-index) whose map point is projected and
        its table row (kp2 / mp2 likewise for pKF2); mps: dict of device tensors pos / min_dist / max_dist / desc.
        Returns (match12 [len(kp1)]: the pKF2 keypoint each side-1 entry is matched to, -1 none; n_found per
        pair), device int32."""
        import torch
        h = self._handle(kfs)
        self.AssignFeaturesToGrid(kfs, stream)
        arr = jobs if not isinstance(jobs, (list, tuple)) else sim3_job_array(jobs)
        n_jobs = len(jobs)
        dev = kfs.kps.device
        n1, n2 = int(kp1.shape[0]), int(kp2.shape[0])
        match12 = torch.empty(max(n1, 1), dtype=torch.int32, device=dev)
        n_found = torch.empty(max(n_jobs, 1), dtype=torch.int32, device=dev)
        m = _lib.KfMps(_lib.ptr(mps["pos"]), None, _lib.ptr(mps["min_dist"]), _lib.ptr(mps["max_dist"]),
                       _lib.ptr(mps["desc"]))
        g = kfs.geom
        log_sf = float(np.float32(np.log(np.float64(np.float32(g.scale_factors[1])))))
        _lib.check(self._lib.omv_matcher_search_by_sim3(
            h, kfs.n_frames, ctypes.byref(g), _lib.ptr(kfs.kps), _lib.ptr(kfs.desc), _lib.ptr(kfs.n_kp), n_jobs, arr,
            n1, _lib.ptr(kp1), _lib.ptr(mp1), n2, _lib.ptr(kp2), _lib.ptr(mp2), ctypes.byref(m), ctypes.c_float(th),
            ctypes.c_float(log_sf), int(g.nlevels), _lib.ptr(match12), _lib.ptr(n_found), self._stream(stream)),
            "omv_matcher_search_by_sim3")
        return match12[:n1], n_found[:n_jobs]


def sim3_job_array(jobs):
    """omv_sim3_job array of dict jobs {kf1, kf2, T1w, T2w ([qx qy qz qw tx ty tz]), S12, S21 ({q, t, scale}),
    fx, fy, cx, cy, start1, count1, start2, count2}."""
    arr = (_lib.Sim3Job * max(len(jobs), 1))()
    for i, jb in enumerate(jobs):
        a = arr[i]
        a.kf1, a.kf2 = int(jb["kf1"]), int(jb["kf2"])
        for dst, T in ((a.T1w, jb["T1w"]), (a.T2w, jb["T2w"])):
            T = np.asarray(T, np.float32).reshape(7)
            for q in range(4):
                dst.q[q] = float(T[q])
            for q in range(3):
                dst.t[q] = float(T[4 + q])
        for dst, S in ((a.S12, jb["S12"]), (a.S21, jb["S21"])):
            for q in range(4):
                dst.q[q] = float(S["q"][q])
            for q in range(3):
                dst.t[q] = float(S["t"][q])
            dst.scale = float(S["scale"])
        a.fx, a.fy, a.cx, a.cy = (float(np.float32(jb[k])) for k in ("fx", "fy", "cx", "cy"))
        a.start1, a.count1, a.start2, a.count2 = (int(jb[k]) for k in ("start1", "count1", "start2", "count2"))
    return arr


def kf_search_params(th, max_dist, cams, scale_factor=1.2, nlevels=8, bf=0.0, uright=None, mp_angle=None):
    """omv_kf_search_params: window factor th, acceptance max_dist (TH_LOW, TH_LOW * ratioHamming or
    ORBdist), KB8 parameters per block, the extractor's scale tables, mbf and mvuRight (Fuse)."""
    p = _lib.KfSearchParams()
    p.th, p.max_dist, p.bf = float(th), float(max_dist), float(bf)
    p.uright = _lib.ptr(uright) if uright is not None else None
    sf = np.float32(scale_factor)
    scales = [np.float32(1.0)]
    for _ in range(1, nlevels):
        scales.append(np.float32(scales[-1] * sf))
    for i, s in enumerate(scales):
        p.inv_level_sigma2[i] = float(np.float32(1.0) / np.float32(s * s))
    p.log_scale_factor = float(np.float32(np.log(np.float64(sf))))
    p.n_levels = nlevels
    c = np.asarray(cams, np.float32).reshape(-1, 8)
    for i in range(c.shape[0]):
        for q in range(8):
            p.cams[i][q] = float(c[i, q])
    p.mp_angle = _lib.ptr(mp_angle) if mp_angle is not None else None
    p._keep = (uright, mp_angle)
    return p


def make_rig(cams, R_cl, t_cl, width, height, scale_factor=1.2, nlevels=8, model="kb8"):
    """omv_rig from per-camera parameters (KannalaBrandt8: fx fy cx cy k1..k4; Pinhole: fx fy cx cy) and the
    block-c-from-block-0 transforms (float32).  model: "kb8" / "pinhole" for every block, or one per block."""
    r = _lib.Rig()
    C = len(cams)
    r.n_cams = C
    models = [model] * C if isinstance(model, str) else list(model)
    for c in range(C):
        r.model[c] = {"kb8": _lib.CAM_KB8, "pinhole": _lib.CAM_PINHOLE}[models[c]]
        for q in range(len(cams[c])):
            r.cam[c][q] = float(cams[c][q])
        Rc = np.asarray(R_cl[c], np.float32).reshape(3, 3)
        tc = np.asarray(t_cl[c], np.float32).reshape(3)
        tlc = (-(Rc.astype(np.float64).T @ tc.astype(np.float64))).astype(np.float32)
        for q in range(9):
            r.R_cl[c][q] = float(Rc.reshape(-1)[q])
        for q in range(3):
            r.t_cl[c][q] = float(tc[q])
            r.t_lc[c][q] = float(tlc[q]) if c else 0.0
    r.min_x, r.max_x, r.min_y, r.max_y = 0.0, float(width), 0.0, float(height)
    r.log_scale_factor = float(np.float32(np.log(np.float64(np.float32(scale_factor)))))
    r.n_levels = nlevels
    return r


def isInFrustum(poses, rig, world, track, viewingCosLimit=0.5, n_in_view=None, stream=None):
    """Frame::isInFrustum for every local map point of every frame (src/Frame.cc:736-826, :1529-1653).

    poses: device float32 [F, 24] (omv_frame_pose); world: dict of device tensors pos [F, M, 3],
    normal [F, M, 3], min_dist / max_dist [F, M]; track: a MapPointBatch whose proj_x / proj_y /
    view_cos / level / in_view / track_depth are written in place (the SearchByProjection inputs)."""
    lib = _lib.load()
    F, M = world["pos"].shape[0], world["pos"].shape[1]
    w = _lib.MpWorld(_lib.ptr(world["pos"]), _lib.ptr(world["normal"]), _lib.ptr(world["min_dist"]),
                     _lib.ptr(world["max_dist"]))
    t = _lib.MpTrack(_lib.ptr(track.proj_x), _lib.ptr(track.proj_y), _lib.ptr(track.view_cos), _lib.ptr(track.level),
                     _lib.ptr(track.in_view), _lib.ptr(track.track_depth))
    s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    _lib.check(lib.omv_frustum(F, _lib.ptr(poses), ctypes.byref(rig), ctypes.byref(w), M, ctypes.c_float(viewingCosLimit),
                               ctypes.byref(t), _lib.ptr(n_in_view), s), "omv_frustum")


def bf_knn2(query, nq, train, nt, stream=None):
    """knnMatch(k=2) over a batch of (query, train) sets: torch uint8 [P, Q, 32], [P, T, 32]; counts
    int32 [P].  Returns (idx2, dist2) int32 [P, Q, 2]."""
    import torch
    lib = _lib.load()
    P, Q = query.shape[0], query.shape[1]
    idx2 = torch.empty((P, Q, 2), dtype=torch.int32, device=query.device)
    dist2 = torch.empty((P, Q, 2), dtype=torch.int32, device=query.device)
    s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
    _lib.check(lib.omv_bf_knn2(P, _lib.ptr(query), Q, _lib.ptr(nq), _lib.ptr(train), train.shape[1], _lib.ptr(nt),
                               _lib.ptr(idx2), _lib.ptr(dist2), s), "omv_bf_knn2")
    return idx2, dist2
