"""LocalMapping's per-keyframe map-point creation on device (LocalMapping::CreateNewMapPoints, src/LocalMapping.cc:
395-783).  Host mirror over include/omv.h:

- CreateNewMapPoints(d, ...)          the reference's whole neighbour loop on the device
                                      (omv_local_mapping_create_new_map_points): per neighbour in order the baseline
                                      gate on the persistent side-1 camera centre, SearchForTriangulation against the
                                      current keyframe's has-map-point flags as the previous neighbours left them, the
                                      geometric checks, AddMapPoint(idx1) of the accepted matches.
- CreateNewMapPointsGeometry(d, ...)  the geometric checks alone on caller-supplied match lists (omv_create_new_map_points;
                                      exact for the reference's loop when each list came from a search that saw the
                                      previous lists' accepted points).

Creating the MapPoint objects and the graph updates stay with the caller (ComputeDistinctiveDescriptors /
UpdateNormalAndDepth of the new points: openmavis_amd.mappoint)."""
import ctypes

import numpy as np

from . import _lib
from .synth_cnmp import chain_kf_struct, cnmp_kf_struct


def _uploader(keep, device):
    import torch

    def arr(a):
        a = np.ascontiguousarray(a)
        if a.dtype.names:   # structured records (keypoints): ship the bytes
            a = a.view(np.uint8).reshape(-1)
        t = torch.from_numpy(a).to(device)
        keep.append(t)
        return ctypes.c_void_p(t.data_ptr())
    return arr


class CnmpCall:
    """One omv_create_new_map_points call with its inputs resident on the device (the keyframes' keypoints, right
    coordinates, depths and the matcher's match12 lists uploaded once); run() launches it on `stream`."""

    def __init__(self, d, inertial=True, far_points=False, th_far=50.0, check_baseline=False, device="cuda:0"):
        import torch
        self._keep = []
        arr = _uploader(self._keep, device)
        self.k1 = cnmp_kf_struct(d["kf1"], d, _lib.CnmpKf, _lib.KfView, arr)
        self.jobs = (_lib.CnmpJob * len(d["jobs"]))()
        n1 = int(d["kf1"]["n"])
        self.outs = []
        for j, jb in enumerate(d["jobs"]):
            self.jobs[j].kf2 = cnmp_kf_struct(jb["kf2"], d, _lib.CnmpKf, _lib.KfView, arr)
            self.jobs[j].match12 = arr(np.ascontiguousarray(jb["match12"], np.int32))
            st = torch.full((n1,), -9, dtype=torch.int32, device=device)
            x = torch.full((n1, 3), float("nan"), dtype=torch.float32, device=device)
            self.jobs[j].x3D, self.jobs[j].status = ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(st.data_ptr())
            self.outs.append((st, x))
        self.has_mp1 = torch.zeros(max(n1, 1), dtype=torch.uint8, device=device)
        self.side1 = torch.zeros(1, dtype=torch.int32, device=device)
        self.cams = np.ascontiguousarray(d["cams"], np.float32)
        self.cm = np.ascontiguousarray(d["cam_model"], np.int32)
        self.args = (len(d["jobs"]), int(d["n_cams"]), int(inertial), int(far_points), float(th_far),
                     float(d["scale_factor"]), int(check_baseline))
        self.lib = _lib.load()

    def run(self, stream=None, side1_state=0):
        import torch
        n, nc, inertial, far, th, sf, cb = self.args
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        self.side1.fill_(int(side1_state))
        _lib.check(self.lib.omv_create_new_map_points(n, ctypes.byref(self.k1), self.jobs, _lib.ptr(self.cams),
                                                      _lib.ptr(self.cm), nc, inertial, far, th, sf, cb,
                                                      ctypes.c_void_p(self.side1.data_ptr()),
                                                      ctypes.c_void_p(self.has_mp1.data_ptr()), s),
                   "omv_create_new_map_points")
        return self.outs


def CreateNewMapPointsGeometry(d, inertial=True, far_points=False, th_far=50.0, check_baseline=False, stream=None,
                               device="cuda:0"):
    """`d`: a keyframe set in synth_cnmp.make_cnmp's layout (kf1, jobs with kf2 / match12, cams, cam_model, n_cams,
    intrinsics, scale factors).  Returns per job (status [kf1.n] int32 device: 1 triangulated, 2 by UnprojectStereo,
    0 none; x3D [kf1.n][3] float32 device)."""
    c = CnmpCall(d, inertial, far_points, th_far, check_baseline, device)
    outs = c.run(stream)
    import torch
    torch.cuda.current_stream().synchronize() if stream is None else stream.synchronize()   # the inputs' lifetime
    return outs


class LocalMappingCall:
    """One omv_local_mapping_create_new_map_points call over a synth_cnmp.make_cnmp_chain set, inputs resident on the
    device.  run() resets the current keyframe's has-map-point flags to d["kf1"]["has_mp"] (or `has_mp1`) and the side-1
    state, then runs the neighbours [lo, hi) (all by default)."""

    def __init__(self, d, matcher, inertial=True, monocular=False, coarse=False, far_points=False, th_far=50.0,
                 device="cuda:0"):
        import torch
        self._keep = []
        self.dev = device
        arr = _uploader(self._keep, device)
        n1 = int(d["kf1"]["n"])
        self.has_mp1 = torch.zeros(max(n1, 1), dtype=torch.uint8, device=device)
        self.has_mp1_init = torch.from_numpy(np.ascontiguousarray(d["kf1"]["has_mp"], np.uint8)).to(device)
        self.k1 = chain_kf_struct(d["kf1"], d, _lib.CnmpKf, _lib.KfView, arr)
        self.nbs = (_lib.CnmpNeighbour * len(d["nbs"]))()
        self.outs = []
        for j, nb in enumerate(d["nbs"]):
            o = self.nbs[j]
            o.kf2 = chain_kf_struct(nb["kf2"], d, _lib.CnmpKf, _lib.KfView, arr)
            ctypes.memmove(ctypes.addressof(o.T), np.ascontiguousarray(nb["T"], np.float32).ctypes.data, 480)
            o.skip = int(nb.get("skip", 0))
            m12 = torch.full((max(n1, 1),), -9, dtype=torch.int32, device=device)
            st = torch.full((max(n1, 1),), -9, dtype=torch.int32, device=device)
            x = torch.full((max(n1, 1), 3), float("nan"), dtype=torch.float32, device=device)
            o.match12, o.x3D, o.status = (ctypes.c_void_p(t.data_ptr()) for t in (m12, x, st))
            self.outs.append((m12, st, x))
        self.n_matches = torch.zeros(len(d["nbs"]), dtype=torch.int32, device=device)
        self.side1 = torch.zeros(1, dtype=torch.int32, device=device)
        self.cams = np.ascontiguousarray(d["cams"], np.float32)
        self.cm = np.ascontiguousarray(d["cam_model"], np.int32)
        self.m = matcher
        self.args = (int(d["n_cams"]), int(inertial), int(not monocular), int(coarse), int(far_points), float(th_far),
                     float(d["scale_factor"]))
        self.lib = _lib.load()

    def run(self, lo=0, hi=None, reset=True, side1_state=0, stream=None):
        import torch
        hi = len(self.outs) if hi is None else hi
        if reset:
            self.has_mp1.copy_(self.has_mp1_init)
            self.side1.fill_(int(side1_state))
        nc, inertial, cb, coarse, far, th, sf = self.args
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        nb = ctypes.cast(ctypes.addressof(self.nbs) + lo * ctypes.sizeof(_lib.CnmpNeighbour), ctypes.c_void_p)
        nm = ctypes.c_void_p(self.n_matches.data_ptr() + 4 * lo)
        _lib.check(self.lib.omv_local_mapping_create_new_map_points(
            self.m._scratch_handle(), ctypes.byref(self.k1), ctypes.c_void_p(self.has_mp1.data_ptr()), hi - lo, nb,
            _lib.ptr(self.cams), _lib.ptr(self.cm), nc, inertial, cb, coarse, far, th, sf, nm,
            ctypes.c_void_p(self.side1.data_ptr()), s), "omv_local_mapping_create_new_map_points")
        return self.outs


def CreateNewMapPoints(d, matcher, inertial=True, monocular=False, coarse=False, far_points=False, th_far=50.0,
                       device="cuda:0"):
    """LocalMapping::CreateNewMapPoints on a synth_cnmp.make_cnmp_chain set: returns (has_mp1 [kf1.n] uint8, n_matches
    [n_neigh], per neighbour (match12, status, x3D)) as numpy, the final side-1 state."""
    c = LocalMappingCall(d, matcher, inertial, monocular, coarse, far_points, th_far, device)
    outs = c.run()
    import torch
    torch.cuda.synchronize()
    n1 = int(d["kf1"]["n"])
    return (c.has_mp1[:n1].cpu().numpy(), c.n_matches.cpu().numpy(),
            [(m[:n1].cpu().numpy(), s[:n1].cpu().numpy(), x[:n1].cpu().numpy()) for m, s, x in outs],
            int(c.side1.item()))


def SearchInNeighborsFuse(s, matcher, th=3.0, device="cuda:0", obs_cap=None, log_cap=None, stream=None):
    """LocalMapping::SearchInNeighbors' fuse sequence (src/LocalMapping.cc:837-889) on a flattened map (the
    synth_fuse.make_fuse_scene layout: keyframes as one multi-camera batch, mvpMapPoints, map points with their
    observations / nObs / isBad and the device table pos / normal / min / max / desc) through
    omv_search_in_neighbors_fuse: every window search on the device (speculative per phase, stale entries re-evaluated
    after Replace's descriptor recomputation, itself on the device), the decisions walked in the reference's order.
    Returns dict(kf_mps, bad, n_obs, replaced, obs_start, obs_kf, obs_idx, log, n_fused, desc (final descriptors,
    numpy), n_reevaluated, n_device_calls)."""
    import torch
    from .matcher import FrameBatch, kf_search_params
    K, C, cap = int(s["n_kf"]), int(s["n_cams"]), int(s["kp_cap"])
    scale = [1.0]
    for _ in range(1, int(s["nlevels"])):
        scale.append(float(np.float32(scale[-1] * np.float32(1.2))))
    kfs = FrameBatch(torch, K, C, cap, s["width"], s["height"], scale, device=device)
    kfs.kps.copy_(torch.from_numpy(np.ascontiguousarray(s["kps"]).view(np.int32).reshape(K, C, cap, 6)))
    kfs.desc.copy_(torch.from_numpy(np.ascontiguousarray(s["desc"])))
    kfs.n_kp.copy_(torch.from_numpy(np.ascontiguousarray(s["n_kp"], np.int32)))
    mps = {k: torch.from_numpy(np.array(v, copy=True)).to(device) for k, v in s["mps"].items()}
    ur = torch.from_numpy(np.ascontiguousarray(s["uright"], np.float32)).to(device)
    p = kf_search_params(th, 50.0, s["cams"], bf=float(s["bf"]), nlevels=int(s["nlevels"]), uright=ur)
    p.mode = _lib.OMV_KF_FUSE
    # the handle's entry capacity: phase A evaluates every (target block, current-keyframe point) at once
    n_cur = int(np.asarray(s["n_kp"])[int(s["current"])].sum())
    n_e = len(s["targets"]) * C * n_cur
    h = matcher._handle(kfs, max(1, -(-n_e // (K * C))))
    matcher.AssignFeaturesToGrid(kfs, stream)
    keep = []

    def arr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return ctypes.c_void_p(a.ctypes.data)

    from .synth_fuse import fuse_graph_struct
    obs_cap = obs_cap or 4 * len(s["obs_kf"]) + 1024
    log_cap = log_cap or 4 * int(s["n_mps"]) + 1024
    out = {}
    G = fuse_graph_struct(s, _lib.FuseGraph, arr, out, obs_cap, log_cap)
    T = len(s["targets"])
    n_fused = np.zeros(T * C + C, np.int32)
    m = _lib.KfMps(*[_lib.ptr(mps[k]) for k in ("pos", "normal", "min_dist", "max_dist", "desc")])
    st = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
    _lib.check(matcher._lib.omv_search_in_neighbors_fuse(
        h, ctypes.byref(kfs.geom), _lib.ptr(kfs.kps), _lib.ptr(kfs.desc), _lib.ptr(kfs.n_kp), cap, ctypes.byref(G),
        int(s["current"]), T, arr(np.ascontiguousarray(s["targets"], np.int32)), ctypes.byref(m), ctypes.byref(p),
        arr(n_fused), st), "omv_search_in_neighbors_fuse")
    n_rows = int(out["out_obs_start"][-1])
    return dict(kf_mps=out["kf_mps"], bad=out["bad"], n_obs=out["n_obs"], replaced=out["replaced"][:int(s["n_mps"])],
                obs_start=out["out_obs_start"], obs_kf=out["out_obs_kf"][:n_rows], obs_idx=out["out_obs_idx"][:n_rows],
                log=out["log"][:G.n_log], n_fused=n_fused, desc=mps["desc"].cpu().numpy(),
                n_reevaluated=int(G.n_reevaluated), n_device_calls=int(G.n_device_calls))
