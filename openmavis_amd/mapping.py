"""LocalMapping's per-keyframe map-point creation on device: the geometric test of SearchForTriangulation's matches
(LocalMapping::CreateNewMapPoints, src/LocalMapping.cc:395-780) over the current keyframe's neighbours.  Thin host
mirror over include/omv.h's omv_create_new_map_points; creating the MapPoint objects and the graph updates stay with the
caller (ComputeDistinctiveDescriptors / UpdateNormalAndDepth of the new points: openmavis_amd.mappoint)."""
import ctypes

import numpy as np

from . import _lib
from .synth_cnmp import cnmp_kf_struct


class CnmpCall:
    """One omv_create_new_map_points call with its inputs resident on the device (the keyframes' keypoints, right
    coordinates, depths and the matcher's match12 lists uploaded once); run() launches it on `stream`."""

    def __init__(self, d, inertial=True, far_points=False, th_far=50.0, device="cuda:0"):
        import torch
        self._keep = []

        def arr(a):
            a = np.ascontiguousarray(a)
            if a.dtype.names:   # structured records (keypoints): ship the bytes
                a = a.view(np.uint8).reshape(-1)
            t = torch.from_numpy(a).to(device)
            self._keep.append(t)
            return ctypes.c_void_p(t.data_ptr())

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
        self.cams = np.ascontiguousarray(d["cams"], np.float32)
        self.cm = np.ascontiguousarray(d["cam_model"], np.int32)
        self.args = (len(d["jobs"]), int(d["n_cams"]), int(inertial), int(far_points), float(th_far),
                     float(d["scale_factor"]))
        self.lib = _lib.load()

    def run(self, stream=None):
        import torch
        n, nc, inertial, far, th, sf = self.args
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        _lib.check(self.lib.omv_create_new_map_points(n, ctypes.byref(self.k1), self.jobs, _lib.ptr(self.cams),
                                                      _lib.ptr(self.cm), nc, inertial, far, th, sf, s),
                   "omv_create_new_map_points")
        return self.outs


def CreateNewMapPoints(d, inertial=True, far_points=False, th_far=50.0, stream=None, device="cuda:0"):
    """`d`: a keyframe set in synth_cnmp.make_cnmp's layout (kf1, jobs with kf2 / match12, cams, cam_model, n_cams,
    intrinsics, scale factors).  Returns per neighbour (status [kf1.n] int32 device: 1 triangulated, 2 by
    UnprojectStereo, 0 none; x3D [kf1.n][3] float32 device)."""
    c = CnmpCall(d, inertial, far_points, th_far, device)
    outs = c.run(stream)
    import torch
    torch.cuda.current_stream().synchronize() if stream is None else stream.synchronize()   # the inputs' lifetime
    return outs
