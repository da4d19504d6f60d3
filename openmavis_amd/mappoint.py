"""Map-point refresh on device for a batch of map points: MapPoint::ComputeDistinctiveDescriptors
(src/MapPoint.cc:405-490) and MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:503-588), the pair LocalMapping calls
for every new or fused point (src/LocalMapping.cc:338-339, :776-778, :897-898).  Thin host mirror over include/omv.h's
omv_mappoint_distinctive_descriptors / omv_mappoint_normal_depth; the map graph (mObservations, mpRefKF, isBad) stays
with the caller, which flattens each point's observations in std::map order."""
import numpy as np

from . import _lib


def _stream(torch, stream):
    return (stream if stream is not None else torch.cuda.current_stream()).cuda_stream


def _dev(torch, a, dtype, device):
    if hasattr(a, "data_ptr"):
        if a.dtype != dtype or not a.is_contiguous():
            raise _lib.OmvError("mappoint: device arrays must be contiguous " + str(dtype))
        return a
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dtype)


def ComputeDistinctiveDescriptors(desc, desc_start, desc_row, with_descriptors=True, stream=None, device="cuda:0"):
    """Per point p the row (of `desc`, [rows][32] u8) of the descriptor with the least median distance to the point's
    other descriptors desc_row[desc_start[p]:desc_start[p+1]] (-1: none, mDescriptor untouched), and the chosen
    descriptors ([P][32] u8) when `with_descriptors`.  Device tensors returned."""
    import torch
    desc = _dev(torch, desc, torch.uint8, device)
    start = _dev(torch, desc_start, torch.int32, device)
    rows = _dev(torch, desc_row, torch.int32, device)
    n = int(start.numel()) - 1
    if desc.dim() != 2 or desc.shape[1] != 32 or n < 0:
        raise _lib.OmvError("ComputeDistinctiveDescriptors: desc must be [rows][32], desc_start [P+1]")
    best = torch.empty(max(n, 0), dtype=torch.int32, device=desc.device)
    out = torch.empty((max(n, 0), 32), dtype=torch.uint8, device=desc.device) if with_descriptors else None
    lib = _lib.load()
    _lib.check(lib.omv_mappoint_distinctive_descriptors(n, _lib.ptr(start), _lib.ptr(rows), _lib.ptr(desc),
                                                        _lib.ptr(best), _lib.ptr(out), _stream(torch, stream)),
               "omv_mappoint_distinctive_descriptors")
    return best, out


def UpdateNormalAndDepth(obs_start, obs_center, pos, ref_center, ref_level_scale, ref_max_scale, stream=None,
                         device="cuda:0"):
    """(mNormalVector [P][3], mfMinDistance [P], mfMaxDistance [P]) as float32 device tensors; points without
    observation entries keep the output buffers' initial NaN (the reference leaves them untouched)."""
    import torch
    start = _dev(torch, obs_start, torch.int32, device)
    cen = _dev(torch, obs_center, torch.float32, device)
    P = _dev(torch, pos, torch.float32, device)
    rc = _dev(torch, ref_center, torch.float32, device)
    ls = _dev(torch, ref_level_scale, torch.float32, device)
    ms = _dev(torch, ref_max_scale, torch.float32, device)
    n = int(start.numel()) - 1
    normal = torch.full((n, 3), float("nan"), dtype=torch.float32, device=P.device)
    dmin = torch.full((n,), float("nan"), dtype=torch.float32, device=P.device)
    dmax = torch.full((n,), float("nan"), dtype=torch.float32, device=P.device)
    lib = _lib.load()
    _lib.check(lib.omv_mappoint_normal_depth(n, _lib.ptr(start), _lib.ptr(cen), _lib.ptr(P), _lib.ptr(rc), _lib.ptr(ls),
                                             _lib.ptr(ms), _lib.ptr(normal), _lib.ptr(dmin), _lib.ptr(dmax),
                                             _stream(torch, stream)), "omv_mappoint_normal_depth")
    return normal, dmin, dmax
