"""The tail of the multi-camera Frame constructor (src/Frame.cc:1913-1939) on device:
mvuRight from the undistorted depth images (GetDepthFromUndistortedPoints, :1659-1765) and the
cv::vconcat of the per-camera keypoints / descriptors into the frame's dense N rows (:1936-1939).
Thin host mirror over include/omv.h's omv_frame_uright / omv_frame_pack."""
import ctypes

import numpy as np

from . import _lib

# GetDepthFromUndistortedPoints' hard-coded Hilti-2022 calibrations (src/Frame.cc:1667-1728), keyed by
# the reference's cam_id: (origK fx, fy, cx, cy), dist_coeff k1..k4, (newK fx, fy, cx, cy).
HILTI_UNDIST = {
    0: ((351.31400364, 351.49117447, 367.85227934, 253.8402145),
        (-0.03696737, -0.00891788, 0.00891297, -0.0037686),
        (269.46230292, 269.59819519, 379.82324304, 245.21372784)),
    1: ((352.64897944, 352.85864986, 347.81700103, 270.58066925),
        (-0.03908665, -0.00552535, 0.00439815, -0.00197013),
        (270.02303235, 270.18357681, 329.41424161, 270.88581184)),
    3: ((352.95148439, 353.32837904, 363.93345228, 266.14511705),
        (-0.03890973, -0.00260468, 0.00046347, -0.00036698),
        (271.39851961, 271.68832899, 369.7572895, 264.14176194)),
    4: ((351.51321487, 351.75575549, 342.84259887, 259.91793255),
        (-0.03842764, -0.00584141, 0.00345104, -0.00114635),
        (269.20586464, 269.39161402, 316.20386976, 254.46723719)),
}
# camera blocks L, R, SL, SR -> cam_id (src/Frame.cc:1916-1922)
BLOCK_CAM_ID = (1, 0, 4, 3)


def undist_params(cam_ids=BLOCK_CAM_ID, table=HILTI_UNDIST):
    """omv_fisheye_undist array for the given blocks (float K / newK like the reference's Mat_<float>)."""
    arr = (_lib.FisheyeUndist * len(cam_ids))()
    for i, c in enumerate(cam_ids):
        K, D, nK = table[c]
        for q in range(4):
            arr[i].K[q] = float(np.float32(K[q]))
            arr[i].D[q] = float(D[q])
            arr[i].newK[q] = float(np.float32(nK[q]))
    return arr


def frame_uright(frames, depth, bf, undist=None, undist_xy=None, stream=None, out=None):
    """mvuRight of every keypoint of `frames` (matcher.FrameBatch) from the undistorted depth images
    `depth` (device float [n_frames][n_blocks][h][w]); the first n_blocks camera blocks (depth's block
    count) are processed.  Returns u_right (written into `out` when given) (device float [n_frames][n_blocks][kp_cap]), -1 where the
    reference writes -1; slots past n_kp are left unset."""
    torch = frames.torch
    nb = int(depth.shape[1])
    if undist is None:
        undist = undist_params(BLOCK_CAM_ID[:nb])
    if len(undist) < nb or depth.dtype != torch.float32 or not depth.is_contiguous():
        raise _lib.OmvError("frame_uright: need float32 contiguous depth and one undist entry per block")
    if frames.n_cams < nb or depth.shape[0] != frames.n_frames or depth.shape[1] != nb:
        raise _lib.OmvError("frame_uright: depth must be [n_frames][n_cams][h][w]")
    lib = _lib.load()
    ur = out if out is not None else torch.empty((frames.n_frames, nb, frames.kp_cap), dtype=torch.float32,
                                                 device=depth.device)
    if tuple(ur.shape) != (frames.n_frames, nb, frames.kp_cap) or ur.dtype != torch.float32 or not ur.is_contiguous():
        raise _lib.OmvError("frame_uright: out must be float32 [n_frames][n_blocks][kp_cap]")
    _lib.check(lib.omv_frame_uright(frames.n_frames, frames.n_cams, nb, frames.kp_cap, _lib.ptr(frames.kps),
                                    _lib.ptr(frames.n_kp), _lib.ptr(depth), int(depth.shape[3]), int(depth.shape[2]),
                                    undist, ctypes.c_float(bf), _lib.ptr(ur), _lib.ptr(undist_xy),
                                    _stream_handle(torch, stream)), "omv_frame_uright")
    return ur


def frame_pack(frames, u_right=None, n_cams=None, stream=None):
    """Dense per-frame rows (the reference's N-indexed mvKeys / mDescriptors / mvuRight order) of the first
    n_cams blocks (default all; u_right in frame_uright's [frame][n_cams][kp_cap] layout):
    returns (offset [n_frames + 1] device int32, kps [total][6] int32 view of omv_kp, desc [total][32],
    uright [total] or None).  Synchronises once to size the outputs."""
    torch = frames.torch
    nb = frames.n_cams if n_cams is None else int(n_cams)
    dev = frames.kps.device
    total = int(frames.n_kp[:, :nb].sum().item())
    off = torch.empty(frames.n_frames + 1, dtype=torch.int32, device=dev)
    k_out = torch.empty((max(total, 1), 6), dtype=torch.int32, device=dev)
    d_out = torch.empty((max(total, 1), 32), dtype=torch.uint8, device=dev)
    u_out = torch.empty(max(total, 1), dtype=torch.float32, device=dev) if u_right is not None else None
    lib = _lib.load()
    _lib.check(lib.omv_frame_pack(frames.n_frames, frames.n_cams, nb, frames.kp_cap, _lib.ptr(frames.kps),
                                  _lib.ptr(frames.desc), _lib.ptr(u_right), _lib.ptr(frames.n_kp), _lib.ptr(off),
                                  _lib.ptr(k_out), _lib.ptr(d_out),
                                  _lib.ptr(u_out), _stream_handle(torch, stream)), "omv_frame_pack")
    return off, k_out[:total], d_out[:total], (u_out[:total] if u_out is not None else None)


def _stream_handle(torch, stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
