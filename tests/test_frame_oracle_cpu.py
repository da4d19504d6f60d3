"""CPU checks of the GetDepthFromUndistortedPoints restatement (oracle/frame_oracle.cpp;
src/Frame.cc:1659-1765 with OpenCV's cv::fisheye::undistortPoints).  OpenCV is absent and the
reference holds no fixtures for this path, so parity with OpenCV is unpinned; these pin the
restatement: the distortion-free case against the closed form, distort -> undistort round trips
on the reference's own Hilti calibrations, and the depth-lookup / u_right rule on designed inputs."""
import numpy as np

from openmavis_amd import _lib
from openmavis_amd.frame import BLOCK_CAM_ID, HILTI_UNDIST, undist_params


def _keys(xy):
    k = np.zeros(len(xy), _lib.KP_DTYPE)
    k["x"], k["y"] = np.asarray(xy, np.float32)[:, 0], np.asarray(xy, np.float32)[:, 1]
    return k


def _distort(cal, u, v):
    """Fisheye (KB) distortion of the undistorted newK pixel (u, v) into the origK image (double)."""
    K, D, nK = cal
    x, y = (u - nK[2]) / nK[0], (v - nK[3]) / nK[1]
    r = np.hypot(x, y)
    th = np.arctan(r)
    thd = th * (1 + D[0] * th ** 2 + D[1] * th ** 4 + D[2] * th ** 6 + D[3] * th ** 8)
    s = np.where(r > 0, thd / np.maximum(r, 1e-300), 1.0)
    return K[0] * x * s + K[2], K[1] * y * s + K[3]


def test_zero_distortion_is_equidistant_to_pinhole(oracle):
    K, nK = (350.0, 351.0, 360.0, 270.0), (270.0, 271.0, 370.0, 260.0)
    U = undist_params((0,), {0: (K, (0.0, 0.0, 0.0, 0.0), nK)})[0]
    rng = np.random.default_rng(0)
    xy = np.stack([rng.uniform(0, 720, 500), rng.uniform(0, 540, 500)], 1).astype(np.float32)
    _, out = oracle.depth_from_undistorted(_keys(xy), np.zeros((540, 720), np.float32), U, 40.0)
    pw = (xy.astype(np.float64) - [K[2], K[3]]) / [K[0], K[1]]
    td = np.hypot(pw[:, 0], pw[:, 1])
    pu = pw * (np.tan(td) / td)[:, None]
    exp = pu * [nK[0], nK[1]] + [nK[2], nK[3]]
    assert np.allclose(out, exp, atol=1e-3, rtol=0)


def test_round_trip_on_the_reference_calibrations(oracle):
    rng = np.random.default_rng(1)
    for cid in BLOCK_CAM_ID:
        cal = HILTI_UNDIST[cid]
        U = undist_params((cid,))[0]
        u, v = rng.uniform(-100, 820, 2000), rng.uniform(-100, 640, 2000)
        xd, yd = _distort(cal, u, v)
        keep = (xd > 0) & (xd < 720) & (yd > 0) & (yd < 540)
        xy = np.stack([xd[keep], yd[keep]], 1).astype(np.float32)
        _, out = oracle.depth_from_undistorted(_keys(xy), np.zeros((540, 720), np.float32), U, 40.0)
        # the float input carries ~3e-5 px; the Newton solve converges to 1e-8 rad
        assert np.abs(out - np.stack([u[keep], v[keep]], 1)).max() < 2e-3, cid


def test_uright_rule(oracle):
    """d = depth(round(y), round(x)); u_R = x - bf / d for 0 < d <= 20, else -1 (incl. outside)."""
    U = undist_params((1,))[0]
    h, w = 540, 720
    depth = np.full((h, w), 5.0, np.float32)
    rng = np.random.default_rng(2)
    depth[rng.random((h, w)) < 0.2] = 0.0
    depth[rng.random((h, w)) < 0.1] = 25.0
    depth[rng.random((h, w)) < 0.05] = 20.0
    depth[rng.random((h, w)) < 0.02] = np.nan
    xy = np.stack([rng.uniform(0, 720, 3000), rng.uniform(0, 540, 3000)], 1).astype(np.float32)
    xy[:5] = [[0, 0], [719.9, 539.9], [0, 539], [719, 0], [360, 270]]   # corners undistort far outside
    keys = _keys(xy)
    bf = np.float32(40.0)
    ur, out = oracle.depth_from_undistorted(keys, depth, U, float(bf))
    for i in range(len(xy)):
        x, y = int(np.round(np.float32(out[i, 0]))), int(np.round(np.float32(out[i, 1])))
        d = depth[y, x] if 0 <= x < w and 0 <= y < h else np.float32(0)
        exp = np.float32(keys["x"][i] - bf / d) if (d > 0 and d <= 20) else np.float32(-1)
        assert ur[i] == exp, (i, ur[i], exp)
    assert (ur == -1).sum() > 100 and (ur != -1).sum() > 100
