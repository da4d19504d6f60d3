"""GPU parity of the Frame constructor tail (openmavis_amd/csrc/frame.hip) against the CPU oracle
(oracle/frame_oracle.cpp): mvuRight from GetDepthFromUndistortedPoints (src/Frame.cc:1659-1765) and the
vconcat of keypoints / descriptors / mvuRight (:1913-1939).  Bar: bit-exact u_right and undistorted
points; the only transcendental, tan(theta) in double, comes from different libms on the two sides,
which can move a float-rounded point only when its double lies within an ulp of a rounding boundary
(none in these seeded cases)."""
import numpy as np
import pytest

from openmavis_amd import _lib
from openmavis_amd.frame import BLOCK_CAM_ID, frame_pack, frame_uright, undist_params

pytestmark = pytest.mark.gpu


def _frames(torch, n_frames, n_cams, kp_cap, seed):
    from openmavis_amd.matcher import FrameBatch
    rng = np.random.default_rng(seed)
    fb = FrameBatch(torch, n_frames, n_cams, kp_cap, 720, 540, [1.0] * 8, device="cuda")
    n_kp = rng.integers(0, kp_cap + 1, (n_frames, n_cams)).astype(np.int32)
    n_kp[0, 0], n_kp[-1, -1] = 0, kp_cap   # an empty block and a full one
    kps = np.zeros((n_frames, n_cams, kp_cap), _lib.KP_DTYPE)
    kps["x"] = rng.uniform(0, 720, kps.shape)
    kps["y"] = rng.uniform(0, 540, kps.shape)
    kps["octave"] = rng.integers(0, 8, kps.shape)
    kps["angle"] = rng.uniform(0, 360, kps.shape)
    fb.kps.copy_(torch.from_numpy(kps.view(np.int32).reshape(n_frames, n_cams, kp_cap, 6)))
    fb.desc.copy_(torch.from_numpy(rng.integers(0, 256, (n_frames, n_cams, kp_cap, 32), dtype=np.uint8)))
    fb.n_kp.copy_(torch.from_numpy(n_kp))
    return fb, kps, n_kp


def _depth(n_frames, n_cams, seed, h=540, w=720):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    d = np.empty((n_frames, n_cams, h, w), np.float32)
    for f in range(n_frames):
        for c in range(n_cams):
            d[f, c] = 2 + 10 * (1 + np.sin(xx / (40 + 7 * c) + f) * np.cos(yy / 55)) + rng.normal(0, 0.2, (h, w))
    d[rng.random(d.shape) < 0.15] = 0.0    # holes
    d[rng.random(d.shape) < 0.05] = 30.0   # beyond the 20 m cut
    return d


def test_uright_matches_oracle(oracle, torch_cuda):
    torch = torch_cuda
    F, C, cap = 6, 4, 700
    fb, kps, n_kp = _frames(torch, F, C, cap, 3)
    depth = _depth(F, C, 4)
    d_dev = torch.from_numpy(depth).cuda()
    xy = torch.zeros((F, C, cap, 2), dtype=torch.float32, device="cuda")
    bf = 47.3
    ur = frame_uright(fb, d_dev, bf, undist_xy=xy).cpu().numpy()
    xy = xy.cpu().numpy()
    U = undist_params(BLOCK_CAM_ID)
    for f in range(F):
        for c in range(C):
            n = int(n_kp[f, c])
            u_o, xy_o = oracle.depth_from_undistorted(kps[f, c, :n], depth[f, c], U[c], bf)
            assert np.array_equal(xy[f, c, :n], xy_o), (f, c)
            assert np.array_equal(ur[f, c, :n], u_o), (f, c)
    valid = np.concatenate([ur[f, c, :n_kp[f, c]] for f in range(F) for c in range(C)])
    assert (valid == -1).sum() > 50 and (valid > -1).sum() > 500


def test_uright_first_blocks_of_wider_frames(oracle, torch_cuda):
    """A 5-camera FrameBatch: the four reference blocks are taken, the fifth is ignored."""
    torch = torch_cuda
    fb, kps, n_kp = _frames(torch, 2, 5, 300, 5)
    depth = _depth(2, 4, 6)
    ur = frame_uright(fb, torch.from_numpy(depth).cuda(), 40.0).cpu().numpy()
    U = undist_params(BLOCK_CAM_ID)
    for f in range(2):
        for c in range(4):
            n = int(n_kp[f, c])
            assert np.array_equal(ur[f, c, :n], oracle.depth_from_undistorted(kps[f, c, :n], depth[f, c], U[c], 40.0)[0])


def test_frame_pack_is_vconcat(torch_cuda):
    torch = torch_cuda
    F, C, cap = 7, 4, 500
    fb, kps, n_kp = _frames(torch, F, C, cap, 7)
    ur = torch.from_numpy(np.random.default_rng(8).normal(0, 1, (F, C, cap)).astype(np.float32)).cuda()
    off, k_out, d_out, u_out = frame_pack(fb, ur)
    off = off.cpu().numpy()
    desc = fb.desc.cpu().numpy()
    urh = ur.cpu().numpy()
    exp_off = np.concatenate([[0], np.cumsum(n_kp.sum(1))])
    assert np.array_equal(off, exp_off)
    k_out = k_out.cpu().numpy().view(_lib.KP_DTYPE).reshape(-1)
    for f in range(F):
        sl = slice(off[f], off[f + 1])
        assert np.array_equal(k_out[sl], np.concatenate([kps[f, c, :n_kp[f, c]] for c in range(C)]))
        assert np.array_equal(d_out.cpu().numpy()[sl], np.concatenate([desc[f, c, :n_kp[f, c]] for c in range(C)]))
        assert np.array_equal(u_out.cpu().numpy()[sl], np.concatenate([urh[f, c, :n_kp[f, c]] for c in range(C)]))


def test_frame_pack_first_blocks(torch_cuda):
    """Dense rows of the four reference blocks of a 5-camera batch (u_right in the 4-block layout)."""
    torch = torch_cuda
    fb, kps, n_kp = _frames(torch, 3, 5, 200, 9)
    ur = torch.from_numpy(np.random.default_rng(10).normal(0, 1, (3, 4, 200)).astype(np.float32)).cuda()
    off, k_out, d_out, u_out = frame_pack(fb, ur, n_cams=4)
    off = off.cpu().numpy()
    assert np.array_equal(off, np.concatenate([[0], np.cumsum(n_kp[:, :4].sum(1))]))
    k_out = k_out.cpu().numpy().view(_lib.KP_DTYPE).reshape(-1)
    urh = ur.cpu().numpy()
    for f in range(3):
        sl = slice(off[f], off[f + 1])
        assert np.array_equal(k_out[sl], np.concatenate([kps[f, c, :n_kp[f, c]] for c in range(4)]))
        assert np.array_equal(u_out.cpu().numpy()[sl], np.concatenate([urh[f, c, :n_kp[f, c]] for c in range(4)]))
