"""Seeded synthetic camera images and map-point sets (BASELINE.md "Workloads").

No datasets are available, so every workload is generated from a seed:
- images: PCG64(seed), 300 random filled rectangles / ellipses with intensity U{0..255} on a
  128-grey background, a 3x3 box blur, then additive N(0, 6^2) noise clipped to u8;
- Hilti-like rig: seed = 20221000 + 1000*cam + frame (5 cams, 720x540);
- 8-cam 1080p rig: seed = 3000 + 1000*cam + frame; EuRoC-like mono: seed = 101 + frame.
"""
import numpy as np

HILTI_SEED = 20221000
P1080_SEED = 3000
EUROC_SEED = 101


def synth_image(seed, w, h, n_shapes=300):
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.full((h, w), 128.0, dtype=np.float32)
    kind = rng.integers(0, 2, n_shapes)
    cx = rng.uniform(0, w, n_shapes)
    cy = rng.uniform(0, h, n_shapes)
    rx = rng.uniform(4, 60, n_shapes)
    ry = rng.uniform(4, 60, n_shapes)
    val = rng.integers(0, 256, n_shapes).astype(np.float32)
    for k in range(n_shapes):
        x0, x1 = int(max(0, cx[k] - rx[k])), int(min(w, cx[k] + rx[k] + 1))
        y0, y1 = int(max(0, cy[k] - ry[k])), int(min(h, cy[k] + ry[k] + 1))
        if x1 <= x0 or y1 <= y0:
            continue
        if kind[k] == 0:
            img[y0:y1, x0:x1] = val[k]
        else:
            yy, xx = np.mgrid[y0:y1, x0:x1]
            m = ((xx - cx[k]) / rx[k]) ** 2 + ((yy - cy[k]) / ry[k]) ** 2 <= 1.0
            img[y0:y1, x0:x1][m] = val[k]
    pad = np.pad(img, 1, mode="edge")
    blur = sum(pad[dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)) / 9.0
    noisy = blur + rng.normal(0.0, 6.0, (h, w)).astype(np.float32)
    return np.clip(np.rint(noisy), 0, 255).astype(np.uint8)


def hilti_frame(frame, n_cams=5, w=720, h=540):
    return np.stack([synth_image(HILTI_SEED + 1000 * c + frame, w, h) for c in range(n_cams)])


def rig_frame(frame, n_cams, w, h, base_seed):
    return np.stack([synth_image(base_seed + 1000 * c + frame, w, h) for c in range(n_cams)])


def flip_bits(desc, rng, max_flips=8):
    """Copy of a (n,32) u8 descriptor array with U{0..max_flips} random bit flips per row."""
    n = desc.shape[0]
    out = desc.copy()
    if n == 0:
        return out
    nflip = rng.integers(0, max_flips + 1, n)
    order = np.argsort(rng.random((n, 256)), axis=1)[:, :max_flips]   # distinct bits per row
    use = np.arange(max_flips)[None, :] < nflip[:, None]
    rows = np.repeat(np.arange(n), max_flips)[use.ravel()]
    bits = order.ravel()[use.ravel()]
    np.bitwise_xor.at(out, (rows, bits >> 3), (1 << (bits & 7)).astype(np.uint8))
    return out


def make_map_points(kps, desc, n_kp, M, seed, width, height, nlevels=8, frac_true=0.6):
    """Synthetic local map: `frac_true` of the points derive from true
    keypoints of the frame (descriptor with U{0..8} bit flips, projection = keypoint + N(0, 1 px),
    level = octave), the rest are random.  30% of the points are also visible in a second, random
    camera at a random position, so the multi-camera claim / `continue` logic is exercised.
    Inputs are host numpy arrays of one frame: kps [C][cap] (KP dtype), desc [C][cap][32], n_kp [C].
    Returns a dict of numpy arrays (the omv_mp_view fields)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    C = kps.shape[0]
    n_kp = np.asarray(n_kp)
    n_true = int(M * frac_true)
    cam0 = rng.integers(0, C, M)
    two = (rng.random(M) < 0.3) & (C > 1)
    cam1 = rng.integers(0, C, M)
    true = (np.arange(M) < n_true) & (n_kp[cam0] > 0)
    kidx = np.minimum((rng.random(M) * np.maximum(n_kp[cam0], 1)).astype(np.int64), np.maximum(n_kp[cam0] - 1, 0))
    src = kps[cam0, kidx]
    out = dict(
        desc=rng.integers(0, 256, (M, 32), dtype=np.uint8),
        proj_x=np.zeros((M, C), np.float32),
        proj_y=np.zeros((M, C), np.float32),
        view_cos=rng.uniform(0.99, 1.0, (M, C)).astype(np.float32),
        level=np.full((M, C), -1, np.int32),
        in_view=np.zeros((M, C), np.uint8),
        track_depth=rng.uniform(1.0, 60.0, M).astype(np.float32),
        is_bad=(rng.random(M) < 0.02).astype(np.uint8),
        has_obs=(rng.random(M) > 0.03).astype(np.uint8),
    )
    ar = np.arange(M)
    rx, ry = rng.uniform(0, width, M), rng.uniform(0, height, M)
    rl = rng.integers(0, nlevels, M)
    nx, ny = rng.normal(0.0, 1.0, M), rng.normal(0.0, 1.0, M)
    out["proj_x"][ar, cam0] = np.where(true, src["x"] + nx, rx)
    out["proj_y"][ar, cam0] = np.where(true, src["y"] + ny, ry)
    out["level"][ar, cam0] = np.where(true, src["octave"], rl)
    out["in_view"][ar, cam0] = 1
    out["desc"][true] = flip_bits(desc[cam0[true], kidx[true]], rng)
    sx, sy = rng.uniform(0, width, M), rng.uniform(0, height, M)
    sl = rng.integers(0, nlevels, M)
    m2 = two & (cam1 != cam0)
    out["proj_x"][ar[m2], cam1[m2]] = sx[m2]
    out["proj_y"][ar[m2], cam1[m2]] = sy[m2]
    out["level"][ar[m2], cam1[m2]] = sl[m2]
    out["in_view"][ar[m2], cam1[m2]] = 1
    return out


# ---- 3-D local maps for Frame::isInFrustum (BASELINE config 2 with geometry) ---------------------------
def hilti_rig(n_cams=5):
    """KB8 parameters [C][8] and the block-c-from-block-0 transforms (R_cl [C][3][3], t_cl [C][3]) of the
    Hilti-2022 rig (block 0 = cam0 left, 1 = cam1 right, >= 2 side cameras), float32."""
    from .synth_ba import rig as ba_rig
    cams, Rbc, tbc = ba_rig()
    Rcb = np.transpose(Rbc, (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc)
    R_cl = np.einsum("cij,jk->cik", Rcb, Rbc[0])
    t_cl = np.einsum("cij,j->ci", Rcb, tbc[0]) + tcb
    return cams[:n_cams].astype(np.float32), R_cl[:n_cams].astype(np.float32), t_cl[:n_cams].astype(np.float32)


def p1080_rig(n_cams=8, width=1920, height=1080):
    """BASELINE config 4's synthetic Pinhole rig: n_cams cameras on a 0.15 m ring, yawed 360/n_cams degrees
    apart (block 0 = left, 1 = right, >= 2 side cameras), fx = fy = 700 px, principal point at the image
    centre.  Returns (Pinhole parameters [C][4], R_cl [C][3][3], t_cl [C][3]) in float32."""
    cams = np.tile(np.array([700.0, 700.0, width / 2.0, height / 2.0]), (n_cams, 1))
    R_cl, t_cl = [], []
    for c in range(n_cams):
        a = 2 * np.pi * c / n_cams
        # camera c's axes in block-0 coordinates: yaw a about the y (down) axis
        Rlc = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
        Ol = 0.15 * np.array([np.sin(a), 0.0, np.cos(a) - 1.0])   # centre on the ring through block 0's
        R_cl.append(Rlc.T)
        t_cl.append(-Rlc.T @ Ol)
    return cams.astype(np.float32), np.array(R_cl, np.float32), np.array(t_cl, np.float32)


def pinhole_unproject(k, u, v):
    """Unit ray of pixel (u, v) through Pinhole k = (fx, fy, cx, cy)."""
    k = np.asarray(k, np.float64)
    ray = np.stack([(np.asarray(u, np.float64) - k[2]) / k[0], (np.asarray(v, np.float64) - k[3]) / k[1],
                    np.ones(np.shape(u))], -1)
    return ray / np.linalg.norm(ray, axis=-1, keepdims=True)


def random_pose(rng):
    """omv_frame_pose as float32[24]: Rcw, tcw, Rwc, Ow of block 0."""
    q = rng.normal(0, 1, 4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    t = rng.uniform(-5, 5, 3)
    Rwc = R.T
    Ow = -Rwc @ t
    return np.concatenate([R.reshape(-1), t, Rwc.reshape(-1), Ow]).astype(np.float32)


def kb8_unproject(k, u, v, iters=10):
    """Ray (unit) of pixel (u, v) through KannalaBrandt8 k (Newton on theta, like unproject())."""
    k = np.asarray(k, np.float64)
    px, py = (np.asarray(u, np.float64) - k[2]) / k[0], (np.asarray(v, np.float64) - k[3]) / k[1]
    r = np.sqrt(px * px + py * py)
    th = r.copy()
    for _ in range(iters):
        t2 = th * th
        f = th * (1 + t2 * (k[4] + t2 * (k[5] + t2 * (k[6] + t2 * k[7])))) - r
        fd = 1 + t2 * (3 * k[4] + t2 * (5 * k[5] + t2 * (7 * k[6] + t2 * 9 * k[7])))
        th = th - f / fd
    s = np.where(r > 1e-12, np.sin(th) / np.maximum(r, 1e-12), 1.0)
    return np.stack([px * s, py * s, np.cos(th)], -1)


def make_world_map(kps, desc, n_kp, M, seed, cams, R_cl, t_cl, pose, width, height, nlevels=8, frac_true=0.6,
                   scale=1.2, model="kb8"):
    """Local map points in 3-D for one frame: `frac_true` are keypoints of a random camera block
    unprojected to a depth U(2, 20) m (descriptor with U{0..8} bit flips, mfMaxDistance chosen so
    PredictScale returns the keypoint's octave), the rest random pixels/depths/octaves.  Normals point
    from the observing camera to the point (+ noise).  Returns (world dict, map-point dict)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    C = kps.shape[0]
    n_kp = np.asarray(n_kp)
    cam = rng.integers(0, C, M)
    true = (np.arange(M) < int(M * frac_true)) & (n_kp[cam] > 0)
    kidx = np.minimum((rng.random(M) * np.maximum(n_kp[cam], 1)).astype(np.int64), np.maximum(n_kp[cam] - 1, 0))
    src = kps[cam, kidx]
    u = np.where(true, src["x"], rng.uniform(0, width, M))
    v = np.where(true, src["y"], rng.uniform(0, height, M))
    octv = np.where(true, src["octave"], rng.integers(0, nlevels, M))
    ray = np.zeros((M, 3))
    for c in range(C):
        sel = cam == c
        ray[sel] = (pinhole_unproject if model == "pinhole" else kb8_unproject)(cams[c], u[sel], v[sel])
    depth = rng.uniform(2.0, 20.0, M)
    Xc = ray * depth[:, None]
    Rcl, tcl = R_cl[cam].astype(np.float64), t_cl[cam].astype(np.float64)
    Xl = np.einsum("mji,mj->mi", Rcl, Xc - tcl)
    Rwc, Ow = pose[12:21].reshape(3, 3).astype(np.float64), pose[21:24].astype(np.float64)
    Xw = Xl @ Rwc.T + Ow
    Oc = np.einsum("mji,mj->mi", Rcl, -tcl) @ Rwc.T + Ow
    d = Xw - Oc
    dist = np.linalg.norm(d, axis=1)
    nrm = d / dist[:, None] + rng.normal(0, 0.05, (M, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    maxd = dist * np.float64(scale) ** octv * rng.uniform(0.86, 0.97, M)
    mind = maxd / np.float64(scale) ** (nlevels - 1)
    world = dict(pos=Xw.astype(np.float32), normal=nrm.astype(np.float32), min_dist=mind.astype(np.float32),
                 max_dist=maxd.astype(np.float32))
    mp = dict(
        desc=rng.integers(0, 256, (M, 32), dtype=np.uint8),
        proj_x=np.full((M, C), -1, np.float32), proj_y=np.full((M, C), -1, np.float32),
        view_cos=np.zeros((M, C), np.float32), level=np.full((M, C), -1, np.int32),
        in_view=np.zeros((M, C), np.uint8), track_depth=rng.uniform(1.0, 60.0, M).astype(np.float32),
        is_bad=(rng.random(M) < 0.02).astype(np.uint8), has_obs=(rng.random(M) > 0.03).astype(np.uint8))
    mp["desc"][true] = flip_bits(desc[cam[true], kidx[true]], rng)
    return world, mp


def quat_from_R(R):
    """Unit quaternion (x, y, z, w) of a rotation matrix (float64)."""
    R = np.asarray(R, np.float64)
    w = np.sqrt(max(0.0, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.copysign(np.sqrt(max(0.0, 1 + R[0, 0] - R[1, 1] - R[2, 2])) / 2, R[2, 1] - R[1, 2])
    y = np.copysign(np.sqrt(max(0.0, 1 - R[0, 0] + R[1, 1] - R[2, 2])) / 2, R[0, 2] - R[2, 0])
    z = np.copysign(np.sqrt(max(0.0, 1 - R[0, 0] - R[1, 1] + R[2, 2])) / 2, R[1, 0] - R[0, 1])
    q = np.array([x, y, z, w])
    return q / np.linalg.norm(q)


def make_last_frame(kps, desc, n_kp, seed, cams, Tcw7, frac_valid=0.7, rand_angle=0.2, pinhole=False):
    """LastFrame for SearchByProjection(Frame&, const Frame&): the current frame's keypoints as the last
    frame's tracked points (unprojected through block 0's camera at depth U(2, 20) and moved to world
    with Tcw), descriptors with U{0..8} bit flips, `frac_valid` valid, angles perturbed (a `rand_angle`
    share at random) so the rotation histogram rejects some.  Returns numpy SoA of omv_last_frame."""
    rng = np.random.Generator(np.random.PCG64(seed))
    C, cap = kps.shape[0], kps.shape[1]
    S = C * cap
    flat = kps.reshape(-1)
    ar = np.arange(S)
    exists = (ar % cap) < np.repeat(np.asarray(n_kp), cap)
    valid = exists & (rng.random(S) < frac_valid)
    if pinhole:   # Pinhole::unprojectEig of block 0's camera
        k = np.asarray(cams[0], np.float64)
        ray = np.stack([(flat["x"] - k[2]) / k[0], (flat["y"] - k[3]) / k[1], np.ones(S)], -1)
    else:
        ray = kb8_unproject(cams[0], flat["x"], flat["y"])
    Xc = ray * rng.uniform(2.0, 20.0, S)[:, None]
    q = np.asarray(Tcw7[:4], np.float64)
    t = np.asarray(Tcw7[4:], np.float64)
    x, y, z, w = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    Xw = (Xc - t) @ R   # R^T (Xc - t)
    lk = flat.copy()
    ang = lk["angle"] + rng.normal(0, 3.0, S)
    rnd = rng.random(S) < rand_angle
    ang = np.where(rnd, rng.uniform(0, 360, S), ang) % 360.0
    lk["angle"] = ang.astype(np.float32)
    d = desc.reshape(S, 32)
    return dict(pos=Xw.astype(np.float32), desc=flip_bits(d, rng), valid=valid.astype(np.uint8),
                has_obs=(rng.random(S) > 0.05).astype(np.uint8), kps=lk)


def random_se3(rng, scale=5.0):
    R = random_pose(rng)[:9].reshape(3, 3).astype(np.float64)
    return np.concatenate([quat_from_R(R), rng.uniform(-scale, scale, 3)]).astype(np.float32)
