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
    out = desc.copy()
    n = desc.shape[0]
    nflip = rng.integers(0, max_flips + 1, n)
    for i in range(n):
        if nflip[i]:
            bits = rng.choice(256, nflip[i], replace=False)
            for b in bits:
                out[i, b >> 3] ^= np.uint8(1 << (b & 7))
    return out


def make_map_points(kps, desc, n_kp, M, seed, width, height, nlevels=8, frac_true=0.6):
    """Synthetic local map: `frac_true` of the points derive from true
    keypoints of the frame (descriptor with U{0..8} bit flips, projection = keypoint + N(0, 1 px),
    level = octave), the rest are random.  Some points are also visible in a second camera so the
    multi-camera claim / `continue` logic is exercised.  Inputs are host numpy arrays of one frame:
    kps [C][cap] (KP dtype), desc [C][cap][32], n_kp [C].  Returns a dict of numpy arrays."""
    rng = np.random.Generator(np.random.PCG64(seed))
    C = kps.shape[0]
    out = dict(
        desc=np.zeros((M, 32), np.uint8),
        proj_x=np.zeros((M, C), np.float32),
        proj_y=np.zeros((M, C), np.float32),
        view_cos=rng.uniform(0.99, 1.0, (M, C)).astype(np.float32),
        level=np.full((M, C), -1, np.int32),
        in_view=np.zeros((M, C), np.uint8),
        track_depth=rng.uniform(1.0, 60.0, M).astype(np.float32),
        is_bad=(rng.random(M) < 0.02).astype(np.uint8),
        has_obs=(rng.random(M) > 0.03).astype(np.uint8),
    )
    n_true = int(M * frac_true)
    for m in range(M):
        cams = [int(rng.integers(0, C))]
        if rng.random() < 0.3 and C > 1:
            cams.append(int(rng.integers(0, C)))
        for j, c in enumerate(cams):
            if m < n_true and n_kp[c] > 0 and j == 0:
                i = int(rng.integers(0, n_kp[c]))
                k = kps[c, i]
                out["desc"][m] = desc[c, i]
                out["proj_x"][m, c] = k["x"] + rng.normal(0.0, 1.0)
                out["proj_y"][m, c] = k["y"] + rng.normal(0.0, 1.0)
                out["level"][m, c] = k["octave"]
            else:
                if j == 0:
                    out["desc"][m] = rng.integers(0, 256, 32, dtype=np.uint8)
                out["proj_x"][m, c] = rng.uniform(0, width)
                out["proj_y"][m, c] = rng.uniform(0, height)
                out["level"][m, c] = int(rng.integers(0, nlevels))
            out["in_view"][m, c] = 1
    out["desc"][:n_true] = flip_bits(out["desc"][:n_true], rng)
    return out
