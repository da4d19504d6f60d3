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
