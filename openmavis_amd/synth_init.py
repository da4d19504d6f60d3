"""Seeded synthetic frame pairs for ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:895-1004).

Monocular initialisation matches the first frame's level-0 keypoints into the second frame around their
previous positions (vbPrevMatched = F1.mvKeysUn at the start).  F1 holds n keypoints (octaves U{0..3},
about half at level 0) on a 752x480 EuRoC-sized image; F2 re-observes 85 % of them moved by a common
image motion + N(0, 1.5 px) with U{0..10} descriptor bit flips and the angle rotated by a common offset +
N(0, 4 deg), plus unrelated distractors (a third at level 0).  Both keypoint lists are in image order
(ascending y, then x), as an extractor leaves them.
"""
import numpy as np

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])
W, H = 752, 480


def _kps(xy, octave, angle):
    k = np.zeros(len(xy), KP_DTYPE)
    k["x"], k["y"] = xy[:, 0], xy[:, 1]
    k["size"] = 31.0
    k["angle"] = angle
    k["response"] = 10.0
    k["octave"] = octave
    return k


def make_init_pair(seed=1, n=1000, n_distract=300, motion=(6.0, -4.0), rot=12.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    xy1 = np.stack([rng.uniform(20, W - 20, n), rng.uniform(20, H - 20, n)], 1).astype(np.float32)
    oct1 = np.where(rng.random(n) < 0.5, 0, rng.integers(1, 4, n)).astype(np.int32)
    ang1 = rng.uniform(0, 360, n).astype(np.float32)
    desc1 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    keep = rng.random(n) < 0.85
    src = np.nonzero(keep)[0]
    xy2 = xy1[src] + np.asarray(motion, np.float32) + rng.normal(0, 1.5, (len(src), 2)).astype(np.float32)
    ang2 = ((ang1[src] + rot + rng.normal(0, 4, len(src))) % 360).astype(np.float32)
    d2 = desc1[src].copy()
    for r in range(len(src)):
        for _ in range(int(rng.integers(0, 11))):
            b = int(rng.integers(0, 256))
            d2[r, b // 8] ^= np.uint8(1 << (b % 8))
    oct2 = oct1[src]
    xyd = np.stack([rng.uniform(20, W - 20, n_distract), rng.uniform(20, H - 20, n_distract)], 1).astype(np.float32)
    octd = np.where(rng.random(n_distract) < 0.33, 0, rng.integers(1, 4, n_distract)).astype(np.int32)
    xy2 = np.concatenate([xy2, xyd])
    oct2 = np.concatenate([oct2, octd])
    ang2 = np.concatenate([ang2, rng.uniform(0, 360, n_distract).astype(np.float32)])
    d2 = np.concatenate([d2, rng.integers(0, 256, (n_distract, 32), dtype=np.uint8)])
    truth2 = np.concatenate([src, np.full(n_distract, -1)]).astype(np.int32)   # F1 index of each F2 keypoint
    o1 = np.lexsort((xy1[:, 0], xy1[:, 1]))
    o2 = np.lexsort((xy2[:, 0], xy2[:, 1]))
    inv1 = np.empty(n, np.int64)
    inv1[o1] = np.arange(n)
    t2 = truth2[o2]
    t2 = np.where(t2 >= 0, inv1[np.maximum(t2, 0)], -1).astype(np.int32)
    f1 = dict(kps=_kps(xy1[o1], oct1[o1], ang1[o1]), desc=desc1[o1])
    f2 = dict(kps=_kps(xy2[o2], oct2[o2], ang2[o2]), desc=d2[o2], truth=t2)
    prev = np.stack([f1["kps"]["x"], f1["kps"]["y"]], 1).astype(np.float32)   # vbPrevMatched = F1.mvKeysUn
    return dict(f1=f1, f2=f2, prev=prev, width=W, height=H)


def scale_factors(nlevels=8, scale=1.2):
    s = [1.0]
    for _ in range(1, nlevels):
        s.append(s[-1] * np.float32(scale))
    return np.asarray(s, np.float32)
