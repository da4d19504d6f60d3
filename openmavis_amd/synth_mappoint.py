"""Synthetic map-point batches for the map-point refresh (ComputeDistinctiveDescriptors / UpdateNormalAndDepth): each
point has N observation descriptors -- noisy copies of one base descriptor (a few bit flips, as the same 3-D point seen
from several keyframes) plus some unrelated ones -- drawn from a shared row table, and N camera centres around it."""
import numpy as np


def make_points(n_points=1000, seed=1, sizes=None, n_rows=None, flip=(0, 12), outlier_frac=0.2, dup_frac=0.1):
    rng = np.random.default_rng(seed)
    if sizes is None:
        sizes = rng.integers(0, 24, n_points)
    sizes = np.asarray(sizes, np.int64)
    n_points = len(sizes)
    rows, start = [], [0]
    table = []
    for p in range(n_points):
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        for _ in range(int(sizes[p])):
            if rng.random() < outlier_frac:
                d = rng.integers(0, 256, 32, dtype=np.uint8)
            elif table and rng.random() < dup_frac:
                d = table[-1].copy()   # duplicates: equal distances / medians (first-index ties)
            else:
                d = base.copy()
                bits = rng.choice(256, int(rng.integers(flip[0], flip[1] + 1)), replace=False)
                for b in bits:
                    d[b >> 3] ^= np.uint8(1 << (b & 7))
            rows.append(len(table))
            table.append(d)
        start.append(len(rows))
    desc = np.array(table, np.uint8).reshape(-1, 32)
    if len(desc) == 0:
        desc = np.zeros((1, 32), np.uint8)
    perm = rng.permutation(len(desc))   # rows scattered over the table (the keyframes' descriptor matrices)
    inv = np.argsort(perm)
    desc = desc[perm]
    rows = inv[np.array(rows, np.int64)].astype(np.int32) if rows else np.zeros(0, np.int32)
    return dict(desc=desc, desc_start=np.array(start, np.int32), desc_row=rows)


def make_geometry(n_points=1000, seed=2, max_obs=12):
    rng = np.random.default_rng(seed)
    cnt = rng.integers(0, max_obs + 1, n_points)
    start = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    pos = rng.normal(0, 20, (n_points, 3)).astype(np.float32)
    cen = (np.repeat(pos, cnt, axis=0) + rng.normal(0, 8, (int(cnt.sum()), 3))).astype(np.float32)
    ref = (pos + rng.normal(0, 8, (n_points, 3))).astype(np.float32)
    scales = (1.2 ** np.arange(8)).astype(np.float32)
    lvl = rng.integers(0, 8, n_points)
    return dict(obs_start=start, obs_center=cen, pos=pos, ref_center=ref, ref_level_scale=scales[lvl],
                ref_max_scale=np.full(n_points, scales[7], np.float32))
