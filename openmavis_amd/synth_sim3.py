"""Seeded synthetic keyframe pairs for ORBmatcher::SearchBySim3 (src/ORBmatcher.cc:1771-1983).

Per pair (kf1 = 2p, kf2 = 2p + 1 of the batch): world points placed in pKF1's camera frame (pinhole pixel,
depth U(2, 15) m) and carried into pKF2's camera by a random similarity S21 (rotation up to ~0.3 rad, scale
U(0.7, 1.4)); the points pKF2 sees get a block-0 keypoint there too.  Keypoints: the pinhole projection
+ N(0, 0.5 px), ORB-like octaves, descriptors = the point's base descriptor with U{0..8} bit flips; map
points: that keypoint's descriptor with U{0..6} flips, world position through a random keyframe pose,
mfMaxDistance chosen so PredictScale returns the other keyframe's octave.  Clutter: 30 % extra block-0
keypoints (some with random map points), keypoints in the other camera blocks with random map points, 10 %
near-copies of another point's map point (agreement failures), 8 % of the mapped keypoints left out of the
side lists (vbAlreadyMatched / isBad).
"""
import numpy as np

from . import synth
from .synth_kfmatch import KP_DTYPE, _R_of

FX, FY, CX, CY = 380.0, 380.0, 360.0, 270.0


def _quat(R):
    return synth.quat_from_R(np.asarray(R, np.float64)).astype(np.float64)


def _sim3(q_unit, s, t):
    q = np.asarray(q_unit, np.float64) * np.sqrt(s)
    qf = q.astype(np.float32)
    scale = np.float32(((qf[0] * qf[0] + qf[1] * qf[1]) + qf[2] * qf[2]) + qf[3] * qf[3])
    return dict(q=qf, t=np.asarray(t, np.float32), scale=scale)


def _rot(rng, max_angle):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    a = rng.uniform(-max_angle, max_angle)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K


def make_sim3_batch(n_pairs=3, n_cams=5, kp_cap=600, n_world=450, seed=1, width=720, height=540, nlevels=8):
    rng = np.random.Generator(np.random.PCG64(seed))
    C, n_kf = n_cams, 2 * n_pairs
    pw = np.float64(1.2) ** (-2.0 * np.arange(nlevels))
    pw /= pw.sum()
    kps = np.zeros((n_kf, C, kp_cap), KP_DTYPE)
    desc = rng.integers(0, 256, (n_kf, C, kp_cap, 32), dtype=np.uint8)
    n_kp = np.zeros((n_kf, C), np.int32)
    wid = np.full((n_kf, kp_cap), -1, np.int64)   # truth: the world point of a block-0 keypoint (per pair)
    kps["size"], kps["response"] = 7.0, 1.0
    kps["angle"] = rng.uniform(0, 360, kps.shape)
    for c in range(1, C):   # the other blocks: random keypoints
        n_kp[:, c] = rng.integers(kp_cap // 2, kp_cap + 1, n_kf)
        kps["x"][:, c] = rng.uniform(0, width, (n_kf, kp_cap))
        kps["y"][:, c] = rng.uniform(0, height, (n_kf, kp_cap))
        kps["octave"][:, c] = rng.choice(nlevels, (n_kf, kp_cap), p=pw)
    tab = {k: [] for k in ("pos", "min_dist", "max_dist", "desc")}
    n_rows = [0]
    jobs, side = [], {1: ([], []), 2: ([], [])}

    def add_mps(pos, maxd, dsc):
        tab["pos"].append(np.asarray(pos, np.float32).reshape(-1, 3))
        tab["max_dist"].append(np.asarray(maxd, np.float32))
        tab["min_dist"].append((np.asarray(maxd, np.float64) / 1.2 ** (nlevels - 1)).astype(np.float32))
        tab["desc"].append(np.asarray(dsc, np.uint8).reshape(-1, 32))
        r = np.arange(n_rows[0], n_rows[0] + len(maxd))
        n_rows[0] += len(maxd)
        return r

    for p in range(n_pairs):
        k1, k2 = 2 * p, 2 * p + 1
        T = [synth.random_se3(rng) for _ in range(2)]
        Rw = [_R_of(t[:4]) for t in T]
        tw = [t[4:].astype(np.float64) for t in T]
        R21, s21, t21 = _rot(rng, 0.3), rng.uniform(0.7, 1.4), rng.uniform(-0.5, 0.5, 3)
        S21 = _sim3(_quat(R21), s21, t21)
        S12 = _sim3(_quat(R21.T), 1.0 / s21, -(R21.T @ t21) / s21)
        # world points in camera 1, carried to camera 2
        u1, v1 = rng.uniform(0, width, n_world), rng.uniform(0, height, n_world)
        z1 = rng.uniform(2.0, 15.0, n_world)
        X1 = np.stack([(u1 - CX) / FX * z1, (v1 - CY) / FY * z1, z1], 1)
        X2 = s21 * X1 @ R21.T + t21
        with np.errstate(divide="ignore", invalid="ignore"):
            u2, v2 = FX * X2[:, 0] / X2[:, 2] + CX, FY * X2[:, 1] / X2[:, 2] + CY
        vis2 = (X2[:, 2] > 0.1) & (u2 >= 0) & (u2 < width) & (v2 >= 0) & (v2 < height)
        base = rng.integers(0, 256, (n_world, 32), dtype=np.uint8)
        oct1 = rng.choice(nlevels, n_world, p=pw)
        oct2 = rng.choice(nlevels, n_world, p=pw)
        views = {}
        for kf, X, uu, vv, oc, sel in ((k1, X1, u1, v1, oct1, np.ones(n_world, bool)), (k2, X2, u2, v2, oct2, vis2)):
            ids = np.nonzero(sel)[0]
            n_cl = int(0.3 * len(ids))
            n0 = min(kp_cap, len(ids) + n_cl)
            ids = ids[:n0 - n_cl] if len(ids) + n_cl > kp_cap else ids
            order = rng.permutation(n0)   # keypoint index of entry e: order[e]
            x = np.concatenate([uu[ids] + rng.normal(0, 0.5, len(ids)), rng.uniform(0, width, n0 - len(ids))])
            y = np.concatenate([vv[ids] + rng.normal(0, 0.5, len(ids)), rng.uniform(0, height, n0 - len(ids))])
            o = np.concatenate([oc[ids], rng.choice(nlevels, n0 - len(ids), p=pw)])
            d = np.concatenate([synth.flip_bits(base[ids], rng, 8),
                                rng.integers(0, 256, (n0 - len(ids), 32), dtype=np.uint8)])
            kps["x"][kf, 0, order], kps["y"][kf, 0, order], kps["octave"][kf, 0, order] = x, y, o
            desc[kf, 0, order] = d
            wid[kf, order[:len(ids)]] = ids
            n_kp[kf, 0] = n0
            views[kf] = (ids, order[:len(ids)])
        for kf, X, Xo, oc_o, tgt_side in ((k1, X1, X2, oct2, 1), (k2, X2, X1, oct1, 2)):
            ids, kidx = views[kf]
            i = 0 if kf == k1 else 1
            Xw = (X[ids] - tw[i]) @ Rw[i]
            # distance in the other camera; points the other keyframe cannot see get a random octave
            dist_o = np.linalg.norm(Xo[ids], axis=1)
            maxd = dist_o * 1.2 ** oc_o[ids] * rng.uniform(0.86, 0.97, len(ids))
            dsc = synth.flip_bits(desc[kf, 0, kidx], rng, 6)
            dup = np.nonzero(rng.random(len(ids)) < 0.1)[0]
            for a in dup:   # near-copy of another point's map point
                b = int(rng.integers(0, len(ids)))
                Xw[a], maxd[a], dsc[a] = Xw[b], maxd[b], synth.flip_bits(dsc[b:b + 1], rng, 4)[0]
            rows = add_mps(Xw, maxd, dsc)
            kp_list, mp_list = list(kidx), list(rows)
            # clutter keypoints of block 0 and the other blocks with random map points
            cl = np.setdiff1d(np.arange(n_kp[kf, 0]), kidx)
            cl = cl[rng.random(len(cl)) < 0.4]
            off = np.concatenate([[0], np.cumsum(n_kp[kf])])
            oth = np.concatenate([off[c] + np.nonzero(rng.random(n_kp[kf, c]) < 0.3)[0] for c in range(1, C)])
            extra = np.concatenate([cl, oth]).astype(np.int64)
            n_x = len(extra)
            Xr = np.stack([rng.uniform(-10, 10, n_x), rng.uniform(-10, 10, n_x), rng.uniform(-5, 20, n_x)], 1)
            rows = add_mps((Xr - tw[i]) @ Rw[i], rng.uniform(2.0, 40.0, n_x), rng.integers(0, 256, (n_x, 32)))
            kp_list += list(extra)
            mp_list += list(rows)
            kp_list, mp_list = np.asarray(kp_list, np.int64), np.asarray(mp_list, np.int64)
            keep = rng.random(len(kp_list)) >= 0.08
            srt = np.argsort(kp_list[keep], kind="stable")
            side[tgt_side][0].append(kp_list[keep][srt].astype(np.int32))
            side[tgt_side][1].append(mp_list[keep][srt].astype(np.int32))
        jobs.append(dict(kf1=k1, kf2=k2, T1w=T[0], T2w=T[1], S12=S12, S21=S21, fx=FX, fy=FY, cx=CX, cy=CY))
    s1 = s2 = 0
    for j, jb in enumerate(jobs):
        jb["start1"], jb["count1"] = s1, len(side[1][0][j])
        jb["start2"], jb["count2"] = s2, len(side[2][0][j])
        s1 += jb["count1"]
        s2 += jb["count2"]
    mps = {k: np.ascontiguousarray(np.concatenate(v)) for k, v in tab.items()}
    mps["normal"] = np.zeros_like(mps["pos"])
    return dict(n_kf=n_kf, n_cams=C, kp_cap=kp_cap, width=width, height=height, nlevels=nlevels, kps=kps, desc=desc,
                n_kp=n_kp, wid=wid, mps=mps, jobs=jobs, kp1=np.concatenate(side[1][0]), mp1=np.concatenate(side[1][1]),
                kp2=np.concatenate(side[2][0]), mp2=np.concatenate(side[2][1]))

