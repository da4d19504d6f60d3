"""Seeded synthetic map for LocalMapping::SearchInNeighbors' fuse sequence (src/LocalMapping.cc:837-889): a current
keyframe and `n_targets` target keyframes of the Hilti-like 4-camera KannalaBrandt8 rig on the synth_ba trajectory, all
seeing one set of world points.  Per keyframe and camera block: keypoints at the visible points' projections (+ N(0,
0.5 px); octave = the point's octave U{0..2}; descriptor = the point's base descriptor with U{0..4} bit flips) plus
distractors; block 0 carries mvuRight for ~30 % of its keypoints (Fuse's stereo gate).  The map holds DUPLICATE map
points -- what Fuse merges: each world point has 1-3 map-point instances, every keyframe observation of the point goes
to one of them with probability 0.75 (else the keypoint has no map point) -- with consistent observations
(mObservations by keyframe index, the L / R / SL / SR slots), mvpMapPoints, nObs, a position near the world point, the
mean viewing normal, mfMaxDistance = distance from the first observing camera x 1.2^octave (so PredictScale lands on the
observed octave) and one observation's descriptor."""
import numpy as np

from . import synth_ba
from .synth_cnmp import KP_DTYPE, _kf_at
from .synth_pose import quat_of


def make_fuse_scene(seed=1, n_targets=8, n_pts=500, n_distract=150, kp_cap=700, bf=40.0, nlevels=8):
    rng = np.random.Generator(np.random.PCG64(seed))
    cams, Rbc, tbc = synth_ba.rig()
    C = 4
    cams = cams[:C].astype(np.float32).copy()
    Rcb = np.transpose(Rbc[:C], (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc[:C])
    t0 = float(rng.uniform(2, 10))
    times = [t0] + [t0 + float(rng.choice([-1, 1])) * float(rng.uniform(0.1, 1.0)) for _ in range(n_targets)]
    poses = [_kf_at(t, C, Rcb, tcb) for t in times]
    n_kf = len(poses)
    R0, t0c = poses[0]
    X = []
    for _ in range(n_pts):
        c = int(rng.integers(0, C))
        d = rng.normal(0, 1, 3)
        d[2] = abs(d[2]) * 1.5 + 0.6
        d /= np.linalg.norm(d)
        X.append(R0[c].T @ (d * rng.uniform(2.0, 20.0) - t0c[c]))
    X = np.array(X)
    base = rng.integers(0, 256, (n_pts, 32), dtype=np.uint8)
    octv = rng.integers(0, 3, n_pts)
    kps = np.zeros((n_kf, C, kp_cap), KP_DTYPE)
    desc = np.zeros((n_kf, C, kp_cap, 32), np.uint8)
    n_kp = np.zeros((n_kf, C), np.int32)
    uright = np.full((n_kf, kp_cap), -1.0, np.float32)
    pt_of = np.full((n_kf, C, kp_cap), -1, np.int32)
    Tcw = np.zeros((n_kf, C, 7), np.float32)
    Ow = np.zeros((n_kf, C, 3), np.float32)
    for k, (Rcw, tcw) in enumerate(poses):
        for c in range(C):
            Tcw[k, c, :4] = quat_of(Rcw[c]).astype(np.float32)
            Tcw[k, c, 4:] = tcw[c].astype(np.float32)
            Ow[k, c] = (-Rcw[c].T @ tcw[c]).astype(np.float32)
            rows = []
            for p in range(n_pts):
                Xc = Rcw[c] @ X[p] + tcw[c]
                if Xc[2] < 0.3:
                    continue
                uv = synth_ba.cam_project(cams[c].astype(np.float64), Xc, False)
                if not (5 <= uv[0] <= 715 and 5 <= uv[1] <= 535):
                    continue
                uv = uv + rng.normal(0, 0.5, 2)
                dd = base[p].copy()
                for _ in range(int(rng.integers(0, 5))):
                    bit = int(rng.integers(0, 256))
                    dd[bit // 8] ^= np.uint8(1 << (bit % 8))
                rows.append((uv[0], uv[1], int(octv[p]), dd, p, Xc[2]))
            for _ in range(n_distract):
                rows.append((float(rng.uniform(10, 710)), float(rng.uniform(10, 530)), int(rng.integers(0, 4)),
                             rng.integers(0, 256, 32, dtype=np.uint8), -1, float(rng.uniform(1, 20))))
            rng.shuffle(rows)
            rows = rows[:kp_cap]
            n = len(rows)
            n_kp[k, c] = n
            kps[k, c, :n]["x"] = [r[0] for r in rows]
            kps[k, c, :n]["y"] = [r[1] for r in rows]
            kps[k, c, :n]["octave"] = [r[2] for r in rows]
            kps[k, c, :n]["angle"] = rng.uniform(0, 360, n)
            kps[k, c, :n]["size"], kps[k, c, :n]["response"] = 31.0, 10.0
            desc[k, c, :n] = np.stack([r[3] for r in rows])
            pt_of[k, c, :n] = [r[4] for r in rows]
            if c == 0:
                z = np.array([r[5] for r in rows])
                has = rng.random(n) < 0.3
                uright[k, :n] = np.where(has, kps[k, 0, :n]["x"] - bf / z, -1.0).astype(np.float32)
    # map-point instances per world point and their observations
    n_inst = rng.choice([1, 2, 3], n_pts, p=[0.5, 0.35, 0.15])
    first = np.concatenate([[0], np.cumsum(n_inst)])
    M0 = int(first[-1])
    obs = [dict() for _ in range(M0)]
    kf_mps = np.full((n_kf, C * kp_cap), -1, np.int32)
    for k in range(n_kf):
        off = 0
        for c in range(C):
            for i in range(n_kp[k, c]):
                p = pt_of[k, c, i]
                if p < 0 or rng.random() >= 0.75:
                    continue
                m = int(first[p] + rng.integers(0, n_inst[p]))
                slots = obs[m].setdefault(k, [-1, -1, -1, -1])
                if slots[c] != -1:   # one keypoint per (keyframe, block) slot: leave the extra one without a point
                    continue
                slots[c] = off + i
                kf_mps[k, off + i] = m
            off += n_kp[k, c]
    keep = [m for m in range(M0) if obs[m]]
    remap = np.full(M0, -1, np.int32)
    remap[keep] = np.arange(len(keep), dtype=np.int32)
    kf_mps = np.where(kf_mps >= 0, remap[np.maximum(kf_mps, 0)], -1).astype(np.int32)
    M = len(keep)
    inst_pt = np.repeat(np.arange(n_pts), n_inst)
    pos = np.zeros((M, 3), np.float32)
    normal = np.zeros((M, 3), np.float32)
    min_d = np.zeros(M, np.float32)
    max_d = np.zeros(M, np.float32)
    mdesc = np.zeros((M, 32), np.uint8)
    n_obs = np.zeros(M, np.int32)
    obs_start, obs_kf, obs_idx = [0], [], []
    for j, m in enumerate(keep):
        p = inst_pt[m]
        pos[j] = (X[p] + rng.normal(0, 0.01, 3)).astype(np.float32)
        nv, first_c = np.zeros(3), None
        for k in sorted(obs[m]):
            sl = obs[m][k]
            obs_kf.append(k)
            obs_idx.append(sl)
            for c in range(C):
                if sl[c] != -1:
                    n_obs[j] += 1
                    v = X[p] - Ow[k, c]
                    nv += v / np.linalg.norm(v)
                    if first_c is None:
                        first_c = (k, c, sl[c])
        obs_start.append(len(obs_kf))
        normal[j] = (nv / np.linalg.norm(nv)).astype(np.float32)
        k, c, idx = first_c
        dist = float(np.linalg.norm(pos[j] - Ow[k, c]))
        max_d[j] = np.float32(dist * 1.2 ** int(octv[p]))
        min_d[j] = np.float32(max_d[j] / 1.2 ** (nlevels - 1))
        off = int(n_kp[k, :c].sum())
        mdesc[j] = desc[k, c, idx - off]
    return dict(n_kf=n_kf, n_cams=C, kp_cap=kp_cap, width=720, height=540, nlevels=nlevels, cams=cams, bf=bf,
                kps=kps, desc=desc, n_kp=n_kp, uright=uright, Tcw=Tcw, Ow=Ow, n_blocks=np.full(n_kf, 4, np.int32),
                kf_mps=kf_mps, n_mps=M, bad=np.zeros(M, np.int32), n_obs=n_obs,
                obs_start=np.array(obs_start, np.int32), obs_kf=np.array(obs_kf, np.int32),
                obs_idx=np.array(obs_idx, np.int32).reshape(-1, 4),
                mps=dict(pos=pos, normal=normal, min_dist=min_d, max_dist=max_d, desc=mdesc),
                current=0, targets=np.arange(1, n_kf, dtype=np.int32))


def fuse_graph_struct(s, struct_cls, arr, out, obs_cap, log_cap):
    """omv_fuse_graph over the scene `s` (host numpy); `out` receives the in/out and output arrays (fresh copies),
    `arr(a)` returns a pointer to a kept-alive numpy array."""
    M = int(s["n_mps"])
    out.update(kf_mps=np.array(s["kf_mps"], np.int32, copy=True), bad=np.array(s["bad"], np.int32, copy=True),
               n_obs=np.array(s["n_obs"], np.int32, copy=True), replaced=np.full(max(M, 1), -7, np.int32),
               out_obs_start=np.zeros(M + 1, np.int32), out_obs_kf=np.zeros(obs_cap, np.int32),
               out_obs_idx=np.zeros((obs_cap, 4), np.int32), log=np.zeros((log_cap, 4), np.int32))
    g = struct_cls()
    g.n_kf, g.n_mps = int(s["n_kf"]), M
    g.n_blocks, g.Tcw, g.Ow = arr(s["n_blocks"]), arr(s["Tcw"]), arr(s["Ow"])
    g.uright = arr(s["uright"])
    for k in ("kf_mps", "bad", "n_obs", "replaced", "out_obs_start", "out_obs_kf", "out_obs_idx", "log"):
        setattr(g, k, arr(out[k]))
    g.obs_start, g.obs_kf, g.obs_idx = arr(s["obs_start"]), arr(s["obs_kf"]), arr(s["obs_idx"])
    g.obs_cap, g.log_cap = int(obs_cap), int(log_cap)
    return g
