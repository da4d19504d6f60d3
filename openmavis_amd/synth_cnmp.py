"""Seeded synthetic inputs for LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:395-780): a current keyframe and
its neighbours on the synth_ba trajectory, each with the rig's cameras (KannalaBrandt8 multi-camera: L, R, SL, SR;
or one Pinhole camera with a stereo baseline: mvuRight / mvDepth), keypoints from projected world points (+ N(0, 0.5
px) noise, octave U{0..3}) and distractors, and per neighbour a match list as SearchForTriangulation returns it
(vMatches12: the true correspondence for most current-keyframe keypoints whose point the neighbour sees, 10 % wrong
ones, the rest -1)."""
import numpy as np

from . import synth_ba

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])


def _kf_at(t, cams_n, Rcb, tcb):
    Rwb, twb, _ = synth_ba._pose_at(t)
    Rbw, tbw = Rwb.T, -Rwb.T @ twb
    Rcw = np.einsum("cij,jk->cik", Rcb[:cams_n], Rbw)
    tcw = np.einsum("cij,j->ci", Rcb[:cams_n], tbw) + tcb[:cams_n]
    return Rcw, tcw


def make_cnmp(seed=1, n_neigh=4, n_pts=600, n_distract=150, multi=True, wrong=0.1, bf=40.0):
    """multi: the Hilti-like 4-camera KannalaBrandt8 rig (n_cams 4, no stereo); else one Pinhole camera with
    mvuRight / mvDepth from a bf-baseline (n_cams 1: the stereo / UnprojectStereo branches)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cams, Rbc, tbc = synth_ba.rig()
    Rcb = np.transpose(Rbc, (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc)
    nc = 4 if multi else 1
    cams = cams[:4].astype(np.float32).copy()
    if not multi:
        cams[:, 4:] = 0.0
    t0 = float(rng.uniform(2, 10))
    times = [t0] + [t0 + float(rng.choice([-1, 1])) * float(rng.uniform(0.15, 1.2)) for _ in range(n_neigh)]
    poses = [_kf_at(t, nc, Rcb, tcb) for t in times]
    # world points in front of keyframe 0's cameras
    R0, t0c = poses[0]
    pts = []
    for _ in range(n_pts):
        c = int(rng.integers(0, nc))
        d = rng.normal(0, 1, 3)
        d[2] = abs(d[2]) * 1.5 + 0.6
        d /= np.linalg.norm(d)
        pts.append(R0[c].T @ (d * rng.uniform(1.5, 30.0) - t0c[c]))
    pts = np.array(pts)
    kfs = []
    for Rcw, tcw in poses:
        blocks = [[] for _ in range(4)]
        for p in range(n_pts):
            for c in range(nc):
                X = Rcw[c] @ pts[p] + tcw[c]
                if X[2] < 0.3:
                    continue
                uv = synth_ba.cam_project(cams[c].astype(np.float64), X, not multi)
                if not (5 <= uv[0] <= 715 and 5 <= uv[1] <= 535):
                    continue
                uv = uv + rng.normal(0, 0.5, 2)
                blocks[c].append((uv[0], uv[1], int(rng.integers(0, 4)), p, X[2]))
        for _ in range(n_distract):
            c = int(rng.integers(0, nc))
            blocks[c].append((float(rng.uniform(20, 700)), float(rng.uniform(20, 520)), int(rng.integers(0, 4)), -1,
                              float(rng.uniform(1, 30))))
        for c in range(4):
            rng.shuffle(blocks[c])
        rows = [r for c in range(4) for r in blocks[c]]
        n = len(rows)
        kps = np.zeros(n, KP_DTYPE)
        kps["x"], kps["y"], kps["octave"] = [r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows]
        kps["size"], kps["response"] = 31.0, 10.0
        z = np.array([r[4] for r in rows], np.float32)
        Tcw = np.zeros((4, 12), np.float32)
        Ow = np.zeros((4, 3), np.float32)
        for c in range(nc):
            Tcw[c] = np.hstack([Rcw[c], tcw[c][:, None]]).astype(np.float32).ravel()
            Ow[c] = (-Rcw[c].T @ tcw[c]).astype(np.float32)
        if multi:
            ur = np.full(n, -1, np.float32)
            depth = np.full(n, -1, np.float32)
        else:   # a stereo pair: half the keypoints carry a right coordinate and a depth
            has = rng.random(n) < 0.5
            depth = np.where(has, z + rng.normal(0, 0.02, n), -1).astype(np.float32)
            ur = np.where(has, kps["x"] - bf / np.maximum(depth, 1e-3), -1).astype(np.float32)
        kfs.append(dict(n=n, n_left=len(blocks[0]) if multi else -1, n_right=len(blocks[1]),
                        n_sideleft=len(blocks[2]), kps=kps, pt=np.array([r[3] for r in rows], np.int32),
                        Tcw=Tcw, Ow=Ow, Rwc=Tcw[0].reshape(3, 4)[:, :3].T.copy().ravel(), twc=Ow[0].copy(),
                        uright=ur, depth=depth))
    cur = kfs[0]
    jobs = []
    for k in range(1, n_neigh + 1):
        kf2 = kfs[k]
        by_pt = {}
        for i, p in enumerate(kf2["pt"]):
            if p >= 0:
                by_pt.setdefault(int(p), []).append(i)
        m12 = np.full(cur["n"], -1, np.int32)
        for i, p in enumerate(cur["pt"]):
            r = rng.random()
            if p >= 0 and int(p) in by_pt and r < 0.8:
                m12[i] = int(rng.choice(by_pt[int(p)]))
            elif r < 0.8 + wrong:
                m12[i] = int(rng.integers(0, kf2["n"]))
        jobs.append(dict(kf2=kf2, match12=m12))
    fx, fy, cx, cy = (float(v) for v in cams[0, :4])
    scale = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    sigma2 = (scale * scale).astype(np.float32)
    return dict(kf1=cur, jobs=jobs, pts=pts, cams=cams, cam_model=np.full(4, 0 if multi else 1, np.int32), n_cams=nc,
                fx=fx, fy=fy, cx=cx, cy=cy, mb=bf / fx, mbf=bf, scale=scale, sigma2=sigma2, scale_factor=1.2)


def cnmp_kf_struct(kf, d, struct_cls, view_cls, arr):
    """omv_cnmp_kf from a make_cnmp keyframe; `arr(array)` returns the pointer to use."""
    import ctypes
    s = struct_cls()
    v = view_cls()
    v.n, v.n_left, v.n_right, v.n_sideleft = int(kf["n"]), int(kf["n_left"]), int(kf["n_right"]), int(kf["n_sideleft"])
    v.kps = arr(kf["kps"])
    for i in range(8):
        v.level_sigma2[i] = float(d["sigma2"][i])
    s.kf = v
    s.kps_raw = None
    for c in range(4):
        for q in range(12):
            s.Tcw[c][q] = float(kf["Tcw"][c, q])
        for q in range(3):
            s.Ow[c][q] = float(kf["Ow"][c, q])
    for q in range(9):
        s.Rwc[q] = float(kf["Rwc"][q])
    for q in range(3):
        s.twc[q] = float(kf["twc"][q])
    s.fx, s.fy, s.cx, s.cy = d["fx"], d["fy"], d["cx"], d["cy"]
    s.invfx, s.invfy = float(np.float32(1) / np.float32(d["fx"])), float(np.float32(1) / np.float32(d["fy"]))
    s.mb, s.mbf = float(np.float32(d["mb"])), float(np.float32(d["mbf"]))
    s.uright, s.depth = arr(kf["uright"]), arr(kf["depth"])
    for i in range(8):
        s.scale_factors[i] = float(d["scale"][i])
    return s


PAIRS = [(0, 0), (0, 1), (1, 0), (1, 1), (0, 2), (2, 0), (2, 2), (1, 3), (3, 1), (3, 3)]


def make_cnmp_chain(seed=1, n_neigh=12, n_pts=700, n_distract=200, n_nodes=120, mp_frac1=0.2, mp_frac2=0.3,
                    close=(0.03, 0.08), bf=40.0):
    """A whole LocalMapping::CreateNewMapPoints input (LocalMapping.cc:439-783) for the Hilti-like 4-camera
    KannalaBrandt8 rig: the current keyframe and `n_neigh` neighbours on the synth_ba trajectory that all see one set of
    world points (so most current-keyframe keypoints are matchable in several neighbours), each keyframe with the
    reference's [L | R | SL | SR] keypoints (projection + N(0, 0.5 px), octave U{0..3}), descriptors (the point's base
    descriptor with U{0..6} bit flips), a FeatureVector (a point's observations share its base descriptor's node with
    probability 0.9), has-map-point flags (mp_frac1 / mp_frac2 of the keypoints), poses, and per neighbour the ten
    camera-pair transforms SearchForTriangulation uses.  Two neighbours sit `close` metres from the current keyframe,
    under the stereo baseline mb = bf / fx, so the baseline gate (:447-454) skips them (or not, by side 1's state)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cams, Rbc, tbc = synth_ba.rig()
    cams = cams[:4].astype(np.float32).copy()
    Rcb = np.transpose(Rbc[:4], (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc[:4])
    t0 = float(rng.uniform(2, 10))
    dts = [float(rng.choice([-1, 1])) * float(rng.uniform(0.15, 1.2)) for _ in range(n_neigh)]
    for k in (0, 5):   # the close ones: the first (side 1 still on the left camera) and one later in the order
        if k < n_neigh:
            dts[k] = float(rng.choice([-1, 1])) * float(rng.uniform(*close))
    poses = [_kf_at(t, 4, Rcb, tcb) for t in [t0] + [t0 + dt for dt in dts]]
    R0, t0c = poses[0]
    pts, base = [], []
    for _ in range(n_pts):
        c = int(rng.integers(0, 4))
        d = rng.normal(0, 1, 3)
        d[2] = abs(d[2]) * 1.5 + 0.6
        d /= np.linalg.norm(d)
        pts.append(R0[c].T @ (d * rng.uniform(2.0, 25.0) - t0c[c]))
        base.append(rng.integers(0, 256, 32, dtype=np.uint8))
    pts = np.array(pts)
    node_of_pt = np.array([int(b[:4].view(np.uint32)[0]) % n_nodes for b in base])
    scale = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    sigma2 = (scale * scale).astype(np.float32)
    kfs = []
    for k, (Rcw, tcw) in enumerate(poses):
        blocks = [[] for _ in range(4)]
        rot_off = float(rng.uniform(-20, 20))
        for p in range(n_pts):
            for c in range(4):
                X = Rcw[c] @ pts[p] + tcw[c]
                if X[2] < 0.3:
                    continue
                uv = synth_ba.cam_project(cams[c].astype(np.float64), X, False)
                if not (5 <= uv[0] <= 715 and 5 <= uv[1] <= 535):
                    continue
                uv = uv + rng.normal(0, 0.5, 2)
                dsc = base[p].copy()
                for _ in range(int(rng.integers(0, 7))):
                    bit = int(rng.integers(0, 256))
                    dsc[bit // 8] ^= np.uint8(1 << (bit % 8))
                ang = ((37.0 * p) % 360.0 + rot_off + float(rng.normal(0, 3))) % 360.0
                node = node_of_pt[p] if rng.random() < 0.9 else int(rng.integers(0, n_nodes))
                blocks[c].append((uv[0], uv[1], int(rng.integers(0, 4)), ang, dsc, node, p))
        for _ in range(n_distract):
            c = int(rng.integers(0, 4))
            blocks[c].append((float(rng.uniform(20, 700)), float(rng.uniform(20, 520)), int(rng.integers(0, 4)),
                              float(rng.uniform(0, 360)), rng.integers(0, 256, 32, dtype=np.uint8),
                              int(rng.integers(0, n_nodes)), -1))
        for c in range(4):
            rng.shuffle(blocks[c])
        rows = [r for c in range(4) for r in blocks[c]]
        n = len(rows)
        kps = np.zeros(n, KP_DTYPE)
        kps["x"], kps["y"], kps["octave"] = [r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows]
        kps["angle"] = [r[3] for r in rows]
        kps["size"], kps["response"] = 31.0, 10.0
        desc = np.stack([r[4] for r in rows]).astype(np.uint8)
        node = np.array([r[5] for r in rows])
        ids = np.unique(node).astype(np.uint32)
        order = np.lexsort((np.arange(n), node))
        node_start = np.concatenate([np.searchsorted(node[order], ids), [n]]).astype(np.int32)
        Tcw = np.zeros((4, 12), np.float32)
        Ow = np.zeros((4, 3), np.float32)
        for c in range(4):
            Tcw[c] = np.hstack([Rcw[c], tcw[c][:, None]]).astype(np.float32).ravel()
            Ow[c] = (-Rcw[c].T @ tcw[c]).astype(np.float32)
        kfs.append(dict(n=n, n_left=len(blocks[0]), n_right=len(blocks[1]), n_sideleft=len(blocks[2]), kps=kps,
                        desc=desc, has_mp=(rng.random(n) < (mp_frac1 if k == 0 else mp_frac2)).astype(np.uint8),
                        node_id=ids, node_start=node_start, node_idx=order.astype(np.int32),
                        pt=np.array([r[6] for r in rows], np.int32), Tcw=Tcw, Ow=Ow,
                        Rwc=Tcw[0].reshape(3, 4)[:, :3].T.copy().ravel(), twc=Ow[0].copy(),
                        uright=np.full(n, -1, np.float32), depth=np.full(n, -1, np.float32)))
    R1, t1 = poses[0]
    nbs = []
    for k in range(1, n_neigh + 1):
        R2, t2 = poses[k]
        T = np.zeros((10, 12), np.float32)
        for i, (c1, c2) in enumerate(PAIRS):
            Rw2, tw2 = R2[c2].T, -R2[c2].T @ t2[c2]
            T[i, :9] = (R1[c1] @ Rw2).ravel()
            T[i, 9:] = R1[c1] @ tw2 + t1[c1]
        nbs.append(dict(kf2=kfs[k], T=T, skip=0))
    fx, fy, cx, cy = (float(v) for v in cams[0, :4])
    return dict(kf1=kfs[0], nbs=nbs, pts=pts, cams=cams, cam_model=np.zeros(4, np.int32), n_cams=4, fx=fx, fy=fy,
                cx=cx, cy=cy, mb=bf / fx, mbf=bf, scale=scale, sigma2=sigma2, scale_factor=1.2)


def chain_kf_struct(kf, d, struct_cls, view_cls, arr, has_mp=None):
    """omv_cnmp_kf with the full omv_kf_view SearchForTriangulation reads (desc, has_mp, FeatureVector)."""
    s = cnmp_kf_struct(kf, d, struct_cls, view_cls, arr)
    s.kf.desc = arr(kf["desc"])
    s.kf.has_mp = arr(kf["has_mp"] if has_mp is None else has_mp)
    s.kf.n_nodes = int(len(kf["node_id"]))
    s.kf.node_id, s.kf.node_start, s.kf.node_idx = arr(kf["node_id"]), arr(kf["node_start"]), arr(kf["node_idx"])
    return s
