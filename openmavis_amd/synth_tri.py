"""Seeded synthetic keyframe pairs for ORBmatcher::SearchForTriangulation (ORBmatcher.cc:1131-1456).

Two keyframes 0.2-0.6 m apart on the synth_ba trajectory, each with the rig's four KannalaBrandt8
cameras in the reference's block order L, R, SL, SR (synth_ba.rig() cameras 0, 1, 2, 3).  World points at
2-25 m are projected into every camera of both keyframes where visible; each projection becomes a
keypoint (projection + N(0, 0.5 px), octave U{0..3}) whose descriptor is the point's base descriptor
with U{0..6} bit flips, plus unrelated distractor keypoints.  30 % of the keypoints already carry a map
point.  DBoW2's FeatureVector (direct index at levelsup 4) is modelled by a node id per keypoint: a
point's observations share the node of its base descriptor (id = hash % n_nodes) with probability 0.9;
distractors get random nodes.  Angles: a keyframe-wide rotation offset + noise for true matches.
"""
import numpy as np

from . import synth_ba


def _se3_inv(R, t):
    return R.T, -R.T @ t


def make_tri_pair(seed=1, n_pts=500, n_distract=200, n_nodes=100, baseline=(0.2, 0.6), mp_frac=0.3,
                  cams_used=4, model="kb8"):
    """model: "kb8", "pinhole" (every camera a Pinhole with the Hilti fx fy cx cy: the configs[3] rig type) or a
    list of 4 per camera ("kb8" / "pinhole", a mixed rig); pair["cam_model"] holds OMV_CAM_* per camera."""
    models = [model] * 4 if isinstance(model, str) else list(model)
    pin = [m == "pinhole" for m in models]
    rng = np.random.Generator(np.random.PCG64(seed))
    cams, Rbc, tbc = synth_ba.rig()
    cams, Rbc, tbc = cams[:4].copy(), Rbc[:4], tbc[:4]
    Rcb = np.transpose(Rbc, (0, 2, 1))
    tcb = -np.einsum("cij,cj->ci", Rcb, tbc)
    t0 = float(rng.uniform(0, 10))
    dt = float(rng.uniform(*baseline))   # 1 m/s
    kfs = []
    for t in (t0, t0 + dt):
        Rwb, twb, _ = synth_ba._pose_at(t)
        Rbw, tbw = _se3_inv(Rwb, twb)
        Rcw = np.einsum("cij,jk->cik", Rcb, Rbw)
        tcw = np.einsum("cij,j->ci", Rcb, tbw) + tcb
        kfs.append((Rcw, tcw))
    # world points in front of a random camera of keyframe 1
    pts, base = [], []
    for _ in range(n_pts):
        c = int(rng.integers(0, cams_used))
        d = rng.normal(0, 1, 3)
        d[2] = abs(d[2]) * 1.5 + 0.6
        d /= np.linalg.norm(d)
        Xc = d * rng.uniform(2.0, 25.0)
        Rcw, tcw = kfs[0]
        pts.append(Rcw[c].T @ (Xc - tcw[c]))
        base.append(rng.integers(0, 256, 32, dtype=np.uint8))
    pts = np.array(pts)
    node_of_pt = np.array([int(b[:4].view(np.uint32)[0]) % n_nodes for b in base])
    rot_off = float(rng.uniform(-20, 20))
    out = []
    for k, (Rcw, tcw) in enumerate(kfs):
        blocks = [[] for _ in range(4)]
        for p in range(n_pts):
            for c in range(cams_used):
                X = Rcw[c] @ pts[p] + tcw[c]
                if X[2] < 0.3:
                    continue
                uv = synth_ba.cam_project(cams[c].astype(np.float64), X, pin[c])
                if not (5 <= uv[0] <= 715 and 5 <= uv[1] <= 535):
                    continue
                uv = uv + rng.normal(0, 0.5, 2)
                d = base[p].copy()
                for _ in range(int(rng.integers(0, 7))):
                    bit = int(rng.integers(0, 256))
                    d[bit // 8] ^= np.uint8(1 << (bit % 8))
                ang = (float(rng.uniform(0, 360)) if False else (37.0 * p) % 360.0) + (rot_off if k else 0.0)
                ang = (ang + float(rng.normal(0, 3))) % 360.0
                node = node_of_pt[p] if rng.random() < 0.9 else int(rng.integers(0, n_nodes))
                blocks[c].append((uv[0], uv[1], int(rng.integers(0, 4)), ang, d, node, p))
        for _ in range(n_distract):
            c = int(rng.integers(0, cams_used))
            blocks[c].append((float(rng.uniform(20, 700)), float(rng.uniform(20, 520)), int(rng.integers(0, 4)),
                              float(rng.uniform(0, 360)), rng.integers(0, 256, 32, dtype=np.uint8),
                              int(rng.integers(0, n_nodes)), -1))
        for c in range(4):   # keypoints in image order like an extractor
            rng.shuffle(blocks[c])
        rows = [r for c in range(4) for r in blocks[c]]
        n = len(rows)
        kps = np.zeros(n, np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                    ("response", "<f4"), ("octave", "<i4")]))
        kps["x"] = [r[0] for r in rows]
        kps["y"] = [r[1] for r in rows]
        kps["size"] = 31.0
        kps["angle"] = [r[3] for r in rows]
        kps["response"] = 10.0
        kps["octave"] = [r[2] for r in rows]
        desc = np.stack([r[4] for r in rows]).astype(np.uint8)
        node = np.array([r[5] for r in rows])
        # FeatureVector: nodes ascending, indices ascending within a node
        ids = np.unique(node).astype(np.uint32)
        order = np.lexsort((np.arange(n), node))
        starts = np.searchsorted(node[order], ids)
        node_start = np.concatenate([starts, [n]]).astype(np.int32)
        out.append(dict(n=n, n_left=len(blocks[0]), n_right=len(blocks[1]), n_sideleft=len(blocks[2]), kps=kps,
                        desc=desc, has_mp=(rng.random(n) < mp_frac).astype(np.uint8), node_id=ids,
                        node_start=node_start, node_idx=order.astype(np.int32),
                        pt=np.array([r[6] for r in rows], np.int32)))
    # camera-pair transforms T_{c1 w}(KF1) * T_{w c2}(KF2), as float R12 | t12
    (R1, t1), (R2, t2) = kfs
    pairs = [(0, 0), (0, 1), (1, 0), (1, 1), (0, 2), (2, 0), (2, 2), (1, 3), (3, 1), (3, 3)]
    T = np.zeros((10, 12), np.float32)
    for i, (c1, c2) in enumerate(pairs):
        Rw2, tw2 = _se3_inv(R2[c2], t2[c2])
        T[i, :9] = (R1[c1] @ Rw2).ravel()
        T[i, 9:] = R1[c1] @ tw2 + t1[c1]
    sigma2 = (np.float32(1.2) ** (2 * np.arange(8))).astype(np.float32)
    cams = cams.astype(np.float32)
    for c in range(4):
        if pin[c]:
            cams[c, 4:] = 0.0   # Pinhole: fx fy cx cy only
    return dict(kf1=out[0], kf2=out[1], T=T, cams=cams, level_sigma2=sigma2,
                cam_model=np.array([1 if p else 0 for p in pin], np.int32))


def kf_struct(kf, struct_cls, sigma2, arr):
    """omv_kf_view from a synth keyframe dict; `arr(name, array)` returns the pointer to use."""
    import ctypes
    s = struct_cls()
    s.n, s.n_left, s.n_right, s.n_sideleft = int(kf["n"]), int(kf["n_left"]), int(kf["n_right"]), int(kf["n_sideleft"])
    s.kps, s.desc, s.has_mp = arr("kps", kf["kps"]), arr("desc", kf["desc"]), arr("has_mp", kf["has_mp"])
    s.n_nodes = int(len(kf["node_id"]))
    s.node_id, s.node_start, s.node_idx = (arr("node_id", kf["node_id"]), arr("node_start", kf["node_start"]),
                                           arr("node_idx", kf["node_idx"]))
    sg = np.ascontiguousarray(np.asarray(sigma2, np.float32)[:16])
    ctypes.memmove(ctypes.addressof(s.level_sigma2), sg.ctypes.data, sg.nbytes)
    return s
