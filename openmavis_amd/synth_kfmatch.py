"""Seeded synthetic batches for the keyframe-side projection searches (omv_matcher_search_kf):
ORBmatcher::Fuse (both overloads), SearchByProjection(KF, Sim3, ...) and SearchByProjection(Frame&, KF, ...)
(src/ORBmatcher.cc:668-893, 1458-1769, 2415-2535).

Per keyframe and camera block: random keypoints (uniform pixels, ORB-like octave mix, random angles and
descriptors) and a random camera pose.  Each job's map points: 70 % derive from a keypoint of the job's
block (its pixel + N(0, 0.6 px) unprojected through the block's Kannala-Brandt model to a depth U(2, 20) m,
descriptor with U{0..10} bit flips, mfMaxDistance chosen so PredictScale returns the keypoint's octave,
source angle = keypoint angle + 15 deg + noise), the rest random pixels / depths / octaves; 8 % fail the
distance invariance, 8 % the viewing angle; 10 % are near-copies of an earlier point of the job (claims
conflict); 10 % are rows of other jobs (mostly out of view).  Block 0 carries mvuRight for about half its
keypoints (Fuse's stereo gate).  Claim modes start with 8 % of the slots already claimed.
"""
import numpy as np

from . import synth
from ._lib import OMV_KF_SBP_FRAME

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])


def _R_of(q):
    x, y, z, w = np.asarray(q, np.float64)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def make_kf_search(mode, n_kf=3, n_cams=5, kp_cap=600, pts_per_job=300, seed=1, width=720, height=540, nlevels=8,
                   bf=40.0, model="kb8"):
    """model: "kb8", "pinhole" or one per block: the camera type of each block (omv_frame_geom::cam_model)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cams = synth.hilti_rig(n_cams)[0]
    C = n_cams
    models = [model] * C if isinstance(model, str) else list(model)
    cam_model = np.array([1 if m == "pinhole" else 0 for m in models], np.int32)
    pw = np.float64(1.2) ** (-2.0 * np.arange(nlevels))
    kps = np.zeros((n_kf, C, kp_cap), KP_DTYPE)
    n_kp = rng.integers(int(kp_cap * 0.7), kp_cap + 1, (n_kf, C)).astype(np.int32)
    kps["x"] = rng.uniform(0, width, kps.shape)
    kps["y"] = rng.uniform(0, height, kps.shape)
    kps["size"] = 7.0
    kps["angle"] = rng.uniform(0, 360, kps.shape)
    kps["response"] = 1.0
    kps["octave"] = rng.choice(nlevels, kps.shape, p=pw / pw.sum())
    desc = rng.integers(0, 256, (n_kf, C, kp_cap, 32), dtype=np.uint8)
    uright = np.full((n_kf, kp_cap), -1.0, np.float32)
    uright[:, :] = np.where(rng.random((n_kf, kp_cap)) < 0.3, kps["x"][:, 0] - rng.uniform(1, 30, (n_kf, kp_cap)),
                            -1.0)
    blocks = [0, 0] if mode == OMV_KF_SBP_FRAME else list(range(C))
    jobs, rows = [], []
    n_rows = 0
    tab = {k: [] for k in ("pos", "normal", "min_dist", "max_dist", "desc", "angle")}
    for kf in range(n_kf):
        for cam in blocks:
            T = synth.random_se3(rng)
            R, t = _R_of(T[:4]), T[4:].astype(np.float64)
            Ow = (-R.T @ t).astype(np.float32)
            n = pts_per_job
            base = n_rows
            true = rng.random(n) < 0.7
            k = rng.integers(0, n_kp[kf, cam], n)
            src = kps[kf, cam, k]
            u = np.where(true, src["x"] + rng.normal(0, 0.6, n), rng.uniform(0, width, n))
            v = np.where(true, src["y"] + rng.normal(0, 0.6, n), rng.uniform(0, height, n))
            octv = np.where(true, src["octave"], rng.integers(0, nlevels, n))
            depth = rng.uniform(2.0, 20.0, n)
            if cam_model[cam]:   # Pinhole::unprojectEig
                kc = np.asarray(cams[cam], np.float64)
                Xc = np.stack([(u - kc[2]) / kc[0], (v - kc[3]) / kc[1], np.ones(n)], -1) * depth[:, None]
            else:
                Xc = synth.kb8_unproject(cams[cam], u, v) * depth[:, None]
            Xw = (Xc - t) @ R
            d = Xw - Ow.astype(np.float64)
            dist = np.linalg.norm(d, axis=1)
            maxd = dist * np.float64(1.2) ** octv * rng.uniform(0.86, 0.97, n)
            mind = maxd / np.float64(1.2) ** (nlevels - 1)
            far = rng.random(n) < 0.08
            mind = np.where(far, dist * 2.0, mind)
            nrm = d / dist[:, None] + rng.normal(0, 0.05, (n, 3))
            nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
            nrm = np.where((rng.random(n) < 0.08)[:, None], -nrm, nrm)
            dsc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
            dsc[true] = synth.flip_bits(desc[kf, cam, k[true]], rng, 10)
            ang = np.where(true, src["angle"] + 15.0 + rng.normal(0, 3.0, n), rng.uniform(0, 360, n)) % 360.0
            if cam == 0:   # mvuRight of the source keypoints: u - bf / z (+ noise) for about half
                st = true & (rng.random(n) < 0.5)
                uright[kf, k[st]] = (u[st] - bf / Xc[st, 2] + rng.normal(0, 0.5, st.sum())).astype(np.float32)
            dup = rng.random(n) < 0.1   # near-copies of an earlier point of the job: they compete for keypoints
            for i in np.nonzero(dup)[0]:
                if i == 0:
                    continue
                j = int(rng.integers(0, i))
                Xw[i], nrm[i], maxd[i], mind[i], ang[i] = Xw[j], nrm[j], maxd[j], mind[j], ang[j]
                dsc[i] = synth.flip_bits(dsc[j:j + 1], rng, 6)[0]
            tab["pos"].append(Xw.astype(np.float32))
            tab["normal"].append(nrm.astype(np.float32))
            tab["min_dist"].append(mind.astype(np.float32))
            tab["max_dist"].append(maxd.astype(np.float32))
            tab["desc"].append(dsc)
            tab["angle"].append(ang.astype(np.float32))
            rows.append(np.arange(base, base + n))
            n_rows += n
            jobs.append(dict(kf=kf, cam=cam, Tcw=T, Ow=Ow))
    tab = {k: np.ascontiguousarray(np.concatenate(v)) for k, v in tab.items()}
    mps = {k: tab[k] for k in ("pos", "normal", "min_dist", "max_dist", "desc")}
    M = mps["pos"].shape[0]
    mp_list, mp_angle = [], []
    start = 0
    for jb, r in zip(jobs, rows):
        extra = rng.integers(0, M, max(1, len(r) // 10))   # rows of other jobs, mostly out of view
        lst = np.concatenate([r, extra])
        perm = rng.permutation(len(lst))
        lst = lst[perm]
        jb["mp_start"], jb["mp_count"] = start, len(lst)
        start += len(lst)
        mp_list.append(lst)
        mp_angle.append(tab["angle"][lst])
    kp_match = np.where(rng.random((n_kf, C * kp_cap)) < 0.08, 1_000_000, -1).astype(np.int32)
    return dict(mode=mode, n_kf=n_kf, n_cams=C, kp_cap=kp_cap, width=width, height=height, nlevels=nlevels,
                cams=cams, kps=kps, desc=desc, n_kp=n_kp, uright=uright, bf=np.float32(bf), jobs=jobs,
                mp_list=np.concatenate(mp_list).astype(np.int32), mp_angle=np.concatenate(mp_angle).astype(np.float32),
                mps=mps, kp_match=kp_match, cam_model=cam_model)


# reference parameters per mode: (th, max_dist) — Fuse th 3 / TH_LOW; Fuse(Sim3) th 4 / TH_LOW;
# SearchByProjection(KF, Sim3) th 10 / TH_LOW * 0.9; SearchByProjection(Frame&, KF) th 10 / ORBdist 100
MODE_PARAMS = {0: (3.0, 50.0), 1: (4.0, 50.0), 2: (10.0, 50.0 * np.float32(0.9)), 3: (10.0, 100.0)}
