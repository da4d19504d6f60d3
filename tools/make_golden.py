"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference cannot be built or run here (OpenCV/Eigen/Pangolin absent) and its tests
hold no fixtures for this path, so these vectors pin the oracle's restated semantics (parity against
real OpenCV stays unpinned).  Images are regenerated from their seed at test time and checked by
SHA-256; keypoints, descriptors and matcher outputs are stored.

    python tools/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from openmavis_amd import synth  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

ORB_CASES = [
    # name, seed, w, h, nfeatures, iniTh, minTh, lapping
    ("orb_hilti_720x540", 20221000, 720, 540, 1200, 15, 7, (0, 720)),
    ("orb_euroc_752x480", 101, 752, 480, 1000, 20, 7, (0, 1000)),
    ("orb_side_320x240", 7, 320, 240, 300, 20, 7, (0, 0)),
]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, seed, w, h, nf, ini, mn, lap in ORB_CASES:
        img = synth.synth_image(seed, w, h)
        mono, kps, desc = oracle.orb_extract(img, nf, 1.2, 8, ini, mn, lap)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), seed=seed, w=w, h=h, nfeatures=nf, ini=ini, mn=mn,
                            lapping=np.array(lap), image_sha256=sha(img), mono=mono,
                            kps=kps.view(np.uint32).reshape(-1, 6), desc=desc)
        print(name, len(kps), mono)
    # matcher: one Hilti-like frame, 1500 map points, lapping knn pairs + SearchByProjection
    lapc = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)
    imgs = synth.hilti_frame(0)
    n_out, mono, kps, desc = oracle.orb_extract_frame(imgs, 1200, lapc)
    cap = kps.shape[1]
    mp = synth.make_map_points(kps, desc, n_out, 1500, 3, 720, 540)
    i2, d2 = oracle.bf_knn2(desc[0, mono[0]:n_out[0]], desc[1, mono[1]:n_out[1]])
    l2r = np.full(cap, -1, np.int32)
    r2l = np.full(cap, -1, np.int32)
    for qi in range(len(i2)):
        if i2[qi, 1] >= 0 and float(d2[qi, 0]) < float(d2[qi, 1]) * 0.8:
            l2r[mono[0] + qi] = mono[1] + i2[qi, 0]
            r2l[mono[1] + i2[qi, 0]] = mono[0] + qi
    tab = oracle.orb_tables(1200)
    g = oracle.frame_geom(5, 720, 540, tab["scale"])
    k2m = np.full(5 * cap, -1, np.int32)
    n = oracle.search_by_projection(g, kps, desc, n_out, mp, 6.0, False, 50.0, 0.8, l2r, r2l, None, k2m)
    np.savez_compressed(os.path.join(OUT, "match_hilti_frame0.npz"), kps=kps.view(np.uint32).reshape(5, cap, 6),
                        desc=desc, n_kp=n_out, mono=mono, knn_idx=i2, knn_dist=d2, l2r=l2r, r2l=r2l,
                        kp_to_mp=k2m, n_matches=n, **{"mp_" + k: v for k, v in mp.items()})
    print("match", n)


if __name__ == "__main__":
    main()
