"""Floating-point contraction sensitivity of the ORB restatement ("Contraction").

The parity mode (oracle + device) rounds every float operation.  The reference is built with
-O3 -march=native (CMakeLists.txt:12-15); on an FMA machine GCC contracts a*b+c in the reference's own
translation units, and OpenCV's contraction depends on how OpenCV was built.  This study extracts the same
images three ways and reports per-field flip rates against the parity mode:

  ref_tu   mode 1 of the parity library: only the reference's own steering products (ORBextractor.cc:56-57)
           fused the way GCC's convert_mult_to_fma fuses them
  all      oracle/liboracle_fma.so: the whole restatement built -O3 -march=x86-64-v3 -ffp-contract=fast
           (GCC's default for GNU C++), i.e. OpenCV's restated fastAtan2 / resize / blur fused as well

Test infrastructure: CPU only, writes profiles/fma_study.json.   python tools/fma_study.py [--frames 10]
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from openmavis_amd import synth  # noqa: E402

FIELDS = ("x", "y", "size", "angle", "response", "octave")


def workloads(n_frames):
    lap = [(0, 720), (0, 720), (0, 0), (0, 0), (0, 0)]
    for f in range(n_frames):
        imgs = synth.hilti_frame(10_000 + f)
        for c in range(imgs.shape[0]):
            yield "hilti_5x720x540_1200", imgs[c], dict(nfeatures=1200, ini_th=15, min_th=7, lapping=lap[c])
    for c in range(8):
        yield "pinhole_8x1920x1080_2000", synth.rig_frame(0, 8, 1920, 1080, synth.P1080_SEED)[c], \
            dict(nfeatures=2000, ini_th=20, min_th=7, lapping=(0, 0))
    for name in ("orb_hilti_720x540", "orb_euroc_752x480", "orb_side_320x240"):
        g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
        img = synth.synth_image(int(g["seed"]), int(g["w"]), int(g["h"]))
        yield "golden_" + name, img, dict(nfeatures=int(g["nfeatures"]), ini_th=int(g["ini"]), min_th=int(g["mn"]),
                                          lapping=tuple(int(v) for v in g["lapping"]))


def extract(img, kw):
    mono, k, d = oracle.orb_extract(img, **kw)
    return mono, k, d


def compare(base, other, acc):
    (m0, k0, d0), (m1, k1, d1) = base, other
    acc["images"] += 1
    acc["keypoints"] += len(k0)
    if len(k0) != len(k1) or m0 != m1:
        acc["count_or_order_changed"] += 1
        return
    for f in FIELDS:
        acc["flips"][f] += int(np.count_nonzero(k0[f].view(np.uint32) != k1[f].view(np.uint32)))
    ulp = np.abs(k0["angle"].view(np.int32).astype(np.int64) - k1["angle"].view(np.int32).astype(np.int64))
    acc["angle_max_ulp"] = max(acc.get("angle_max_ulp", 0), int(ulp.max()) if len(ulp) else 0)
    acc["flips"]["descriptor"] += int(np.count_nonzero(np.any(d0 != d1, axis=1)))
    acc["flips"]["descriptor_bits"] += int(np.unpackbits(d0 ^ d1).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so", "liboracle_fma.so"])
    items = list(workloads(a.frames))
    base_lib = os.path.join(ROOT, "oracle", "liboracle.so")
    fma_lib = os.path.join(ROOT, "oracle", "liboracle_fma.so")
    runs = {}
    oracle.use_library(base_lib)
    oracle.set_contract(0)
    runs["parity"] = [extract(img, kw) for _, img, kw in items]
    oracle.set_contract(1)
    runs["ref_tu"] = [extract(img, kw) for _, img, kw in items]
    oracle.set_contract(0)
    oracle.use_library(fma_lib)
    oracle.set_contract(0)
    runs["all"] = [extract(img, kw) for _, img, kw in items]
    oracle.use_library(base_lib)
    out = {"note": "flip counts vs the parity mode (no contraction); a keypoint flips a field if its raw bits differ",
           "modes": {}}
    for mode in ("ref_tu", "all"):
        per = {}
        for (wl, _, _), b, o in zip(items, runs["parity"], runs[mode]):
            acc = per.setdefault(wl, {"images": 0, "keypoints": 0, "count_or_order_changed": 0,
                                      "flips": {f: 0 for f in FIELDS + ("descriptor", "descriptor_bits")}})
            compare(b, o, acc)
        for acc in per.values():
            acc["rates"] = {f: round(v / max(acc["keypoints"], 1), 6) for f, v in acc["flips"].items()
                            if f != "descriptor_bits"}
        out["modes"][mode] = per
    path = os.path.join(ROOT, "profiles", "fma_study.json")
    json.dump(out, open(path, "w"), indent=1)
    for mode, per in out["modes"].items():
        for wl, acc in per.items():
            fl = {k: v for k, v in acc["flips"].items() if v}
            print(f"{mode:7s} {wl:28s} images {acc['images']:3d} keypoints {acc['keypoints']:6d} "
                  f"count/order changed {acc['count_or_order_changed']} flips {fl} "
                  f"angle max {acc.get('angle_max_ulp', 0)} ulp")


if __name__ == "__main__":
    main()
