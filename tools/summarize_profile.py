"""Summarise a tools/profile_gpu.sh run into profiles/<tag>_*.

- <tag>_kernel_stats.md : rocprofv3 --kernel-trace --stats table (calls, total/avg ns, share)
- pmc_<kernel>.json     : HBM traffic per launch from the separate FETCH_SIZE / WRITE_SIZE passes,
                          corrected per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
                          WRITE_SIZE are KB; on gfx950 FETCH_SIZE counts 64 B per 128-B request, so
                          the read side is doubled (calibrated for wide coalesced streams only; our
                          byte-granular kernels are uncalibrated, so read the value as an estimate).
    python tools/summarize_profile.py gpurun_out/prof_r01 r01
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"pyr_resize": "pyr_resize", "fast_cells": "fast_cells", "octree": "octree", "describe": "describe",
         "grid_kernel": "grid", "knn2": "stereo_knn", "stereo_pairs": "stereo_pairs", "cand_kernel": "proj_candidates",
         "resolve": "proj_resolve"}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return name


def main(src, tag, images_per_launch=None, command=None):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats ({tag})", "",
             "Command: `" + (command or "rocprofv3 --kernel-trace --stats -T -- python3 bench.py --no-cpu-baseline "
                             "--steps 5 --warmup 1 --lba-steps 3 --pose-frames 256 --tri-pairs 64") + "` (MI355X, one GPU).", "",
             "| kernel | calls | total ms | avg us | min us | max us | share |", "|---|---|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        lines.append(f"| {r['Name'][:60]} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                     f"{float(r['MaxNs']) / 1e3:.1f} | {100 * float(r['TotalDurationNs']) / tot:.1f}% |")
    pmc = defaultdict(lambda: defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            pmc[short(r["Kernel_Name"])][c].append(float(r["Counter_Value"]))
    lines += ["", "## HBM traffic per launch (separate --pmc passes; KB x 1024; FETCH doubled for gfx950)", "",
              "| kernel | launches | FETCH_SIZE KB/launch | WRITE_SIZE KB/launch | corrected bytes/launch |",
              "|---|---|---|---|---|"]
    for k, d in sorted(pmc.items()):
        f = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
        w = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
        b = (2 * f + w) * 1024
        lines.append(f"| {k} | {len(d['FETCH_SIZE'])} | {f:.1f} | {w:.1f} | {b:.0f} |")
        if k in SHORT.values():
            rec = {"kernel": k, "tag": tag, "fetch_kb_per_launch": f, "write_kb_per_launch": w,
                   "hbm_bytes_per_launch": round(b), "correction": "2*FETCH_SIZE + WRITE_SIZE, KB*1024"}
            if images_per_launch:   # extraction kernels: one launch covers images_per_launch images
                rec["images_per_launch"] = images_per_launch
                rec["hbm_bytes_per_image"] = round(b / images_per_launch)
            json.dump(rec, open(os.path.join(prof, f"pmc_{k}.json"), "w"), indent=1)
    open(os.path.join(prof, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01",
         int(sys.argv[3]) if len(sys.argv) > 3 else None, sys.argv[4] if len(sys.argv) > 4 else None)
