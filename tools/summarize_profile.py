"""Summarise a tools/profile_gpu.sh run into profiles/<tag>_*.

- <tag>_kernel_stats.md : rocprofv3 --kernel-trace --stats table (calls, total/avg ns, share)
- <tag>_pmc_<kernel>.json : HBM traffic per launch from the separate FETCH_SIZE / WRITE_SIZE passes,
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
# substring -> short name, first match wins: the more specific names come before the ones they contain
SHORT = {"bow_build_kernel": "bow_build", "bow_resolve": "bow_resolve", "build_all_kernel": "lba_build", "build_big_kernel": "lba_build_big",
         "cur_copy_kernel": "lba_cur_copy", "trial_scalars_kernel": "lba_trial_scalars", "pyr_resize": "pyr_resize", "fast_cells": "fast_cells", "octree": "octree", "describe": "describe",
         "grid_kernel": "grid", "knn2": "stereo_knn", "stereo_pairs": "stereo_pairs",
         "stereo_tri_kernel": "stereo_tri", "cand_stage_kernel": "proj_candidates", "cand_kernel": "proj_candidates", "resolve": "proj_resolve",
         "frustum_kernel": "frustum", "uright_kernel": "uright", "err_kernel": "lba_err", "build_land_kernel": "lba_build_land", "build_kernel": "lba_build_split",
         "schur_kernel": "lba_schur", "assemble_kernel": "lba_assemble", "ldlt_kernel": "lba_ldlt",
         "update_kernel": "lba_update", "finish_trial_kernel": "lba_finish_trial", "accept_copy_kernel": "lba_accept",
         "epilogue_kernel": "lba_epilogue", "ctl_init_kernel": "lba_ctl_init"}
# PMC programs (tools/profile_gpu.sh): units one launch covers
PMC_SOURCES = {"orb": ("images", 160), "match": ("frames", 32), "lba": ("launches", 1)}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return name


def main(src, tag, command=None):
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
    # per (kernel, grid) from the dispatch trace: launches of one kernel at different batch sizes differ
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        by = defaultdict(list)
        for r in csv.DictReader(open(tr)):
            by[(short(r["Kernel_Name"]), "x".join(r.get(f"Grid_Size_{a}", "?") for a in "XYZ"))].append(
                (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
        lines += ["", "## Per kernel and grid size (dispatch trace)", "",
                  "| kernel | grid (work-items) | calls | avg us | min us |", "|---|---|---|---|---|"]
        grid_rows = []
        for (k, g), v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            if sum(v) < 50:   # skip sub-50-us totals
                continue
            lines.append(f"| {k} | {g} | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} |")
            grid_rows.append({"kernel": k, "grid": g, "calls": len(v), "avg_us": round(sum(v) / len(v), 2),
                              "min_us": round(min(v), 2), "total_us": round(sum(v), 1)})
        # read by bench.py (roofline.rocprof): the dominant kernel's dispatch-trace average beside its HIP-event time
        json.dump({"tag": tag, "command": command, "rows": grid_rows},
                  open(os.path.join(prof, f"{tag}_kernel_grid.json"), "w"), indent=1)
    pmc = defaultdict(lambda: defaultdict(list))
    for srcname in PMC_SOURCES:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            p = os.path.join(src, f"pmc_{srcname}_{c}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            for r in csv.DictReader(open(p)):
                pmc[(srcname, short(r["Kernel_Name"]))][c].append(float(r["Counter_Value"]))
    lines += ["", "## HBM traffic per launch (separate --pmc passes; KB x 1024; FETCH doubled for gfx950)", "",
              "| program | kernel | launches | FETCH_SIZE KB/launch | WRITE_SIZE KB/launch | corrected bytes/launch | per unit (all launches of a pass) |",
              "|---|---|---|---|---|---|---|"]
    # passes of a program = launches of its once-per-pass kernel; a kernel launched several times per pass (pyr_resize:
    # one launch per pyramid level, 7 per extraction) has its per-unit bytes summed over all its launches of a pass
    per_pass = {"orb": "describe", "match": "proj_resolve", "lba": None}
    passes = {src: len(pmc[(src, k)]["FETCH_SIZE"]) for src, k in per_pass.items() if k and (src, k) in pmc}
    for (srcname, k), d in sorted(pmc.items()):
        f = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
        w = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
        b = (2 * f + w) * 1024
        unit, n = PMC_SOURCES[srcname]
        lpp = len(d["FETCH_SIZE"]) / passes[srcname] if passes.get(srcname) else 1.0
        lines.append(f"| {srcname} | {k} | {len(d['FETCH_SIZE'])} | {f:.1f} | {w:.1f} | {b:.0f} | "
                     f"{b * lpp / n:.0f} B per {unit[:-1]} ({lpp:g} launches per pass) |")
        if k in SHORT.values():
            rec = {"kernel": k, "tag": tag, "program": srcname, "fetch_kb_per_launch": f, "write_kb_per_launch": w,
                   "hbm_bytes_per_launch": round(b), "correction": "2*FETCH_SIZE + WRITE_SIZE, KB*1024",
                   f"{unit}_per_launch": n, "launches_per_pass": lpp,
                   f"hbm_bytes_per_{unit[:-1]}": round(b * lpp / n),
                   "per_unit_note": f"all launches of one pass (one batched call over {n} {unit}) summed, / {n}"}
            out = os.path.join(prof, f"{tag}_pmc_{k}.json")
            if srcname == "match" and os.path.exists(out) and json.load(open(out)).get("program") == "orb":
                continue   # extraction kernels keep the extraction-only program's numbers
            json.dump(rec, open(out, "w"), indent=1)
    # LocalInertialBA: every kernel of the lba program (tools/lba_time.py), per LM trial
    lba = [(k, d) for (s, k), d in pmc.items() if s == "lba" and k.startswith("lba_")]
    trials = 0
    tf = os.path.join(src, "lba_FETCH_SIZE.txt")
    if os.path.exists(tf):
        for line in open(tf):
            if line.startswith("{"):
                trials += int(json.loads(line).get("trials", 0))
    if lba and trials:
        tot = sum(2 * sum(d["FETCH_SIZE"]) + sum(d["WRITE_SIZE"]) for _, d in lba) * 1024
        rec = {"kernel": "lba_trial", "tag": tag, "program": "lba", "trials": trials, "hbm_bytes_per_trial": round(tot / trials),
               "kernels": sorted(k for k, _ in lba), "correction": "2*FETCH_SIZE + WRITE_SIZE, KB*1024, summed over the "
               "LocalInertialBA kernels of tools/lba_time.py (set-up uploads excluded), per LM trial"}
        json.dump(rec, open(os.path.join(prof, f"{tag}_pmc_lba_trial.json"), "w"), indent=1)
        lines += ["", f"LocalInertialBA per LM trial: {rec['hbm_bytes_per_trial']} B of HBM traffic ({trials} trials)"]
    open(os.path.join(prof, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01", sys.argv[3] if len(sys.argv) > 3 else None)
