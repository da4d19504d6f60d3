#!/bin/bash
# Whole-step VALU issue of the headline chain (one --pmc pass): tools/match_once.py runs the bench's stream-group step
# (extract -> grid -> knn -> TriangulateMatches -> mvuRight -> isInFrustum -> SearchByProjection) on 32 frames,
# --reps 1 after its warm-up step = 2 passes = 64 frames.  Prints and writes profiles-ready JSON:
#   VALU wave-instructions per frame (SQ_INSTS_VALU summed over every kernel of the step), and the share of the
#   chip's VALU issue capacity that rate takes at a given frames/s (256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64
#   VALU instruction, MI355X_MICROARCH.md "Wave scheduling").
# Usage (on the box, repo root): bash tools/pmc_step_valu.sh <tag> <frames_per_s>
set -euo pipefail
TAG=${1:-valu}
FPS=${2:-35000}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $CTR -d $OUT/step -o run --output-format csv -- \
    python3 $R/tools/match_once.py --frames 32 --reps 1 > $OUT/step.txt 2> $OUT/step.err
python3 - $OUT $FPS $TAG <<'PY'
import csv, sys, collections, re, os, json
out, fps, tag = sys.argv[1], float(sys.argv[2]), sys.argv[3]
frames = 64
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(os.path.join(out, "step", "run_counter_collection.csv"))):
    m = re.search(r"::(\w+_kernel)", r["Kernel_Name"])
    d[m.group(1) if m else "other"][r["Counter_Name"]] += float(r["Counter_Value"])
tot = collections.defaultdict(float)
for v in d.values():
    for k, x in v.items():
        tot[k] += x
cap = 256 * 4 * 2.4e9 / 2
per_frame = tot["SQ_INSTS_VALU"] / frames
res = {"tag": tag, "program": "tools/match_once.py --frames 32 --reps 1 (2 passes, 64 frames)",
       "counters": sorted(tot), "valu_wave_instr_per_frame": round(per_frame),
       "salu_per_frame": round(tot["SQ_INSTS_SALU"] / frames), "lds_per_frame": round(tot["SQ_INSTS_LDS"] / frames),
       "vmem_per_frame": round(tot["SQ_INSTS_VMEM"] / frames), "frames_per_s": fps,
       "chip_valu_issue_per_s": cap, "valu_issue_share_at_fps": round(per_frame * fps / cap, 4),
       "per_kernel_valu_per_frame": {k: round(v["SQ_INSTS_VALU"] / frames) for k, v in
                                     sorted(d.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"])}}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, f"valu_{tag}.json"), "w"), indent=1)
PY
