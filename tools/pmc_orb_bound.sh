#!/bin/bash
# The bound of the extraction kernels: two 8-counter SQ passes over one batched extraction (tools/orb_once.py,
# 32 frames = 160 images per launch), per kernel VALU / LDS issue and wait shares per wave-cycle, plus the isolated
# per-stage HIP-event times.  bash tools/pmc_orb_bound.sh <tag>   (on the box, from the repo root)
set -euo pipefail
TAG=${1:-bound}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/orb_once.py --frames 128 --reps 3 --timing > $OUT/timing.txt 2>&1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d $OUT/p1 -o run --output-format csv -- python3 $R/tools/orb_once.py --frames 32 --reps 1 > $OUT/p1.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc $P2 -d $OUT/p2 -o run --output-format csv -- python3 $R/tools/orb_once.py --frames 32 --reps 1 > $OUT/p2.txt 2>&1
python3 - $OUT <<'PY'
import csv, sys, collections, re, os, glob, json
out = {}
for p in ("p1", "p2"):
    f = glob.glob(os.path.join(sys.argv[1], p, "**", "*counter_collection.csv"), recursive=True)
    for r in csv.DictReader(open(f[0])):
        m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
        if not m:
            continue
        out.setdefault(m.group(1), collections.defaultdict(float))[r["Counter_Name"] + ("" if p == "p1" else "_2")] += float(r["Counter_Value"])
res = {}
for k, v in out.items():
    w = max(v["SQ_WAVES"], 1); wc = max(v["SQ_WAVE_CYCLES"], 1); wc2 = max(v.get("SQ_WAVE_CYCLES_2", 0), 1)
    res[k] = dict(waves=v["SQ_WAVES"], cycles_per_wave=4 * wc / w, active_any=v["SQ_ACTIVE_INST_ANY"] / wc,
                  wait_any=v["SQ_WAIT_ANY"] / wc, wait_inst_any=v["SQ_WAIT_INST_ANY"] / wc,
                  valu_per_wave=v["SQ_INSTS_VALU"] / w, lds_per_wave=v["SQ_INSTS_LDS"] / w,
                  active_valu=v.get("SQ_ACTIVE_INST_VALU_2", 0) / wc2, active_lds=v.get("SQ_ACTIVE_INST_LDS_2", 0) / wc2,
                  wait_inst_lds=v.get("SQ_WAIT_INST_LDS_2", 0) / wc2, salu_per_wave=v.get("SQ_INSTS_SALU_2", 0) / w,
                  lds_bank_conflict_per_wave=v.get("SQ_LDS_BANK_CONFLICT_2", 0) / w,
                  vmem_rd_per_wave=v.get("SQ_INSTS_VMEM_RD_2", 0) / w)
json.dump(res, open(os.path.join(sys.argv[1], "bound.json"), "w"), indent=1)
for k, r in sorted(res.items(), key=lambda kv: -kv[1]["cycles_per_wave"] * kv[1]["waves"]):
    print(k, {a: round(b, 3) for a, b in r.items()})
PY
