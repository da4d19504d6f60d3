"""Per-kernel HBM bytes of one tools/quick_lba.sh PMC pair (FETCH_SIZE doubled for gfx950, KB x 1024), per launch and
per LM trial: python tools/pmc_lba_summary.py gpurun_out/prof_<tag> [trials_per_run]
Writes <src>/pmc_lba_trial.json (bench.py reads it once copied to profiles/<tag>_pmc_lba_trial.json)."""
import os
import csv
import json
import sys
from collections import defaultdict

src = sys.argv[1]
out = defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    d = defaultdict(list)
    for r in csv.DictReader(open(f"{src}/pmc_lba_{c}/run_counter_collection.csv")):
        d[r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")].append(float(r["Counter_Value"]))
    for k, v in d.items():
        out[k][c] = (len(v), sum(v) * 1024 * (2 if c == "FETCH_SIZE" else 1))
trials = None
for line in open(f"{src}/lba_FETCH_SIZE.txt"):
    pass
rows, tot = [], 0.0
for k, v in sorted(out.items()):
    n = v.get("FETCH_SIZE", (0, 0))[0]
    b = v.get("FETCH_SIZE", (0, 0))[1] + v.get("WRITE_SIZE", (0, 0))[1]
    rows.append((k, n, b))
n_trials = int(sys.argv[2]) if len(sys.argv) > 2 else max(n for k, n, b in rows if k.startswith("ldlt"))
for k, n, b in rows:
    print(f"{k:40s} launches {n:4d}  {b / max(n, 1) / 1e6:8.3f} MB/launch  {b / n_trials / 1e6:8.3f} MB/trial")
    tot += b
print(f"total {tot / n_trials / 1e6:.2f} MB per trial over {n_trials} trials")
tag = os.path.basename(os.path.normpath(src)).replace("prof_", "")
json.dump({"kernel": "lba_trial", "tag": tag, "program": "tools/quick_lba.sh (tools/lba_time.py under --pmc)",
           "hbm_bytes_per_trial": int(tot / n_trials), "trials": n_trials,
           "correction": "2*FETCH_SIZE + WRITE_SIZE, KB*1024, summed over every kernel of the run, per LM trial",
           "per_kernel_mb_per_trial": {k: round(b / n_trials / 1e6, 3) for k, n, b in rows}},
          open(f"{src}/pmc_lba_trial.json", "w"), indent=1)
