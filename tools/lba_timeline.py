"""Per-kernel timeline of the last LocalInertialBA optimize() in a rocprofv3 kernel trace:
python tools/lba_timeline.py <run_kernel_trace.csv>"""
import csv
import sys

tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last optimize() starts at its initial error launch: the first err_kernel after the previous optimize()'s
# epilogue (the control block reset rides on that launch; older traces have a separate ctl_init launch)
epi = [i for i, r in enumerate(tr) if "epilogue_kernel" in r["Kernel_Name"]]
idx = [i for i, r in enumerate(tr) if "ctl_init" in r["Kernel_Name"]]
if idx:
    s = idx[-1]
else:
    s0 = epi[-2] + 1 if len(epi) >= 2 else 0
    s = next(i for i in range(s0, len(tr)) if "err_kernel" in tr[i]["Kernel_Name"]) + 1
t0 = int(tr[s]["Start_Timestamp"])
prev = None
tot = {}
for r in tr[s - 1:]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    gap = (st - prev) / 1e3 if prev else 0.0
    print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:7.1f} gap {gap:6.1f}  {name[:60]}")
    tot[name] = tot.get(name, 0.0) + (en - st) / 1e3
    prev = en
print("span us", (prev - t0) / 1e3)
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.1f}  {k}")
