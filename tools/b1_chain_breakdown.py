"""Per-frame kernel breakdown of bench.py's B=1 latency leg from a rocprofv3 --kernel-trace database: the frames
after the 5th PoseInertialOptimizationLastFrame launch (warm), each kernel's device time per frame and launches per
frame, the sum and the wall span per frame.  Usage: python tools/b1_chain_breakdown.py gpurun_out/prof_lat"""
import collections
import glob
import re
import sqlite3
import sys


def main():
    db = glob.glob(sys.argv[1].rstrip("/") + "/*.db")[0]
    rows = list(sqlite3.connect(db).execute("select name, start, end, duration from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if "pose_lat" in r[0]]
    sub = rows[marks[5] + 1:marks[-1] + 1]
    nf = sum(1 for r in sub if "pose_lat" in r[0])
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in sub:
        n = re.sub(r"\(anonymous namespace\)::", "", r[0]).replace("void ", "").split("(")[0]
        agg[n][0] += 1
        agg[n][1] += r[3]
    print(f"| kernel | us / frame | launches / frame |\n|---|---|---|")
    tot = 0.0
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"| {k} | {v[1] / nf / 1e3:.1f} | {v[0] / nf:.2f} |")
        tot += v[1] / nf / 1e3
    print(f"\n{nf} frames; kernel time {tot:.1f} us / frame; wall span {(sub[-1][2] - sub[0][1]) / nf / 1e3:.1f} us / frame")


if __name__ == "__main__":
    main()
