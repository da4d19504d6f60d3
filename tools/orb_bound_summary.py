"""profiles/<tag>_orb_bound.json from tools/pmc_orb_bound.sh's gpurun_out/<dir>/bound.json (SQ PMC passes over one
32-frame extraction, 160 images per launch): per extraction kernel the waves per image and the per-wave instruction
and wait shares that bench.py turns into chip-level VALU / LDS issue fractions.
    python3 tools/orb_bound_summary.py gpurun_out/<dir> <tag>"""
import json
import os
import sys

IMAGES = 160   # tools/orb_once.py --frames 32 x 5 cameras


def main():
    src, tag = sys.argv[1], sys.argv[2]
    b = json.load(open(os.path.join(src, "bound.json")))
    out = {"tag": tag, "program": "tools/orb_once.py --frames 32 (160 images per launch), tools/pmc_orb_bound.sh",
           "images": IMAGES, "kernels": {}}
    for k in ("pyr_resize_kernel", "fast_cells_kernel", "octree_kernel", "describe_kernel"):
        if k not in b:
            continue
        r = b[k]
        d = {a: round(v, 4) for a, v in r.items()}
        d["waves_per_image"] = round(r["waves"] / IMAGES, 2)
        out["kernels"][k.replace("_kernel", "")] = d
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", f"{tag}_orb_bound.json")
    json.dump(out, open(path, "w"), indent=1)
    print(path)


if __name__ == "__main__":
    main()
