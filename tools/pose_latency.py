"""Single-frame latency of the pose-inertial optimisations on cuda:0 (Tracking's call pattern: one frame, its pose
needed before the next frame starts): PoseInertialOptimizationLastKeyFrame / LastFrame on ONE frame of --pts matched
keypoints, per kernel path (one workgroup per frame, the grouped kernel at several part counts).  Per call: device
time by HIP events around the call on its stream, and the host wall time of call + synchronise.  JSON lines out."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("OMV_LIB"):   # e.g. the -DOMV_POSE_PROFILE variant of the library
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pts", type=int, default=1000)
    ap.add_argument("--stereo", type=float, default=0.0)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--parts", default="0,2,4,8")
    ap.add_argument("--modes", default="batch,grouped")
    a = ap.parse_args()
    import numpy as np
    import torch
    from openmavis_amd import synth_pose
    from openmavis_amd.optimizer import PoseInertialOptimizer
    dev = "cuda:0"
    for lf in (False, True):
        b = (synth_pose.make_last_frame_batch if lf else synth_pose.make_pose_batch)(
            n_frames=1, n_pts=a.pts, seed=1, outlier_frac=0.1, stereo_frac=a.stereo)
        init = {k: torch.tensor(np.asarray(b[k], np.float64), device=dev) for k in synth_pose.STATE_KEYS}
        arrays = {k: v.clone() for k, v in init.items()}
        for k in synth_pose.INPUT_KEYS + (synth_pose.PRIOR_KEYS if lf else ()):
            arrays[k] = torch.from_numpy(np.ascontiguousarray(b[k])).to(dev)
        kpo = torch.zeros((1, int(b["kp_cap"])), dtype=torch.uint8, device=dev)
        H = torch.zeros((1, 225), dtype=torch.float64, device=dev)
        opt = PoseInertialOptimizer(max_frames=1, max_edges=max(len(b["mono_cam"]), len(b["stereo_cam"]), 1))
        fn = opt.PoseInertialOptimizationLastFrame if lf else opt.PoseInertialOptimizationLastKeyFrame
        s = torch.cuda.current_stream()
        modes = ([("batch", PoseInertialOptimizer.BATCH, 0)] if "batch" in a.modes else []) + ([
            (f"grouped{p}", PoseInertialOptimizer.GROUPED, int(p)) for p in a.parts.split(",")] if "grouped" in a.modes else [])
        for name, mode, parts in modes:
            opt.set_mode(mode, parts)
            for _ in range(3):
                fn(b, arrays, kpo, H)
            torch.cuda.synchronize()
            dev_ms, wall_ms = [], []
            for _ in range(a.reps):
                for k in init:
                    arrays[k].copy_(init[k])
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record(s)
                n = fn(b, arrays, kpo, H)
                e1.record(s)
                torch.cuda.synchronize()
                wall_ms.append((time.perf_counter() - t0) * 1e3)
                dev_ms.append(e0.elapsed_time(e1))
            err = opt.last_error()
            print(json.dumps({"op": "LastFrame" if lf else "LastKeyFrame", "mode": name, "edges": int(
                len(b["mono_cam"]) + len(b["stereo_cam"])), "n_good": int(n.cpu()[0]), "err": err,
                "dev_ms_p50": round(float(np.median(dev_ms)), 4), "dev_ms_min": round(float(np.min(dev_ms)), 4),
                "wall_ms_p50": round(float(np.median(wall_ms)), 4)}), flush=True)


if __name__ == "__main__":
    main()
