"""Time the batched PoseInertialOptimizationLastKeyFrame kernel (frames/s) on cuda:0."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--pts", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    from openmavis_amd import synth_pose
    from openmavis_amd.optimizer import PoseInertialOptimizer
    b = synth_pose.make_pose_batch(n_frames=min(a.frames, 32), n_pts=a.pts, seed=1, outlier_frac=0.1)
    # tile the generated frames up to the batch size (generation is slow in Python)
    reps = (a.frames + 31) // 32
    F = a.frames
    def tile(x, n):
        return np.concatenate([x] * reps)[:n]
    bb = dict(b)
    for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba", "kf_Rwb", "kf_twb", "kf_vel", "kf_bg", "kf_ba", "preint"):
        bb[k] = tile(b[k], F)
    per = np.diff(b["mono_start"])
    counts = tile(per, F)
    starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    idx = np.concatenate([np.arange(b["mono_start"][f % len(per)], b["mono_start"][f % len(per) + 1]) for f in range(F)])
    for k in ("mono_cam", "mono_kp", "mono_obs", "mono_inv_sigma2", "mono_xw", "mono_close"):
        bb[k] = b[k][idx]
    bb["mono_start"] = starts
    bb["stereo_start"] = np.zeros(F + 1, np.int32)
    bb["n_frames"] = F
    dev = "cuda:0"
    init = {k: torch.tensor(np.asarray(bb[k], np.float64), device=dev) for k in synth_pose.STATE_KEYS}
    arrays = {k: v.clone() for k, v in init.items()}
    for k in synth_pose.INPUT_KEYS:
        arrays[k] = torch.from_numpy(np.ascontiguousarray(bb[k])).to(dev)
    kpo = torch.zeros((F, int(bb["kp_cap"])), dtype=torch.uint8, device=dev)
    H = torch.zeros((F, 225), dtype=torch.float64, device=dev)
    opt = PoseInertialOptimizer(max_frames=F, max_edges=len(idx))
    for _ in range(3):
        opt.PoseInertialOptimizationLastKeyFrame(bb, arrays, kpo, H)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        for k in init:
            arrays[k].copy_(init[k])
        opt.PoseInertialOptimizationLastKeyFrame(bb, arrays, kpo, H)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(f"pose_inertial_last_kf: {F} frames x {a.pts} edges: {dt * 1e3:.3f} ms/batch, {F / dt:.0f} frames/s")


if __name__ == "__main__":
    main()
