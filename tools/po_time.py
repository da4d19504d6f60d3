"""Optimizer::PoseOptimization on one frame (bench.py's pose_optimization_b1 shape: 4-camera rig, ~400 edges), timed
with HIP events on the launch stream.  OMV_LIB=<variant .so> loads an instrumented build (e.g. -DOMV_PO_PROFILE)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("OMV_LIB"):
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])


def main():
    import numpy as np
    import torch
    from openmavis_amd import synth_pose
    from openmavis_amd.optimizer import PoseInertialOptimizer
    dev = torch.device("cuda", 0)
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    pb0 = synth_pose.make_pose_only_batch(n_frames=16, n_pts=400, seed=9, n_cams=4)
    pb = synth_pose.tile_batch(pb0, F)
    sel = [f % 16 for f in range(F)]
    q0 = torch.tensor(np.asarray(pb0["pose_q"])[sel], dtype=torch.float64, device=dev)
    t0 = torch.tensor(np.asarray(pb0["pose_t"])[sel], dtype=torch.float64, device=dev)
    pb["rig_q"], pb["rig_t"] = pb0["rig_q"], pb0["rig_t"]
    q, t = q0.clone(), t0.clone()
    arr = {k: torch.from_numpy(np.ascontiguousarray(pb[k])).to(dev) for k in PoseInertialOptimizer.EDGE_KEYS}
    kpo = torch.zeros((F, int(pb["kp_cap"])), dtype=torch.uint8, device=dev)
    po = PoseInertialOptimizer(max_frames=F, max_edges=max(len(pb["mono_cam"]), 1))
    ms = []
    for r in range(reps):
        q.copy_(q0)
        t.copy_(t0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        po.PoseOptimization(pb, arr, q, t, kpo)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(f"PoseOptimization frames {F}: median {np.median(ms[1:]):.4f} ms (host call included), first {ms[0]:.3f}")


if __name__ == "__main__":
    main()
