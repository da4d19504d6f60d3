"""One batched ORB extraction (+ grid / knn / SearchByProjection) of B Hilti-like frames on cuda:0, for
profiling runs (rocprofv3 --pmc) that must stay short."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("OMV_LIB"):   # e.g. a -DOMV_OCT_PROFILE build of the library
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch
    from openmavis_amd import synth
    from openmavis_amd.orb import ORBextractor
    from openmavis_amd.matcher import FrameBatch
    W, H, C = 720, 540, 5
    lap = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)
    imgs = np.concatenate([synth.hilti_frame(f) for f in range(a.frames)])
    ex = ORBextractor(1200, 1.2, 8, 15, 7, width=W, height=H, max_images=a.frames * C)
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, a.frames, C, cap, W, H, ex.GetScaleFactors(), device="cuda:0")
    d = torch.from_numpy(imgs).cuda()
    for _ in range(a.reps):
        ex.extract_batch(d, np.tile(lap, (a.frames, 1)), fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32),
                         fb.n_kp.view(-1), fb.mono.view(-1))
    torch.cuda.synchronize()
    print("keypoints", int(fb.n_kp.sum()))


if __name__ == "__main__":
    main()
