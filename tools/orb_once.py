"""One batched ORB extraction of B Hilti-like frames on cuda:0 (one stream), for profiling runs (rocprofv3 --pmc)
that must stay short.  --timing: per-stage HIP-event times of the extraction launches (ms per launch).
--p1080: the configs[3] 8 x 1920x1080 rig instead."""
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
    ap.add_argument("--timing", action="store_true")
    ap.add_argument("--p1080", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    from openmavis_amd import synth
    from openmavis_amd.orb import ORBextractor
    from openmavis_amd.matcher import FrameBatch
    if a.p1080:
        W, H, C, NF, INI = 1920, 1080, 8, 2000, 20
        lap = np.zeros((C, 2), np.int32)
        imgs = np.concatenate([synth.rig_frame(f, C, W, H, synth.P1080_SEED) for f in range(a.frames)])
    else:
        W, H, C, NF, INI = 720, 540, 5, 1200, 15
        lap = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)
        imgs = np.concatenate([synth.hilti_frame(f) for f in range(a.frames)])
    ex = ORBextractor(NF, 1.2, 8, INI, 7, width=W, height=H, max_images=a.frames * C)
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, a.frames, C, cap, W, H, ex.GetScaleFactors(), device="cuda:0")
    d = torch.from_numpy(imgs).cuda()

    def run():
        ex.extract_batch(d, np.tile(lap, (a.frames, 1)), fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32),
                         fb.n_kp.view(-1), fb.mono.view(-1))

    run()
    torch.cuda.synchronize()
    if a.timing:
        ex.enable_timing(True)
        ex.stage_ms(reset=True)
    for _ in range(a.reps):
        run()
    torch.cuda.synchronize()
    assert ex.last_error() == 0
    msg = f"images {a.frames * C} keypoints {int(fb.n_kp.sum())}"
    if a.timing:
        st, calls = ex.stage_ms(reset=True)
        msg += " " + " ".join(f"{k} {v / max(calls, 1):.4f}" for k, v in st.items()) + " (ms per launch)"
    print(msg)


if __name__ == "__main__":
    main()
