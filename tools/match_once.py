"""One stream group of the headline pipeline (bench.py's step for B frames, no other stream running), for the
PMC passes of the matcher kernels (rocprofv3 --pmc must stay short): extract 5 x 720x540 per frame, grid,
lapping knn + TriangulateMatches, mvuRight, isInFrustum, SearchByProjection — `--reps` times.
--timing: per-stage HIP-event times per launch (ms)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("OMV_LIB"):   # an instrumented variant of the library
    from openmavis_amd import _lib  # noqa: E402
    _lib.load(os.environ["OMV_LIB"])
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--timing", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    from openmavis_amd import synth
    from openmavis_amd.frame import frame_uright
    from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher, isInFrustum, make_rig
    from openmavis_amd.orb import ORBextractor
    B, C, W, H = a.frames, bench.C, bench.W, bench.H
    imgs = np.concatenate([bench._gen_frame(f) for f in range(B)])
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    ex = ORBextractor(bench.NFEAT, bench.SCALE, bench.NLEV, bench.INI_TH, bench.MIN_TH, width=W, height=H,
                      max_images=B * C)
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, B, C, cap, W, H, ex.GetScaleFactors(), device=dev)
    lap = np.tile(bench.LAP, (B, 1))
    m = ORBmatcher(bench.NNRATIO)

    def extract():
        ex.extract_batch(d_img, lap, fb.kps.view(-1, cap, 6), fb.desc.view(-1, cap, 32), fb.n_kp.view(-1),
                         fb.mono.view(-1))

    extract()
    torch.cuda.synchronize()
    from openmavis_amd._lib import KP_DTYPE
    kps_h = fb.kps.cpu().numpy().view(KP_DTYPE).reshape(B, C, cap)
    desc_h, nk = fb.desc.cpu().numpy(), fb.n_kp.cpu().numpy()
    per = [bench._gen_map((kps_h[f], desc_h[f], nk[f], 7000 + f)) for f in range(B)]
    poses = torch.from_numpy(np.stack([p[0] for p in per])).to(dev)
    world = {k: torch.from_numpy(np.stack([p[1][k] for p in per])).to(dev) for k in per[0][1]}
    mps = MapPointBatch(**{k: torch.from_numpy(np.stack([p[2][k] for p in per])).to(dev) for k in per[0][2]})
    cams_r, R_cl, t_cl = synth.hilti_rig(C)
    rig = make_rig(cams_r, R_cl, t_cl, W, H, bench.SCALE, bench.NLEV)
    Rlr = R_cl[1].T.astype(np.float32)
    tlr = (-R_cl[1].T @ t_cl[1]).astype(np.float32)
    BF = float(cams_r[0][0] * np.linalg.norm(tlr))
    sigma2 = (np.float32(bench.SCALE) ** (2 * np.arange(bench.NLEV))).astype(np.float32)
    depth = torch.rand((B, min(4, C), H, W), device=dev, dtype=torch.float32) * 25.0
    uright = torch.empty((B, min(4, C), cap), dtype=torch.float32, device=dev)

    def step():
        extract()
        fb.kp_to_mp.fill_(-1)
        m.AssignFeaturesToGrid(fb)
        m.StereoLapping(fb, 0.8)
        m.StereoTriangulate(fb, cams_r[:2], Rlr, tlr, sigma2)
        frame_uright(fb, depth, BF, out=uright)
        isInFrustum(poses, rig, world, mps, 0.5)
        m.SearchByProjection(fb, mps, bench.TH, False, 50.0, grid_ready=True)

    step()
    torch.cuda.synchronize()
    if a.timing:
        ex.enable_timing(True)
        m.enable_timing(True)
        ex.stage_ms(reset=True)
        m.stage_ms(reset=True)
    for _ in range(a.reps):
        step()
    torch.cuda.synchronize()
    assert ex.last_error() == 0 and m.last_error() == 0
    msg = f"frames {B} matches {int(fb.n_matches.sum())}"
    if a.timing:
        st, calls = ex.stage_ms(reset=True)
        st.update(m.stage_ms(reset=True))
        msg += " " + " ".join(f"{k} {v / max(a.reps, 1):.4f}" for k, v in st.items()) + " (ms per launch)"
    print(msg)


if __name__ == "__main__":
    main()
