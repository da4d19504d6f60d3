"""One rank of the camera-sharded multi-camera frame (BASELINE configs[2]), launched by torch.distributed.run.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/camshard_run.py --out result.npz [--backend gloo|nccl] [--frames 2]

Rank r extracts cameras r, r + world, ... of every frame on its GPU (cuda:LOCAL_RANK modulo the visible devices,
so 2 ranks can share one card with gloo), the slabs are all-gathered once (openmavis_amd.dist.CameraShard), and
the tracking rank (0) runs the frame's matching on the gathered batch: grid, lapping knn cam0 <-> cam1 (Lowe
0.8), SearchByProjection of a seeded local map (matching is not split across GPUs).  Rank 0 writes
the gathered keypoints / descriptors and the match outcome (tests/test_camshard_gpu.py compares them with the
single-GPU batched path and the oracle).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H, C, NF = 720, 540, 5, 1200
LAP = [[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", default="gloo", choices=("gloo", "nccl"))
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--map-seed", type=int, default=31)
    args = ap.parse_args()

    import numpy as np
    from openmavis_amd import synth
    F = args.frames
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    my_cams = list(range(rank, C, world))
    # this rank's images only, cam-major ([cam][frame]), generated before anything touches the GPU
    imgs = np.stack([synth.synth_image(synth.HILTI_SEED + 1000 * c + args.first + f, W, H)
                     for c in my_cams for f in range(F)]) if my_cams else np.zeros((0, H, W), np.uint8)

    import torch
    import torch.distributed as dist
    from openmavis_amd.dist import CameraShard
    from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher
    from openmavis_amd.orb import ORBextractor

    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo")
    try:
        ex = ORBextractor(NF, 1.2, 8, 15, 7, width=W, height=H, max_images=max(1, len(my_cams) * F))
        cap = ex.max_keypoints()
        sh = CameraShard(rank, world, C, F, cap, torch.device("cuda", dev),
                         mode="device" if args.backend == "nccl" else "host")
        if my_cams:
            kps, desc, n_kp, mono = sh.outputs()
            lap = np.array([LAP[c] for c in my_cams for _ in range(F)], np.int32)
            ex.extract_batch(torch.from_numpy(imgs).cuda(dev), lap, kps, desc, n_kp, mono)
            torch.cuda.synchronize(dev)
            assert ex.last_error() == 0
        fb = FrameBatch(torch, F, C, cap, W, H, ex.GetScaleFactors(), device=torch.device("cuda", dev))
        sh.gather(fb)
        torch.cuda.synchronize(dev)
        if rank == 0:
            kps_h = fb.kps.cpu().numpy()
            desc_h = fb.desc.cpu().numpy()
            n_h = fb.n_kp.cpu().numpy()
            kpv = kps_h.view(np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                                       ("response", "<f4"), ("octave", "<i4")])).reshape(F, C, cap)
            per = [synth.make_map_points(kpv[f], desc_h[f], n_h[f], 3000, args.map_seed + f, W, H) for f in range(F)]
            mps = MapPointBatch(**{k: torch.from_numpy(np.stack([p[k] for p in per])).cuda(dev) for k in per[0]})
            m = ORBmatcher(0.8)
            m.AssignFeaturesToGrid(fb)
            m.StereoLapping(fb, 0.8)
            fb.kp_to_mp.fill_(-1)
            m.SearchByProjection(fb, mps, 6.0, False, 50.0, grid_ready=True)
            torch.cuda.synchronize(dev)
            assert m.last_error() == 0
            np.savez(args.out, world=world, kps=kps_h, desc=desc_h, n_kp=n_h, mono=fb.mono.cpu().numpy(),
                     l2r=fb.l2r.cpu().numpy(), r2l=fb.r2l.cpu().numpy(), kp_to_mp=fb.kp_to_mp.cpu().numpy(),
                     n_matches=fb.n_matches.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
