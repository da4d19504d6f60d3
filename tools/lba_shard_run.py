"""One rank of a landmark-sharded LocalInertialBA, launched by torch.distributed.run.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/lba_shard_run.py --out result.npz [--backend gloo] [--n-kf 20 --n-opt 10 --n-pts 3000]

Every rank builds the same seeded window, keeps its share of the landmarks on its GPU
(cuda:LOCAL_RANK modulo the visible devices, so 2 ranks can share one card with gloo) and runs the
LM; the partial Schur systems and chi2 sums are all-reduced once per trial.  Rank 0 merges the
ranks' landmarks / edges and writes the outcome (tests/test_lba_gpu.py compares it to the oracle).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--backend", default="gloo", choices=("gloo", "nccl"))
    ap.add_argument("--n-kf", type=int, default=20)
    ap.add_argument("--n-opt", type=int, default=10)
    ap.add_argument("--n-pts", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--large", type=int, default=1)
    ap.add_argument("--host-driver", type=int, default=0, help="1: the host-driven LM loop (read-back per trial)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from openmavis_amd import synth_ba
    from openmavis_amd.dist import LbaAllReduce
    from openmavis_amd.optimizer import LocalInertialBA, lba_options

    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    prob = synth_ba.make_lba_problem(n_kf=args.n_kf, n_opt=args.n_opt, n_pts=args.n_pts, seed=args.seed)
    ar = LbaAllReduce("device" if args.backend == "nccl" else "host", device=dev)
    ba = LocalInertialBA(max_kf=prob["n_kf"], max_cams=prob["n_cams"], max_pts=len(prob["pts"]),
                         max_mono=len(prob["mono_pt"]), max_imu=max(1, len(prob["imu_kf1"])), rank=rank, world=world,
                         allreduce=ar)
    ba.set_driver(bool(args.host_driver))
    ba.set_problem(prob)
    idx, n_e = ba.shard()
    res, st = ba.optimize(max_trials=10, large=bool(args.large), **lba_options(bool(args.large)))
    syncs, trials = ba.host_syncs()
    mine = np.isin(prob["mono_pt"], idx)
    assert int(mine.sum()) == n_e
    part = dict(rank=rank, idx=idx, pts=st["pts"][idx], edges=np.nonzero(mine)[0],
                chi2=res["mono_chi2"][mine], outl=res["mono_outlier"][mine],
                kf={k: st[k] for k in ("Rwb", "twb", "Rcw", "tcw", "vel", "bg", "ba")},
                scal={k: res[k] for k in ("err", "err_end", "status", "iterations", "trials")}, syncs=syncs,
                ar_calls=ar.calls)
    parts = [None] * world
    dist.all_gather_object(parts, part)
    if rank == 0:
        P, E = len(prob["pts"]), len(prob["mono_pt"])
        pts = np.full((P, 3), np.nan)
        chi2 = np.full(E, np.nan)
        outl = np.zeros(E, np.uint8)
        owner = np.full(P, -1)
        for q in parts:
            assert (owner[q["idx"]] == -1).all(), "a landmark owned by two ranks"
            owner[q["idx"]] = q["rank"]
            pts[q["idx"]] = q["pts"]
            chi2[q["edges"]] = q["chi2"]
            outl[q["edges"]] = q["outl"]
            for k, v in q["kf"].items():   # every rank solved the identical reduced system
                assert np.array_equal(v, parts[0]["kf"][k]), ("keyframe state differs across ranks", k)
            assert q["scal"] == parts[0]["scal"], "LM outcome differs across ranks"
        out = dict(pts=pts, mono_chi2=chi2, mono_outlier=outl, owner=owner, world=world,
                   host_syncs=max(q["syncs"] for q in parts), ar_calls=min(q["ar_calls"] for q in parts),
                   **{k: v for k, v in parts[0]["kf"].items()}, **parts[0]["scal"])
        np.savez(args.out, **out)
        print(f"lba shard ok: world {world}, trials {out['trials']}, err {out['err']:.6g} -> {out['err_end']:.6g}")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
