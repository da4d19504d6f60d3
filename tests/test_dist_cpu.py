"""world_size-2 gloo tests of the multi-GPU plumbing on CPU (the driver runs the RCCL version)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from openmavis_amd import dist as od
    od.init_from_env("gloo")
    try:
        kp_cap = 37
        g = torch.Generator().manual_seed(rank)
        kps = torch.randint(-2**31, 2**31 - 1, (kp_cap, 6), dtype=torch.int32, generator=g)
        desc = torch.randint(0, 256, (kp_cap, 32), dtype=torch.uint8, generator=g)
        n = torch.tensor([10 + rank], dtype=torch.int32)
        gk, gd, gn = od.allgather_camera_slabs(kps, desc, n)
        ok = True
        for r in range(world):
            g2 = torch.Generator().manual_seed(r)
            ek = torch.randint(-2**31, 2**31 - 1, (kp_cap, 6), dtype=torch.int32, generator=g2)
            ed = torch.randint(0, 256, (kp_cap, 32), dtype=torch.uint8, generator=g2)
            ok &= bool(torch.equal(gk[r], ek)) and bool(torch.equal(gd[r], ed)) and int(gn[r]) == 10 + r
        t = od.job_seconds(1.0 + rank)
        q.put((rank, ok, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_allgather_slabs_and_max_time_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(abs(t - world) < 1e-9 for _, _, t in res), res   # max over ranks = 1.0 + (world-1)


def _shard_worker(rank, world, port, q, n_cams, F, cap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from openmavis_amd import dist as od
    od.init_from_env("gloo")
    try:
        class FB:   # the FrameBatch tensors CameraShard.gather fills
            pass
        fb = FB()
        fb.kps = torch.zeros((F, n_cams, cap, 6), dtype=torch.int32)
        fb.desc = torch.zeros((F, n_cams, cap, 32), dtype=torch.uint8)
        fb.n_kp = torch.zeros((F, n_cams), dtype=torch.int32)
        fb.mono = torch.zeros((F, n_cams), dtype=torch.int32)
        sh = od.CameraShard(rank, world, n_cams, F, cap, "cpu", mode="device")
        kps, desc, n, mono = sh.outputs()
        # "extract": image i of this rank = (camera cams[i // F], frame i % F), values derived from (camera, frame)
        for i in range(len(sh.cams) * F):
            c, f = sh.cams[i // F], i % F
            g = torch.Generator().manual_seed(1000 * c + f)
            kps[i] = torch.randint(-2**31, 2**31 - 1, (cap, 6), dtype=torch.int32, generator=g)
            desc[i] = torch.randint(0, 256, (cap, 32), dtype=torch.uint8, generator=g)
            n[i], mono[i] = 7 * c + f, 3 * c + f
        sh.gather(fb)
        ok = True
        for c in range(n_cams):
            for f in range(F):
                g = torch.Generator().manual_seed(1000 * c + f)
                ok &= bool(torch.equal(fb.kps[f, c], torch.randint(-2**31, 2**31 - 1, (cap, 6), dtype=torch.int32,
                                                                   generator=g)))
                ok &= bool(torch.equal(fb.desc[f, c], torch.randint(0, 256, (cap, 32), dtype=torch.uint8, generator=g)))
                ok &= int(fb.n_kp[f, c]) == 7 * c + f and int(fb.mono[f, c]) == 3 * c + f
        q.put((rank, ok, sh.cams))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_cams", [(2, 5), (2, 2), (5, 5), (8, 5)])
def test_camera_shard_gather_gloo(world, n_cams):
    """configs[2]: one camera per rank (5 cameras on 2 ranks: 3 + 2 slots; on 5 ranks one each; on 8 ranks --
    the real 5-of-8 layout -- ranks 5-7 hold no camera and send empty sections), one all-gather, every rank holds
    every camera's keypoints / descriptors in camera order."""
    F, cap = 3, 17
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, q, n_cams, F, cap)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert sorted(c for _, _, cams in res for c in cams) == list(range(n_cams))
