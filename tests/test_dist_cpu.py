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
