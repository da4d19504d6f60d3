"""BASELINE configs[2]: cameras sharded over ranks with one all-gather of the keypoint / descriptor slabs, then
the tracking rank's matching — identical to the single-GPU batched path (and that to the oracle).

Runs 2 ranks on this box: gloo with the slabs staged through host memory when one GPU is visible (both ranks
share it), RCCL (nccl) with device slabs when two or more are."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from openmavis_amd import synth
from openmavis_amd.matcher import FrameBatch, MapPointBatch, ORBmatcher
from openmavis_amd.orb import ORBextractor

pytestmark = pytest.mark.gpu

W, H, C, NF, F = 720, 540, 5, 1200, 2
LAP = np.array([[0, 720], [0, 720], [0, 0], [0, 0], [0, 0]], np.int32)


def _run_ranks(tmp_path, backend, world=2):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / f"camshard_{backend}.npz"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(root, "tools", "camshard_run.py"),
           "--out", str(out), "--backend", backend, "--frames", str(F)]
    r = subprocess.run(cmd, cwd=root, env=dict(os.environ, OMP_NUM_THREADS="2"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return dict(np.load(out))


def test_camera_sharded_frame_equals_batched(oracle, torch_cuda, tmp_path):
    torch = torch_cuda
    backend = "nccl" if torch.cuda.device_count() >= 2 else "gloo"
    g = _run_ranks(tmp_path, backend)
    assert int(g["world"]) == 2
    _check_against_batched(g, oracle, torch)


def test_camera_shard_rccl_one_rank(oracle, torch_cuda, tmp_path):
    """CameraShard(mode="device") under torch's nccl backend (RCCL) with one rank: the slab all-gather runs through
    RCCL on the device (all five cameras on rank 0) and the gathered frame equals the batched path bit for bit."""
    g = _run_ranks(tmp_path, "nccl", world=1)
    assert int(g["world"]) == 1
    _check_against_batched(g, oracle, torch_cuda)


def test_camera_shard_five_ranks_one_camera_each(oracle, torch_cuda, tmp_path):
    """configs[2]'s layout: five ranks, one camera of the Hilti rig each (rank r extracts camera r with the HIP
    extractor on its GPU — all five share this box's card, gloo stages the slabs through host memory), one all-gather,
    rank 0 matches the gathered frame: identical to the single-GPU batched path bit for bit, and that to the oracle."""
    g = _run_ranks(tmp_path, "gloo", world=5)
    assert int(g["world"]) == 5
    _check_against_batched(g, oracle, torch_cuda)


def _check_against_batched(g, oracle, torch):
    # the single-GPU batched path on the same frames
    imgs = np.concatenate([synth.hilti_frame(f) for f in range(F)])
    ex = ORBextractor(NF, 1.2, 8, 15, 7, width=W, height=H, max_images=F * C)
    cap = ex.max_keypoints()
    fb = FrameBatch(torch, F, C, cap, W, H, ex.GetScaleFactors())
    ex.extract_batch(torch.from_numpy(imgs).cuda(), np.tile(LAP, (F, 1)), fb.kps.view(-1, cap, 6),
                     fb.desc.view(-1, cap, 32), fb.n_kp.view(-1), fb.mono.view(-1))
    torch.cuda.synchronize()
    n_kp = fb.n_kp.cpu().numpy()
    assert np.array_equal(g["n_kp"], n_kp) and np.array_equal(g["mono"], fb.mono.cpu().numpy())
    kps, desc = fb.kps.cpu().numpy(), fb.desc.cpu().numpy()
    for f in range(F):
        for c in range(C):
            n = n_kp[f, c]
            assert np.array_equal(g["kps"][f, c, :n], kps[f, c, :n]), (f, c)
            assert np.array_equal(g["desc"][f, c, :n], desc[f, c, :n]), (f, c)
    kpv = kps.view(oracle.KP_DTYPE).reshape(F, C, cap)
    per = [synth.make_map_points(kpv[f], desc[f], n_kp[f], 3000, 31 + f, W, H) for f in range(F)]
    mps = MapPointBatch(**{k: torch.from_numpy(np.stack([p[k] for p in per])).cuda() for k in per[0]})
    m = ORBmatcher(0.8)
    m.AssignFeaturesToGrid(fb)
    m.StereoLapping(fb, 0.8)
    fb.kp_to_mp.fill_(-1)
    m.SearchByProjection(fb, mps, 6.0, False, 50.0, grid_ready=True)
    torch.cuda.synchronize()
    assert np.array_equal(g["l2r"], fb.l2r.cpu().numpy()) and np.array_equal(g["r2l"], fb.r2l.cpu().numpy())
    assert np.array_equal(g["kp_to_mp"], fb.kp_to_mp.cpu().numpy())
    assert np.array_equal(g["n_matches"], fb.n_matches.cpu().numpy())
    # and the batched path against the oracle's sequential SearchByProjection
    geom = oracle.frame_geom(C, W, H, ex.GetScaleFactors())
    for f in range(F):
        exp = np.full(C * cap, -1, np.int32)
        n = oracle.search_by_projection(geom, kpv[f], desc[f], n_kp[f], per[f], 6.0, False, 50.0, 0.8, g["l2r"][f],
                                        g["r2l"][f], None, exp)
        assert n == g["n_matches"][f] and np.array_equal(exp, g["kp_to_mp"][f]), f
        assert n > 300
