"""GPU parity of the batched IMU preintegration (openmavis_amd/csrc/imu.hip) against the float oracle
(oracle/imu_oracle.cpp, src/ImuTypes.cc:160-239): bit-exact records and averages (both evaluate every float
expression in the same order with the same sinf / cosf / sqrtf)."""
import numpy as np
import pytest

from openmavis_amd import synth_imu
from openmavis_amd.imu import Calib, PreintegratedBatch

pytestmark = pytest.mark.gpu
CAL = Calib(1.7e-4, 2.0e-3, 1.9e-5, 3.0e-3, freq=200.0)


@pytest.mark.parametrize("seed,n_rec", [(1, 64), (2, 300)])
def test_preintegration_matches_oracle(oracle, seed, n_rec):
    import torch
    b = synth_imu.make_imu_batch(n_rec=n_rec, seed=seed)
    pre = PreintegratedBatch(n_rec, CAL).Initialize(b["bias"])
    pre.IntegrateNewMeasurements(torch.from_numpy(b["meas"]).cuda(), torch.from_numpy(b["start"]).cuda())
    torch.cuda.synchronize()
    rec, avg = oracle.preintegrate(b, CAL.Cov, CAL.CovWalk)
    g = pre.rec.cpu().numpy()
    assert np.array_equal(g.view(np.int32), rec.view(np.int32)), np.argwhere(g != rec)[:5]
    assert np.array_equal(pre.avg.cpu().numpy(), avg)


def test_empty_runs_and_two_calls():
    """Records with no measurements stay as initialised; two calls chain like one."""
    import torch
    b = synth_imu.make_imu_batch(n_rec=8, seed=5)
    st = b["start"].copy()
    st[3] = st[2]   # record 2 empty: shift is fine since start is non-decreasing
    st[3:] = np.maximum(st[3:], st[3])
    pre = PreintegratedBatch(8, CAL).Initialize(b["bias"])
    pre.IntegrateNewMeasurements(torch.from_numpy(b["meas"]).cuda(), torch.from_numpy(st).cuda())
    torch.cuda.synchronize()
    g = pre.rec.cpu().numpy()
    assert g[2, 66] == 0 and g[2, 0] == 1
    one = PreintegratedBatch(8, CAL).Initialize(b["bias"])
    one.IntegrateNewMeasurements(torch.from_numpy(b["meas"]).cuda(), torch.from_numpy(b["start"]).cuda())
    a = PreintegratedBatch(8, CAL).Initialize(b["bias"])
    mid = (b["start"][:-1] + b["start"][1:]) // 2
    s1 = np.stack([b["start"][:-1], mid], 1)
    s2 = np.stack([mid, b["start"][1:]], 1)
    # per-record halves via gathered measurement arrays
    m1 = np.concatenate([b["meas"][s:e] for s, e in s1])
    m2 = np.concatenate([b["meas"][s:e] for s, e in s2])
    c1 = np.concatenate([[0], np.cumsum(s1[:, 1] - s1[:, 0])]).astype(np.int32)
    c2 = np.concatenate([[0], np.cumsum(s2[:, 1] - s2[:, 0])]).astype(np.int32)
    a.IntegrateNewMeasurements(torch.from_numpy(m1).cuda(), torch.from_numpy(c1).cuda())
    a.IntegrateNewMeasurements(torch.from_numpy(m2).cuda(), torch.from_numpy(c2).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(a.rec.cpu().numpy(), one.rec.cpu().numpy())
