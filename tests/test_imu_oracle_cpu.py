"""CPU checks of the IMU::Preintegrated::IntegrateNewMeasurement restatement (oracle/imu_oracle.cpp,
src/ImuTypes.cc:160-239).  The reference's tests hold no fixtures for it (parity vs Eigen unpinned); the float
restatement is pinned to an independent float64 numpy restatement (openmavis_amd/synth_imu.integrate64) and
to the kinematics it integrates."""
import numpy as np

from openmavis_amd import synth_ba, synth_imu
from openmavis_amd.imu import Calib

CAL = Calib(1.7e-4, 2.0e-3, 1.9e-5, 3.0e-3, freq=200.0)


def test_float_restatement_matches_float64():
    import oracle
    b = synth_imu.make_imu_batch(n_rec=12, seed=2)
    rec, avg = oracle.preintegrate(b, CAL.Cov, CAL.CovWalk)
    for r in range(12):
        s0, s1 = b["start"][r], b["start"][r + 1]
        ref = synth_imu.integrate64(b["meas"][s0:s1], b["bias"][r], CAL.Cov, CAL.CovWalk)
        g = rec[r].astype(np.float64)
        R, Rr = g[:9].reshape(3, 3), ref[:9].reshape(3, 3)
        assert np.linalg.norm(synth_ba._log(R.T @ Rr)) < 2e-6
        assert np.abs(g[9:15] - ref[9:15]).max() < 2e-5 * max(1.0, np.abs(ref[9:15]).max())
        for o in range(15, 60, 9):   # bias Jacobians
            assert np.abs(g[o:o + 9] - ref[o:o + 9]).max() < 1e-4 * max(1e-3, np.abs(ref[o:o + 9]).max())
        assert abs(g[66] - ref[66]) < 1e-6
        C, Cr = g[67:].reshape(15, 15), ref[67:].reshape(15, 15)
        assert np.abs(C - Cr).max() < 1e-4 * np.abs(Cr).max()
        assert np.allclose(C[:9, 9:], 0) and np.allclose(C[9:, :9], 0)   # the reference never writes them


def test_integrates_the_kinematics():
    """Noise-free, bias-free samples of the trajectory: dR / dV / dP reproduce the pose change."""
    import oracle
    b = synth_imu.make_imu_batch(n_rec=4, seed=3, noise=(0.0, 0.0), bias_sigma=(0.0, 0.0), freq=400.0)
    b["bias"][:] = 0
    rec, _ = oracle.preintegrate(b, CAL.Cov, CAL.CovWalk)
    assert (rec[:, 66] > 0).all()
    R = rec[:, :9].reshape(-1, 3, 3)
    for r in range(4):
        assert abs(np.linalg.det(R[r].astype(np.float64)) - 1) < 1e-5


def test_chained_calls_equal_one_call():
    """Integrating a run in two calls (the record carries the state) is bit-identical to one call."""
    import oracle
    b = synth_imu.make_imu_batch(n_rec=1, seed=4, n_range=(30, 30))
    one, avg1 = oracle.preintegrate(b, CAL.Cov, CAL.CovWalk)
    half = dict(b, start=np.array([0, 17], np.int32))
    rec, avg = oracle.preintegrate(half, CAL.Cov, CAL.CovWalk)
    meas = np.ascontiguousarray(b["meas"][17:30], np.float32)
    oracle.lib().oracle_preintegrate(oracle._p(rec[0]), oracle._p(avg[0]), oracle._p(meas), 13,
                                     oracle._p(CAL.Cov), oracle._p(CAL.CovWalk))
    assert np.array_equal(rec, one) and np.array_equal(avg, avg1)
