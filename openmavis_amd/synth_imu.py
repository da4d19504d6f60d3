"""Seeded synthetic IMU streams for IMU::Preintegrated::IntegrateNewMeasurement (src/ImuTypes.cc:160-239):
per record an interval of synth_ba's smooth trajectory (arc + pitch wobble) sampled at `freq` Hz, the
exact body-frame specific force / angular rate of each step plus white noise and a constant bias, with the
first / last steps shortened like Tracking::PreintegrateIMU's interpolation at the frame times
(src/Tracking.cc:1675-1706).  integrate64() is an independent float64 numpy restatement used to pin the
float oracle."""
import numpy as np

from . import synth_ba


def make_imu_batch(n_rec=16, seed=1, freq=200.0, n_range=(4, 40), noise=(1.7e-3, 2.0e-2), bias_sigma=(2e-3, 5e-2)):
    rng = np.random.Generator(np.random.PCG64(seed))
    meas, start, bias = [], [0], []
    for r in range(n_rec):
        t0 = float(rng.uniform(0, 30))
        n = int(rng.integers(n_range[0], n_range[1] + 1))
        h = 1.0 / freq
        steps = np.full(n, h)
        steps[0] *= rng.uniform(0.2, 1.0)
        steps[-1] *= rng.uniform(0.2, 1.0)
        b = np.concatenate([rng.normal(0, bias_sigma[1], 3), rng.normal(0, bias_sigma[0], 3)])
        t = t0
        for dt in steps:
            Ra, pa, va = synth_ba._pose_at(t)
            Rb, pb, vb = synth_ba._pose_at(t + dt)
            w = synth_ba._log(Ra.T @ Rb) / dt
            a = Ra.T @ ((vb - va) / dt - synth_ba.G)
            m = np.concatenate([a + b[:3] + rng.normal(0, noise[1], 3), w + b[3:] + rng.normal(0, noise[0], 3), [dt]])
            meas.append(m)
            t += dt
        start.append(start[-1] + n)
        bias.append(b + np.concatenate([rng.normal(0, 1e-3, 3), rng.normal(0, 1e-4, 3)]))   # estimate != truth
    return dict(meas=np.array(meas, np.float32), start=np.array(start, np.int32), bias=np.array(bias, np.float32))


def integrate64(meas, b, Nga, NgaWalk):
    """Float64 IntegrateNewMeasurement chain from Initialize(b) (numpy; NormalizeRotation by SVD)."""
    b = np.asarray(b, np.float64)
    dR, dV, dP = np.eye(3), np.zeros(3), np.zeros(3)
    JRg, JVg, JVa, JPg, JPa = (np.zeros((3, 3)) for _ in range(5))
    C = np.zeros((15, 15))
    dT = 0.0
    N, NW = np.diag(np.asarray(Nga, np.float64)), np.diag(np.asarray(NgaWalk, np.float64))
    for m in np.asarray(meas, np.float64):
        dt = m[6]
        acc, w = m[:3] - b[:3], m[3:6] - b[3:]
        th = np.linalg.norm(w)
        W = synth_ba._hat(w)
        J1 = dt * np.eye(3) + (1 - np.cos(dt * th)) / th ** 2 * W + (dt * th - np.sin(dt * th)) / th ** 3 * W @ W
        J2 = (0.5 * dt * dt * np.eye(3) + (dt * th - np.sin(dt * th)) / th ** 3 * W
              + (0.5 * dt * dt * th ** 2 + np.cos(dt * th) - 1) / th ** 4 * W @ W)
        dP = dP + dV * dt + dR @ J2 @ acc
        dV = dV + dR @ J1 @ acc
        A = np.eye(9, 15)
        B = np.zeros((9, 6))
        Wa = synth_ba._hat(acc)
        A[3:6, 0:3] = -dR @ synth_ba._hat(J1 @ acc)
        A[6:9, 0:3] = -dR @ synth_ba._hat(J2 @ acc)
        A[6:9, 3:6] = dt * np.eye(3)
        A[0:3, 9:12] = -dt * np.eye(3)
        A[3:6, 12:15] = -dR @ J1
        A[6:9, 12:15] = -dR @ J2
        B[3:6, 3:6] = dR @ J1
        B[6:9, 3:6] = dR @ J2
        JPa = JPa + JVa * dt - dR @ J2
        JPg = JPg + JVg * dt - dR @ J2 @ Wa @ JRg
        JVa = JVa - dR @ J1
        JVg = JVg - dR @ J1 @ Wa @ JRg
        dRi, rJ = synth_ba._exp(w * dt), synth_ba._rightJ(w * dt)
        u, _, vt = np.linalg.svd(dR @ dRi)
        dR = u @ vt
        A[0:3, 0:3] = dRi.T
        B[0:3, 0:3] = rJ * dt
        C[:9, :9] = A @ C @ A.T + B @ N @ B.T
        C[9:, 9:] += dt * dt * NW
        JRg = dRi.T @ JRg - rJ * dt
        dT += dt
    return np.concatenate([dR.ravel(), dV, dP, JRg.ravel(), JVg.ravel(), JVa.ravel(), JPg.ravel(), JPa.ravel(),
                           b, [dT], C.ravel()])
