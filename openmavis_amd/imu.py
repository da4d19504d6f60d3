"""Host-side mirror of IMU::Preintegrated (include/ImuTypes.h, src/ImuTypes.cc) for a batch of records on
the device (openmavis_amd/csrc/imu.hip).

    pre = PreintegratedBatch(n, calib=Calib(ng, na, ngw, naw, freq), device="cuda:0")
    pre.Initialize(bias)                       # Preintegrated::Initialize (:132-150), bias [n][6]
    pre.IntegrateNewMeasurements(meas, start)  # IntegrateNewMeasurement (:160-239) per record run

`pre.rec` is the [n][OMV_PREINT_FLOATS] float32 tensor the pose optimisations and LocalInertialBA read
(dR dV dP JRg JVg JVa JPg JPa b dT C), `pre.avg` avgA | avgW.  There is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib

PREINT_FLOATS = 292


class Calib:
    """IMU::Calib::Set (src/ImuTypes.cc:388-405) with Tracking's per-frequency scaling (Tracking.cc:601):
    Cov = diag(ng^2 x3, na^2 x3), CovWalk = diag(ngw^2 x3, naw^2 x3) of Ng*sf, Na*sf, Ngw/sf, Naw/sf,
    sf = sqrt(freq), all float."""

    def __init__(self, ng, na, ngw, naw, freq=None):
        f32 = np.float32
        if freq is not None:
            sf = f32(np.sqrt(f32(freq)))
            ng, na, ngw, naw = f32(ng) * sf, f32(na) * sf, f32(ngw) / sf, f32(naw) / sf
        ng, na, ngw, naw = f32(ng), f32(na), f32(ngw), f32(naw)
        self.Cov = np.array([ng * ng] * 3 + [na * na] * 3, np.float32)
        self.CovWalk = np.array([ngw * ngw] * 3 + [naw * naw] * 3, np.float32)


class PreintegratedBatch:
    def __init__(self, n, calib, device="cuda:0"):
        import torch
        self.n, self.calib = n, calib
        self.rec = torch.zeros((n, PREINT_FLOATS), dtype=torch.float32, device=device)
        self.avg = torch.zeros((n, 6), dtype=torch.float32, device=device)
        self._lib = _lib.load()

    def Initialize(self, bias):
        """dR = I, everything else zero, b = bias ([n][6]: bax bay baz bwx bwy bwz)."""
        import torch
        self.rec.zero_()
        self.avg.zero_()
        self.rec[:, [0, 4, 8]] = 1.0
        self.rec[:, 60:66] = torch.as_tensor(np.asarray(bias, np.float32), device=self.rec.device)
        return self

    def IntegrateNewMeasurements(self, meas, start, stream=None):
        """meas: device float32 [m][7] (acc xyz, angVel xyz, dt) in integration order; start: device int32
        [n+1]: record r integrates meas[start[r]:start[r+1]]."""
        import torch
        st = stream if stream is not None else torch.cuda.current_stream(self.rec.device).cuda_stream
        _lib.check(self._lib.omv_imu_preintegrate(self.n, _lib.ptr(self.rec), _lib.ptr(self.avg), _lib.ptr(meas),
                                                  _lib.ptr(start), _lib.ptr(self.calib.Cov),
                                                  _lib.ptr(self.calib.CovWalk), ctypes.c_void_p(st)),
                   "omv_imu_preintegrate")
        return self
