// MI355X-native IMU preintegration: IMU::Preintegrated::IntegrateNewMeasurement (src/ImuTypes.cc:160-239,
// IntegratedRotation :58-80) over a batch of independent preintegrations, as Tracking::PreintegrateIMU
// feeds them (src/Tracking.cc:1675-1712: per frame one record from the last keyframe and one from the last
// frame).  The chain over measurements is sequential; the batch is not: one wavefront per record.
//
// Per measurement, lane 0 runs the float 3x3 algebra (deltas, bias Jacobians, IntegratedRotation, the
// polar-factor NormalizeRotation) and writes the 9x15 A and 9x6 B of the covariance step into LDS; the
// wavefront then forms T = A C (135 dot products), A C A^T + B Nga B^T (81) and the random-walk block.
// Every float expression follows the oracle's (oracle/imu_oracle.cpp) written order, so the two agree bit
// for bit: glibc sinf / cosf restated (omv_device.h), correctly rounded sqrt and division.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../include/omv.h"
#include "omv_device.h"

namespace {

#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

// record offsets (include/omv.h OMV_PREINT_FLOATS layout)
constexpr int kR = 0, kV = 9, kP = 12, kJRg = 15, kJVg = 24, kJVa = 33, kJPg = 42, kJPa = 51, kB = 60, kT = 66,
              kC = 67;

__device__ __forceinline__ void mul3(const float *a, const float *b, float *r) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
__device__ __forceinline__ void mulv3(const float *a, const float *x, float *y) {
    for (int i = 0; i < 3; ++i) y[i] = a[3 * i] * x[0] + a[3 * i + 1] * x[1] + a[3 * i + 2] * x[2];
}
__device__ __forceinline__ void hat3(const float *w, float *W) {
    W[0] = 0, W[1] = -w[2], W[2] = w[1], W[3] = w[2], W[4] = 0, W[5] = -w[0], W[6] = -w[1], W[7] = w[0], W[8] = 0;
}
__device__ void polar3f(float *r) {   // NormalizeRotation: X <- (X + X^-T) / 2
    for (int it = 0; it < 20; ++it) {
        float c[9];
        c[0] = r[4] * r[8] - r[5] * r[7];
        c[1] = r[5] * r[6] - r[3] * r[8];
        c[2] = r[3] * r[7] - r[4] * r[6];
        c[3] = r[2] * r[7] - r[1] * r[8];
        c[4] = r[0] * r[8] - r[2] * r[6];
        c[5] = r[1] * r[6] - r[0] * r[7];
        c[6] = r[1] * r[5] - r[2] * r[4];
        c[7] = r[2] * r[3] - r[0] * r[5];
        c[8] = r[0] * r[4] - r[1] * r[3];
        const float det = r[0] * c[0] + r[1] * c[1] + r[2] * c[2];
        const float id = 1.0f / det;
        float diff = 0;
        for (int k = 0; k < 9; ++k) {
            const float nv = (r[k] + c[k] * id) * 0.5f;
            diff = fmaxf(diff, fabsf(nv - r[k]));
            r[k] = nv;
        }
        if (diff <= 2.5e-7f) break;
    }
}

struct Calib {   // IMU::Calib::Cov / CovWalk: Eigen::DiagonalMatrix<float, 6> (include/ImuTypes.h:126)
    float Nga[6], NgaWalk[6];
};

// Lane 0's part of one measurement: updates the record's deltas and Jacobians in `s` (LDS) and writes the
// covariance step's A (9x15) and B (9x6).
__device__ void step_scalar(float *s, float *avg, const float *meas, float *A, float *B) {
    const float eps = 1e-4f;
    const float dt = meas[6];
    float acc[3], accW[3];
    for (int q = 0; q < 3; ++q) acc[q] = meas[q] - s[kB + q], accW[q] = meas[3 + q] - s[kB + 3 + q];
    float dR[9];
    for (int k = 0; k < 9; ++k) dR[k] = s[kR + k];
    const float dT = s[kT];
    {
        float ra[3];
        mulv3(dR, acc, ra);
        for (int q = 0; q < 3; ++q) avg[q] = (dT * avg[q] + ra[q] * dt) / (dT + dt);
        for (int q = 0; q < 3; ++q) avg[3 + q] = (dT * avg[3 + q] + accW[q] * dt) / (dT + dt);
    }
    const float theta = omv::sqrtf_cr(accW[0] * accW[0] + accW[1] * accW[1] + accW[2] * accW[2]);
    const float theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta3 * theta;
    float W[9], W2[9];
    hat3(accW, W);
    mul3(W, W, W2);
    float sn, cs;
    omv::glibc_sincosf(dt * theta, &sn, &cs);
    const float c1 = (1.0f - cs) / theta2, c2 = (dt * theta - sn) / theta3;
    const float h2 = 0.5f * dt * dt, c3 = (0.5f * dt * dt * theta2 + cs - 1) / theta4;
    float J1[9], J2[9];
    for (int k = 0; k < 9; ++k) {
        const float I = (k % 4 == 0) ? 1.0f : 0.0f;
        J1[k] = (dt * I + c1 * W[k]) + c2 * W2[k];
        J2[k] = (h2 * I + c2 * W[k]) + c3 * W2[k];
    }
    float dRJ1[9], dRJ2[9];
    mul3(dR, J1, dRJ1);
    mul3(dR, J2, dRJ2);
    {
        float p2[3], p1[3];
        mulv3(dRJ2, acc, p2);
        mulv3(dRJ1, acc, p1);
        for (int q = 0; q < 3; ++q) s[kP + q] = (s[kP + q] + s[kV + q] * dt) + p2[q];
        for (int q = 0; q < 3; ++q) s[kV + q] = s[kV + q] + p1[q];
    }
    for (int q = 0; q < 135; ++q) A[q] = (q / 15 == q % 15) ? 1.0f : 0.0f;
    for (int q = 0; q < 54; ++q) B[q] = 0.0f;
    float Wacc[9];
    hat3(acc, Wacc);
    {
        float j1a[3], j2a[3], H1[9], H2[9], a30[9], a60[9];
        mulv3(J1, acc, j1a);
        mulv3(J2, acc, j2a);
        hat3(j1a, H1);
        hat3(j2a, H2);
        mul3(dR, H1, a30);
        mul3(dR, H2, a60);
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) {
                A[(3 + r) * 15 + q] = -a30[3 * r + q];
                A[(6 + r) * 15 + q] = -a60[3 * r + q];
                A[(6 + r) * 15 + 3 + q] = r == q ? dt : 0.0f;
                A[r * 15 + 9 + q] = r == q ? -dt : 0.0f;
                A[(3 + r) * 15 + 12 + q] = -dRJ1[3 * r + q];
                A[(6 + r) * 15 + 12 + q] = -dRJ2[3 * r + q];
                B[(3 + r) * 6 + 3 + q] = dRJ1[3 * r + q];
                B[(6 + r) * 6 + 3 + q] = dRJ2[3 * r + q];
            }
    }
    {   // bias Jacobians (old dR, old JVa / JVg)
        float t[9], t2[9], t1[9];
        mul3(dRJ2, Wacc, t);
        mul3(t, s + kJRg, t2);
        mul3(dRJ1, Wacc, t);
        mul3(t, s + kJRg, t1);
        for (int k = 0; k < 9; ++k) {
            const float jva = s[kJVa + k], jvg = s[kJVg + k];
            s[kJPa + k] = (s[kJPa + k] + jva * dt) - dRJ2[k];
            s[kJPg + k] = (s[kJPg + k] + jvg * dt) - t2[k];
            s[kJVa + k] = jva - dRJ1[k];
            s[kJVg + k] = jvg - t1[k];
        }
    }
    float dRi[9], rJ[9];
    {   // IntegratedRotation(angVel, b, dt)
        const float x = (meas[3] - s[kB + 3]) * dt, y = (meas[4] - s[kB + 4]) * dt, z = (meas[5] - s[kB + 5]) * dt;
        const float d2 = x * x + y * y + z * z, d = omv::sqrtf_cr(d2);
        const float v[3] = {x, y, z};
        float Wr[9], Wr2[9];
        hat3(v, Wr);
        mul3(Wr, Wr, Wr2);
        if (d < eps) {
            for (int k = 0; k < 9; ++k) dRi[k] = ((k % 4 == 0) ? 1.0f : 0.0f) + Wr[k], rJ[k] = (k % 4 == 0) ? 1.0f : 0.0f;
        } else {
            float sd, cd;
            omv::glibc_sincosf(d, &sd, &cd);
            for (int k = 0; k < 9; ++k) {
                const float I = (k % 4 == 0) ? 1.0f : 0.0f;
                dRi[k] = (I + Wr[k] * sd / d) + Wr2[k] * (1.0f - cd) / d2;
                rJ[k] = (I - Wr[k] * (1.0f - cd) / d2) + Wr2[k] * (d - sd) / (d2 * d);
            }
        }
    }
    float nR[9];
    mul3(dR, dRi, nR);
    polar3f(nR);
    for (int k = 0; k < 9; ++k) s[kR + k] = nR[k];
    float dRit[9];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) dRit[3 * r + q] = dRi[3 * q + r];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) A[r * 15 + q] = dRit[3 * r + q], B[r * 6 + q] = rJ[3 * r + q] * dt;
    {   // JRg = dRi^T * JRg - rightJ * dt
        float a[9];
        mul3(dRit, s + kJRg, a);
        for (int k = 0; k < 9; ++k) s[kJRg + k] = a[k] - rJ[k] * dt;
    }
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wavefront per record.
__global__ void __launch_bounds__(64) preint_kernel(float *rec, float *avg_io, const float *meas, const int32_t *start,
                                                    Calib cal) {
    __shared__ float s[OMV_PREINT_FLOATS];
    __shared__ float A[135], B[54], T[135], U[54], avg[6];
    const int r = blockIdx.x, lane = threadIdx.x;
    float *g = rec + (size_t)r * OMV_PREINT_FLOATS;
    for (int q = lane; q < OMV_PREINT_FLOATS; q += 64) s[q] = g[q];
    if (lane < 6) avg[lane] = avg_io ? avg_io[(size_t)r * 6 + lane] : 0.0f;
    wave_sync();
    const int m0 = start[r], m1 = start[r + 1];
    for (int m = m0; m < m1; ++m) {
        const float *ms = meas + (size_t)m * 7;
        if (lane == 0) step_scalar(s, avg, ms, A, B);
        wave_sync();
        // T = A C (9x15), U = B Nga (9x6)
        for (int q = lane; q < 135 + 54; q += 64) {
            if (q < 135) {
                const int i = q / 15, k = q % 15;
                float t = 0;
                for (int j = 0; j < 15; ++j) t += A[i * 15 + j] * s[kC + j * 15 + k];
                T[q] = t;
            } else {   // B * Nga: column scaling by the diagonal
                const int k = (q - 135) % 6;
                U[q - 135] = B[q - 135] * cal.Nga[k];
            }
        }
        wave_sync();
        // C[0:9, 0:9] = T A^T + U B^T; diag C[9:15, 9:15] += dt^2 NgaWalk (disjoint elements)
        const float dt = ms[6];
        float cn[2];
        for (int q = lane, n = 0; q < 81; q += 64, ++n) {
            const int i = q / 9, l = q % 9;
            float t = 0, u = 0;
            for (int k = 0; k < 15; ++k) t += T[i * 15 + k] * A[l * 15 + k];
            for (int k = 0; k < 6; ++k) u += U[i * 6 + k] * B[l * 6 + k];
            cn[n] = t + u;
        }
        wave_sync();
        for (int q = lane, n = 0; q < 81; q += 64, ++n) s[kC + (q / 9) * 15 + q % 9] = cn[n];
        if (lane < 6) s[kC + (9 + lane) * 15 + 9 + lane] += (dt * dt) * cal.NgaWalk[lane];   // += a diagonal
        if (lane == 0) s[kT] += dt;
        wave_sync();
    }
    for (int q = lane; q < OMV_PREINT_FLOATS; q += 64) g[q] = s[q];
    if (avg_io && lane < 6) avg_io[(size_t)r * 6 + lane] = avg[lane];
}

}  // namespace

extern "C" {

omv_status omv_imu_preintegrate(int n, float *preint, float *avg, const float *meas, const int32_t *start,
                                const float *Nga, const float *NgaWalk, void *stream) {
    if (n < 0 || (n > 0 && (!preint || !meas || !start || !Nga || !NgaWalk))) return OMV_ERR_ARG;
    if (n == 0) return OMV_OK;
    Calib cal;
    for (int q = 0; q < 6; ++q) cal.Nga[q] = Nga[q], cal.NgaWalk[q] = NgaWalk[q];
    preint_kernel<<<n, 64, 0, (hipStream_t)stream>>>(preint, avg, meas, start, cal);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

}  // extern "C"
