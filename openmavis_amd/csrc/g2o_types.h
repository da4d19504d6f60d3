// Device-side restatement of the g2o vertex / edge math OpenMAVIS defines in src/G2oTypes.cc and
// include/G2oTypes.h (ImuCamPose, KannalaBrandt8 projection, EdgeMono / EdgeStereo rows, EdgeInertial
// with IMU::Preintegrated's bias-corrected deltas, Huber), shared by the LocalInertialBA kernels
// (lba.hip) and the batched pose-inertial optimisation (pose.hip).  Header-only, f64 unless the
// reference computes in float (marked where it does).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/omv.h"
#include "omv_device.h"

namespace omv_g2o {

constexpr int kMaxCams = 8;
constexpr int kPF = OMV_PREINT_FLOATS;

using omv::glibc_atan2f;
using omv::sqrtf_cr;

// sin / cos in double of |x| < 1e5 (every argument on these paths: angles of rotation vectors and atan2f outputs):
// x - n pi/2 by two fused multiply-adds (pi/2 as a double pair), then Taylor polynomials to degree 17 / 18 on
// |r| <= pi/4 (truncation < 1e-19) -- within 1-2 ulp of the C library's results in ~40 instructions, where the
// general ocml routines (Payne-Hanek reduction for any argument) inline to several hundred.  Larger arguments take
// those routines.
__device__ __attribute__((noinline)) void sincos_slow(double x, double *s, double *c) { *s = sin(x), *c = cos(x); }
__device__ __forceinline__ void sincos_d(double x, double &s, double &c) {
    if (!(fabs(x) < 1e5)) {
        sincos_slow(x, &s, &c);
        return;
    }
    const double n = rint(x * 0.63661977236758134308);
    double r = __builtin_fma(-n, 1.5707963267948966192e+00, x);
    r = __builtin_fma(-n, 6.1232339957367660359e-17, r);
    const double r2 = r * r;
    double ps = 1.0 / 355687428096000.0;
    ps = __builtin_fma(ps, r2, -1.0 / 1307674368000.0);
    ps = __builtin_fma(ps, r2, 1.0 / 6227020800.0);
    ps = __builtin_fma(ps, r2, -1.0 / 39916800.0);
    ps = __builtin_fma(ps, r2, 1.0 / 362880.0);
    ps = __builtin_fma(ps, r2, -1.0 / 5040.0);
    ps = __builtin_fma(ps, r2, 1.0 / 120.0);
    ps = __builtin_fma(ps, r2, -1.0 / 6.0);
    const double sr = __builtin_fma(ps * r2, r, r);
    double pc = 1.0 / 6402373705728000.0;
    pc = __builtin_fma(pc, r2, -1.0 / 20922789888000.0);
    pc = __builtin_fma(pc, r2, 1.0 / 87178291200.0);
    pc = __builtin_fma(pc, r2, -1.0 / 479001600.0);
    pc = __builtin_fma(pc, r2, 1.0 / 3628800.0);
    pc = __builtin_fma(pc, r2, -1.0 / 40320.0);
    pc = __builtin_fma(pc, r2, 1.0 / 720.0);
    pc = __builtin_fma(pc, r2, -1.0 / 24.0);
    pc = __builtin_fma(pc, r2, 0.5);
    const double cr = __builtin_fma(-pc, r2, 1.0);
    const int q = (int)n & 3;
    s = q == 0 ? sr : q == 1 ? cr : q == 2 ? -sr : -cr;
    c = q == 0 ? cr : q == 1 ? -sr : q == 2 ? -cr : sr;
}

// ---- small f64 helpers (row-major 3x3) ----------------------------------------------------------
struct D3 {
    double v[3];
};
__device__ __forceinline__ void mv3(const double *R, const double *x, double *y) {
    for (int i = 0; i < 3; ++i) y[i] = R[3 * i] * x[0] + R[3 * i + 1] * x[1] + R[3 * i + 2] * x[2];
}
__device__ __forceinline__ void mtv3(const double *R, const double *x, double *y) {   // R^T x
    for (int i = 0; i < 3; ++i) y[i] = R[i] * x[0] + R[3 + i] * x[1] + R[6 + i] * x[2];
}
__device__ __forceinline__ void mm3(const double *a, const double *b, double *r) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
__device__ __forceinline__ void mtm3(const double *a, const double *b, double *r) {   // a^T b
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[i] * b[j] + a[3 + i] * b[3 + j] + a[6 + i] * b[6 + j];
}
__device__ __forceinline__ void tr3(const double *a, double *r) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * j + i];
}
__device__ __forceinline__ void hat3(const double *w, double *W) {
    W[0] = 0, W[1] = -w[2], W[2] = w[1], W[3] = w[2], W[4] = 0, W[5] = -w[0], W[6] = -w[1], W[7] = w[0], W[8] = 0;
}
template <typename T>
__host__ __device__ inline bool inv3(const T *a, T *r) {
    T c[9];
    c[0] = a[4] * a[8] - a[5] * a[7];
    c[1] = a[2] * a[7] - a[1] * a[8];
    c[2] = a[1] * a[5] - a[2] * a[4];
    c[3] = a[5] * a[6] - a[3] * a[8];
    c[4] = a[0] * a[8] - a[2] * a[6];
    c[5] = a[2] * a[3] - a[0] * a[5];
    c[6] = a[3] * a[7] - a[4] * a[6];
    c[7] = a[1] * a[6] - a[0] * a[7];
    c[8] = a[0] * a[4] - a[1] * a[3];
    const T det = a[0] * c[0] + a[1] * c[3] + a[2] * c[6];
    const T id = T(1) / det;
    for (int k = 0; k < 9; ++k) r[k] = c[k] * id;
    return det != T(0);
}
// NormalizeRotation (Eigen JacobiSVD U V^T) = polar factor, by Newton iteration X <- (X + X^-T)/2
template <typename T>
__host__ __device__ inline void polar3(T *r) {
    for (int it = 0; it < 20; ++it) {
        T c[9];
        c[0] = r[4] * r[8] - r[5] * r[7];
        c[1] = r[5] * r[6] - r[3] * r[8];
        c[2] = r[3] * r[7] - r[4] * r[6];
        c[3] = r[2] * r[7] - r[1] * r[8];
        c[4] = r[0] * r[8] - r[2] * r[6];
        c[5] = r[1] * r[6] - r[0] * r[7];
        c[6] = r[1] * r[5] - r[2] * r[4];
        c[7] = r[2] * r[3] - r[0] * r[5];
        c[8] = r[0] * r[4] - r[1] * r[3];
        const T det = r[0] * c[0] + r[1] * c[1] + r[2] * c[2];
        const T id = T(1) / det;
        T diff = 0;
        for (int k = 0; k < 9; ++k) {
            const T nv = (r[k] + c[k] * id) * T(0.5);
            const T dd = nv > r[k] ? nv - r[k] : r[k] - nv;
            diff = dd > diff ? dd : diff;
            r[k] = nv;
        }
        if (diff <= (sizeof(T) == 4 ? T(2.5e-7) : T(5e-16))) break;   // within ~2 ulp of a fixed point
    }
}

// ---- camera + pose math -------------------------------------------------------------------------
struct Rig {
    int n_cams;
    float cam[kMaxCams][8];
    double Rcb[kMaxCams][9], tcb[kMaxCams][3], Rbc[kMaxCams][9], tbc[kMaxCams][3];
    double bf;   // ImuCamPose::bf = KeyFrame::mbf (EdgeStereo)
    int model[kMaxCams];   // OMV_CAM_KB8 / OMV_CAM_PINHOLE (GeometricCamera::mnType)
};

// KannalaBrandt8::project(const Eigen::Vector3d&) (KannalaBrandt8.cpp:28-46)
__device__ __forceinline__ void kb8_project(const float *k, const double *X, double &u, double &v) {
    const double x2y2 = X[0] * X[0] + X[1] * X[1];
    const double theta = glibc_atan2f(sqrtf_cr((float)x2y2), (float)X[2]);
    const double psi = glibc_atan2f((float)X[1], (float)X[0]);
    const double t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
    const double r = theta + (double)k[4] * t3 + (double)k[5] * t5 + (double)k[6] * t7 + (double)k[7] * t9;
    double sp, cp;
    sincos_d(psi, sp, cp);
    u = (double)k[0] * r * cp + (double)k[2];
    v = (double)k[1] * r * sp + (double)k[3];
}
// KannalaBrandt8::projectJac (:128-158), 2x3 row-major
__device__ __forceinline__ void kb8_jac(const float *k, const double *X, double *J) {
    const double x2 = X[0] * X[0], y2 = X[1] * X[1], z2 = X[2] * X[2];
    const double r2 = x2 + y2, r = sqrt(r2), r3 = r2 * r;
    const double theta = atan2(r, X[2]);
    const double t2 = theta * theta, t3 = t2 * theta, t4 = t2 * t2, t5 = t4 * theta, t6 = t2 * t4, t7 = t6 * theta,
                 t8 = t4 * t4, t9 = t8 * theta;
    const double k4 = k[4], k5 = k[5], k6 = k[6], k7 = k[7];
    const double f = theta + t3 * k4 + t5 * k5 + t7 * k6 + t9 * k7;
    // `3 * mvParameters[4]` is an int x float product in the reference: rounded to float first
    const double fd = 1 + (double)(3.0f * k[4]) * t2 + (double)(5.0f * k[5]) * t4 + (double)(7.0f * k[6]) * t6 +
                      (double)(9.0f * k[7]) * t8;
    // three reciprocals for the eight quotients (each within an ulp of the division)
    const double iz = 1.0 / (r2 + z2), iq = iz / r2, ir3 = 1.0 / r3;
    const double xy = fd * X[2] * X[1] * X[0] * iq - f * X[1] * X[0] * ir3;
    J[0] = (double)k[0] * (fd * X[2] * x2 * iq + f * y2 * ir3);
    J[3] = (double)k[1] * xy;
    J[1] = (double)k[0] * xy;
    J[4] = (double)k[1] * (fd * X[2] * y2 * iq + f * x2 * ir3);
    J[2] = -(double)k[0] * fd * X[0] * iz;
    J[5] = -(double)k[1] * fd * X[1] * iz;
}

// Pinhole::project(const Eigen::Vector3d&) (Pinhole.cpp:18-24): float parameters, double arithmetic
__device__ __forceinline__ void pinhole_project(const float *k, const double *X, double &u, double &v) {
    u = (double)k[0] * X[0] / X[2] + (double)k[2];
    v = (double)k[1] * X[1] / X[2] + (double)k[3];
}
// Pinhole::projectJac (Pinhole.cpp:55-65), 2x3 row-major
__device__ __forceinline__ void pinhole_jac(const float *k, const double *X, double *J) {
    J[0] = (double)k[0] / X[2];
    J[1] = 0.0;
    J[2] = (double)(-k[0]) * X[0] / (X[2] * X[2]);
    J[3] = 0.0;
    J[4] = (double)k[1] / X[2];
    J[5] = (double)(-k[1]) * X[1] / (X[2] * X[2]);
}
// pCamera[c]->project / projectJac by the camera's type
__device__ __forceinline__ void cam_project(const Rig &rig, int c, const double *X, double &u, double &v) {
    if (rig.model[c] == OMV_CAM_PINHOLE) pinhole_project(rig.cam[c], X, u, v);
    else kb8_project(rig.cam[c], X, u, v);
}
__device__ __forceinline__ void cam_jac(const Rig &rig, int c, const double *X, double *J) {
    if (rig.model[c] == OMV_CAM_PINHOLE) pinhole_jac(rig.cam[c], X, J);
    else kb8_jac(rig.cam[c], X, J);
}

struct State {   // one of the two state buffers
    double *Rwb, *twb, *Rcw, *tcw, *vel, *bg, *ba, *pts;
};

struct Edges {   // landmark-major visual edges (EdgeMono, and EdgeStereo where ur >= 0)
    const int32_t *pt, *kf, *cam, *slot;
    const double *obs;
    const float *w;    // invSigma2
    const float *ur;   // EdgeStereo's third measurement (mvuRight >= 0); -1 on an EdgeMono
    int n;
};

// ImuCamPose::ProjectStereo's third row (G2oTypes.cc:198-205): u - bf * (1 / z)
__device__ __forceinline__ double stereo_ur(double u, double bf, double z) {
    const double invZ = 1 / z;
    return u - bf * invZ;
}

// Huber (robust_kernel_impl.cpp:78-91)
__device__ __forceinline__ void huber(double e2, double delta, double dsqr, double &r0, double &r1) {
    if (e2 <= dsqr) {
        r0 = e2, r1 = 1.0;
    } else {
        const double s = sqrt(e2);
        r0 = 2 * s * delta - dsqr;
        r1 = delta / s;
    }
}

// ---- errors ------------------------------------------------------------------------------------
__device__ double block_reduce_sum(double v, double *sh) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double t = 0;
    for (int q = 0; q < nw; ++q) t += sh[q];
    return t;
}

struct Imu {
    int n;
    const int32_t *kf1, *kf2;
    const float *pre;        // [n][kPF]
    const double *info9;     // [n][81] (scaled)
    const double *infoG, *infoA;   // [n][9]
    const uint8_t *robust;
    const int *offP, *offV, *offG, *offA;   // per keyframe, -1 if not in the reduced system
};

// IMU::Preintegrated::GetDeltaRotation/Velocity/Position (ImuTypes.cc:288-309) in float
__device__ void so3f_exp(const float *w, float *R) {
    const float theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    float imag, real;
    if (theta_sq < 1e-5f * 1e-5f) {
        const float t4 = theta_sq * theta_sq;
        imag = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * t4;
        real = 1.0f - (float)(1.0 / 8.0) * theta_sq + (float)(1.0 / 384.0) * t4;
    } else {
        const float theta = sqrtf_cr(theta_sq);
        const float half = 0.5f * theta;
        float sh, ch;
        omv::glibc_sincosf(half, &sh, &ch);
        imag = sh / theta;
        real = ch;
    }
    const float qw = real, qx = imag * w[0], qy = imag * w[1], qz = imag * w[2];
    const float tx = 2.0f * qx, ty = 2.0f * qy, tz = 2.0f * qz;
    const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
    const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    R[0] = 1.0f - (tyy + tzz), R[1] = txy - twz, R[2] = txz + twy;
    R[3] = txy + twz, R[4] = 1.0f - (txx + tzz), R[5] = tyz - twx;
    R[6] = txz - twy, R[7] = tyz + twx, R[8] = 1.0f - (txx + tyy);
}
__device__ void f33mulv(const float *a, const float *x, float *r) {
    for (int i = 0; i < 3; ++i) r[i] = a[3 * i] * x[0] + a[3 * i + 1] * x[1] + a[3 * i + 2] * x[2];
}
struct PreView {   // offsets inside one preintegration record
    static constexpr int dR = 0, dV = 9, dP = 12, JRg = 15, JVg = 24, JVa = 33, JPg = 42, JPa = 51, b = 60, dT = 66,
                         C = 67;
};
__device__ void delta_rot(const float *p, const float *b1, double *dR) {
    const float dbg[3] = {b1[3] - p[PreView::b + 3], b1[4] - p[PreView::b + 4], b1[5] - p[PreView::b + 5]};
    float w[3], E[9], R[9];
    f33mulv(p + PreView::JRg, dbg, w);
    so3f_exp(w, E);
    const float *A = p + PreView::dR;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = A[3 * i] * E[j] + A[3 * i + 1] * E[3 + j] + A[3 * i + 2] * E[6 + j];
    polar3(R);
    for (int q = 0; q < 9; ++q) dR[q] = (double)R[q];
}
__device__ void delta_vp(const float *p, int d, int jg, int ja, const float *b1, double *out) {
    const float dbg[3] = {b1[3] - p[PreView::b + 3], b1[4] - p[PreView::b + 4], b1[5] - p[PreView::b + 5]};
    const float dba[3] = {b1[0] - p[PreView::b], b1[1] - p[PreView::b + 1], b1[2] - p[PreView::b + 2]};
    float g[3], a[3];
    f33mulv(p + jg, dbg, g);
    f33mulv(p + ja, dba, a);
    for (int q = 0; q < 3; ++q) out[q] = (double)((p[d + q] + g[q]) + a[q]);
}
__device__ void log_so3(const double *R, double *w) {
    const double t = R[0] + R[4] + R[8];
    w[0] = (R[7] - R[5]) / 2, w[1] = (R[2] - R[6]) / 2, w[2] = (R[3] - R[1]) / 2;
    const double costheta = (t - 1.0) * 0.5f;
    if (costheta > 1 || costheta < -1) return;
    const double theta = acos(costheta);
    double s, c_unused;
    sincos_d(theta, s, c_unused);
    if (fabs(s) < 1e-5) return;
    for (int q = 0; q < 3; ++q) w[q] = theta * w[q] / s;
}

// EdgeInertial::computeError (G2oTypes.cc:502-531)
__device__ void imu_error(const State &s, const Imu &I, int i, double *e, double *eR_out = nullptr) {
    const int k1 = I.kf1[i], k2 = I.kf2[i];
    const float *p = I.pre + (size_t)i * kPF;
    float b1[6];
    for (int q = 0; q < 3; ++q) b1[q] = (float)s.ba[3 * k1 + q], b1[3 + q] = (float)s.bg[3 * k1 + q];
    double dR[9], dV[3], dP[3];
    delta_rot(p, b1, dR);
    delta_vp(p, PreView::dV, PreView::JVg, PreView::JVa, b1, dV);
    delta_vp(p, PreView::dP, PreView::JPg, PreView::JPa, b1, dP);
    const double dt = (double)p[PreView::dT];
    const double g[3] = {0, 0, -(double)9.81f};
    const double *R1 = s.Rwb + 9 * k1, *R2 = s.Rwb + 9 * k2;
    double A[9], B[9];
    double R1t[9];
    tr3(R1, R1t);
    double dRt[9];
    tr3(dR, dRt);
    mm3(dRt, R1t, A);
    mm3(A, R2, B);
    if (eR_out)
        for (int q = 0; q < 9; ++q) eR_out[q] = B[q];
    log_so3(B, e);
    double t[3];
    for (int q = 0; q < 3; ++q) t[q] = s.vel[3 * k2 + q] - s.vel[3 * k1 + q] - g[q] * dt;
    double ev[3];
    mtv3(R1, t, ev);
    for (int q = 0; q < 3; ++q) e[3 + q] = ev[q] - dV[q];
    for (int q = 0; q < 3; ++q)
        t[q] = s.twb[3 * k2 + q] - s.twb[3 * k1 + q] - s.vel[3 * k1 + q] * dt - g[q] * dt * dt / 2;
    mtv3(R1, t, ev);
    for (int q = 0; q < 3; ++q) e[6 + q] = ev[q] - dP[q];
}

__device__ void inv_right_jac(const double *v, double *J) {
    const double d2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double d = sqrt(d2);
    if (d < 1e-5) {
        for (int q = 0; q < 9; ++q) J[q] = (q % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double W[9], WW[9];
    hat3(v, W);
    mm3(W, W, WW);
    double sd, cd;
    sincos_d(d, sd, cd);
    const double k = 1.0 / d2 - (1.0 + cd) / (2.0 * d * sd);
    for (int q = 0; q < 9; ++q) J[q] = ((q % 4 == 0) ? 1.0 : 0.0) + W[q] / 2 + WW[q] * k;
}
__device__ void right_jac(const double *v, double *J) {
    const double d2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double d = sqrt(d2);
    if (d < 1e-5) {
        for (int q = 0; q < 9; ++q) J[q] = (q % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double W[9], WW[9];
    hat3(v, W);
    mm3(W, W, WW);
    double sd, cd;
    sincos_d(d, sd, cd);
    for (int q = 0; q < 9; ++q) J[q] = ((q % 4 == 0) ? 1.0 : 0.0) - W[q] * (1.0 - cd) / d2 + WW[q] * (d - sd) / (d2 * d);
}

// EdgeInertial::linearizeOplus (G2oTypes.cc:533-599): J [9][24], columns P1(6) V1 G1 A1 P2(6) V2
__device__ void imu_jacobian(const State &s, const Imu &I, int i, double *J) {
    const int k1 = I.kf1[i], k2 = I.kf2[i];
    const float *p = I.pre + (size_t)i * kPF;
    float b1[6];
    for (int q = 0; q < 3; ++q) b1[q] = (float)s.ba[3 * k1 + q], b1[3 + q] = (float)s.bg[3 * k1 + q];
    const float dbgf[3] = {b1[3] - p[PreView::b + 3], b1[4] - p[PreView::b + 4], b1[5] - p[PreView::b + 5]};
    const double dbg[3] = {(double)dbgf[0], (double)dbgf[1], (double)dbgf[2]};
    const double *Rwb1 = s.Rwb + 9 * k1, *Rwb2 = s.Rwb + 9 * k2;
    double Rbw1[9];
    tr3(Rwb1, Rbw1);
    double dR[9], dRt[9], t1[9], eR[9], er[3], invJr[9];
    delta_rot(p, b1, dR);
    tr3(dR, dRt);
    mm3(dRt, Rbw1, t1);
    mm3(t1, Rwb2, eR);
    log_so3(eR, er);
    inv_right_jac(er, invJr);
    double JRg[9], JVg[9], JPg[9], JVa[9], JPa[9];
    for (int q = 0; q < 9; ++q) {
        JRg[q] = p[PreView::JRg + q], JVg[q] = p[PreView::JVg + q], JPg[q] = p[PreView::JPg + q];
        JVa[q] = p[PreView::JVa + q], JPa[q] = p[PreView::JPa + q];
    }
    const double dt = (double)p[PreView::dT];
    const double g[3] = {0, 0, -(double)9.81f};
    for (int q = 0; q < 216; ++q) J[q] = 0;
    auto put = [&](int r0, int c0, const double *B, double sgn) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) J[(r0 + r) * 24 + c0 + c] = sgn * B[3 * r + c];
    };
    double R2t[9], A[9], B[9], W[9], v[3], w[3];
    tr3(Rwb2, R2t);
    mm3(invJr, R2t, A);
    mm3(A, Rwb1, B);
    put(0, 0, B, -1.0);
    for (int q = 0; q < 3; ++q) v[q] = s.vel[3 * k2 + q] - s.vel[3 * k1 + q] - g[q] * dt;
    mv3(Rbw1, v, w);
    hat3(w, W);
    put(3, 0, W, 1.0);
    for (int q = 0; q < 3; ++q)
        v[q] = s.twb[3 * k2 + q] - s.twb[3 * k1 + q] - s.vel[3 * k1 + q] * dt - 0.5 * g[q] * dt * dt;
    mv3(Rbw1, v, w);
    hat3(w, W);
    put(6, 0, W, 1.0);
    for (int q = 0; q < 3; ++q) J[(6 + q) * 24 + 3 + q] = -1.0;
    put(3, 6, Rbw1, -1.0);
    put(6, 6, Rbw1, -dt);
    double eRt[9], Jg[9], RJ[9], w3[3];
    tr3(eR, eRt);
    mv3(JRg, dbg, w3);
    right_jac(w3, RJ);
    mm3(invJr, eRt, A);
    mm3(A, RJ, B);
    mm3(B, JRg, Jg);
    put(0, 9, Jg, -1.0);
    put(3, 9, JVg, -1.0);
    put(6, 9, JPg, -1.0);
    put(3, 12, JVa, -1.0);
    put(6, 12, JPa, -1.0);
    put(0, 15, invJr, 1.0);
    mm3(Rbw1, Rwb2, A);
    put(6, 18, A, 1.0);
    put(3, 21, Rbw1, 1.0);
}

// EdgeInertial::linearizeOplus (G2oTypes.cc:533-599) from the rotation error the error pass cached (eR = dR^T Rbw1
// Rwb2, er = LogSO3(eR): the same values imu_jacobian recomputes), spread over a block's threads: thread 0 forms
// invJr = InverseRightJacobianSO3(er) and the blocks that use it, thread 1 RightJacobianSO3(JRg dbg), threads 2..9
// the blocks of the velocity / position rows; J [9][24] in shared memory, zeroed by the caller.  Same arithmetic,
// entry for entry, as imu_jacobian.
__device__ void imu_jacobian_par(const State &s, const Imu &I, int i, const double *eR, const double *er, double *J,
                                 double *RJ) {
    const int tid = threadIdx.x;
    const int k1 = I.kf1[i], k2 = I.kf2[i];
    const float *p = I.pre + (size_t)i * kPF;
    const double *Rwb1 = s.Rwb + 9 * k1, *Rwb2 = s.Rwb + 9 * k2;
    auto put = [&](int r0, int c0, const double *B, double sgn) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) J[(r0 + r) * 24 + c0 + c] = sgn * B[3 * r + c];
    };
    const double dt = (double)p[PreView::dT];
    const double g[3] = {0, 0, -(double)9.81f};
    double Rbw1[9];
    tr3(Rwb1, Rbw1);
    if (tid == 1) {
        float b1[6];
        for (int q = 0; q < 3; ++q) b1[q] = (float)s.ba[3 * k1 + q], b1[3 + q] = (float)s.bg[3 * k1 + q];
        const float dbgf[3] = {b1[3] - p[PreView::b + 3], b1[4] - p[PreView::b + 4], b1[5] - p[PreView::b + 5]};
        const double dbg[3] = {(double)dbgf[0], (double)dbgf[1], (double)dbgf[2]};
        double JRg[9], w3[3];
        for (int q = 0; q < 9; ++q) JRg[q] = p[PreView::JRg + q];
        mv3(JRg, dbg, w3);
        right_jac(w3, RJ);
    } else if (tid == 2) {
        double v[3], w[3], W[9];
        for (int q = 0; q < 3; ++q) v[q] = s.vel[3 * k2 + q] - s.vel[3 * k1 + q] - g[q] * dt;
        mv3(Rbw1, v, w);
        hat3(w, W);
        put(3, 0, W, 1.0);
    } else if (tid == 3) {
        double v[3], w[3], W[9];
        for (int q = 0; q < 3; ++q)
            v[q] = s.twb[3 * k2 + q] - s.twb[3 * k1 + q] - s.vel[3 * k1 + q] * dt - 0.5 * g[q] * dt * dt;
        mv3(Rbw1, v, w);
        hat3(w, W);
        put(6, 0, W, 1.0);
    } else if (tid == 4) {
        for (int q = 0; q < 3; ++q) J[(6 + q) * 24 + 3 + q] = -1.0;
        put(3, 6, Rbw1, -1.0);
        put(3, 21, Rbw1, 1.0);
    } else if (tid == 5) {
        put(6, 6, Rbw1, -dt);
    } else if (tid == 6) {
        double B[9];
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JVg + q];
        put(3, 9, B, -1.0);
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JVa + q];
        put(3, 12, B, -1.0);
    } else if (tid == 7) {
        double B[9];
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JPg + q];
        put(6, 9, B, -1.0);
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JPa + q];
        put(6, 12, B, -1.0);
    } else if (tid == 8) {
        double A[9];
        mm3(Rbw1, Rwb2, A);
        put(6, 18, A, 1.0);
    }
    double invJr[9];
    if (tid == 0) {
        inv_right_jac(er, invJr);
        double R2t[9], A[9], B[9];
        tr3(Rwb2, R2t);
        mm3(invJr, R2t, A);
        mm3(A, Rwb1, B);
        put(0, 0, B, -1.0);
        put(0, 15, invJr, 1.0);
    }
    __syncthreads();   // RJ
    if (tid == 0) {
        double eRt[9], A[9], B[9], Jg[9], JRg[9];
        for (int q = 0; q < 9; ++q) JRg[q] = p[PreView::JRg + q];
        tr3(eR, eRt);
        mm3(invJr, eRt, A);
        mm3(A, RJ, B);
        mm3(B, JRg, Jg);
        put(0, 9, Jg, -1.0);
    }
}

__device__ void exp_so3(const double *w, double *R) {   // ExpSO3 (G2oTypes.cc:802-815)
    const double x = w[0], y = w[1], z = w[2];
    const double d2 = x * x + y * y + z * z;
    const double d = sqrt(d2);
    double W[9], WW[9];
    hat3(w, W);
    mm3(W, W, WW);
    if (d < 1e-5) {
        for (int q = 0; q < 9; ++q) R[q] = ((q % 4 == 0) ? 1.0 : 0.0) + W[q] + 0.5 * WW[q];
    } else {
        double s, c;
        sincos_d(d, s, c);
        for (int q = 0; q < 9; ++q) R[q] = ((q % 4 == 0) ? 1.0 : 0.0) + W[q] * s / d + WW[q] * (1.0 - c) / d2;
    }
    polar3(R);
}

}  // namespace omv_g2o

namespace omv_g2o {

}  // namespace omv_g2o

namespace omv_g2o {

// EdgeInertial error and the Jacobian columns of its second pose / velocity vertices (4, 5: columns
// 15-23 of the 9x24 layout; the only free ones when the first keyframe's vertices are fixed, as in
// PoseInertialOptimizationLastKeyFrame).  Same arithmetic as imu_error + imu_jacobian; other entries
// of J are left untouched.
__device__ inline void imu_error_jac_p2v2(const State &s, const Imu &I, int i, double *e, double *J) {
    imu_error(s, I, i, e);
    const int k1 = I.kf1[i], k2 = I.kf2[i];
    double Rbw1[9], A[9], invJr[9];
    tr3(s.Rwb + 9 * k1, Rbw1);
    inv_right_jac(e, invJr);
    mm3(Rbw1, s.Rwb + 9 * k2, A);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            J[r * 24 + 15 + c] = invJr[3 * r + c];
            J[(6 + r) * 24 + 18 + c] = A[3 * r + c];
            J[(3 + r) * 24 + 21 + c] = Rbw1[3 * r + c];
        }
}

// Fixed-order wavefront sum of N <= 64 per-lane values at once (a transposing butterfly): at distance d = 32 .. 1
// each lane keeps one half of its current values -- the lower half when (lane & d) == 0 -- adds the partner's
// copy of that half, and sends the other; after six steps lane l holds the wave total of value l (l < N), in an
// order fixed by the lane numbering.  63 shuffles instead of the 6 N of N separate xor trees.
template <int N>
__device__ __forceinline__ double wave_transpose_sum(const double (&v)[N], int lane) {
    static_assert(N <= 64, "at most one value per lane");
    double a[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {   // d = 32: values j and 32 + j
        const double lo = j < N ? v[j] : 0.0, hi = j + 32 < N ? v[j + 32] : 0.0;
        const bool up = (lane & 32) != 0;
        a[j] = (up ? hi : lo) + __shfl_xor(up ? lo : hi, 32, 64);
    }
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) {
        const bool up = (lane & d) != 0;
#pragma unroll
        for (int j = 0; j < d; ++j) {
            const double lo = a[j], hi = a[j + d];
            a[j] = (up ? hi : lo) + __shfl_xor(up ? lo : hi, d, 64);
        }
    }
    return a[0];
}

// Lane l's value of x to every lane (v_readlane on both halves; l wave-uniform).
__device__ __forceinline__ double lane_f64(double x, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Cyclic Jacobi eigen-decomposition of the symmetric N x N matrix A (row-major, LDS) over one wavefront:
// A is driven to diag(w) in place, V (LDS, N x N) receives the eigenvectors (columns).  Per element the same
// operations in the same order as the oracle's sym_eig (ba_oracle.cpp).  Every lane of the wave must call it.
template <int N>
__device__ inline void sym_eig_wave(double *A, double *V, int lane) {
    static_assert(N <= 64, "one row per lane");
    for (int q = lane; q < N * N; q += 64) V[q] = (q / N == q % N) ? 1.0 : 0.0;
    wave_lds_sync();
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0, dg = 0;   // converged: off-diagonal mass below 1e-32 of the diagonal's
        for (int p = 0; p < N; ++p) {
            dg += A[p * N + p] * A[p * N + p];
            for (int q = p + 1; q < N; ++q) off += A[p * N + q] * A[p * N + q];
        }
        if (off <= 1e-32 * dg || off < 1e-300) break;
        for (int p = 0; p < N; ++p)
            for (int q = p + 1; q < N; ++q) {
                const double apq = A[p * N + q];
                if (apq == 0) continue;
                const double th = (A[q * N + q] - A[p * N + p]) / (2 * apq);
                const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
                const double c = 1 / sqrt(t * t + 1), s = t * c;
                wave_lds_sync();
                if (lane < N) {
                    const double akp = A[lane * N + p], akq = A[lane * N + q];
                    A[lane * N + p] = c * akp - s * akq, A[lane * N + q] = s * akp + c * akq;
                }
                wave_lds_sync();
                if (lane < N) {
                    const double apk = A[p * N + lane], aqk = A[q * N + lane];
                    A[p * N + lane] = c * apk - s * aqk, A[q * N + lane] = s * apk + c * aqk;
                    const double vkp = V[lane * N + p], vkq = V[lane * N + q];
                    V[lane * N + p] = c * vkp - s * vkq, V[lane * N + q] = s * vkp + c * vkq;
                }
                wave_lds_sync();
            }
    }
}

// The same eigen-decomposition in parallel order: per sweep NP - 1 rounds of a round-robin tournament over the
// (even-padded) indices, each round NP / 2 disjoint rotations at once (angles from the round-start matrix, by the
// same formula as sym_eig_wave), then all their column updates (A and V), then all their row updates -- a
// rotation order different from the cyclic one, so the result differs from sym_eig_wave's by rounding only.
// cs / pq: LDS scratch [NP] doubles / [NP] ints.  Every lane of the wave must call it.
template <int N>
__device__ inline void sym_eig_wave_par(double *A, double *V, double *cs, int *pq, int lane) {
    static_assert(N <= 64, "one row per lane");
    constexpr int NP = (N + 1) & ~1, HP = NP / 2;
    for (int q = lane; q < N * N; q += 64) V[q] = (q / N == q % N) ? 1.0 : 0.0;
    wave_lds_sync();
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0, dg = 0;   // converged: off-diagonal mass below 1e-32 of the diagonal's
        for (int e = lane; e < N * N; e += 64) {
            const int r = e / N, c = e - (e / N) * N;
            const double v = A[e];
            if (r == c) dg += v * v;
            else if (c > r) off += v * v;
        }
        for (int d = 32; d >= 1; d >>= 1) off += __shfl_xor(off, d, 64), dg += __shfl_xor(dg, d, 64);
        if (off <= 1e-32 * dg || off < 1e-300) break;
        for (int round = 0; round < NP - 1; ++round) {
            if (lane < HP) {
                const int a = lane == 0 ? 0 : (round + lane - 1) % (NP - 1) + 1;
                const int bpos = NP - 1 - lane, b = (round + bpos - 1) % (NP - 1) + 1;
                const int p = min(a, b), q = max(a, b);
                double c = 1.0, sn = 0.0;
                int qq = N;   // dummy pair (padding index) or a zero entry: no rotation
                if (q < N) {
                    const double apq = A[p * N + q];
                    if (apq != 0) {
                        const double th = (A[q * N + q] - A[p * N + p]) / (2 * apq);
                        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
                        c = 1 / sqrt(t * t + 1), sn = t * c;
                        qq = q;
                    }
                }
                cs[2 * lane] = c, cs[2 * lane + 1] = sn, pq[2 * lane] = p, pq[2 * lane + 1] = qq;
            }
            wave_lds_sync();
            for (int tk = lane; tk < HP * N; tk += 64) {   // columns p, q of A and V
                const int i = tk / N, k = tk - (tk / N) * N;
                const int p = pq[2 * i], q = pq[2 * i + 1];
                if (q >= N) continue;
                const double c = cs[2 * i], sn = cs[2 * i + 1];
                const double akp = A[k * N + p], akq = A[k * N + q];
                A[k * N + p] = c * akp - sn * akq, A[k * N + q] = sn * akp + c * akq;
                const double vkp = V[k * N + p], vkq = V[k * N + q];
                V[k * N + p] = c * vkp - sn * vkq, V[k * N + q] = sn * vkp + c * vkq;
            }
            wave_lds_sync();
            for (int tk = lane; tk < HP * N; tk += 64) {   // rows p, q of A
                const int i = tk / N, k = tk - (tk / N) * N;
                const int p = pq[2 * i], q = pq[2 * i + 1];
                if (q >= N) continue;
                const double c = cs[2 * i], sn = cs[2 * i + 1];
                const double apk = A[p * N + k], aqk = A[q * N + k];
                A[p * N + k] = c * apk - sn * aqk, A[q * N + k] = sn * apk + c * aqk;
            }
            wave_lds_sync();
        }
    }
}

// LDL^T without pivoting of the symmetric N x N A - shift I (LDS, row-major), one wavefront (lane = row, the row in
// registers, v_readlane broadcasts of the pivot row).  True iff every pivot is > 0; then, when L is given, the factor
// is stored there (strict lower triangle L, D on the diagonal).  All lanes get the same verdict.
template <int N>
__device__ inline bool ldl_nopiv_wave(const double *A, double shift, double *L, int lane) {
    static_assert(N <= 32, "rows on lanes 0..31");
    const bool in = lane < N;
    double r[N];
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? A[lane * N + j] - (j == lane ? shift : 0.0) : 0.0;
    bool pos = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double d = lane_f64(r[k], k);
        pos = pos && d > 0.0;
        const double inv = d > 0.0 ? 1.0 / d : 0.0;
        const bool below = lane > k;
        const double l = below ? r[k] * inv : 0.0;
#pragma unroll
        for (int j = k + 1; j < N; ++j) r[j] = r[j] - l * lane_f64(r[j], k);
        r[k] = below ? l : r[k];
    }
    if (pos && L && in) {
#pragma unroll
        for (int j = 0; j < N; ++j) L[lane * N + j] = r[j];
    }
    wave_lds_sync();
    return pos;
}

// X = A^-1 (N x N, LDS) from ldl_nopiv_wave's factor L: lane m solves column m (L D L^T x = e_m), the factor read by
// broadcast LDS loads.
template <int N>
__device__ inline void ldl_inverse_wave(const double *L, double *X, int lane) {
    if (lane < N) {
        double y[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double t = i == lane ? 1.0 : 0.0;
#pragma unroll
            for (int k = 0; k < i; ++k) t -= L[i * N + k] * y[k];
            y[i] = t;
            asm volatile("" ::: "memory");   // one row of L live at a time (hoisting all 225 loads spills)
        }
#pragma unroll
        for (int i = 0; i < N; ++i) y[i] = y[i] / L[i * N + i];
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {
            double t = y[i];
#pragma unroll
            for (int k = i + 1; k < N; ++k) t -= L[k * N + i] * y[k];
            y[i] = t;
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < N; ++i) X[i * N + lane] = y[i];
    }
    wave_lds_sync();
}

// Largest |diagonal| of the N x N A (wave-uniform).
template <int N>
__device__ inline double max_abs_diag(const double *A, int lane) {
    double m = lane < N ? fabs(A[lane * (N + 1)]) : 0.0;
    for (int d = 32; d >= 1; d >>= 1) m = fmax(m, __shfl_xor(m, d, 64));
    return m;
}

// P = pinv(A) of the symmetric 15 x 15 A (LDS; overwritten) with eigenvalues |w| <= 1e-6 dropped (Marginalize,
// Optimizer.cc:3388-3455), one wavefront.  When A - tau I factors with positive pivots (tau = 1e-6 plus a margin for
// the factorisation's rounding), every eigenvalue exceeds 1e-6 and pinv(A) = A^-1: LDL^T and 15 triangular solves.
// Otherwise the Jacobi eigen-decomposition and V diag(1/w over |w| > 1e-6) V^T.  The two agree up to rounding.
// V: LDS [225] scratch; cs / pq: sym_eig_wave_par's scratch.
__device__ __attribute__((noinline)) void pinv15_wave(double *A, double *V, double *P, double *cs, int *pq, int lane) {
    const double tau = 1e-6 + 1e-12 * max_abs_diag<15>(A, lane);
    if (ldl_nopiv_wave<15>(A, tau, nullptr, lane) && ldl_nopiv_wave<15>(A, 0.0, V, lane)) {
        ldl_inverse_wave<15>(V, P, lane);
        return;
    }
    sym_eig_wave_par<15>(A, V, cs, pq, lane);
    for (int q = lane; q < 225; q += 64) {
        const int r = q / 15, c = q % 15;
        double s = 0;
        for (int k = 0; k < 15; ++k) {
            const double w = A[k * 16];
            s += V[r * 15 + k] * (fabs(w) > 1e-6 ? 1.0 / w : 0.0) * V[c * 15 + k];
        }
        P[q] = s;
    }
    wave_lds_sync();
}

// EdgePriorPoseImu::computeError / linearizeOplus (G2oTypes.cc:758-785) at the vertex state (R, t, v, bg, ba)
// against the ConstraintPoseImu state pr = [Rwb 9 | twb 3 | vwb 3 | bg 3 | ba 3]; J (15x15 over pose 6,
// v 3, bg 3, ba 3) may be null.
__device__ inline void prior_error_jac(const double *pr, const double *R, const double *t, const double *v,
                                       const double *bg, const double *ba, double *e, double *J) {
    double RR[9], d[3], et[3];
    mtm3(pr, R, RR);
    log_so3(RR, e);
    for (int q = 0; q < 3; ++q) d[q] = t[q] - pr[9 + q];
    mtv3(pr, d, et);
    for (int q = 0; q < 3; ++q) {
        e[3 + q] = et[q];
        e[6 + q] = v[q] - pr[12 + q];
        e[9 + q] = bg[q] - pr[15 + q];
        e[12 + q] = ba[q] - pr[18 + q];
    }
    if (!J) return;
    double iJ[9];
    inv_right_jac(e, iJ);
    for (int q = 0; q < 225; ++q) J[q] = 0.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) J[r * 15 + c] = iJ[3 * r + c], J[(3 + r) * 15 + 3 + c] = RR[3 * r + c];
    for (int q = 6; q < 15; ++q) J[q * 15 + q] = 1.0;
}

// EdgeInertial's information (ctor, G2oTypes.cc:486-495): Info = C[0:9,0:9]^-1, symmetrised, projected onto
// its non-negative eigen-space (eigenvalues < 1e-12 zeroed) — Gauss-Jordan with partial pivoting and cyclic
// Jacobi, per element the same operations in the same order as lba.hip's host path and the oracle, spread
// over one wavefront (lane = row / column index).  sm: 243 doubles of LDS (A | I | V) + 10 (kPar: the parallel-order
// Jacobi's scratch).  kPar: sym_eig_wave_par instead of the cyclic order (equal up to rounding; the pose path, where
// this runs per call on the latency chain).  Every lane of the wave must call it.
template <bool kPar = false>
__device__ inline void inertial_info9_wave(const float *C15, double *out, double *sm, int lane) {
    double *A = sm, *I = sm + 81, *V = sm + 162;
    for (int q = lane; q < 81; q += 64) {
        const int r = q / 9, c = q % 9;
        A[q] = (double)C15[r * 15 + c], I[q] = r == c ? 1.0 : 0.0, V[q] = r == c ? 1.0 : 0.0;
    }
    wave_lds_sync();
    for (int c = 0; c < 9; ++c) {   // Gauss-Jordan, partial pivoting
        int p = c;
        for (int r = c + 1; r < 9; ++r)
            if (fabs(A[r * 9 + c]) > fabs(A[p * 9 + c])) p = r;
        wave_lds_sync();
        if (p != c && lane < 9) {
            double t = A[p * 9 + lane];
            A[p * 9 + lane] = A[c * 9 + lane], A[c * 9 + lane] = t;
            t = I[p * 9 + lane];
            I[p * 9 + lane] = I[c * 9 + lane], I[c * 9 + lane] = t;
        }
        wave_lds_sync();
        const double d = A[c * 9 + c];
        wave_lds_sync();
        if (lane < 9) A[c * 9 + lane] /= d, I[c * 9 + lane] /= d;
        wave_lds_sync();
        if (lane < 9 && lane != c && A[lane * 9 + c] != 0) {
            const double f = A[lane * 9 + c];
            for (int k = 0; k < 9; ++k) A[lane * 9 + k] -= f * A[c * 9 + k], I[lane * 9 + k] -= f * I[c * 9 + k];
        }
        wave_lds_sync();
    }
    for (int q = lane; q < 81; q += 64) {   // symmetrise: (I + I^T) / 2 in the upper-then-lower write order
        const int r = q / 9, c = q % 9;
        A[q] = r < c ? (I[r * 9 + c] + I[c * 9 + r]) / 2 : (r > c ? (I[c * 9 + r] + I[r * 9 + c]) / 2 : I[q]);
    }
    wave_lds_sync();
    for (int q = lane; q < 81; q += 64) I[q] = A[q];
    wave_lds_sync();
    if constexpr (kPar) {
        // every eigenvalue above the 1e-12 cut (I - tau I factors with positive pivots): the projection is I itself
        const double tau = 1e-12 + 1e-12 * max_abs_diag<9>(I, lane);
        if (ldl_nopiv_wave<9>(I, tau, nullptr, lane)) {
            for (int q = lane; q < 81; q += 64) out[q] = I[q];
            return;
        }
        sym_eig_wave_par<9>(I, V, sm + 243, reinterpret_cast<int *>(sm + 253), lane);
    } else {
        sym_eig_wave<9>(I, V, lane);
    }
    for (int q = lane; q < 81; q += 64) {
        const int r = q / 9, c = q % 9;
        double s = 0;
        for (int k = 0; k < 9; ++k) {
            const double wk = I[k * 9 + k] < 1e-12 ? 0.0 : I[k * 9 + k];
            s += V[r * 9 + k] * wk * V[c * 9 + k];
        }
        out[q] = s;
    }
}

// Eigen::LDLT<MatrixXd> (lower, diagonal pivoting; ldlt_inplace::unblocked) + LDLT::_solve_impl with the
// D pseudo-inverse below DBL_MIN, spread over one wavefront (lane = row); per element the same operations
// in the same order as the oracle's ldlt_pivot_solve.  Returns isPositive().  A (N x N,
// row-major), b, x and the scratch t[2N] live in LDS; every lane of the wave must call it.
template <int N>
__device__ inline bool ldlt_pivot_solve_wave(double *A, const double *b, double *x, double *t, int *tr, int lane) {
    static_assert(N <= 64, "one row per lane");
    int sign = 0;
    for (int k = 0; k < N; ++k) {
        // largest |diagonal| in the trailing corner, first index on ties (Eigen maxCoeff)
        double v = (lane >= k && lane < N) ? fabs(A[lane * N + lane]) : -1.0;
        int idx = lane;
        for (int d = 1; d < 64; d <<= 1) {
            const double ov = __shfl_xor(v, d, 64);
            const int oi = __shfl_xor(idx, d, 64);
            if (ov > v || (ov == v && oi < idx)) v = ov, idx = oi;
        }
        const int big = idx;
        if (lane == 0) tr[k] = big;
        if (k != big) {
            if (lane < k) {
                const double u = A[k * N + lane];
                A[k * N + lane] = A[big * N + lane], A[big * N + lane] = u;
            }
            if (lane > big && lane < N) {
                const double u = A[lane * N + k];
                A[lane * N + k] = A[lane * N + big], A[lane * N + big] = u;
            }
            if (lane > k && lane < big) {
                const double u = A[lane * N + k];
                A[lane * N + k] = A[big * N + lane], A[big * N + lane] = u;
            }
            if (lane == 0) {
                const double u = A[k * N + k];
                A[k * N + k] = A[big * N + big], A[big * N + big] = u;
            }
        }
        wave_lds_sync();
        if (k > 0) {
            if (lane < k) t[lane] = A[lane * N + lane] * A[k * N + lane];
            wave_lds_sync();
            if (lane >= k && lane < N) {   // lane k: the pivot, lanes > k: the column below it
                double s = 0;
                for (int j = 0; j < k; ++j) s += A[lane * N + j] * t[j];
                A[lane * N + k] -= s;
            }
            wave_lds_sync();
        }
        const double akk = A[k * N + k];
        const bool valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            sign = 0;
            if (lane < N) tr[lane] = lane;
            wave_lds_sync();
            break;
        }
        if (valid && lane > k && lane < N) A[lane * N + k] /= akk;
        if (sign == 1) {
            if (akk < 0) sign = 3;
        } else if (sign == 2) {
            if (akk > 0) sign = 3;
        } else if (sign == 0) {
            if (akk > 0) sign = 1;
            else if (akk < 0) sign = 2;
        }
        wave_lds_sync();
    }
    if (!(sign == 1 || sign == 0)) return false;
    // y = P b; L y' = y (column-oriented); D pseudo-inverse; L^T x = y'' (column-oriented, j descending)
    double *y = t;
    if (lane == 0) {
        for (int i = 0; i < N; ++i) y[i] = b[i];
        for (int k = 0; k < N; ++k) {
            const double u = y[k];
            y[k] = y[tr[k]], y[tr[k]] = u;
        }
    }
    wave_lds_sync();
    for (int j = 0; j < N; ++j) {
        const double yj = y[j];
        if (lane > j && lane < N) y[lane] -= A[lane * N + j] * yj;
        wave_lds_sync();
    }
    if (lane < N) y[lane] = fabs(A[lane * N + lane]) > 2.2250738585072014e-308 ? y[lane] / A[lane * N + lane] : 0.0;
    wave_lds_sync();
    for (int j = N - 1; j >= 0; --j) {
        const double yj = y[j];
        if (lane < j) y[lane] -= A[j * N + lane] * yj;
        wave_lds_sync();
    }
    if (lane == 0) {
        for (int k = N - 1; k >= 0; --k) {
            const double u = y[k];
            y[k] = y[tr[k]], y[tr[k]] = u;
        }
        for (int i = 0; i < N; ++i) x[i] = y[i];
    }
    wave_lds_sync();
    return true;
}

}  // namespace omv_g2o
