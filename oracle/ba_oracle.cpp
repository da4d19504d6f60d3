// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for the LocalInertialBA inner loop. Never linked into the
// product path.
//
// Scalar restatement (double, single thread like g2o with OpenMP off, Thirdparty/g2o/CMakeLists.txt:48) of
//   ImuCamPose::Update / isDepthPositive        src/G2oTypes.cc:192-235
//   EdgeMono computeError / linearizeOplus      include/G2oTypes.h:293-299, src/G2oTypes.cc:356-380
//   EdgeInertial ctor / computeError / lin.     src/G2oTypes.cc:478-599
//   EdgeGyroRW / EdgeAccRW                      include/G2oTypes.h:567-633
//   ExpSO3 / LogSO3 / (Inverse)RightJacobianSO3 src/G2oTypes.cc:797-860
//   IMU::Preintegrated::GetDelta*               src/ImuTypes.cc:277-309 (float, Sophus SO3f::exp)
//   KannalaBrandt8::project(Vector3d) / projectJac  src/CameraModels/KannalaBrandt8.cpp:28-46, 128-158
//   RobustKernelHuber::robustify                Thirdparty/g2o/g2o/core/robust_kernel_impl.cpp:78-91
//   constructQuadraticForm (binary / multi)     base_binary_edge.hpp:55-116, base_multi_edge.hpp:36-48,171+
//   BlockSolver::solve / setLambda (Schur)      block_solver.hpp:353-486, 563-604
//   OptimizationAlgorithmLevenberg::solve        optimization_algorithm_levenberg.cpp:61-169
//   LocalInertialBA: err / optimize / outlier test / FAIL guard   src/Optimizer.cc:3270-3321
// Linear-algebra kernels the reference takes from Eigen (absent here) are replaced by textbook
// equivalents: 3x3 inverse by cofactors, 9x9 inverse by Gauss-Jordan with partial pivoting, symmetric
// eigen-decomposition by cyclic Jacobi, NormalizeRotation (JacobiSVD U*V^T) by the polar factor
// (Newton iteration), SimplicialLDLT by a dense LDL^T without pivoting.  These agree with the Eigen
// results to rounding, so BA parity is tolerance-based (north star: 1e-5 relative).
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <vector>

#include "../include/omv.h"

namespace {

// ---- glibc atan2f (fdlibm e_atan2f.c / s_atanf.c), float, no contraction ---------------------------
// KannalaBrandt8::project(Vector3d) evaluates theta and psi with atan2f (:30-31); the host libm is the
// reference here, so the oracle simply calls it.

// ---- small fixed-size linear algebra (row-major) -------------------------------------------------
struct M3 {
    double m[9];
    double &operator()(int r, int c) { return m[3 * r + c]; }
    double operator()(int r, int c) const { return m[3 * r + c]; }
};
struct V3 {
    double v[3];
    double &operator[](int i) { return v[i]; }
    double operator[](int i) const { return v[i]; }
};
M3 eye() {
    M3 r{};
    r(0, 0) = r(1, 1) = r(2, 2) = 1;
    return r;
}
M3 mul(const M3 &a, const M3 &b) {
    M3 r{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r(i, j) = a(i, 0) * b(0, j) + a(i, 1) * b(1, j) + a(i, 2) * b(2, j);
    return r;
}
V3 mul(const M3 &a, const V3 &x) {
    V3 r;
    for (int i = 0; i < 3; ++i) r[i] = a(i, 0) * x[0] + a(i, 1) * x[1] + a(i, 2) * x[2];
    return r;
}
M3 tr(const M3 &a) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r(i, j) = a(j, i);
    return r;
}
M3 add(const M3 &a, const M3 &b) {
    M3 r;
    for (int k = 0; k < 9; ++k) r.m[k] = a.m[k] + b.m[k];
    return r;
}
M3 scale(const M3 &a, double s) {
    M3 r;
    for (int k = 0; k < 9; ++k) r.m[k] = a.m[k] * s;
    return r;
}
V3 add(const V3 &a, const V3 &b) { return V3{{a[0] + b[0], a[1] + b[1], a[2] + b[2]}}; }
V3 sub(const V3 &a, const V3 &b) { return V3{{a[0] - b[0], a[1] - b[1], a[2] - b[2]}}; }
V3 scale(const V3 &a, double s) { return V3{{a[0] * s, a[1] * s, a[2] * s}}; }
M3 hat(const V3 &w) {
    M3 r{};
    r(0, 1) = -w[2], r(0, 2) = w[1], r(1, 0) = w[2], r(1, 2) = -w[0], r(2, 0) = -w[1], r(2, 1) = w[0];
    return r;
}
M3 inv3(const M3 &a) {   // cofactors / determinant
    M3 c;
    c(0, 0) = a(1, 1) * a(2, 2) - a(1, 2) * a(2, 1);
    c(0, 1) = a(0, 2) * a(2, 1) - a(0, 1) * a(2, 2);
    c(0, 2) = a(0, 1) * a(1, 2) - a(0, 2) * a(1, 1);
    c(1, 0) = a(1, 2) * a(2, 0) - a(1, 0) * a(2, 2);
    c(1, 1) = a(0, 0) * a(2, 2) - a(0, 2) * a(2, 0);
    c(1, 2) = a(0, 2) * a(1, 0) - a(0, 0) * a(1, 2);
    c(2, 0) = a(1, 0) * a(2, 1) - a(1, 1) * a(2, 0);
    c(2, 1) = a(0, 1) * a(2, 0) - a(0, 0) * a(2, 1);
    c(2, 2) = a(0, 0) * a(1, 1) - a(0, 1) * a(1, 0);
    const double det = a(0, 0) * c(0, 0) + a(0, 1) * c(1, 0) + a(0, 2) * c(2, 0);
    return scale(c, 1.0 / det);
}

// Polar factor (NormalizeRotation's U*V^T) by Newton iteration X <- (X + X^-T) / 2.
template <typename T>
void polar3(T *r) {
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
        const T det = r[0] * c[0] + r[1] * c[1] + r[2] * c[2];   // cofactor matrix = det * inv^T
        const T id = T(1) / det;
        T diff = 0;
        for (int k = 0; k < 9; ++k) {
            const T nv = (r[k] + c[k] * id) * T(0.5);
            diff = std::max(diff, (T)std::fabs(nv - r[k]));
            r[k] = nv;
        }
        if (diff <= (sizeof(T) == 4 ? T(2.5e-7) : T(5e-16))) break;   // within ~2 ulp of a fixed point
    }
}

M3 normalize_rotation(M3 r) {
    polar3(r.m);
    return r;
}

// ---- SO3 helpers (src/G2oTypes.cc:797-860) -----------------------------------------------------------
M3 expSO3(double x, double y, double z) {
    const double d2 = x * x + y * y + z * z;
    const double d = std::sqrt(d2);
    const M3 W = hat(V3{{x, y, z}});
    M3 res;
    if (d < 1e-5) {
        const M3 WW = mul(W, W);
        for (int k = 0; k < 9; ++k) res.m[k] = eye().m[k] + W.m[k] + 0.5 * WW.m[k];
    } else {
        const M3 WW = mul(W, W);
        const double s = std::sin(d), c = std::cos(d);
        for (int k = 0; k < 9; ++k) res.m[k] = eye().m[k] + W.m[k] * s / d + WW.m[k] * (1.0 - c) / d2;
    }
    return normalize_rotation(res);
}
V3 logSO3(const M3 &R) {
    const double t = R(0, 0) + R(1, 1) + R(2, 2);
    V3 w{{(R(2, 1) - R(1, 2)) / 2, (R(0, 2) - R(2, 0)) / 2, (R(1, 0) - R(0, 1)) / 2}};
    const double costheta = (t - 1.0) * 0.5f;
    if (costheta > 1 || costheta < -1) return w;
    const double theta = std::acos(costheta);
    const double s = std::sin(theta);
    if (std::fabs(s) < 1e-5) return w;
    return V3{{theta * w[0] / s, theta * w[1] / s, theta * w[2] / s}};
}
M3 invRightJ(const V3 &v) {
    const double x = v[0], y = v[1], z = v[2];
    const double d2 = x * x + y * y + z * z;
    const double d = std::sqrt(d2);
    const M3 W = hat(v);
    if (d < 1e-5) return eye();
    const M3 WW = mul(W, W);
    const double k = 1.0 / d2 - (1.0 + std::cos(d)) / (2.0 * d * std::sin(d));
    M3 r;
    for (int q = 0; q < 9; ++q) r.m[q] = eye().m[q] + W.m[q] / 2 + WW.m[q] * k;
    return r;
}
M3 rightJ(const V3 &v) {
    const double x = v[0], y = v[1], z = v[2];
    const double d2 = x * x + y * y + z * z;
    const double d = std::sqrt(d2);
    const M3 W = hat(v);
    if (d < 1e-5) return eye();
    const M3 WW = mul(W, W);
    M3 r;
    for (int q = 0; q < 9; ++q)
        r.m[q] = eye().m[q] - W.m[q] * (1.0 - std::cos(d)) / d2 + WW.m[q] * (d - std::sin(d)) / (d2 * d);
    return r;
}

// ---- float preintegration getters (src/ImuTypes.cc:283-309) ----------------------------------------
struct Preint {
    float dR[9], dV[3], dP[3], JRg[9], JVg[9], JVa[9], JPg[9], JPa[9], b[6], dT, C[225];
};
constexpr size_t kPreintC = offsetof(Preint, C) / sizeof(float);   // C's offset in an OMV_PREINT_FLOATS record
void f33mul(const float *a, const float *b, float *r) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
void f33mulv(const float *a, const float *x, float *r) {
    for (int i = 0; i < 3; ++i) r[i] = a[3 * i] * x[0] + a[3 * i + 1] * x[1] + a[3 * i + 2] * x[2];
}
// Sophus::SO3f::exp(w).matrix() (sophus/so3.hpp:583-621 + Eigen Quaternion::toRotationMatrix)
void so3f_exp(const float *w, float *R) {
    const float theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    float imag, real;
    if (theta_sq < 1e-5f * 1e-5f) {
        const float t4 = theta_sq * theta_sq;
        imag = 0.5f - (float)(1.0 / 48.0) * theta_sq + (float)(1.0 / 3840.0) * t4;
        real = 1.0f - (float)(1.0 / 8.0) * theta_sq + (float)(1.0 / 384.0) * t4;
    } else {
        const float theta = std::sqrt(theta_sq);
        const float half = 0.5f * theta;
        imag = sinf(half) / theta;
        real = cosf(half);
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
// b1 = (bax bay baz bwx bwy bwz) as floats (IMU::Bias ctor)
void delta_rotation(const Preint &p, const float *b1, M3 &out) {
    const float dbg[3] = {b1[3] - p.b[3], b1[4] - p.b[4], b1[5] - p.b[5]};
    float w[3], E[9], R[9];
    f33mulv(p.JRg, dbg, w);
    so3f_exp(w, E);
    f33mul(p.dR, E, R);
    polar3(R);
    for (int k = 0; k < 9; ++k) out.m[k] = (double)R[k];
}
V3 delta_vp(const float *d, const float *Jg, const float *Ja, const Preint &p, const float *b1) {
    const float dbg[3] = {b1[3] - p.b[3], b1[4] - p.b[4], b1[5] - p.b[5]};
    const float dba[3] = {b1[0] - p.b[0], b1[1] - p.b[1], b1[2] - p.b[2]};
    float g[3], a[3];
    f33mulv(Jg, dbg, g);
    f33mulv(Ja, dba, a);
    return V3{{(double)((d[0] + g[0]) + a[0]), (double)((d[1] + g[1]) + a[1]), (double)((d[2] + g[2]) + a[2])}};
}

// ---- KannalaBrandt8 (src/CameraModels/KannalaBrandt8.cpp:28-46, 128-158) ---------------------------
void kb8_project(const float *k, const V3 &X, double &u, double &v) {
    const double x2y2 = X[0] * X[0] + X[1] * X[1];
    const double theta = atan2f(sqrtf((float)x2y2), (float)X[2]);
    const double psi = atan2f((float)X[1], (float)X[0]);
    const double t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
    const double r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9;
    u = k[0] * r * std::cos(psi) + k[2];
    v = k[1] * r * std::sin(psi) + k[3];
}
void kb8_jac(const float *k, const V3 &X, double J[6]) {   // 2x3 row-major
    const double x2 = X[0] * X[0], y2 = X[1] * X[1], z2 = X[2] * X[2];
    const double r2 = x2 + y2, r = std::sqrt(r2), r3 = r2 * r;
    const double theta = std::atan2(r, X[2]);
    const double t2 = theta * theta, t3 = t2 * theta, t4 = t2 * t2, t5 = t4 * theta, t6 = t2 * t4, t7 = t6 * theta,
                 t8 = t4 * t4, t9 = t8 * theta;
    const double f = theta + t3 * k[4] + t5 * k[5] + t7 * k[6] + t9 * k[7];
    const double fd = 1 + 3 * k[4] * t2 + 5 * k[5] * t4 + 7 * k[6] * t6 + 9 * k[7] * t8;
    J[0] = k[0] * (fd * X[2] * x2 / (r2 * (r2 + z2)) + f * y2 / r3);
    J[3] = k[1] * (fd * X[2] * X[1] * X[0] / (r2 * (r2 + z2)) - f * X[1] * X[0] / r3);
    J[1] = k[0] * (fd * X[2] * X[1] * X[0] / (r2 * (r2 + z2)) - f * X[1] * X[0] / r3);
    J[4] = k[1] * (fd * X[2] * y2 / (r2 * (r2 + z2)) + f * x2 / r3);
    J[2] = -k[0] * fd * X[0] / (r2 + z2);
    J[5] = -k[1] * fd * X[1] / (r2 + z2);
}

// ---- Pinhole (src/CameraModels/Pinhole.cpp:18-24, :55-65) ------------------------------------------------
void pinhole_project(const float *k, const V3 &X, double &u, double &v) {
    u = k[0] * X[0] / X[2] + k[2];
    v = k[1] * X[1] / X[2] + k[3];
}
void pinhole_jac(const float *k, const V3 &X, double J[6]) {
    J[0] = k[0] / X[2];
    J[1] = 0.f;
    J[2] = -k[0] * X[0] / (X[2] * X[2]);
    J[3] = 0.f;
    J[4] = k[1] / X[2];
    J[5] = -k[1] * X[1] / (X[2] * X[2]);
}
// pCamera[c]->project / projectJac by GeometricCamera type (model NULL: KannalaBrandt8)
void cam_project(const int32_t *model, int c, const float *k, const V3 &X, double &u, double &v) {
    if (model && model[c] == OMV_CAM_PINHOLE) pinhole_project(k, X, u, v);
    else kb8_project(k, X, u, v);
}
void cam_jac(const int32_t *model, int c, const float *k, const V3 &X, double J[6]) {
    if (model && model[c] == OMV_CAM_PINHOLE) pinhole_jac(k, X, J);
    else kb8_jac(k, X, J);
}

// ---- dense helpers ---------------------------------------------------------------------------------
bool invert_gj(std::vector<double> &A, int n) {   // in place, partial pivoting
    std::vector<double> I(n * n, 0.0);
    for (int i = 0; i < n; ++i) I[i * n + i] = 1;
    for (int c = 0; c < n; ++c) {
        int p = c;
        for (int r = c + 1; r < n; ++r)
            if (std::fabs(A[r * n + c]) > std::fabs(A[p * n + c])) p = r;
        if (A[p * n + c] == 0) return false;
        if (p != c)
            for (int k = 0; k < n; ++k) std::swap(A[p * n + k], A[c * n + k]), std::swap(I[p * n + k], I[c * n + k]);
        const double d = A[c * n + c];
        for (int k = 0; k < n; ++k) A[c * n + k] /= d, I[c * n + k] /= d;
        for (int r = 0; r < n; ++r)
            if (r != c) {
                const double f = A[r * n + c];
                if (f == 0) continue;
                for (int k = 0; k < n; ++k) A[r * n + k] -= f * A[c * n + k], I[r * n + k] -= f * I[c * n + k];
            }
    }
    A = I;
    return true;
}
// cyclic Jacobi eigen-decomposition of a symmetric n x n matrix: A = V diag(w) V^T
void sym_eig(std::vector<double> A, int n, std::vector<double> &w, std::vector<double> &V) {
    V.assign(n * n, 0.0);
    for (int i = 0; i < n; ++i) V[i * n + i] = 1;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0, dg = 0;   // converged: off-diagonal mass below 1e-32 of the diagonal's
        for (int p = 0; p < n; ++p) {
            dg += A[p * n + p] * A[p * n + p];
            for (int q = p + 1; q < n; ++q) off += A[p * n + q] * A[p * n + q];
        }
        if (off <= 1e-32 * dg || off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = A[p * n + q];
                if (apq == 0) continue;
                const double th = (A[q * n + q] - A[p * n + p]) / (2 * apq);
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1));
                const double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; ++k) {
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    w.resize(n);
    for (int i = 0; i < n; ++i) w[i] = A[i * n + i];
}

// ---- the problem -------------------------------------------------------------------------------------
// ---- EdgeInertial over explicit vertex states (vertex 1 = previous, 2 = current) ---------------------
struct ImuVerts {
    M3 Rwb1;
    V3 twb1, v1, bg1, ba1;
    M3 Rwb2;
    V3 twb2, v2;
};
// EdgeInertial::computeError (G2oTypes.cc:502-531)
void inertial_error(const Preint &p, const ImuVerts &s, double out[9]) {
    float b1[6];   // IMU::Bias(ba, bg) of vertex 1 as floats
    for (int q = 0; q < 3; ++q) b1[q] = (float)s.ba1[q], b1[3 + q] = (float)s.bg1[q];
    M3 dR;
    delta_rotation(p, b1, dR);
    const V3 dV = delta_vp(p.dV, p.JVg, p.JVa, p, b1);
    const V3 dP = delta_vp(p.dP, p.JPg, p.JPa, p, b1);
    const double dt = (double)p.dT;
    const V3 g{{0, 0, -(double)9.81f}};
    const V3 er = logSO3(mul(mul(tr(dR), tr(s.Rwb1)), s.Rwb2));
    const V3 ev = sub(mul(tr(s.Rwb1), sub(sub(s.v2, s.v1), scale(g, dt))), dV);
    const V3 gdt2 = V3{{g[0] * dt * dt / 2, g[1] * dt * dt / 2, g[2] * dt * dt / 2}};
    const V3 ep = sub(mul(tr(s.Rwb1), sub(sub(sub(s.twb2, s.twb1), scale(s.v1, dt)), gdt2)), dP);
    for (int q = 0; q < 3; ++q) out[q] = er[q], out[3 + q] = ev[q], out[6 + q] = ep[q];
}
// EdgeInertial::linearizeOplus (:542-599): J[v] 9 x dim(v), v = P1 V1 G1 A1 P2 V2
void inertial_jac(const Preint &p, const ImuVerts &s, std::vector<double> J[6]) {
    float b1[6];
    for (int q = 0; q < 3; ++q) b1[q] = (float)s.ba1[q], b1[3 + q] = (float)s.bg1[q];
    const float dbgf[3] = {b1[3] - p.b[3], b1[4] - p.b[4], b1[5] - p.b[5]};
    const V3 dbg{{(double)dbgf[0], (double)dbgf[1], (double)dbgf[2]}};
    const M3 Rwb1 = s.Rwb1, Rbw1 = tr(Rwb1), Rwb2 = s.Rwb2;
    M3 dR;
    delta_rotation(p, b1, dR);
    const M3 eR = mul(mul(tr(dR), Rbw1), Rwb2);
    const V3 er = logSO3(eR);
    const M3 invJr = invRightJ(er);
    M3 JRg, JVg, JPg, JVa, JPa;
    for (int q = 0; q < 9; ++q)
        JRg.m[q] = p.JRg[q], JVg.m[q] = p.JVg[q], JPg.m[q] = p.JPg[q], JVa.m[q] = p.JVa[q], JPa.m[q] = p.JPa[q];
    const double dt = (double)p.dT;
    const V3 g{{0, 0, -(double)9.81f}};
    const int dims[6] = {6, 3, 3, 3, 6, 3};
    for (int v = 0; v < 6; ++v) J[v].assign(9 * dims[v], 0.0);
    auto put = [&](std::vector<double> &A, int cols, int r0, int c0, const M3 &B) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) A[(r0 + r) * cols + c0 + c] = B(r, c);
    };
    put(J[0], 6, 0, 0, scale(mul(mul(invJr, tr(Rwb2)), Rwb1), -1.0));
    put(J[0], 6, 3, 0, hat(mul(Rbw1, sub(sub(s.v2, s.v1), scale(g, dt)))));
    const V3 half{{0.5 * g[0] * dt * dt, 0.5 * g[1] * dt * dt, 0.5 * g[2] * dt * dt}};
    put(J[0], 6, 6, 0, hat(mul(Rbw1, sub(sub(sub(s.twb2, s.twb1), scale(s.v1, dt)), half))));
    put(J[0], 6, 6, 3, scale(eye(), -1.0));
    put(J[1], 3, 3, 0, scale(Rbw1, -1.0));
    put(J[1], 3, 6, 0, scale(Rbw1, -dt));
    put(J[2], 3, 0, 0, scale(mul(mul(mul(invJr, tr(eR)), rightJ(mul(JRg, dbg))), JRg), -1.0));
    put(J[2], 3, 3, 0, scale(JVg, -1.0));
    put(J[2], 3, 6, 0, scale(JPg, -1.0));
    put(J[3], 3, 3, 0, scale(JVa, -1.0));
    put(J[3], 3, 6, 0, scale(JPa, -1.0));
    put(J[4], 6, 0, 0, invJr);
    put(J[4], 6, 6, 3, mul(Rbw1, Rwb2));
    put(J[5], 3, 3, 0, Rbw1);
}
// EdgeInertial ctor information (:486-495): sym(C[0:9,0:9]^-1) with eigenvalues < 1e-12 zeroed
std::vector<double> inertial_info(const Preint &p) {
    std::vector<double> A(81);
    for (int r = 0; r < 9; ++r)
        for (int c = 0; c < 9; ++c) A[r * 9 + c] = (double)p.C[r * 15 + c];
    invert_gj(A, 9);
    for (int r = 0; r < 9; ++r)
        for (int c = r + 1; c < 9; ++c) {
            const double s = (A[r * 9 + c] + A[c * 9 + r]) / 2;
            A[r * 9 + c] = A[c * 9 + r] = s;
        }
    std::vector<double> w, V;
    sym_eig(A, 9, w, V);
    for (double &x : w)
        if (x < 1e-12) x = 0;
    std::vector<double> I9(81, 0.0);
    for (int r = 0; r < 9; ++r)
        for (int c = 0; c < 9; ++c) {
            double s = 0;
            for (int k = 0; k < 9; ++k) s += V[r * 9 + k] * w[k] * V[c * 9 + k];
            I9[r * 9 + c] = s;
        }
    return I9;
}

struct Pose {
    M3 Rwb;
    V3 twb;
    std::vector<M3> Rcw;
    std::vector<V3> tcw;
};

struct Solver {
    const omv_lba_problem &P;
    int C;
    std::vector<M3> Rcb, Rbc;
    std::vector<V3> tcb, tbc;
    // state
    std::vector<Pose> pose;
    std::vector<V3> vel, bg, ba, pts;
    // inertial edges
    std::vector<Preint> pre;
    std::vector<std::vector<double>> info9;   // 81 each (robust/scale applied to scale only)
    std::vector<M3> infoG, infoA;
    // reduced-system layout
    std::vector<int> offP, offV, offG, offA;
    int nred = 0;
    // errors (last computeActiveErrors)
    std::vector<double> e_mono;   // 2 per edge
    std::vector<double> e_st;     // 3 per EdgeStereo
    std::vector<double> e_imu;    // 9 per edge
    std::vector<V3> e_gr, e_ar;
    double delta_mono, dsqr_mono, delta_st, dsqr_st, delta_imu, dsqr_imu;
    int NS;

    explicit Solver(const omv_lba_problem &p) : P(p), C(p.n_cams) {
        for (int c = 0; c < C; ++c) {
            M3 a, b;
            std::memcpy(a.m, p.Rcb + 9 * c, 72);
            std::memcpy(b.m, p.Rbc + 9 * c, 72);
            Rcb.push_back(a), Rbc.push_back(b);
            tcb.push_back(V3{{p.tcb[3 * c], p.tcb[3 * c + 1], p.tcb[3 * c + 2]}});
            tbc.push_back(V3{{p.tbc[3 * c], p.tbc[3 * c + 1], p.tbc[3 * c + 2]}});
        }
        pose.resize(p.n_kf);
        vel.resize(p.n_kf), bg.resize(p.n_kf), ba.resize(p.n_kf);
        for (int k = 0; k < p.n_kf; ++k) {
            std::memcpy(pose[k].Rwb.m, p.Rwb + 9 * k, 72);
            std::memcpy(pose[k].twb.v, p.twb + 3 * k, 24);
            pose[k].Rcw.resize(C), pose[k].tcw.resize(C);
            for (int c = 0; c < C; ++c) {
                std::memcpy(pose[k].Rcw[c].m, p.Rcw + 9 * (k * C + c), 72);
                std::memcpy(pose[k].tcw[c].v, p.tcw + 3 * (k * C + c), 24);
            }
            std::memcpy(vel[k].v, p.vel + 3 * k, 24);
            std::memcpy(bg[k].v, p.bg + 3 * k, 24);
            std::memcpy(ba[k].v, p.ba + 3 * k, 24);
        }
        pts.resize(p.n_pts);
        for (int i = 0; i < p.n_pts; ++i) std::memcpy(pts[i].v, p.pts + 3 * i, 24);
        // EdgeInertial ctor: Info = sym(C[0:9,0:9]^-1), eigenvalues < 1e-12 zeroed (:486-495)
        pre.resize(p.n_imu);
        info9.resize(p.n_imu);
        infoG.resize(p.n_imu), infoA.resize(p.n_imu);
        for (int i = 0; i < p.n_imu; ++i) {
            std::memcpy(&pre[i], p.preint + (size_t)i * OMV_PREINT_FLOATS, sizeof(float) * OMV_PREINT_FLOATS);
            std::vector<double> I9 = inertial_info(pre[i]);
            const double sc = p.imu_info_scale ? (double)p.imu_info_scale[i] : 1.0;
            for (double &x : I9) x *= sc;
            info9[i] = I9;
            M3 g, a;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    g(r, c) = (double)pre[i].C[(9 + r) * 15 + 9 + c];
                    a(r, c) = (double)pre[i].C[(12 + r) * 15 + 12 + c];
                }
            infoG[i] = inv3(g), infoA[i] = inv3(a);
        }
        // vertex layout of the non-marginalised part: per optimisable KF pose (6) [+ v, bg, ba]
        offP.assign(p.n_kf, -1), offV.assign(p.n_kf, -1), offG.assign(p.n_kf, -1), offA.assign(p.n_kf, -1);
        for (int k = 0; k < p.n_opt; ++k) {
            offP[k] = nred, nred += 6;
            if (p.kf_imu[k]) offV[k] = nred, offG[k] = nred + 3, offA[k] = nred + 6, nred += 9;
        }
        delta_mono = (double)(float)std::sqrt(5.991);   // thHuberMono is a float (:3036)
        dsqr_mono = delta_mono * delta_mono;           // RobustKernel::setDelta: dsqr = delta * delta
        delta_imu = std::sqrt(16.92);
        dsqr_imu = delta_imu * delta_imu;
        e_mono.assign(2 * (size_t)p.n_mono, 0.0);
        NS = p.n_stereo > 0 ? p.n_stereo : 0;
        e_st.assign(3 * (size_t)NS, 0.0);
        delta_st = (double)(float)std::sqrt(7.815);    // thHuberStereo (:3030)
        dsqr_st = delta_st * delta_st;
        e_imu.assign(9 * (size_t)p.n_imu, 0.0);
        e_gr.resize(p.n_imu), e_ar.resize(p.n_imu);
    }

    const float *camk(int c) const { return P.cam + 8 * c; }

    // --- errors ---
    void mono_error(int e, double out[2]) const {
        const int k = P.mono_kf[e], c = P.mono_cam[e];
        const V3 Xc = add(mul(pose[k].Rcw[c], pts[P.mono_pt[e]]), pose[k].tcw[c]);
        double u, v;
        cam_project(P.cam_model, c, camk(c), Xc, u, v);
        out[0] = P.mono_obs[2 * e] - u;
        out[1] = P.mono_obs[2 * e + 1] - v;
    }
    // EdgeStereo::computeError (G2oTypes.h:364-380): obs - ProjectStereo(X, 0) (G2oTypes.cc:198-205)
    void stereo_error(int e, double out[3]) const {
        const int k = P.stereo_kf[e];
        const V3 Xc = add(mul(pose[k].Rcw[0], pts[P.stereo_pt[e]]), pose[k].tcw[0]);
        double u, v;
        cam_project(P.cam_model, 0, camk(0), Xc, u, v);
        const double invZ = 1 / Xc[2];
        const double ur = u - (double)P.bf * invZ;
        out[0] = P.stereo_obs[3 * e] - u;
        out[1] = P.stereo_obs[3 * e + 1] - v;
        out[2] = P.stereo_obs[3 * e + 2] - ur;
    }
    double stereo_chi2(int e) const {
        const double w = (double)P.stereo_inv_sigma2[e];
        const double *r = &e_st[3 * e];
        return r[0] * w * r[0] + r[1] * w * r[1] + r[2] * w * r[2];
    }
    ImuVerts imu_verts(int i) const {
        const int k1 = P.imu_kf1[i], k2 = P.imu_kf2[i];
        return ImuVerts{pose[k1].Rwb, pose[k1].twb, vel[k1], bg[k1], ba[k1], pose[k2].Rwb, pose[k2].twb, vel[k2]};
    }
    void imu_error(int i, double out[9]) const { inertial_error(pre[i], imu_verts(i), out); }
    void compute_errors() {
        for (int e = 0; e < P.n_mono; ++e) mono_error(e, &e_mono[2 * e]);
        for (int e = 0; e < NS; ++e) stereo_error(e, &e_st[3 * e]);
        for (int i = 0; i < P.n_imu; ++i) {
            imu_error(i, &e_imu[9 * i]);
            e_gr[i] = sub(bg[P.imu_kf2[i]], bg[P.imu_kf1[i]]);
            e_ar[i] = sub(ba[P.imu_kf2[i]], ba[P.imu_kf1[i]]);
        }
    }
    double mono_chi2(int e) const {
        const double w = (double)P.mono_inv_sigma2[e];
        return e_mono[2 * e] * w * e_mono[2 * e] + e_mono[2 * e + 1] * w * e_mono[2 * e + 1];
    }
    double imu_chi2(int i) const {
        const double *e = &e_imu[9 * i];
        const std::vector<double> &I = info9[i];
        double s = 0;
        for (int r = 0; r < 9; ++r) {
            double t = 0;
            for (int c = 0; c < 9; ++c) t += I[r * 9 + c] * e[c];
            s += e[r] * t;
        }
        return s;
    }
    static double quad3(const V3 &e, const M3 &I) {
        const V3 t = mul(I, e);
        return e[0] * t[0] + e[1] * t[1] + e[2] * t[2];
    }
    static void huber(double e2, double delta, double dsqr, double rho[3]) {
        if (e2 <= dsqr) {
            rho[0] = e2, rho[1] = 1, rho[2] = 0;
        } else {
            const double s = std::sqrt(e2);
            rho[0] = 2 * s * delta - dsqr;
            rho[1] = delta / s;
            rho[2] = -0.5 * rho[1] / e2;
        }
    }
    double robust_chi2() const {
        double chi = 0, rho[3];
        for (int i = 0; i < P.n_imu; ++i) {
            const double c = imu_chi2(i);
            if (P.imu_robust && P.imu_robust[i]) {
                huber(c, delta_imu, dsqr_imu, rho);
                chi += rho[0];
            } else {
                chi += c;
            }
            chi += quad3(e_gr[i], infoG[i]);
            chi += quad3(e_ar[i], infoA[i]);
        }
        for (int e = 0; e < P.n_mono; ++e) {
            huber(mono_chi2(e), delta_mono, dsqr_mono, rho);
            chi += rho[0];
        }
        for (int e = 0; e < NS; ++e) {
            huber(stereo_chi2(e), delta_st, dsqr_st, rho);
            chi += rho[0];
        }
        return chi;
    }

    // --- linearisation (Jacobians at the current state) ---
    void mono_jac(int e, double JX[6], double JP[12]) const {
        const int k = P.mono_kf[e], c = P.mono_cam[e];
        const M3 &Rcw = pose[k].Rcw[c];
        const V3 Xc = add(mul(Rcw, pts[P.mono_pt[e]]), pose[k].tcw[c]);
        const V3 Xb = add(mul(Rbc[c], Xc), tbc[c]);
        double pj[6];
        cam_jac(P.cam_model, c, camk(c), Xc, pj);
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 3; ++q)
                JX[3 * r + q] = -(pj[3 * r] * Rcw(0, q) + pj[3 * r + 1] * Rcw(1, q) + pj[3 * r + 2] * Rcw(2, q));
        const double x = Xb[0], y = Xb[1], z = Xb[2];
        const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
        double pr[6];   // proj_jac * Rcb
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 3; ++q)
                pr[3 * r + q] = pj[3 * r] * Rcb[c](0, q) + pj[3 * r + 1] * Rcb[c](1, q) + pj[3 * r + 2] * Rcb[c](2, q);
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 6; ++q)
                JP[6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
    }
    // EdgeStereo::linearizeOplus (G2oTypes.cc:402-431): proj_jac row 2 = row 0 with (2,2) += bf / z^2
    void stereo_jac(int e, double JX[9], double JP[18]) const {
        const int k = P.stereo_kf[e], c = 0;
        const M3 &Rcw = pose[k].Rcw[c];
        const V3 Xc = add(mul(Rcw, pts[P.stereo_pt[e]]), pose[k].tcw[c]);
        const V3 Xb = add(mul(Rbc[c], Xc), tbc[c]);
        double pj[9];
        cam_jac(P.cam_model, c, camk(c), Xc, pj);
        const double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
        pj[6] = pj[0], pj[7] = pj[1], pj[8] = pj[2] + (double)P.bf * inv_z2;
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q)
                JX[3 * r + q] = -(pj[3 * r] * Rcw(0, q) + pj[3 * r + 1] * Rcw(1, q) + pj[3 * r + 2] * Rcw(2, q));
        const double x = Xb[0], y = Xb[1], z = Xb[2];
        const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
        double pr[9];
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q)
                pr[3 * r + q] = pj[3 * r] * Rcb[c](0, q) + pj[3 * r + 1] * Rcb[c](1, q) + pj[3 * r + 2] * Rcb[c](2, q);
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 6; ++q)
                JP[6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
    }
    void imu_jac(int i, std::vector<double> J[6]) const { inertial_jac(pre[i], imu_verts(i), J); }

    // --- system: dense reduced part + per-landmark blocks ---
    struct Landmark {
        double Hll[9] = {0}, bl[3] = {0};
        std::map<int, std::vector<double>> Hpl;   // kf -> 6x3 (pose rows x point cols)
    };
    std::vector<double> H, b;   // nred x nred, nred
    std::vector<Landmark> lm;

    void add_block(int r0, int rdim, int c0, int cdim, const double *A, int lda) {
        for (int r = 0; r < rdim; ++r)
            for (int c = 0; c < cdim; ++c) H[(size_t)(r0 + r) * nred + c0 + c] += A[r * lda + c];
    }

    void build_system() {
        H.assign((size_t)nred * nred, 0.0);
        b.assign(nred, 0.0);
        lm.assign(P.n_pts, Landmark());
        double rho[3];
        // inertial + random-walk edges
        for (int i = 0; i < P.n_imu; ++i) {
            const int k1 = P.imu_kf1[i], k2 = P.imu_kf2[i];
            std::vector<double> J[6];
            imu_jac(i, J);
            const double *e = &e_imu[9 * i];
            double w = 1.0;
            if (P.imu_robust && P.imu_robust[i]) {
                huber(imu_chi2(i), delta_imu, dsqr_imu, rho);
                w = rho[1];
            }
            const std::vector<double> &I = info9[i];
            double Ie[9];
            for (int r = 0; r < 9; ++r) {
                double t = 0;
                for (int c = 0; c < 9; ++c) t += I[r * 9 + c] * e[c];
                Ie[r] = -t * w;   // omega_r = -Omega e, times rho'
            }
            const int off[6] = {offP[k1], offV[k1], offG[k1], offA[k1], offP[k2], offV[k2]};
            const int dims[6] = {6, 3, 3, 3, 6, 3};
            for (int a = 0; a < 6; ++a) {
                if (off[a] < 0) continue;
                // AtO = J_a^T Omega' (dims[a] x 9)
                std::vector<double> AtO(dims[a] * 9, 0.0);
                for (int r = 0; r < dims[a]; ++r)
                    for (int c = 0; c < 9; ++c) {
                        double s = 0;
                        for (int k = 0; k < 9; ++k) s += J[a][k * dims[a] + r] * I[k * 9 + c];
                        AtO[r * 9 + c] = s * w;
                    }
                for (int r = 0; r < dims[a]; ++r) {
                    double s = 0;
                    for (int k = 0; k < 9; ++k) s += J[a][k * dims[a] + r] * Ie[k];
                    b[off[a] + r] += s;
                }
                for (int bb = a; bb < 6; ++bb) {
                    if (off[bb] < 0) continue;
                    std::vector<double> blk(dims[a] * dims[bb], 0.0);
                    for (int r = 0; r < dims[a]; ++r)
                        for (int c = 0; c < dims[bb]; ++c) {
                            double s = 0;
                            for (int k = 0; k < 9; ++k) s += AtO[r * 9 + k] * J[bb][k * dims[bb] + c];
                            blk[r * dims[bb] + c] = s;
                        }
                    add_block(off[a], dims[a], off[bb], dims[bb], blk.data(), dims[bb]);
                    if (bb != a) {   // keep H symmetric (dense storage of both triangles)
                        std::vector<double> t(dims[a] * dims[bb]);
                        for (int r = 0; r < dims[a]; ++r)
                            for (int c = 0; c < dims[bb]; ++c) t[c * dims[a] + r] = blk[r * dims[bb] + c];
                        add_block(off[bb], dims[bb], off[a], dims[a], t.data(), dims[a]);
                    }
                }
            }
            // EdgeGyroRW / EdgeAccRW: J1 = -I, J2 = I, no robust kernel
            for (int which = 0; which < 2; ++which) {
                const V3 &er = which ? e_ar[i] : e_gr[i];
                const M3 &Iw = which ? infoA[i] : infoG[i];
                const int o1 = which ? offA[k1] : offG[k1], o2 = which ? offA[k2] : offG[k2];
                const V3 Oe = mul(Iw, er);
                if (o1 >= 0) {
                    add_block(o1, 3, o1, 3, Iw.m, 3);
                    for (int r = 0; r < 3; ++r) b[o1 + r] += Oe[r];   // (-I)^T (-Omega e)
                }
                if (o2 >= 0) {
                    add_block(o2, 3, o2, 3, Iw.m, 3);
                    for (int r = 0; r < 3; ++r) b[o2 + r] -= Oe[r];
                }
                if (o1 >= 0 && o2 >= 0) {
                    const M3 m = scale(Iw, -1.0);
                    add_block(o1, 3, o2, 3, m.m, 3);
                    add_block(o2, 3, o1, 3, tr(m).m, 3);
                }
            }
        }
        // visual edges
        for (int e = 0; e < P.n_mono; ++e) {
            double JX[6], JP[12];
            mono_jac(e, JX, JP);
            huber(mono_chi2(e), delta_mono, dsqr_mono, rho);
            const double w = (double)P.mono_inv_sigma2[e] * rho[1];   // robust information
            const double om0 = -(double)P.mono_inv_sigma2[e] * e_mono[2 * e] * rho[1];
            const double om1 = -(double)P.mono_inv_sigma2[e] * e_mono[2 * e + 1] * rho[1];
            Landmark &L = lm[P.mono_pt[e]];
            for (int r = 0; r < 3; ++r) {
                L.bl[r] += JX[r] * om0 + JX[3 + r] * om1;
                for (int c = 0; c < 3; ++c) L.Hll[3 * r + c] += w * (JX[r] * JX[c] + JX[3 + r] * JX[3 + c]);
            }
            const int k = P.mono_kf[e];
            const int o = offP[k];
            if (o < 0) continue;
            for (int r = 0; r < 6; ++r) {
                b[o + r] += JP[r] * om0 + JP[6 + r] * om1;
                for (int c = 0; c < 6; ++c) H[(size_t)(o + r) * nred + o + c] += w * (JP[r] * JP[c] + JP[6 + r] * JP[6 + c]);
            }
            std::vector<double> &B = L.Hpl[k];
            if (B.empty()) B.assign(18, 0.0);
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c < 3; ++c) B[3 * r + c] += w * (JP[r] * JX[c] + JP[6 + r] * JX[3 + c]);
        }
        // EdgeStereo: 3 residual rows; the third row's terms are added after the first two
        for (int e = 0; e < NS; ++e) {
            double JX[9], JP[18];
            stereo_jac(e, JX, JP);
            huber(stereo_chi2(e), delta_st, dsqr_st, rho);
            const double wi = (double)P.stereo_inv_sigma2[e];
            const double w = wi * rho[1];
            const double om[3] = {-wi * e_st[3 * e] * rho[1], -wi * e_st[3 * e + 1] * rho[1], -wi * e_st[3 * e + 2] * rho[1]};
            auto rows = [](const double *A, int ia, const double *B, int ib, int lda, int ldb) {
                return A[ia] * B[ib] + A[lda + ia] * B[ldb + ib] + A[2 * lda + ia] * B[2 * ldb + ib];
            };
            auto rows_om = [&](const double *A, int ia, int lda) {
                return A[ia] * om[0] + A[lda + ia] * om[1] + A[2 * lda + ia] * om[2];
            };
            Landmark &L = lm[P.stereo_pt[e]];
            for (int r = 0; r < 3; ++r) {
                L.bl[r] += rows_om(JX, r, 3);
                for (int c = 0; c < 3; ++c) L.Hll[3 * r + c] += w * rows(JX, r, JX, c, 3, 3);
            }
            const int k = P.stereo_kf[e];
            const int o = offP[k];
            if (o < 0) continue;
            for (int r = 0; r < 6; ++r) {
                b[o + r] += rows_om(JP, r, 6);
                for (int c = 0; c < 6; ++c) H[(size_t)(o + r) * nred + o + c] += w * rows(JP, r, JP, c, 6, 6);
            }
            std::vector<double> &B = L.Hpl[k];
            if (B.empty()) B.assign(18, 0.0);
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c < 3; ++c) B[3 * r + c] += w * rows(JP, r, JX, c, 6, 3);
        }
    }

    // --- one LM trial: damped Schur solve; x = [poses | landmarks] ---
    bool solve(double lambda, std::vector<double> &xp, std::vector<double> &xl) {
        std::vector<double> S = H;
        for (int i = 0; i < nred; ++i) S[(size_t)i * nred + i] += lambda;
        std::vector<double> coef(nred, 0.0);
        std::vector<M3> Dinv(P.n_pts);
        for (int p = 0; p < P.n_pts; ++p) {
            Landmark &L = lm[p];
            M3 D;
            std::memcpy(D.m, L.Hll, 72);
            for (int q = 0; q < 3; ++q) D(q, q) += lambda;
            Dinv[p] = inv3(D);
            const V3 db = mul(Dinv[p], V3{{L.bl[0], L.bl[1], L.bl[2]}});
            for (auto it = L.Hpl.begin(); it != L.Hpl.end(); ++it) {
                const double *Bi = it->second.data();
                const int oi = offP[it->first];
                for (int r = 0; r < 6; ++r) coef[oi + r] += Bi[3 * r] * db[0] + Bi[3 * r + 1] * db[1] + Bi[3 * r + 2] * db[2];
                double BD[18];   // Bi * Dinv
                for (int r = 0; r < 6; ++r)
                    for (int c = 0; c < 3; ++c)
                        BD[3 * r + c] = Bi[3 * r] * Dinv[p](0, c) + Bi[3 * r + 1] * Dinv[p](1, c) + Bi[3 * r + 2] * Dinv[p](2, c);
                for (auto jt = L.Hpl.begin(); jt != L.Hpl.end(); ++jt) {
                    const double *Bj = jt->second.data();
                    const int oj = offP[jt->first];
                    for (int r = 0; r < 6; ++r)
                        for (int c = 0; c < 6; ++c)
                            S[(size_t)(oi + r) * nred + oj + c] -=
                                BD[3 * r] * Bj[3 * c] + BD[3 * r + 1] * Bj[3 * c + 1] + BD[3 * r + 2] * Bj[3 * c + 2];
                }
            }
        }
        std::vector<double> bs(nred);
        for (int i = 0; i < nred; ++i) bs[i] = b[i] - coef[i];
        // dense LDL^T without pivoting (SimplicialLDLT fails only on a zero pivot)
        const int n = nred;
        std::vector<double> Lm(S), d(n);
        for (int j = 0; j < n; ++j) {
            double dj = Lm[(size_t)j * n + j];
            for (int k = 0; k < j; ++k) dj -= Lm[(size_t)j * n + k] * Lm[(size_t)j * n + k] * d[k];
            if (dj == 0 || !std::isfinite(dj)) return false;
            d[j] = dj;
            for (int i = j + 1; i < n; ++i) {
                double s = Lm[(size_t)i * n + j];
                for (int k = 0; k < j; ++k) s -= Lm[(size_t)i * n + k] * Lm[(size_t)j * n + k] * d[k];
                Lm[(size_t)i * n + j] = s / dj;
            }
        }
        xp.assign(n, 0.0);
        for (int i = 0; i < n; ++i) {
            double s = bs[i];
            for (int k = 0; k < i; ++k) s -= Lm[(size_t)i * n + k] * xp[k];
            xp[i] = s;
        }
        for (int i = 0; i < n; ++i) xp[i] /= d[i];
        for (int i = n - 1; i >= 0; --i) {
            double s = xp[i];
            for (int k = i + 1; k < n; ++k) s -= Lm[(size_t)k * n + i] * xp[k];
            xp[i] = s;
        }
        xl.assign(3 * (size_t)P.n_pts, 0.0);
        for (int p = 0; p < P.n_pts; ++p) {
            const Landmark &L = lm[p];
            V3 c{{L.bl[0], L.bl[1], L.bl[2]}};
            for (auto it = L.Hpl.begin(); it != L.Hpl.end(); ++it) {
                const double *Bi = it->second.data();
                const int oi = offP[it->first];
                for (int q = 0; q < 3; ++q)
                    for (int r = 0; r < 6; ++r) c[q] -= Bi[3 * r + q] * xp[oi + r];
            }
            const V3 x = mul(Dinv[p], c);
            for (int q = 0; q < 3; ++q) xl[3 * p + q] = x[q];
        }
        return true;
    }

    // ImuCamPose::its of the optimisable keyframes (every one is created with its 0 and updated by every step, so one
    // counter serves all; a rejected step's pop restores it): Rwb normalised after every third Update (:220-225)
    int its = 0;
    void update(const std::vector<double> &xp, const std::vector<double> &xl) {
        const bool norm = ++its >= 3;
        if (norm) its = 0;
        for (int k = 0; k < P.n_opt; ++k) {
            const double *u = &xp[offP[k]];
            Pose &ps = pose[k];
            ps.twb = add(ps.twb, mul(ps.Rwb, V3{{u[3], u[4], u[5]}}));
            ps.Rwb = mul(ps.Rwb, expSO3(u[0], u[1], u[2]));
            if (norm) polar3(ps.Rwb.m);
            const M3 Rbw = tr(ps.Rwb);
            const V3 tbw = scale(mul(Rbw, ps.twb), -1.0);
            for (int c = 0; c < C; ++c) {
                ps.Rcw[c] = mul(Rcb[c], Rbw);
                ps.tcw[c] = add(mul(Rcb[c], tbw), tcb[c]);
            }
            if (offV[k] >= 0) {
                for (int q = 0; q < 3; ++q) {
                    vel[k][q] += xp[offV[k] + q];
                    bg[k][q] += xp[offG[k] + q];
                    ba[k][q] += xp[offA[k] + q];
                }
            }
        }
        for (int p = 0; p < P.n_pts; ++p)
            for (int q = 0; q < 3; ++q) pts[p][q] += xl[3 * p + q];
    }

    double scale_of(const std::vector<double> &xp, const std::vector<double> &xl, double lambda) const {
        // computeScale: sum_j x_j (lambda x_j + b_j) over the full vector [poses | landmarks]
        double s = 0;
        for (int i = 0; i < nred; ++i) s += xp[i] * (lambda * xp[i] + b[i]);
        for (int p = 0; p < P.n_pts; ++p)
            for (int q = 0; q < 3; ++q) s += xl[3 * p + q] * (lambda * xl[3 * p + q] + lm[p].bl[q]);
        return s;
    }

    struct Snapshot {
        std::vector<Pose> pose;
        std::vector<V3> vel, bg, ba, pts;
        int its;
    };
    Snapshot push() const { return Snapshot{pose, vel, bg, ba, pts, its}; }
    void pop(const Snapshot &s) { pose = s.pose, vel = s.vel, bg = s.bg, ba = s.ba, pts = s.pts, its = s.its; }

    void write_state(omv_lba_problem &p) const {
        for (int k = 0; k < p.n_kf; ++k) {
            std::memcpy(p.Rwb + 9 * k, pose[k].Rwb.m, 72);
            std::memcpy(p.twb + 3 * k, pose[k].twb.v, 24);
            for (int c = 0; c < C; ++c) {
                std::memcpy(p.Rcw + 9 * (k * C + c), pose[k].Rcw[c].m, 72);
                std::memcpy(p.tcw + 3 * (k * C + c), pose[k].tcw[c].v, 24);
            }
            std::memcpy(p.vel + 3 * k, vel[k].v, 24);
            std::memcpy(p.bg + 3 * k, bg[k].v, 24);
            std::memcpy(p.ba + 3 * k, ba[k].v, 24);
        }
        for (int i = 0; i < p.n_pts; ++i) std::memcpy(p.pts + 3 * i, pts[i].v, 24);
    }
};

}  // namespace

extern "C" {

// Residuals and Jacobians at the given state (parity of the edge math).
int oracle_lba_evaluate(const omv_lba_problem *p, double *mono_err, double *mono_jx, double *mono_jp,
                        double *imu_err, double *imu_jac /* [n_imu][9*24] v = P1 V1 G1 A1 P2 V2 */,
                        double *st_err, double *st_jx, double *st_jp /* [n_stereo][3 | 9 | 18] */) {
    Solver s(*p);
    s.compute_errors();
    for (int e = 0; e < s.NS; ++e) {
        if (st_err) std::memcpy(st_err + 3 * e, &s.e_st[3 * e], 24);
        if (st_jx || st_jp) {
            double JX[9], JP[18];
            s.stereo_jac(e, JX, JP);
            if (st_jx) std::memcpy(st_jx + 9 * e, JX, 72);
            if (st_jp) std::memcpy(st_jp + 18 * e, JP, 144);
        }
    }
    for (int e = 0; e < p->n_mono; ++e) {
        if (mono_err) mono_err[2 * e] = s.e_mono[2 * e], mono_err[2 * e + 1] = s.e_mono[2 * e + 1];
        if (mono_jx || mono_jp) {
            double JX[6], JP[12];
            s.mono_jac(e, JX, JP);
            if (mono_jx) std::memcpy(mono_jx + 6 * e, JX, 48);
            if (mono_jp) std::memcpy(mono_jp + 12 * e, JP, 96);
        }
    }
    for (int i = 0; i < p->n_imu; ++i) {
        if (imu_err) std::memcpy(imu_err + 9 * i, &s.e_imu[9 * i], 72);
        if (imu_jac) {
            std::vector<double> J[6];
            s.imu_jac(i, J);
            const int dims[6] = {6, 3, 3, 3, 6, 3};
            int c0 = 0;
            for (int v = 0; v < 6; ++v) {
                for (int r = 0; r < 9; ++r)
                    for (int c = 0; c < dims[v]; ++c) imu_jac[(size_t)i * 216 + r * 24 + c0 + c] = J[v][r * dims[v] + c];
                c0 += dims[v];
            }
        }
    }
    return 0;
}

// Optimizer::LocalInertialBA's optimisation (:3270-3321): err, optimize(opt_it), err_end, outlier test,
// FAIL guard.  Writes the final state into p; trial_log (optional) gets [chi2_before, chi2_after,
// lambda] per trial.
int oracle_lba_optimize(omv_lba_problem *p, const omv_lba_opts *o, omv_lba_result *r, double *trial_log,
                        int log_cap) {
    Solver s(*p);
    s.compute_errors();
    r->err = (float)s.robust_chi2();
    double lambda = 0, ni = 2;
    int nBad = 0, trials = 0, its = 0;
    for (int it = 0; it < o->opt_it; ++it) {
        ++its;
        s.compute_errors();
        double currentChi = s.robust_chi2();
        const double iniChi = currentChi;
        s.build_system();
        if (it == 0) {
            lambda = o->lambda_init;   // user lambda init > 0 (:171-176)
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            Solver::Snapshot snap = s.push();
            std::vector<double> xp, xl;
            const bool ok = s.solve(lambda, xp, xl);
            if (ok) s.update(xp, xl);
            s.compute_errors();
            double tempChi = s.robust_chi2();
            if (!ok) tempChi = std::numeric_limits<double>::max();
            double sc = ok ? s.scale_of(xp, xl, lambda) : 0.0;
            sc += 1e-3;
            rho = (currentChi - tempChi) / sc;
            if (trial_log && trials < log_cap) {
                trial_log[3 * trials] = currentChi;
                trial_log[3 * trials + 1] = tempChi;
                trial_log[3 * trials + 2] = lambda;
            }
            ++trials;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                s.pop(snap);   // errors stay those of the rejected trial, as in g2o
            }
            qmax++;
        } while (rho < 0 && qmax < o->max_trials);
        if (qmax == o->max_trials || rho == 0) break;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) break;
    }
    r->err_end = (float)s.robust_chi2();
    r->iterations = its;
    r->trials = trials;
    r->lambda = lambda;
    for (int e = 0; e < p->n_mono; ++e) {
        const double c = s.mono_chi2(e);
        if (r->mono_chi2) r->mono_chi2[e] = c;
        if (r->mono_outlier) {
            const bool close = p->pt_track_depth[p->mono_pt[e]] < 10.f;
            const int k = p->mono_kf[e], cam = p->mono_cam[e];
            const M3 &R = s.pose[k].Rcw[cam];
            const V3 &X = s.pts[p->mono_pt[e]];
            const bool depth_pos = (R(2, 0) * X[0] + R(2, 1) * X[1] + R(2, 2) * X[2] + s.pose[k].tcw[cam][2]) > 0.0;
            r->mono_outlier[e] = ((c > 5.991f && !close) || (c > 1.5f * 5.991f && close) || !depth_pos) ? 1 : 0;
        }
    }
    for (int e = 0; e < s.NS; ++e) {   // :3299-3311
        const double c = s.stereo_chi2(e);
        if (r->stereo_chi2) r->stereo_chi2[e] = c;
        if (r->stereo_outlier) r->stereo_outlier[e] = c > 7.815f ? 1 : 0;
    }
    const bool fail = (2 * r->err < r->err_end || std::isnan(r->err) || std::isnan(r->err_end)) && !o->large;
    r->status = fail ? OMV_LBA_FAIL : OMV_LBA_OK;
    s.write_state(*p);
    return 0;
}

}  // extern "C"

// =============================================================================================
// Optimizer::PoseInertialOptimizationLastKeyFrame (src/Optimizer.cc:5021-5578), one frame.
namespace {

// Eigen::LDLT<MatrixXd> (lower, diagonal pivoting) as Eigen 3.3's ldlt_inplace::unblocked computes it,
// and LDLT::_solve_impl (D pseudo-inverse below the smallest normal double).  Returns isPositive().
bool ldlt_pivot_solve(std::vector<double> A, int n, const double *b, double *x) {
    std::vector<int> tr(n);
    std::vector<double> temp(n);
    int sign = 0;   // 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
    bool found_zero = false;
    auto a = [&](int i, int j) -> double & { return A[(size_t)i * n + j]; };
    for (int k = 0; k < n; ++k) {
        int big = k;
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(a(i, i)) > std::fabs(a(big, big))) big = i;
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; ++j) std::swap(a(k, j), a(big, j));
            for (int i = big + 1; i < n; ++i) std::swap(a(i, k), a(i, big));
            std::swap(a(k, k), a(big, big));
            for (int i = k + 1; i < big; ++i) {
                const double t = a(i, k);
                a(i, k) = a(big, i);
                a(big, i) = t;
            }
        }
        if (k > 0) {
            for (int j = 0; j < k; ++j) temp[j] = a(j, j) * a(k, j);
            double s = 0;
            for (int j = 0; j < k; ++j) s += a(k, j) * temp[j];
            a(k, k) -= s;
            for (int i = k + 1; i < n; ++i) {
                double t = 0;
                for (int j = 0; j < k; ++j) t += a(i, j) * temp[j];
                a(i, k) -= t;
            }
        }
        const double akk = a(k, k);
        const bool valid = std::fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            sign = 0;
            for (int j = 0; j < n; ++j) tr[j] = j;
            break;
        }
        if (valid)
            for (int i = k + 1; i < n; ++i) a(i, k) /= akk;
        if (!(found_zero && valid) && !valid) found_zero = true;
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    const bool positive = sign == 1 || sign == 0;
    if (!positive) return false;
    std::vector<double> y(b, b + n);
    for (int k = 0; k < n; ++k) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) y[i] -= a(i, j) * y[j];
    for (int i = 0; i < n; ++i) {
        if (std::fabs(a(i, i)) > std::numeric_limits<double>::min()) y[i] /= a(i, i);
        else y[i] = 0;
    }
    for (int i = n - 1; i >= 0; --i)   // L^T x = y, column-oriented (j descending)
        for (int j = n - 1; j > i; --j) y[i] -= a(j, i) * y[j];
    for (int k = n - 1; k >= 0; --k) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; ++i) x[i] = y[i];
    return true;
}

struct PoseEdge {
    int cam, kp;
    bool stereo;
    double obs[3];
    double w;
    V3 Xw;
    bool close;
    bool active = true;    // level 0
    bool robust = true;    // Huber (dropped after round 3)
    double chi2 = 0;       // e->chi2() of the last computeError
};

struct PoseProblem {
    int C;
    const float *cam;
    const int32_t *model = nullptr;   // omv_pose_batch::cam_model (NULL: KannalaBrandt8)
    std::vector<M3> Rcb, Rbc;
    std::vector<V3> tcb, tbc;
    double bf;
    // frame vertices
    M3 Rwb;
    V3 twb, v, bg, ba;
    std::vector<M3> Rcw;
    std::vector<V3> tcw;
    // fixed keyframe vertices (LastFrame: the previous frame's, optimised)
    M3 kRwb;
    V3 ktwb, kv, kbg, kba;
    // ImuCamPose::its of the two pose vertices (0 when the vertex is created, G2oTypes.cc:6 / :74): every third
    // Update normalises Rwb (:220-225)
    int its = 0, kits = 0;
    Preint pre;
    std::vector<double> info9;
    M3 infoG, infoA;
    std::vector<PoseEdge> E;   // EdgeMonoOnlyPose first, then EdgeStereoOnlyPose (creation order)
    double dmono = (double)(float)std::sqrt(5.991), dst = (double)(float)std::sqrt(7.815);

    // computeError of one visual edge (ImuCamPose::Project / ProjectStereo, G2oTypes.cc:192-205)
    void error(const PoseEdge &e, double r[3]) const {
        const V3 Xc = add(mul(Rcw[e.cam], e.Xw), tcw[e.cam]);
        double u, vv;
        cam_project(model, e.cam, cam + 8 * e.cam, Xc, u, vv);
        r[0] = e.obs[0] - u;
        r[1] = e.obs[1] - vv;
        r[2] = 0;
        if (e.stereo) {
            const double invZ = 1 / Xc[2];
            r[2] = e.obs[2] - (u - bf * invZ);
        }
    }
    double chi2_of(const PoseEdge &e, const double r[3]) const {
        double c = r[0] * e.w * r[0] + r[1] * e.w * r[1];
        if (e.stereo) c += r[2] * e.w * r[2];
        return c;
    }
    void compute_error(PoseEdge &e) const {
        double r[3];
        error(e, r);
        e.chi2 = chi2_of(e, r);
    }
    bool depth_positive(const PoseEdge &e) const {   // ImuCamPose::isDepthPositive (:207-209)
        const M3 &R = Rcw[e.cam];
        return (R(2, 0) * e.Xw[0] + R(2, 1) * e.Xw[1] + R(2, 2) * e.Xw[2] + tcw[e.cam][2]) > 0.0;
    }
    // EdgeMonoOnlyPose / EdgeStereoOnlyPose::linearizeOplus: J = proj_jac Rcb SE3deriv (rows 2 or 3)
    void jac(const PoseEdge &e, double JP[18]) const {
        const int c = e.cam;
        const V3 Xc = add(mul(Rcw[c], e.Xw), tcw[c]);
        const V3 Xb = add(mul(Rbc[c], Xc), tbc[c]);
        double pj[9];
        cam_jac(model, c, cam + 8 * c, Xc, pj);
        const int nr = e.stereo ? 3 : 2;
        if (e.stereo) {
            const double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
            pj[6] = pj[0], pj[7] = pj[1], pj[8] = pj[2] + bf * inv_z2;
        }
        double pr[9];
        for (int r = 0; r < nr; ++r)
            for (int q = 0; q < 3; ++q)
                pr[3 * r + q] = pj[3 * r] * Rcb[c](0, q) + pj[3 * r + 1] * Rcb[c](1, q) + pj[3 * r + 2] * Rcb[c](2, q);
        const double x = Xb[0], y = Xb[1], z = Xb[2];
        const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
        for (int r = 0; r < nr; ++r)
            for (int q = 0; q < 6; ++q)
                JP[6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
    }
    ImuVerts verts() const { return ImuVerts{kRwb, ktwb, kv, kbg, kba, Rwb, twb, v}; }

    // one Gauss-Newton iteration (optimization_algorithm_gauss_newton.cpp:50-95): computeActiveErrors,
    // buildSystem, dense LDLT solve, update.  Returns the solve's ok.
    bool gn_iteration(std::vector<double> &x_prev) {
        for (PoseEdge &e : E)
            if (e.active) compute_error(e);
        double H[225] = {0}, b[15] = {0}, rho[3];
        for (PoseEdge &e : E) {
            if (!e.active) continue;
            double r[3], JP[18];
            error(e, r);
            jac(e, JP);
            const int nr = e.stereo ? 3 : 2;
            double w1 = 1.0;
            if (e.robust) {
                Solver::huber(e.chi2, e.stereo ? dst : dmono, e.stereo ? dst * dst : dmono * dmono, rho);
                w1 = rho[1];
            }
            const double w = e.w * w1;
            double om[3];
            for (int q = 0; q < nr; ++q) om[q] = -e.w * r[q] * w1;
            for (int i = 0; i < 6; ++i) {
                double t = JP[i] * om[0] + JP[6 + i] * om[1];
                if (nr == 3) t += JP[12 + i] * om[2];
                b[i] += t;
                for (int j = 0; j < 6; ++j) {
                    double h = JP[i] * JP[j] + JP[6 + i] * JP[6 + j];
                    if (nr == 3) h += JP[12 + i] * JP[12 + j];
                    H[15 * i + j] += w * h;
                }
            }
        }
        // EdgeInertial: vertices 4 (pose, columns 15-20 of the 9x24 Jacobian) and 5 (velocity, 21-23)
        {
            double e9[9];
            inertial_error(pre, verts(), e9);
            std::vector<double> J[6];
            inertial_jac(pre, verts(), J);
            double Jc[9][9];   // [row][state col 0..8]: pose 0-5, v 6-8
            for (int r = 0; r < 9; ++r) {
                for (int c = 0; c < 6; ++c) Jc[r][c] = J[4][r * 6 + c];
                for (int c = 0; c < 3; ++c) Jc[r][6 + c] = J[5][r * 3 + c];
            }
            double Oe[9];
            for (int r = 0; r < 9; ++r) {
                double t = 0;
                for (int c = 0; c < 9; ++c) t += info9[r * 9 + c] * e9[c];
                Oe[r] = t;
            }
            for (int i = 0; i < 9; ++i) {
                double t = 0;
                for (int r = 0; r < 9; ++r) t += Jc[r][i] * Oe[r];
                b[i] -= t;
                for (int j = 0; j < 9; ++j) {
                    double h = 0;
                    for (int r = 0; r < 9; ++r) {
                        double oj = 0;
                        for (int c = 0; c < 9; ++c) oj += info9[r * 9 + c] * Jc[c][j];
                        h += Jc[r][i] * oj;
                    }
                    H[15 * i + j] += h;
                }
            }
        }
        // EdgeGyroRW / EdgeAccRW (G2oTypes.h:567-633): e = b - b_kf, J = I on the frame's bias
        for (int which = 0; which < 2; ++which) {
            const V3 er = which ? sub(ba, kba) : sub(bg, kbg);
            const M3 &Iw = which ? infoA : infoG;
            const int o = which ? 12 : 9;
            const V3 Oe = mul(Iw, er);
            for (int i = 0; i < 3; ++i) {
                b[o + i] -= Oe[i];
                for (int j = 0; j < 3; ++j) H[15 * (o + i) + o + j] += Iw(i, j);
            }
        }
        std::vector<double> Hv(H, H + 225);
        double x[15];
        const bool ok = ldlt_pivot_solve(Hv, 15, b, x);
        if (!ok)   // the solver's x keeps the previous solution (zero before the first)
            for (int i = 0; i < 15; ++i) x[i] = x_prev[i];
        for (int i = 0; i < 15; ++i) x_prev[i] = x[i];
        // VertexPose::oplusImpl -> ImuCamPose::Update (:211-235); velocity / biases additive
        twb = add(twb, mul(Rwb, V3{{x[3], x[4], x[5]}}));
        Rwb = mul(Rwb, expSO3(x[0], x[1], x[2]));
        if (++its >= 3) polar3(Rwb.m), its = 0;   // NormalizeRotation after every third update
        const M3 Rbw = tr(Rwb);
        const V3 tbw = scale(mul(Rbw, twb), -1.0);
        for (int c = 0; c < C; ++c) {
            Rcw[c] = mul(Rcb[c], Rbw);
            tcw[c] = add(mul(Rcb[c], tbw), tcb[c]);
        }
        for (int q = 0; q < 3; ++q) v[q] += x[6 + q], bg[q] += x[9 + q], ba[q] += x[12 + q];
        return ok;
    }
};

void load_pose_frame(const omv_pose_batch *b, int f, const float *C_rw, PoseProblem &P);

}  // namespace

extern "C" {

// One frame of the batch (host pointers in `b`); kp_outlier [kp_cap], H [225] (may be NULL).
int oracle_pose_inertial_last_kf(const omv_pose_batch *b, int f, int rec_init, uint8_t *kp_outlier, int32_t *n_good,
                                 double *Hout) {
    PoseProblem P;
    const int C = b->n_cams;
    // EdgeGyroRW / EdgeAccRW information from the same preintegration as the EdgeInertial
    load_pose_frame(b, f, b->preint + (size_t)f * OMV_PREINT_FLOATS + kPreintC, P);
    const int n_edges = (int)P.E.size();
    for (const PoseEdge &e : P.E) kp_outlier[e.kp] = 0;   // mvbOutlier[i] = false at edge creation
    const float chi2Mono[4] = {12, 7.5, 5.991, 5.991};
    const float chi2Stereo[4] = {15.6, 9.8, 7.815, 7.815};
    int nBad = 0, nInliers = 0;
    std::vector<double> x_prev(15, 0.0);
    for (int it = 0; it < 4; ++it) {
        for (int i = 0; i < 10; ++i)   // optimize(its[it]): stops after a failed solve
            if (!P.gn_iteration(x_prev)) break;
        nBad = 0, nInliers = 0;
        const float chi2close = 1.5f * chi2Mono[it];
        for (int q = 0; q < n_edges; ++q) {   // mono loop, then stereo loop (:5439-5490)
            PoseEdge &e = P.E[q];
            if (kp_outlier[e.kp]) P.compute_error(e);
            const float chi2 = (float)e.chi2;
            bool out;
            if (!e.stereo) out = (chi2 > chi2Mono[it] && !e.close) || (e.close && chi2 > chi2close) || !P.depth_positive(e);
            else out = chi2 > chi2Stereo[it];
            kp_outlier[e.kp] = out ? 1 : 0;
            e.active = !out;
            if (out) ++nBad;
            else ++nInliers;
            if (it == 2) e.robust = false;
        }
        if (n_edges + 3 < 10) break;   // optimizer.edges().size() < 10
    }
    if (nInliers < 30 && !rec_init) {   // recover not too bad points (:5503-5526)
        nBad = 0;
        for (int q = 0; q < n_edges; ++q) {
            PoseEdge &e = P.E[q];
            P.compute_error(e);
            if (e.chi2 < (e.stereo ? 24.f : 18.f)) kp_outlier[e.kp] = 0;
            else ++nBad;
        }
    }
    // state back
    std::memcpy(b->Rwb + 9 * f, P.Rwb.m, 72);
    std::memcpy(b->twb + 3 * f, P.twb.v, 24);
    std::memcpy(b->vel + 3 * f, P.v.v, 24);
    std::memcpy(b->bg + 3 * f, P.bg.v, 24);
    std::memcpy(b->ba + 3 * f, P.ba.v, 24);
    for (int c = 0; c < C; ++c) {
        std::memcpy(b->Rcw + 9 * ((size_t)f * C + c), P.Rcw[c].m, 72);
        std::memcpy(b->tcw + 3 * ((size_t)f * C + c), P.tcw[c].v, 24);
    }
    *n_good = n_edges - nBad;
    if (Hout) {   // ConstraintPoseImu Hessian (:5533-5571), information without robust weights
        double H[225] = {0};
        std::vector<double> J[6];
        inertial_jac(P.pre, P.verts(), J);
        double Jc[9][9];
        for (int r = 0; r < 9; ++r) {
            for (int c = 0; c < 6; ++c) Jc[r][c] = J[4][r * 6 + c];
            for (int c = 0; c < 3; ++c) Jc[r][6 + c] = J[5][r * 3 + c];
        }
        for (int i = 0; i < 9; ++i)
            for (int j = 0; j < 9; ++j) {
                double h = 0;
                for (int r = 0; r < 9; ++r) {
                    double oj = 0;
                    for (int c = 0; c < 9; ++c) oj += P.info9[r * 9 + c] * Jc[c][j];
                    h += Jc[r][i] * oj;
                }
                H[15 * i + j] += h;
            }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) H[15 * (9 + i) + 9 + j] += P.infoG(i, j), H[15 * (12 + i) + 12 + j] += P.infoA(i, j);
        for (const PoseEdge &e : P.E) {
            if (kp_outlier[e.kp]) continue;
            double JP[18];
            P.jac(e, JP);
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) {
                    double h = JP[i] * JP[j] + JP[6 + i] * JP[6 + j];
                    if (e.stereo) h += JP[12 + i] * JP[12 + j];
                    H[15 * i + j] += e.w * h;
                }
        }
        std::memcpy(Hout, H, sizeof H);
    }
    return 0;
}

}  // extern "C"

// =============================================================================================
// Optimizer::PoseInertialOptimizationLastFrame (src/Optimizer.cc:5580-6170), one frame, and the
// ConstraintPoseImu ctor (include/G2oTypes.h:639-659).
namespace {

// Symmetric 15x15: V diag(g(w)) V^T from the cyclic-Jacobi eigen-decomposition (sym_eig).
void sym_recompose(const std::vector<double> &w, const std::vector<double> &V, int n, double *out) {
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
            double s = 0;
            for (int k = 0; k < n; ++k) s += V[r * n + k] * w[k] * V[c * n + k];
            out[r * n + c] = s;
        }
}

// ConstraintPoseImu ctor: H = (H + H) / 2 (exactly H), eigenvalues < 1e-12 zeroed.  Eigen's
// SelfAdjointEigenSolver (tridiagonalisation + implicit QR) is restated by cyclic Jacobi.
void constraint_pose_imu(const double *Hin, double *Hout) {
    std::vector<double> A(225);
    for (int q = 0; q < 225; ++q) A[q] = (Hin[q] + Hin[q]) / 2;
    std::vector<double> w, V;
    sym_eig(A, 15, w, V);
    for (double &x : w)
        if (x < 1e-12) x = 0;
    sym_recompose(w, V, 15, Hout);
}

struct PoseLFProblem : PoseProblem {
    // ConstraintPoseImu of the previous frame (pFp->mpcpi): EdgePriorPoseImu's measurement and information
    M3 pRwb;
    V3 ptwb, pv, pbg, pba;
    std::vector<double> pH;   // 15x15
    double dprior = 5.0;      // rkp->setDelta(5) (:5986)

    // EdgePriorPoseImu::computeError (G2oTypes.cc:758-771) at the previous frame's vertices (k*)
    void prior_error(double e[15]) const {
        const V3 er = logSO3(mul(tr(pRwb), kRwb));
        const V3 et = mul(tr(pRwb), sub(ktwb, ptwb));
        const V3 ev = sub(kv, pv), eg = sub(kbg, pbg), ea = sub(kba, pba);
        for (int q = 0; q < 3; ++q) e[q] = er[q], e[3 + q] = et[q], e[6 + q] = ev[q], e[9 + q] = eg[q], e[12 + q] = ea[q];
    }
    // EdgePriorPoseImu::linearizeOplus (:773-785): J 15x15 over (pose 6, v 3, bg 3, ba 3)
    void prior_jac(double J[225]) const {
        std::fill(J, J + 225, 0.0);
        const M3 RR = mul(tr(pRwb), kRwb);
        const M3 iJ = invRightJ(logSO3(RR));
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) J[r * 15 + c] = iJ(r, c), J[(3 + r) * 15 + 3 + c] = RR(r, c);
        for (int q = 6; q < 15; ++q) J[q * 15 + q] = 1.0;
    }
    // EdgeInertial's 9x24 Jacobian [P1 V1 G1 A1 P2 V2] (GetHessian's column order, G2oTypes.h:445-455)
    void inertial_j24(double Jc[9][24]) const {
        std::vector<double> J[6];
        inertial_jac(pre, verts(), J);
        const int off[6] = {0, 6, 9, 12, 15, 21}, dim[6] = {6, 3, 3, 3, 6, 3};
        for (int v = 0; v < 6; ++v)
            for (int r = 0; r < 9; ++r)
                for (int c = 0; c < dim[v]; ++c) Jc[r][off[v] + c] = J[v][r * dim[v] + c];
    }

    // One Gauss-Newton iteration over the 30 free states in g2o's hessian-index order (vertex ids
    // 0-7): frame pose 0-5, v 6-8, bg 9-11, ba 12-14, previous frame pose 15-20, v 21-23, bg 24-26,
    // ba 27-29.  Edges in creation order: visual, EdgeInertial, EdgeGyroRW, EdgeAccRW, EdgePriorPoseImu.
    bool gn_iteration(std::vector<double> &x_prev) {
        for (PoseEdge &e : E)
            if (e.active) compute_error(e);
        std::vector<double> H(900, 0.0);
        double b[30] = {0}, rho[3];
        auto h = [&](int i, int j) -> double & { return H[(size_t)i * 30 + j]; };
        for (PoseEdge &e : E) {
            if (!e.active) continue;
            double r[3], JP[18];
            error(e, r);
            jac(e, JP);
            const int nr = e.stereo ? 3 : 2;
            double w1 = 1.0;
            if (e.robust) {
                Solver::huber(e.chi2, e.stereo ? dst : dmono, e.stereo ? dst * dst : dmono * dmono, rho);
                w1 = rho[1];
            }
            const double w = e.w * w1;
            double om[3];
            for (int q = 0; q < nr; ++q) om[q] = -e.w * r[q] * w1;
            for (int i = 0; i < 6; ++i) {
                double t = JP[i] * om[0] + JP[6 + i] * om[1];
                if (nr == 3) t += JP[12 + i] * om[2];
                b[i] += t;
                for (int j = 0; j < 6; ++j) {
                    double hh = JP[i] * JP[j] + JP[6 + i] * JP[6 + j];
                    if (nr == 3) hh += JP[12 + i] * JP[12 + j];
                    h(i, j) += w * hh;
                }
            }
        }
        // EdgeInertial over all six vertex blocks: ei column c -> state index
        {
            double e9[9], Jc[9][24];
            inertial_error(pre, verts(), e9);
            inertial_j24(Jc);
            int smap[24];
            for (int c = 0; c < 15; ++c) smap[c] = 15 + c;    // P1 V1 G1 A1: the previous frame
            for (int c = 15; c < 24; ++c) smap[c] = c - 15;   // P2 V2: the frame
            double Oe[9];
            for (int r = 0; r < 9; ++r) {
                double t = 0;
                for (int c = 0; c < 9; ++c) t += info9[r * 9 + c] * e9[c];
                Oe[r] = t;
            }
            double OJ[9][24];
            for (int r = 0; r < 9; ++r)
                for (int j = 0; j < 24; ++j) {
                    double t = 0;
                    for (int c = 0; c < 9; ++c) t += info9[r * 9 + c] * Jc[c][j];
                    OJ[r][j] = t;
                }
            for (int i = 0; i < 24; ++i) {
                double t = 0;
                for (int r = 0; r < 9; ++r) t += Jc[r][i] * Oe[r];
                b[smap[i]] -= t;
                for (int j = 0; j < 24; ++j) {
                    double hh = 0;
                    for (int r = 0; r < 9; ++r) hh += Jc[r][i] * OJ[r][j];
                    h(smap[i], smap[j]) += hh;
                }
            }
        }
        // EdgeGyroRW / EdgeAccRW (G2oTypes.h:567-633): e = b_frame - b_prev, J_prev = -I, J_frame = I
        for (int which = 0; which < 2; ++which) {
            const V3 er = which ? sub(ba, kba) : sub(bg, kbg);
            const M3 &Iw = which ? infoA : infoG;
            const int of = which ? 12 : 9, op = which ? 27 : 24;
            const V3 Oe = mul(Iw, er);
            for (int i = 0; i < 3; ++i) {
                b[op + i] += Oe[i];
                b[of + i] -= Oe[i];
                for (int j = 0; j < 3; ++j) {
                    h(op + i, op + j) += Iw(i, j);
                    h(op + i, of + j) -= Iw(i, j);
                    h(of + i, op + j) -= Iw(i, j);
                    h(of + i, of + j) += Iw(i, j);
                }
            }
        }
        // EdgePriorPoseImu, Huber(5) on chi2 = e^T H e (base_multi_edge.hpp: omega_r = -rho' H e,
        // weighted information rho' H)
        {
            double e[15], J[225], Oe[15];
            prior_error(e);
            prior_jac(J);
            double chi2 = 0;
            for (int k = 0; k < 15; ++k) {
                double t = 0;
                for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * e[l];
                Oe[k] = t;
            }
            for (int k = 0; k < 15; ++k) chi2 += e[k] * Oe[k];
            Solver::huber(chi2, dprior, dprior * dprior, rho);
            const double w1 = rho[1];
            double WJ[225];
            for (int k = 0; k < 15; ++k)
                for (int j = 0; j < 15; ++j) {
                    double t = 0;
                    for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * J[l * 15 + j];
                    WJ[k * 15 + j] = w1 * t;
                }
            for (int i = 0; i < 15; ++i) {
                double t = 0;
                for (int k = 0; k < 15; ++k) t += J[k * 15 + i] * (-Oe[k] * w1);
                b[15 + i] += t;
                for (int j = 0; j < 15; ++j) {
                    double hh = 0;
                    for (int k = 0; k < 15; ++k) hh += J[k * 15 + i] * WJ[k * 15 + j];
                    h(15 + i, 15 + j) += hh;
                }
            }
        }
        double x[30];
        const bool ok = ldlt_pivot_solve(H, 30, b, x);
        if (!ok)
            for (int i = 0; i < 30; ++i) x[i] = x_prev[i];
        for (int i = 0; i < 30; ++i) x_prev[i] = x[i];
        // VertexPose::oplusImpl -> ImuCamPose::Update (G2oTypes.cc:211-235) on both frames
        twb = add(twb, mul(Rwb, V3{{x[3], x[4], x[5]}}));
        Rwb = mul(Rwb, expSO3(x[0], x[1], x[2]));
        if (++its >= 3) polar3(Rwb.m), its = 0;   // NormalizeRotation after every third update
        const M3 Rbw = tr(Rwb);
        const V3 tbw = scale(mul(Rbw, twb), -1.0);
        for (int c = 0; c < C; ++c) {
            Rcw[c] = mul(Rcb[c], Rbw);
            tcw[c] = add(mul(Rcb[c], tbw), tcb[c]);
        }
        for (int q = 0; q < 3; ++q) v[q] += x[6 + q], bg[q] += x[9 + q], ba[q] += x[12 + q];
        ktwb = add(ktwb, mul(kRwb, V3{{x[18], x[19], x[20]}}));
        kRwb = mul(kRwb, expSO3(x[15], x[16], x[17]));
        if (++kits >= 3) polar3(kRwb.m), kits = 0;
        for (int q = 0; q < 3; ++q) kv[q] += x[21 + q], kbg[q] += x[24 + q], kba[q] += x[27 + q];
        return ok;
    }
};

// Load one frame of an omv_pose_batch (frame vertices, the k* vertices, rig, preintegration, visual edges
// in creation order: EdgeMonoOnlyPose, then EdgeStereoOnlyPose).  InfoG / InfoA from `C_rw`.
void load_pose_frame(const omv_pose_batch *b, int f, const float *C_rw, PoseProblem &P) {
    const int C = b->n_cams;
    P.C = C, P.cam = b->cam, P.model = b->cam_model, P.bf = (double)b->bf;
    for (int c = 0; c < C; ++c) {
        M3 a, r;
        std::memcpy(a.m, b->Rcb + 9 * c, 72);
        std::memcpy(r.m, b->Rbc + 9 * c, 72);
        P.Rcb.push_back(a), P.Rbc.push_back(r);
        P.tcb.push_back(V3{{b->tcb[3 * c], b->tcb[3 * c + 1], b->tcb[3 * c + 2]}});
        P.tbc.push_back(V3{{b->tbc[3 * c], b->tbc[3 * c + 1], b->tbc[3 * c + 2]}});
    }
    auto v3 = [](const double *p) { return V3{{p[0], p[1], p[2]}}; };
    std::memcpy(P.Rwb.m, b->Rwb + 9 * f, 72);
    P.twb = v3(b->twb + 3 * f), P.v = v3(b->vel + 3 * f), P.bg = v3(b->bg + 3 * f), P.ba = v3(b->ba + 3 * f);
    P.Rcw.resize(C), P.tcw.resize(C);
    for (int c = 0; c < C; ++c) {
        std::memcpy(P.Rcw[c].m, b->Rcw + 9 * ((size_t)f * C + c), 72);
        P.tcw[c] = v3(b->tcw + 3 * ((size_t)f * C + c));
    }
    std::memcpy(P.kRwb.m, b->kf_Rwb + 9 * f, 72);
    P.ktwb = v3(b->kf_twb + 3 * f), P.kv = v3(b->kf_vel + 3 * f), P.kbg = v3(b->kf_bg + 3 * f),
    P.kba = v3(b->kf_ba + 3 * f);
    std::memcpy(&P.pre, b->preint + (size_t)f * OMV_PREINT_FLOATS, sizeof(float) * OMV_PREINT_FLOATS);
    P.info9 = inertial_info(P.pre);
    {
        M3 g, a;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                g(r, c) = (double)C_rw[(9 + r) * 15 + 9 + c];
                a(r, c) = (double)C_rw[(12 + r) * 15 + 12 + c];
            }
        P.infoG = inv3(g), P.infoA = inv3(a);
    }
    for (int e = b->mono_start[f]; e < b->mono_start[f + 1]; ++e) {
        PoseEdge q;
        q.cam = b->mono_cam[e], q.kp = b->mono_kp[e], q.stereo = false;
        q.obs[0] = b->mono_obs[2 * e], q.obs[1] = b->mono_obs[2 * e + 1], q.obs[2] = 0;
        q.w = (double)b->mono_inv_sigma2[e];
        q.Xw = V3{{(double)b->mono_xw[3 * e], (double)b->mono_xw[3 * e + 1], (double)b->mono_xw[3 * e + 2]}};
        q.close = b->mono_close[e] != 0;
        P.E.push_back(q);
    }
    for (int e = b->stereo_start[f]; e < b->stereo_start[f + 1]; ++e) {
        PoseEdge q;
        q.cam = b->stereo_cam[e], q.kp = b->stereo_kp[e], q.stereo = true;
        for (int d = 0; d < 3; ++d) q.obs[d] = b->stereo_obs[3 * e + d];
        q.w = (double)b->stereo_inv_sigma2[e];
        q.Xw = V3{{(double)b->stereo_xw[3 * e], (double)b->stereo_xw[3 * e + 1], (double)b->stereo_xw[3 * e + 2]}};
        q.close = false;
        P.E.push_back(q);
    }
}

}  // namespace

extern "C" {

int oracle_pose_constraint(const double *Hin, double *Hout) {
    constraint_pose_imu(Hin, Hout);
    return 0;
}

// One frame of the batch (host pointers in `b` / `pr`); kp_outlier [kp_cap], H [225] (may be NULL):
// the frame's block of Marginalize(H, 0, 14), before the ConstraintPoseImu ctor.
int oracle_pose_inertial_last_frame(const omv_pose_batch *b, const omv_pose_prior *pr, int f, int rec_init,
                                    uint8_t *kp_outlier, int32_t *n_good, double *Hout) {
    PoseLFProblem P;
    load_pose_frame(b, f, pr->preint_kf + (size_t)f * OMV_PREINT_FLOATS + kPreintC, P);
    std::memcpy(P.pRwb.m, pr->Rwb + 9 * f, 72);
    for (int q = 0; q < 3; ++q) {
        P.ptwb[q] = pr->twb[3 * f + q], P.pv[q] = pr->vel[3 * f + q];
        P.pbg[q] = pr->bg[3 * f + q], P.pba[q] = pr->ba[3 * f + q];
    }
    P.pH.assign(pr->H + 225 * (size_t)f, pr->H + 225 * (size_t)f + 225);
    const int n_edges = (int)P.E.size();
    for (const PoseEdge &e : P.E) kp_outlier[e.kp] = 0;   // mvbOutlier[i] = false at edge creation
    const float chi2Mono[4] = {5.991f, 5.991f, 5.991f, 5.991f};
    const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
    int nBad = 0, nInliers = 0;
    std::vector<double> x_prev(30, 0.0);
    for (int it = 0; it < 4; ++it) {
        for (int i = 0; i < 10; ++i)   // optimize(its[it]): stops after a failed solve
            if (!P.gn_iteration(x_prev)) break;
        nBad = 0, nInliers = 0;
        const float chi2close = 1.5f * chi2Mono[it];
        for (int q = 0; q < n_edges; ++q) {   // mono loop, then stereo loop (:6014-6064)
            PoseEdge &e = P.E[q];
            if (kp_outlier[e.kp]) P.compute_error(e);
            const float chi2 = (float)e.chi2;
            bool out;
            if (!e.stereo) out = (chi2 > chi2Mono[it] && !e.close) || (e.close && chi2 > chi2close) || !P.depth_positive(e);
            else out = chi2 > chi2Stereo[it];
            kp_outlier[e.kp] = out ? 1 : 0;
            e.active = !out;
            if (out) ++nBad;
            else ++nInliers;
            if (it == 2) e.robust = false;
        }
        if (n_edges + 4 < 10) break;   // optimizer.edges().size() < 10 (ei, egr, ear, ep)
    }
    if (nInliers < 30 && !rec_init) {   // :6074-6098
        nBad = 0;
        for (int q = 0; q < n_edges; ++q) {
            PoseEdge &e = P.E[q];
            P.compute_error(e);
            if (e.chi2 < (e.stereo ? 24.f : 18.f)) kp_outlier[e.kp] = 0;
            else ++nBad;
        }
    }
    const int C = b->n_cams;
    std::memcpy(b->Rwb + 9 * f, P.Rwb.m, 72);
    std::memcpy(b->twb + 3 * f, P.twb.v, 24);
    std::memcpy(b->vel + 3 * f, P.v.v, 24);
    std::memcpy(b->bg + 3 * f, P.bg.v, 24);
    std::memcpy(b->ba + 3 * f, P.ba.v, 24);
    for (int c = 0; c < C; ++c) {
        std::memcpy(b->Rcw + 9 * ((size_t)f * C + c), P.Rcw[c].m, 72);
        std::memcpy(b->tcw + 3 * ((size_t)f * C + c), P.tcw[c].v, 24);
    }
    *n_good = n_edges - nBad;
    if (Hout) {   // :6112-6156 in the reference's layout: previous frame 0-14, frame 15-29
        std::vector<double> H(900, 0.0);
        auto h = [&](int i, int j) -> double & { return H[(size_t)i * 30 + j]; };
        double Jc[9][24];
        P.inertial_j24(Jc);
        for (int i = 0; i < 24; ++i)   // ei->GetHessian(): J^T Info J
            for (int j = 0; j < 24; ++j) {
                double s = 0;
                for (int r = 0; r < 9; ++r) {
                    double oj = 0;
                    for (int c = 0; c < 9; ++c) oj += P.info9[r * 9 + c] * Jc[c][j];
                    s += Jc[r][i] * oj;
                }
                h(i, j) += s;
            }
        for (int which = 0; which < 2; ++which) {   // egr / ear->GetHessian(): [[I, -I], [-I, I]] blocks
            const M3 &Iw = which ? P.infoA : P.infoG;
            const int o1 = which ? 12 : 9, o2 = which ? 27 : 24;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    h(o1 + i, o1 + j) += Iw(i, j);
                    h(o1 + i, o2 + j) += -Iw(i, j);
                    h(o2 + i, o1 + j) += -Iw(i, j);
                    h(o2 + i, o2 + j) += Iw(i, j);
                }
        }
        {   // ep->GetHessian(): J^T H_prior J (no robust weight)
            double J[225];
            P.prior_jac(J);
            for (int i = 0; i < 15; ++i)
                for (int j = 0; j < 15; ++j) {
                    double s = 0;
                    for (int k = 0; k < 15; ++k) {
                        double oj = 0;
                        for (int l = 0; l < 15; ++l) oj += P.pH[k * 15 + l] * J[l * 15 + j];
                        s += J[k * 15 + i] * oj;
                    }
                    h(i, j) += s;
                }
        }
        for (const PoseEdge &e : P.E) {   // inlier visual edges' GetHessian()
            if (kp_outlier[e.kp]) continue;
            double JP[18];
            P.jac(e, JP);
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) {
                    double s = JP[i] * JP[j] + JP[6 + i] * JP[6 + j];
                    if (e.stereo) s += JP[12 + i] * JP[12 + j];
                    h(15 + i, 15 + j) += e.w * s;
                }
        }
        // Marginalize(H, 0, 14): Hff - Hfp pinv(Hpp) Hpf; JacobiSVD's pseudo-inverse of the symmetric Hpp
        // (singular values = |eigenvalues|, U = V sign) is V diag(1/w) V^T over |w| > 1e-6
        std::vector<double> A(225), w, V;
        for (int i = 0; i < 15; ++i)
            for (int j = 0; j < 15; ++j) A[i * 15 + j] = h(i, j);
        sym_eig(A, 15, w, V);
        for (double &x : w) x = std::fabs(x) > 1e-6 ? 1.0 / x : 0.0;
        double inv[225], T[225];
        sym_recompose(w, V, 15, inv);
        for (int i = 0; i < 15; ++i)
            for (int j = 0; j < 15; ++j) {
                double s = 0;
                for (int k = 0; k < 15; ++k) s += h(15 + i, k) * inv[k * 15 + j];
                T[i * 15 + j] = s;
            }
        for (int i = 0; i < 15; ++i)
            for (int j = 0; j < 15; ++j) {
                double s = 0;
                for (int k = 0; k < 15; ++k) s += T[i * 15 + k] * h(k, 15 + j);
                Hout[i * 15 + j] = h(15 + i, 15 + j) - s;
            }
    }
    return 0;
}

}  // extern "C"

// =============================================================================================
// Optimizer::PoseOptimization (src/Optimizer.cc:855-1278), one frame: the non-inertial pose-only optimisation
// Tracking runs before the IMU is initialised (Tracking.cc:2924) and in the visual-only configurations.
//   vertex     VertexSE3Expmap (types_six_dof_expmap.h:57-77): SE3Quat Tcw of camera 0, oplus = exp(dx) * T
//              (se3quat.h:104-110, :223-257), the quaternion kept normalised with w >= 0 (:280-285)
//   edges      EdgeSE3ProjectXYZOnlyPose / ...PoseToBody / ...SLPoseToBody / ...SRPoseToBody (OptimizableTypes.h:12-38,
//              OptimizableTypes.cpp:30-171): camera c of the rig through T_c0 (mTrl / mTsll / mTsrl), Huber sqrt(5.991);
//              EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.cpp:339-404, float invz), Huber sqrt(7.815)
//   optimizer  OptimizationAlgorithmLevenberg (tau 1e-5, 10 trials) over BlockSolver_6_3 with no landmark (Hpp only) and
//              LinearSolverDense (Eigen::LDLT): 4 rounds of optimize(10), each from the frame's initial pose
//              (:1136-1142), outliers re-classified between rounds (chi2 5.991 / 7.815), robust kernels dropped
//              after round 3, early stop when fewer than 10 edges.
// Summation order = edge creation order (keypoint order), as g2o's id-sorted active edge list.
namespace {

struct Quat {   // Eigen::Quaterniond coefficients
    double x, y, z, w;
};
Quat qmul(const Quat &a, const Quat &b) {   // Eigen quat_product
    return Quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
V3 qrot(const Quat &q, const V3 &v) {   // Eigen _transformVector: uv = 2 q.vec x v; v + w uv + q.vec x uv
    V3 uv{{q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]}};
    uv = add(uv, uv);
    const V3 c{{q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]}};
    return V3{{v[0] + q.w * uv[0] + c[0], v[1] + q.w * uv[1] + c[1], v[2] + q.w * uv[2] + c[2]}};
}
M3 qmat(const Quat &q) {   // QuaternionBase::toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w, txx = tx * q.x, txy = ty * q.x, txz = tz * q.x,
                 tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    M3 r;
    r(0, 0) = 1 - (tyy + tzz), r(0, 1) = txy - twz, r(0, 2) = txz + twy;
    r(1, 0) = txy + twz, r(1, 1) = 1 - (txx + tzz), r(1, 2) = tyz - twx;
    r(2, 0) = txz - twy, r(2, 1) = tyz + twx, r(2, 2) = 1 - (txx + tyy);
    return r;
}
Quat qfrom(const M3 &m) {   // Quaternion(const Matrix3&): quaternionbase_assign_impl
    Quat q;
    double t = m(0, 0) + m(1, 1) + m(2, 2);
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m(2, 1) - m(1, 2)) * t, q.y = (m(0, 2) - m(2, 0)) * t, q.z = (m(1, 0) - m(0, 1)) * t;
    } else {
        int i = 0;
        if (m(1, 1) > m(0, 0)) i = 1;
        if (m(2, 2) > m(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double c[3];
        t = std::sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0);
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m(k, j) - m(j, k)) * t;
        c[j] = (m(j, i) + m(i, j)) * t;
        c[k] = (m(k, i) + m(i, k)) * t;
        q.x = c[0], q.y = c[1], q.z = c[2];
    }
    return q;
}
void qnormalize_pos(Quat &q) {   // SE3Quat::normalizeRotation
    if (q.w < 0) q.x = -q.x, q.y = -q.y, q.z = -q.z, q.w = -q.w;
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n, q.y /= n, q.z /= n, q.w /= n;
}
struct SE3Q {
    Quat q;
    V3 t;
    V3 map(const V3 &X) const { return add(qrot(q, X), t); }
};
// VertexSE3Expmap::oplusImpl: SE3Quat::exp(dx) * T (rotation part dx[0..2], translation dx[3..5])
SE3Q se3_oplus(const double *dx, const SE3Q &T) {
    const V3 om{{dx[0], dx[1], dx[2]}}, up{{dx[3], dx[4], dx[5]}};
    const double theta = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    const M3 O = hat(om), I = eye();
    M3 R, V;
    if (theta < 0.00001) {
        R = add(add(I, O), mul(O, O));
        V = R;
    } else {
        const M3 O2 = mul(O, O);
        R = add(add(I, scale(O, std::sin(theta) / theta)), scale(O2, (1 - std::cos(theta)) / (theta * theta)));
        V = add(add(I, scale(O, (1 - std::cos(theta)) / (theta * theta))),
                scale(O2, (theta - std::sin(theta)) / std::pow(theta, 3)));
    }
    SE3Q e{qfrom(R), mul(V, up)};
    qnormalize_pos(e.q);
    SE3Q r{qmul(e.q, T.q), add(e.t, qrot(e.q, T.t))};
    qnormalize_pos(r.q);
    return r;
}

struct PoseOnlyEdge {
    int cam, kp;
    bool stereo;
    double obs[3];
    double w;
    V3 Xw;
    bool active = true;
    double chi2 = 0;   // e->chi2() of the last computeError
};

struct PoseOnlyProblem {
    const float *cam;
    const int32_t *model;
    std::vector<SE3Q> rig;   // T_c0 (entry 0 unused)
    std::vector<M3> rigR;    // T_c0.rotation().toRotationMatrix()
    double fx, fy, cx, cy, bf;
    std::vector<PoseOnlyEdge> E;   // creation order (keypoint order)
    bool robust = true;
    const double dmono = (double)(float)std::sqrt(5.991), dst = (double)(float)std::sqrt(7.815);

    // computeError at pose T; returns chi2 and the residual
    double error(const SE3Q &T, const PoseOnlyEdge &e, double r[3]) const {
        const V3 Xl = T.map(e.Xw);
        r[2] = 0;
        if (e.stereo) {   // EdgeStereoSE3ProjectXYZOnlyPose::cam_project: float invz
            const float invz = (float)(1.0f / Xl[2]);
            const double u = Xl[0] * invz * fx + cx;
            r[0] = e.obs[0] - u;
            r[1] = e.obs[1] - (Xl[1] * invz * fy + cy);
            r[2] = e.obs[2] - (u - bf * invz);
            return r[0] * (e.w * r[0]) + r[1] * (e.w * r[1]) + r[2] * (e.w * r[2]);
        }
        const V3 Xc = e.cam ? rig[e.cam].map(Xl) : Xl;
        double u, v;
        cam_project(model, e.cam, cam + 8 * e.cam, Xc, u, v);
        r[0] = e.obs[0] - u, r[1] = e.obs[1] - v;
        return r[0] * (e.w * r[0]) + r[1] * (e.w * r[1]);
    }
    void jac(const SE3Q &T, const PoseOnlyEdge &e, double J[18]) const {
        const V3 Xl = T.map(e.Xw);
        if (e.stereo) {
            const double x = Xl[0], y = Xl[1], invz = 1.0 / Xl[2], invz_2 = invz * invz;
            J[0] = x * y * invz_2 * fx, J[1] = -(1 + (x * x * invz_2)) * fx, J[2] = y * invz * fx;
            J[3] = -invz * fx, J[4] = 0, J[5] = x * invz_2 * fx;
            J[6] = (1 + y * y * invz_2) * fy, J[7] = -x * y * invz_2 * fy, J[8] = -x * invz * fy;
            J[9] = 0, J[10] = -invz * fy, J[11] = y * invz_2 * fy;
            J[12] = J[0] - bf * y * invz_2, J[13] = J[1] + bf * x * invz_2, J[14] = J[2];
            J[15] = J[3], J[16] = 0, J[17] = J[5] - bf * invz_2;
            return;
        }
        const V3 Xc = e.cam ? rig[e.cam].map(Xl) : Xl;
        double pj[6];
        cam_jac(model, e.cam, cam + 8 * e.cam, Xc, pj);
        double pr[6];   // -projectJac(Xc) * R_c0
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 3; ++q)
                pr[3 * r + q] = e.cam ? (-pj[3 * r]) * rigR[e.cam](0, q) + (-pj[3 * r + 1]) * rigR[e.cam](1, q) +
                                            (-pj[3 * r + 2]) * rigR[e.cam](2, q)
                                      : -pj[3 * r + q];
        const double x = Xl[0], y = Xl[1], z = Xl[2];
        const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
        for (int r = 0; r < 2; ++r)
            for (int q = 0; q < 6; ++q)
                J[6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
    }
    double rho0(const PoseOnlyEdge &e) const {   // the edge's term of activeRobustChi2
        if (!robust) return e.chi2;
        double rho[3];
        const double d = e.stereo ? dst : dmono;
        Solver::huber(e.chi2, d, d * d, rho);
        return rho[0];
    }
    double compute_active_errors(const SE3Q &T) {
        double chi = 0, r[3];
        for (PoseOnlyEdge &e : E)
            if (e.active) e.chi2 = error(T, e, r), chi += rho0(e);
        return chi;
    }
    // buildSystem (base_unary_edge constructQuadraticForm): H = sum J^T (rho' Omega) J, b = sum J^T (-rho' Omega e)
    void build(const SE3Q &T, double H[36], double b[6]) const {
        std::fill(H, H + 36, 0.0), std::fill(b, b + 6, 0.0);
        for (const PoseOnlyEdge &e : E) {
            if (!e.active) continue;
            double r[3], J[18], rho[3] = {0, 1, 0};
            error(T, e, r);
            jac(T, e, J);
            const int nr = e.stereo ? 3 : 2;
            if (robust) {
                const double d = e.stereo ? dst : dmono;
                Solver::huber(e.chi2, d, d * d, rho);
            }
            for (int i = 0; i < 6; ++i) {
                double t = 0;
                for (int k = 0; k < nr; ++k) t += J[6 * k + i] * (-e.w * r[k] * rho[1]);
                b[i] += t;
                for (int j = 0; j < 6; ++j) {
                    double h = 0;
                    for (int k = 0; k < nr; ++k) h += J[6 * k + i] * (rho[1] * e.w) * J[6 * k + j];
                    H[6 * i + j] += h;
                }
            }
        }
    }
};

}  // namespace

extern "C" {

// One frame of the batch (host pointers in `b`): rig_q / rig_t [n_cams][4] (x y z w) / [3] = T_c0 (mTrl, mTsll, mTsrl;
// entry 0 unused); pose_q / pose_t [4] / [3] in/out (frame f's Tcw); kp_outlier [kp_cap] (edge keypoints only).
// Returns the reference's return value (nInitialCorrespondences - nBad, or 0 below 3 correspondences).
int oracle_pose_optimization(const omv_pose_batch *b, const double *rig_q, const double *rig_t, int f, double *pose_q,
                             double *pose_t, uint8_t *kp_outlier) {
    PoseOnlyProblem P;
    P.cam = b->cam, P.model = b->cam_model;
    P.fx = b->cam[0], P.fy = b->cam[1], P.cx = b->cam[2], P.cy = b->cam[3], P.bf = b->bf;
    P.rig.resize(b->n_cams), P.rigR.resize(b->n_cams);
    for (int c = 0; c < b->n_cams; ++c) {
        SE3Q T{Quat{rig_q[4 * c], rig_q[4 * c + 1], rig_q[4 * c + 2], rig_q[4 * c + 3]},
               V3{{rig_t[3 * c], rig_t[3 * c + 1], rig_t[3 * c + 2]}}};
        qnormalize_pos(T.q);   // SE3Quat(q, t) ctor
        P.rig[c] = T, P.rigR[c] = qmat(T.q);
    }
    // creation order: keypoint order over the mono and stereo lists
    std::vector<PoseOnlyEdge> E;
    for (int e = b->mono_start[f]; e < b->mono_start[f + 1]; ++e) {
        PoseOnlyEdge x;
        x.cam = b->mono_cam[e], x.kp = b->mono_kp[e], x.stereo = false;
        x.obs[0] = b->mono_obs[2 * e], x.obs[1] = b->mono_obs[2 * e + 1], x.obs[2] = 0;
        x.w = (double)b->mono_inv_sigma2[e];
        for (int q = 0; q < 3; ++q) x.Xw[q] = (double)b->mono_xw[3 * e + q];
        E.push_back(x);
    }
    for (int e = b->stereo_start[f]; e < b->stereo_start[f + 1]; ++e) {
        PoseOnlyEdge x;
        x.cam = 0, x.kp = b->stereo_kp[e], x.stereo = true;
        for (int q = 0; q < 3; ++q) x.obs[q] = b->stereo_obs[3 * e + q], x.Xw[q] = (double)b->stereo_xw[3 * e + q];
        x.w = (double)b->stereo_inv_sigma2[e];
        E.push_back(x);
    }
    std::stable_sort(E.begin(), E.end(), [](const PoseOnlyEdge &a, const PoseOnlyEdge &c) { return a.kp < c.kp; });
    P.E = E;
    const int n = (int)P.E.size();
    for (const PoseOnlyEdge &e : P.E) kp_outlier[e.kp] = 0;
    if (n < 3) return 0;
    SE3Q T0{Quat{pose_q[0], pose_q[1], pose_q[2], pose_q[3]}, V3{{pose_t[0], pose_t[1], pose_t[2]}}};
    qnormalize_pos(T0.q);
    SE3Q T = T0;
    int nBad = 0;
    double x[6] = {0};   // the dense solver's x: kept when a factorisation is not positive
    for (int round = 0; round < 4; ++round) {
        T = T0;
        int n_active = 0;
        for (const PoseOnlyEdge &e : P.E) n_active += e.active ? 1 : 0;
        if (n_active > 0) {   // initializeOptimization(0) found the vertex; otherwise optimize() returns -1
            double lambda = 0, ni = 2;
            int nb = 0;
            for (int it = 0; it < 10; ++it) {
                double currentChi = P.compute_active_errors(T);
                const double iniChi = currentChi;
                double H[36], g[6];
                P.build(T, H, g);
                if (it == 0) {
                    double md = 0;
                    for (int j = 0; j < 6; ++j) md = std::max(std::fabs(H[7 * j]), md);
                    lambda = 1e-5 * md, ni = 2, nb = 0;
                }
                double rho = 0;
                int qmax = 0;
                do {
                    std::vector<double> A(H, H + 36);
                    for (int j = 0; j < 6; ++j) A[7 * j] += lambda;
                    const bool ok = ldlt_pivot_solve(A, 6, g, x);
                    const SE3Q Tt = se3_oplus(x, T);
                    double tempChi = P.compute_active_errors(Tt);
                    if (!ok) tempChi = std::numeric_limits<double>::max();
                    double sc = 0;
                    for (int j = 0; j < 6; ++j) sc += x[j] * (lambda * x[j] + g[j]);
                    sc += 1e-3;
                    rho = (currentChi - tempChi) / sc;
                    if (rho > 0 && std::isfinite(tempChi)) {
                        double alpha = 1. - std::pow((2 * rho - 1), 3);
                        alpha = std::min(alpha, 2. / 3.);
                        lambda *= std::max(1. / 3., alpha);
                        ni = 2;
                        currentChi = tempChi;
                        T = Tt;
                    } else {
                        lambda *= ni;
                        ni *= 2;   // pop(): the pose restored, the edges keep the rejected trial's errors
                    }
                    qmax++;
                } while (rho < 0 && qmax < 10);
                if (qmax == 10 || rho == 0) break;
                if ((iniChi - currentChi) * 1e3 < iniChi) nb++;
                else nb = 0;
                if (nb >= 3) break;
            }
        }
        nBad = 0;
        for (int pass = 0; pass < 2; ++pass)   // mono loops (:1145-1239), then the stereo loop (:1241-1263)
            for (PoseOnlyEdge &e : P.E) {
                if (e.stereo != (pass == 1)) continue;
                if (kp_outlier[e.kp]) {
                    double r[3];
                    e.chi2 = P.error(T, e, r);
                }
                const float chi2 = (float)e.chi2;
                const bool out = chi2 > (e.stereo ? 7.815f : 5.991f);
                kp_outlier[e.kp] = out ? 1 : 0;
                e.active = !out;
                nBad += out ? 1 : 0;
            }
        if (round == 2) P.robust = false;
        if (n < 10) break;
    }
    pose_q[0] = T.q.x, pose_q[1] = T.q.y, pose_q[2] = T.q.z, pose_q[3] = T.q.w;
    pose_t[0] = T.t[0], pose_t[1] = T.t[1], pose_t[2] = T.t[2];
    return n - nBad;
}

}  // extern "C"
