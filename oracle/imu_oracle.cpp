// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for IMU preintegration. Never linked into the product path.
//
// Scalar float restatement of IMU::Preintegrated::IntegrateNewMeasurement (src/ImuTypes.cc:160-239) with
// IntegratedRotation (:58-80), as Tracking::PreintegrateIMU drives it (src/Tracking.cc:1675-1712), over one
// preintegration record in the omv layout (include/omv.h, OMV_PREINT_FLOATS):
//   dR 9 | dV 3 | dP 3 | JRg 9 | JVg 9 | JVa 9 | JPg 9 | JPa 9 | b 6 (bax bay baz bwx bwy bwz) | dT | C 225
// Eigen's fixed-size float expressions are evaluated here as written, left to right: a matrix product's
// coefficient is the dot product of a row and a column summed in index order, a chain A * B * C is
// (A * B) * C, matrix sums are elementwise in the written order.  Eigen's own kernels may vectorise those
// dot products (a different summation order) — against the real Eigen the result is "parity unpinned"; the
// device restatement (csrc/imu.hip) follows the same order as this file.  NormalizeRotation (JacobiSVD
// U V^T) is the polar factor by Newton iteration (as for the getters, ba_oracle.cpp).  sin / cos / sqrt of
// floats are the float functions (Eigen's float expressions need float scalars).
// =====================================================================================================
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../include/omv.h"

namespace {

struct M {   // 3x3 float, row-major
    float m[9];
    float &operator()(int r, int c) { return m[3 * r + c]; }
    float operator()(int r, int c) const { return m[3 * r + c]; }
};
M eye() {
    M r{};
    r(0, 0) = r(1, 1) = r(2, 2) = 1.0f;
    return r;
}
M mul(const M &a, const M &b) {
    M r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r(i, j) = a(i, 0) * b(0, j) + a(i, 1) * b(1, j) + a(i, 2) * b(2, j);
    return r;
}
void mulv(const M &a, const float *x, float *y) {
    for (int i = 0; i < 3; ++i) y[i] = a(i, 0) * x[0] + a(i, 1) * x[1] + a(i, 2) * x[2];
}
M tr(const M &a) {
    M r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r(i, j) = a(j, i);
    return r;
}
M hat(const float *w) {   // Sophus::SO3f::hat
    M r{};
    r(0, 1) = -w[2], r(0, 2) = w[1], r(1, 0) = w[2], r(1, 2) = -w[0], r(2, 0) = -w[1], r(2, 1) = w[0];
    return r;
}
// NormalizeRotation: polar factor X <- (X + X^-T) / 2 (the same iteration as ba_oracle.cpp's polar3<float>)
void polar3f(float *r) {
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
            diff = std::fmax(diff, std::fabs(nv - r[k]));
            r[k] = nv;
        }
        if (diff <= 2.5e-7f) break;
    }
}

struct Rec {   // one OMV_PREINT_FLOATS record
    float dR[9], dV[3], dP[3], JRg[9], JVg[9], JVa[9], JPg[9], JPa[9], b[6], dT, C[225];
};
static_assert(sizeof(Rec) == OMV_PREINT_FLOATS * sizeof(float), "record layout");

M load(const float *p) {
    M r;
    std::memcpy(r.m, p, 36);
    return r;
}
void store(const M &a, float *p) { std::memcpy(p, a.m, 36); }

void integrate(Rec &R, float *avg, const float *meas, const float *Nga, const float *NgaWalk) {
    const float eps = 1e-4f;
    const float dt = meas[6];
    float acc[3], accW[3];
    for (int q = 0; q < 3; ++q) acc[q] = meas[q] - R.b[q], accW[q] = meas[3 + q] - R.b[3 + q];
    const M dR = load(R.dR);
    {   // avgA = (dT * avgA + dR * acc * dt) / (dT + dt); avgW likewise
        float ra[3];
        mulv(dR, acc, ra);
        for (int q = 0; q < 3; ++q) avg[q] = (R.dT * avg[q] + ra[q] * dt) / (R.dT + dt);
        for (int q = 0; q < 3; ++q) avg[3 + q] = (R.dT * avg[3 + q] + accW[q] * dt) / (R.dT + dt);
    }
    const float theta = std::sqrt(accW[0] * accW[0] + accW[1] * accW[1] + accW[2] * accW[2]);
    const float theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta3 * theta;
    const M W = hat(accW), W2 = mul(W, W);
    const float s = sinf(dt * theta), c = cosf(dt * theta);
    const float c1 = (1.0f - c) / theta2, c2 = (dt * theta - s) / theta3;
    const float h2 = 0.5f * dt * dt, c3 = (0.5f * dt * dt * theta2 + c - 1) / theta4;
    M J1, J2;
    for (int k = 0; k < 9; ++k) {
        const float I = (k % 4 == 0) ? 1.0f : 0.0f;
        J1.m[k] = (dt * I + c1 * W.m[k]) + c2 * W2.m[k];
        J2.m[k] = (h2 * I + c2 * W.m[k]) + c3 * W2.m[k];
    }
    const M dRJ1 = mul(dR, J1), dRJ2 = mul(dR, J2);
    {   // dP = dP + dV * dt + dR * J2 * acc; dV = dV + dR * J1 * acc
        float p2[3], p1[3];
        mulv(dRJ2, acc, p2);
        mulv(dRJ1, acc, p1);
        for (int q = 0; q < 3; ++q) R.dP[q] = (R.dP[q] + R.dV[q] * dt) + p2[q];
        for (int q = 0; q < 3; ++q) R.dV[q] = R.dV[q] + p1[q];
    }
    float A[9][15] = {}, B[9][6] = {};
    for (int q = 0; q < 9; ++q) A[q][q] = 1.0f;
    const M Wacc = hat(acc);
    {
        float j1a[3], j2a[3];
        mulv(J1, acc, j1a);
        mulv(J2, acc, j2a);
        const M a30 = mul(dR, hat(j1a)), a60 = mul(dR, hat(j2a));
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) {
                A[3 + r][q] = -a30(r, q);
                A[6 + r][q] = -a60(r, q);
                A[6 + r][3 + q] = r == q ? dt : 0.0f;
                A[r][9 + q] = r == q ? -dt : 0.0f;
                A[3 + r][12 + q] = -dRJ1(r, q);
                A[6 + r][12 + q] = -dRJ2(r, q);
                B[3 + r][3 + q] = dRJ1(r, q);
                B[6 + r][3 + q] = dRJ2(r, q);
            }
    }
    {   // Jacobians wrt the bias (old dR)
        const M JRg = load(R.JRg), JVg = load(R.JVg), JVa = load(R.JVa), JPg = load(R.JPg), JPa = load(R.JPa);
        const M t2 = mul(mul(dRJ2, Wacc), JRg), t1 = mul(mul(dRJ1, Wacc), JRg);
        M nPa, nPg, nVa, nVg;
        for (int k = 0; k < 9; ++k) {
            nPa.m[k] = (JPa.m[k] + JVa.m[k] * dt) - dRJ2.m[k];
            nPg.m[k] = (JPg.m[k] + JVg.m[k] * dt) - t2.m[k];
            nVa.m[k] = JVa.m[k] - dRJ1.m[k];
            nVg.m[k] = JVg.m[k] - t1.m[k];
        }
        store(nPa, R.JPa), store(nPg, R.JPg), store(nVa, R.JVa), store(nVg, R.JVg);
    }
    // IntegratedRotation(angVel, b, dt)
    M dRi, rJ;
    {
        const float x = (meas[3] - R.b[3]) * dt, y = (meas[4] - R.b[4]) * dt, z = (meas[5] - R.b[5]) * dt;
        const float d2 = x * x + y * y + z * z, d = std::sqrt(d2);
        const float v[3] = {x, y, z};
        const M Wr = hat(v), Wr2 = mul(Wr, Wr);
        if (d < eps) {
            for (int k = 0; k < 9; ++k) dRi.m[k] = ((k % 4 == 0) ? 1.0f : 0.0f) + Wr.m[k];
            rJ = eye();
        } else {
            const float sd = sinf(d), cd = cosf(d);
            for (int k = 0; k < 9; ++k) {
                const float I = (k % 4 == 0) ? 1.0f : 0.0f;
                dRi.m[k] = (I + Wr.m[k] * sd / d) + Wr2.m[k] * (1.0f - cd) / d2;
                rJ.m[k] = (I - Wr.m[k] * (1.0f - cd) / d2) + Wr2.m[k] * (d - sd) / (d2 * d);
            }
        }
    }
    M nR = mul(dR, dRi);
    polar3f(nR.m);
    store(nR, R.dR);
    const M dRit = tr(dRi);
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) A[r][q] = dRit(r, q), B[r][q] = rJ(r, q) * dt;
    {   // C[0:9, 0:9] = A * C * A^T + B * Nga * B^T;  C[9:15, 9:15] += dt * dt * NgaWalk
        float T[9][15], U[9][6];
        for (int i = 0; i < 9; ++i)
            for (int k = 0; k < 15; ++k) {
                float t = 0;
                for (int j = 0; j < 15; ++j) t += A[i][j] * R.C[j * 15 + k];
                T[i][k] = t;
            }
        for (int i = 0; i < 9; ++i)   // B * Nga with Nga an Eigen::DiagonalMatrix: column scaling
            for (int k = 0; k < 6; ++k) U[i][k] = B[i][k] * Nga[k];
        float Cn[81];
        for (int i = 0; i < 9; ++i)
            for (int l = 0; l < 9; ++l) {
                float t = 0, u = 0;
                for (int k = 0; k < 15; ++k) t += T[i][k] * A[l][k];
                for (int k = 0; k < 6; ++k) u += U[i][k] * B[l][k];
                Cn[i * 9 + l] = t + u;
            }
        for (int i = 0; i < 9; ++i)
            for (int l = 0; l < 9; ++l) R.C[i * 15 + l] = Cn[i * 9 + l];
        const float dt2 = dt * dt;   // += a DiagonalMatrix: the diagonal only
        for (int i = 0; i < 6; ++i) R.C[(9 + i) * 15 + 9 + i] += dt2 * NgaWalk[i];
    }
    {   // JRg = dRi^T * JRg - rightJ * dt
        const M a = mul(dRit, load(R.JRg));
        M n;
        for (int k = 0; k < 9; ++k) n.m[k] = a.m[k] - rJ.m[k] * dt;
        store(n, R.JRg);
    }
    R.dT += dt;
}

}  // namespace

extern "C" {

// Record `rec` (in/out, OMV_PREINT_FLOATS floats), avg (in/out avgA | avgW, 6 floats, may be NULL),
// n measurements meas[n][7] = (ax ay az wx wy wz dt), Nga / NgaWalk the 6 diagonal entries of
// IMU::Calib::Cov / CovWalk (Eigen::DiagonalMatrix<float, 6>, include/ImuTypes.h:126).
int oracle_preintegrate(float *rec, float *avg, const float *meas, int n, const float *Nga, const float *NgaWalk) {
    Rec R;
    std::memcpy(&R, rec, sizeof R);
    float a[6] = {0, 0, 0, 0, 0, 0};
    if (avg) std::memcpy(a, avg, sizeof a);
    for (int i = 0; i < n; ++i) integrate(R, a, meas + 7 * (size_t)i, Nga, NgaWalk);
    std::memcpy(rec, &R, sizeof R);
    if (avg) std::memcpy(avg, a, sizeof a);
    return 0;
}

}  // extern "C"
