// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for ORBmatcher::SearchForTriangulation. Never linked into the product.
//
// Scalar restatement of
//   ORBmatcher::SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse)
//                                                    src/ORBmatcher.cc:1131-1456 (+ ComputeThreeMaxima :2537-2573)
//   KannalaBrandt8::epipolarConstrain                src/CameraModels/KannalaBrandt8.cpp:219-229
//   KannalaBrandt8::TriangulateMatches               src/CameraModels/KannalaBrandt8.cpp:319-395
//   KannalaBrandt8::unproject / unprojectEig         src/CameraModels/KannalaBrandt8.cpp:96-126, 91-94
//   KannalaBrandt8::project(const Eigen::Vector3f&)  src/CameraModels/KannalaBrandt8.cpp:48-67
//   KannalaBrandt8::Triangulate                      src/CameraModels/KannalaBrandt8.cpp:414-429
//   Pinhole::epipolarConstrain                       src/CameraModels/Pinhole.cpp:103-132
//   Pinhole::unprojectEig / project(Vector3f)        src/CameraModels/Pinhole.cpp:26-32, :40-45
//   Eigen::Matrix3f::inverse()                       Eigen/src/LU/InverseImpl.h compute_inverse<.., 3>
//       (third-party; the cofactor formula: cofactors of column 0, det = their dot with column 0,
//       result(i, j) = cofactor(j, i) * (1 / det))
// pCamera1->epipolarConstrain is a virtual call (ORBmatcher.cc:1380-1387): dispatched on camera 1's type;
// inside KannalaBrandt8::TriangulateMatches pCamera2->unprojectEig / project are camera 2's own.
//   Eigen::JacobiSVD<Eigen::Matrix4f>(A, ComputeFullV)  Eigen 3.3.5+ / 3.4 two-sided Jacobi SVD
//       (third-party, not under /root/reference; restated from its published algorithm: square input, so
//       no QR preconditioner; scale by max|a_ij|; sweeps over (p, q) with threshold
//       max(FLT_MIN, 2 eps maxDiagEntry); real_2x2_jacobi_svd + JacobiRotation::makeJacobi; singular
//       values sorted descending by first-max selection, V columns swapped with them)
// Multi-camera keyframes only (mpCamera2 present): the single-camera epipole test and the monocular
// bStereo branch are not part of this path.  Float arithmetic without contraction; Eigen's 3-element
// products / dot products / norms are taken left to right (the convention of the other restatements
// here).  glibc's sqrtf / atan2f / tanf and double cos / sin are used as the reference's
// KannalaBrandt8.cpp resolves them.
// Parity status: no reference test pins these functions; Eigen's exact JacobiSVD
// rounding (version, FMA contraction) is unpinned.  The device path is bit-exact to THIS restatement.
// =====================================================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/omv.h"

namespace {

const int TH_LOW = 50;
const int HISTO_LENGTH = 30;

int hamming(const uint8_t *a, const uint8_t *b) {
    int d = 0;
    for (int k = 0; k < 32; ++k) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
    return d;
}

// KannalaBrandt8::project(const Eigen::Vector3f&): no `using namespace std` in KannalaBrandt8.cpp, so
// cos(float) / sin(float) are the C double functions on the promoted argument.
void kb8_project_f(const float *k, const float *X, float &u, float &v) {
    const float x2y2 = X[0] * X[0] + X[1] * X[1];
    const float theta = atan2f(sqrtf(x2y2), X[2]);
    const float psi = atan2f(X[1], X[0]);
    const float t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
    const float r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9;
    u = (float)(k[0] * r * std::cos((double)psi) + k[2]);
    v = (float)(k[1] * r * std::sin((double)psi) + k[3]);
}

// KannalaBrandt8::unproject (precision 1e-6, 10 Newton steps, scale = std::tan(theta) / theta_d)
void kb8_unproject_f(const float *k, float px, float py, float *ray) {
    const float pwx = (px - k[2]) / k[0], pwy = (py - k[3]) / k[1];
    float scale = 1.f;
    float theta_d = sqrtf(pwx * pwx + pwy * pwy);
    theta_d = fminf(fmaxf((float)(-M_PI / 2.f), theta_d), (float)(M_PI / 2.f));
    if (theta_d > 1e-8) {
        float theta = theta_d;
        for (int j = 0; j < 10; j++) {
            const float theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2,
                        theta8 = theta4 * theta4;
            const float k0_theta2 = k[4] * theta2, k1_theta4 = k[5] * theta4;
            const float k2_theta6 = k[6] * theta6, k3_theta8 = k[7] * theta8;
            const float theta_fix = (theta * (1 + k0_theta2 + k1_theta4 + k2_theta6 + k3_theta8) - theta_d) /
                                    (1 + 3 * k0_theta2 + 5 * k1_theta4 + 7 * k2_theta6 + 9 * k3_theta8);
            theta = theta - theta_fix;
            if (fabsf(theta_fix) < 1e-6f) break;
        }
        scale = std::tan(theta) / theta_d;
    }
    ray[0] = pwx * scale, ray[1] = pwy * scale, ray[2] = 1.f;
}

// Pinhole::unprojectEig / project(const Eigen::Vector3f&): float, left to right
void pinhole_unproject_f(const float *k, float px, float py, float *ray) {
    ray[0] = (px - k[2]) / k[0], ray[1] = (py - k[3]) / k[1], ray[2] = 1.f;
}
void pinhole_project_f(const float *k, const float *X, float &u, float &v) {
    u = k[0] * X[0] / X[2] + k[2];
    v = k[1] * X[1] / X[2] + k[3];
}
void cam_unproject_f(int model, const float *k, float px, float py, float *ray) {
    if (model == OMV_CAM_PINHOLE) pinhole_unproject_f(k, px, py, ray);
    else kb8_unproject_f(k, px, py, ray);
}
void cam_project_f(int model, const float *k, const float *X, float &u, float &v) {
    if (model == OMV_CAM_PINHOLE) pinhole_project_f(k, X, u, v);
    else kb8_project_f(k, X, u, v);
}

// Eigen Matrix3f::inverse() (row-major in / out)
float cofactor3(const float *m, int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[3 * i1 + j1] * m[3 * i2 + j2] - m[3 * i1 + j2] * m[3 * i2 + j1];
}
void eigen_inverse3(const float *m, float *r) {
    const float c0 = cofactor3(m, 0, 0), c1 = cofactor3(m, 1, 0), c2 = cofactor3(m, 2, 0);
    const float det = c0 * m[0] + c1 * m[3] + c2 * m[6];
    const float invdet = 1.f / det;
    r[0] = c0 * invdet, r[1] = c1 * invdet, r[2] = c2 * invdet;
    for (int i = 1; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = cofactor3(m, j, i) * invdet;
}
void mat3_mul(const float *A, const float *B, float *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// Pinhole::epipolarConstrain(pCamera2, kp1, kp2, R12, t12, sigmaLevel, unc): F12 = K1.transpose().inverse() *
// SO3f::hat(t12) * R12 * K2.inverse(); a b c the epipolar line of kp1; dsqr < 3.84 * unc in double
bool pinhole_epipolar(const float *k1, const float *k2, const omv_kp &kp1, const omv_kp &kp2, const float *R12,
                      const float *t12, float unc) {
    const float K1t[9] = {k1[0], 0.f, 0.f, 0.f, k1[1], 0.f, k1[2], k1[3], 1.f};
    const float K2[9] = {k2[0], 0.f, k2[2], 0.f, k2[1], k2[3], 0.f, 0.f, 1.f};
    const float tx[9] = {0.f, -t12[2], t12[1], t12[2], 0.f, -t12[0], -t12[1], t12[0], 0.f};
    float K1ti[9], K2i[9], A[9], B[9], F[9];
    eigen_inverse3(K1t, K1ti);
    eigen_inverse3(K2, K2i);
    mat3_mul(K1ti, tx, A);
    mat3_mul(A, R12, B);
    mat3_mul(B, K2i, F);
    const float a = kp1.x * F[0] + kp1.y * F[3] + F[6];
    const float b = kp1.x * F[1] + kp1.y * F[4] + F[7];
    const float c = kp1.x * F[2] + kp1.y * F[5] + F[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * unc;
}

// Eigen::JacobiSVD<Matrix4f>(A, ComputeFullV).matrixV(), A and V row-major.
void jacobi_svd4_v(const float *A, float *V) {
    float W[16];
    float scale = 0.f;
    for (int c = 0; c < 4; ++c)   // cwiseAbs().maxCoeff() (column-major visit; max is order-free)
        for (int r = 0; r < 4; ++r) scale = std::max(scale, std::fabs(A[4 * r + c]));
    if (scale == 0.f) scale = 1.f;
    for (int i = 0; i < 16; ++i) W[i] = A[i] / scale, V[i] = (i % 5 == 0) ? 1.f : 0.f;
    const float considerAsZero = FLT_MIN, precision = 2.f * FLT_EPSILON;
    float maxDiag = std::fabs(W[0]);
    for (int i = 1; i < 4; ++i) maxDiag = std::max(maxDiag, std::fabs(W[5 * i]));
    bool finished = false;
    while (!finished) {
        finished = true;
        for (int p = 1; p < 4; ++p)
            for (int q = 0; q < p; ++q) {
                const float threshold = std::max(considerAsZero, precision * maxDiag);
                if (!(std::fabs(W[4 * p + q]) > threshold || std::fabs(W[4 * q + p]) > threshold)) continue;
                finished = false;
                // real_2x2_jacobi_svd
                const float m00 = W[4 * p + p], m01 = W[4 * p + q], m10 = W[4 * q + p], m11 = W[4 * q + q];
                float c1, s1;
                const float t = m00 + m11, d = m10 - m01;
                if (std::fabs(d) < FLT_MIN) {
                    s1 = 0.f, c1 = 1.f;
                } else {
                    const float u = t / d;
                    const float tmp = sqrtf(1.f + u * u);
                    s1 = 1.f / tmp, c1 = u / tmp;
                }
                float n00 = m00, n01 = m01, n11 = m11;
                if (!(c1 == 1.f && s1 == 0.f)) {   // m.applyOnTheLeft(0, 1, rot1)
                    n00 = c1 * m00 + s1 * m10, n01 = c1 * m01 + s1 * m11;
                    n11 = -s1 * m01 + c1 * m11;
                }
                float cr, sr;   // j_right.makeJacobi(m, 0, 1)
                const float deno = 2.f * std::fabs(n01);
                if (deno < FLT_MIN) {
                    cr = 1.f, sr = 0.f;
                } else {
                    const float tau = (n00 - n11) / deno;
                    const float w = sqrtf(tau * tau + 1.f);
                    const float tt = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
                    const float sign_t = tt > 0.f ? 1.f : -1.f;
                    const float n = 1.f / sqrtf(tt * tt + 1.f);
                    sr = -sign_t * (n01 / std::fabs(n01)) * std::fabs(tt) * n;
                    cr = n;
                }
                // j_left = rot1 * j_right.transpose()
                const float cl = c1 * cr - s1 * -sr, sl = c1 * -sr + s1 * cr;
                if (!(cl == 1.f && sl == 0.f))   // W.applyOnTheLeft(p, q, j_left): rows p, q
                    for (int k = 0; k < 4; ++k) {
                        const float xi = W[4 * p + k], yi = W[4 * q + k];
                        W[4 * p + k] = cl * xi + sl * yi;
                        W[4 * q + k] = -sl * xi + cl * yi;
                    }
                if (!(cr == 1.f && -sr == 0.f))   // applyOnTheRight(p, q, j_right): columns p, q, rotation (cr, -sr)
                    for (int k = 0; k < 4; ++k) {
                        float xi = W[4 * k + p], yi = W[4 * k + q];
                        W[4 * k + p] = cr * xi + -sr * yi;
                        W[4 * k + q] = -(-sr) * xi + cr * yi;
                        xi = V[4 * k + p], yi = V[4 * k + q];
                        V[4 * k + p] = cr * xi + -sr * yi;
                        V[4 * k + q] = -(-sr) * xi + cr * yi;
                    }
                maxDiag = std::max(maxDiag, std::max(std::fabs(W[4 * p + p]), std::fabs(W[4 * q + q])));
            }
    }
    float sv[4];
    for (int i = 0; i < 4; ++i) sv[i] = std::fabs(W[5 * i]) * scale;
    for (int i = 0; i < 4; ++i) {   // sort descending: tail(4 - i).maxCoeff(&pos), first max
        int pos = i;
        for (int j = i + 1; j < 4; ++j)
            if (sv[j] > sv[pos]) pos = j;
        if (sv[pos] == 0.f) break;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int k = 0; k < 4; ++k) std::swap(V[4 * k + i], V[4 * k + pos]);
        }
    }
}

// KannalaBrandt8::TriangulateMatches (returns z1, or -1 .. -5)
float triangulate_matches(const float *cam1, const float *cam2, const omv_kp &kp1, const omv_kp &kp2, const float *R12,
                          const float *t12, float sigmaLevel, float unc, float *p3D = nullptr, int model2 = OMV_CAM_KB8) {
    float r1[3], r2[3], r21[3];
    kb8_unproject_f(cam1, kp1.x, kp1.y, r1);
    cam_unproject_f(model2, cam2, kp2.x, kp2.y, r2);
    for (int i = 0; i < 3; ++i) r21[i] = R12[3 * i] * r2[0] + R12[3 * i + 1] * r2[1] + R12[3 * i + 2] * r2[2];
    const float dot = r1[0] * r21[0] + r1[1] * r21[1] + r1[2] * r21[2];
    const float n1 = sqrtf(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
    const float n21 = sqrtf(r21[0] * r21[0] + r21[1] * r21[1] + r21[2] * r21[2]);
    const float cosParallaxRays = dot / (n1 * n21);
    if (cosParallaxRays > 0.9998) return -1;
    float R21[9], t2[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R21[3 * i + j] = R12[3 * j + i];
    for (int i = 0; i < 3; ++i) t2[i] = -R21[3 * i] * t12[0] + -R21[3 * i + 1] * t12[1] + -R21[3 * i + 2] * t12[2];
    // Triangulate: rows p.x * T.row(2) - T.row(0), p.y * T.row(2) - T.row(1); Tcw1 = [I | 0], Tcw2 = [R21 | t2]
    const float T1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const float T2[12] = {R21[0], R21[1], R21[2], t2[0], R21[3], R21[4], R21[5], t2[1], R21[6], R21[7], R21[8], t2[2]};
    float A[16], V[16];
    for (int j = 0; j < 4; ++j) {
        A[j] = r1[0] * T1[8 + j] - T1[j];
        A[4 + j] = r1[1] * T1[8 + j] - T1[4 + j];
        A[8 + j] = r2[0] * T2[8 + j] - T2[j];
        A[12 + j] = r2[1] * T2[8 + j] - T2[4 + j];
    }
    jacobi_svd4_v(A, V);
    float x3D[3];
    for (int i = 0; i < 3; ++i) x3D[i] = V[4 * i + 3] / V[4 * 3 + 3];
    const float z1 = x3D[2];
    if (z1 <= 0) return -2;
    const float z2 = R21[6] * x3D[0] + R21[7] * x3D[1] + R21[8] * x3D[2] + t2[2];
    if (z2 <= 0) return -3;
    float u1, v1;
    kb8_project_f(cam1, x3D, u1, v1);
    const float ex1 = u1 - kp1.x, ey1 = v1 - kp1.y;
    if ((ex1 * ex1 + ey1 * ey1) > 5.991 * sigmaLevel) return -4;
    float x3D2[3];
    for (int i = 0; i < 3; ++i) x3D2[i] = R21[3 * i] * x3D[0] + R21[3 * i + 1] * x3D[1] + R21[3 * i + 2] * x3D[2] + t2[i];
    float u2, v2;
    cam_project_f(model2, cam2, x3D2, u2, v2);
    const float ex2 = u2 - kp2.x, ey2 = v2 - kp2.y;
    if ((ex2 * ex2 + ey2 * ey2) > 5.991 * unc) return -5;
    if (p3D) p3D[0] = x3D[0], p3D[1] = x3D[1], p3D[2] = x3D[2];
    return z1;
}

int cam_of(const omv_kf_view &k, int idx) {
    return idx < k.n_left ? 0 : idx < k.n_left + k.n_right ? 1 : idx < k.n_left + k.n_right + k.n_sideleft ? 2 : 3;
}

// (cameraId1, cameraId2) -> pair index in OMV_TRI_PAIRS order, -1 if the reference leaves R12/t12 as they were
// LL=0, LR=1, RL=2, RR=3, L-SL=4, SL-L=5, SL-SL=6, R-SR=7, SR-R=8, SR-SR=9 (ORBmatcher.cc:1300-1392)
int pair_of(int c1, int c2) {
    if (c1 == 0 && c2 == 0) return 0;
    if (c1 == 0 && c2 == 1) return 1;
    if (c1 == 1 && c2 == 0) return 2;
    if (c1 == 1 && c2 == 1) return 3;
    if (c1 == 0 && c2 == 2) return 4;
    if (c1 == 2 && c2 == 0) return 5;
    if (c1 == 2 && c2 == 2) return 6;
    if (c1 == 1 && c2 == 3) return 7;
    if (c1 == 3 && c2 == 1) return 8;
    if (c1 == 3 && c2 == 3) return 9;
    return -1;
}

// ComputeThreeMaxima (ORBmatcher.cc:2537-2573)
void three_maxima(const int *cnt, int &ind1, int &ind2, int &ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = cnt[i];
        if (s > max1) {
            max3 = max2, max2 = max1, max1 = s;
            ind3 = ind2, ind2 = ind1, ind1 = i;
        } else if (s > max2) {
            max3 = max2, max2 = s;
            ind3 = ind2, ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1, ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

}  // namespace

extern "C" {

// One keyframe pair (host pointers in the views); writes match12 [kf1.n]; returns nmatches.
int oracle_search_for_triangulation(const omv_tri_pair *P, const float *cams, const int32_t *cam_model,
                                    int only_stereo, int coarse, int check_ori) {
    const omv_kf_view &K1 = P->kf1, &K2 = P->kf2;
    for (int i = 0; i < K1.n; ++i) P->match12[i] = -1;
    int nmatches = 0;
    std::vector<int> hist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;
    // the persistent camera-pair state (R12, t12, pCamera1, pCamera2); LL before any assignment
    int state = 0;
    int a = 0, b = 0;
    while (a < K1.n_nodes && b < K2.n_nodes) {
        if (K1.node_id[a] == K2.node_id[b]) {
            for (int i1 = K1.node_start[a]; i1 < K1.node_start[a + 1]; ++i1) {
                const int idx1 = K1.node_idx[i1];
                if (K1.has_mp[idx1]) continue;
                if (only_stereo) continue;   // bStereo1 = (!mpCamera2 && ...) is false on multi-camera keyframes
                const omv_kp &kp1 = K1.kps[idx1];
                const int cam1 = cam_of(K1, idx1);
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int i2 = K2.node_start[b]; i2 < K2.node_start[b + 1]; ++i2) {
                    const int idx2 = K2.node_idx[i2];
                    if (K2.has_mp[idx2]) continue;
                    const int dist = hamming(K1.desc + 32 * (size_t)idx1, K2.desc + 32 * (size_t)idx2);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const omv_kp &kp2 = K2.kps[idx2];
                    const int cam2 = cam_of(K2, idx2);
                    const int pr = pair_of(cam1, cam2);
                    if (pr >= 0) state = pr;
                    static const int pc1[10] = {0, 0, 1, 1, 0, 2, 2, 1, 3, 3}, pc2[10] = {0, 1, 0, 1, 2, 0, 2, 3, 1, 3};
                    bool ok = coarse != 0;
                    const int m1 = cam_model ? cam_model[pc1[state]] : OMV_CAM_KB8;
                    const int m2 = cam_model ? cam_model[pc2[state]] : OMV_CAM_KB8;
                    if (!ok && m1 == OMV_CAM_PINHOLE)   // pCamera1->epipolarConstrain: Pinhole
                        ok = pinhole_epipolar(cams + 8 * pc1[state], cams + 8 * pc2[state], kp1, kp2, P->T[state],
                                              P->T[state] + 9, K2.level_sigma2[kp2.octave]);
                    else if (!ok)                       // KannalaBrandt8: TriangulateMatches(...) > 0.0001
                        ok = triangulate_matches(cams + 8 * pc1[state], cams + 8 * pc2[state], kp1, kp2, P->T[state],
                                                 P->T[state] + 9, K1.level_sigma2[kp1.octave],
                                                 K2.level_sigma2[kp2.octave], nullptr, m2) > 0.0001f;
                    if (ok) bestIdx2 = idx2, bestDist = dist;
                }
                if (bestIdx2 >= 0) {
                    const omv_kp &kp2 = K2.kps[bestIdx2];
                    P->match12[idx1] = bestIdx2;
                    nmatches++;
                    if (check_ori) {
                        float rot = kp1.angle - kp2.angle;
                        if (rot < 0.0) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        hist[bin].push_back(idx1);
                    }
                }
            }
            ++a, ++b;
        } else if (K1.node_id[a] < K2.node_id[b]) {
            ++a;   // lower_bound(f2it->first)
        } else {
            ++b;
        }
    }
    if (check_ori) {
        int cnt[HISTO_LENGTH], ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < HISTO_LENGTH; ++i) cnt[i] = (int)hist[i].size();
        three_maxima(cnt, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx1 : hist[i]) P->match12[idx1] = -1, nmatches--;
        }
    }
    return nmatches;
}

// Frame::ComputeMultiFishEyeMatches' depth check (src/Frame.cc:1488-1512) for one frame: l2r holds the
// Lowe-filtered candidates (right index or -1) of the nL left keypoints; on return the kept pairs, r2l
// (right block, the later left index wins), depth (-1 where none) and p3d [nL][3].
void oracle_stereo_triangulate(const omv_kp *kpsL, int nL, const omv_kp *kpsR, int nR, const float *camL,
                               const float *camR, const float *Rlr, const float *tlr, const float *sigma2,
                               int32_t *l2r, int32_t *r2l, float *depth, float *p3d) {
    for (int j = 0; j < nR; ++j) r2l[j] = -1;
    for (int i = 0; i < nL; ++i) {
        depth[i] = -1.0f;
        const int r = l2r[i];
        if (r < 0) continue;
        float p[3];
        const float d = triangulate_matches(camL, camR, kpsL[i], kpsR[r], Rlr, tlr, sigma2[kpsL[i].octave],
                                            sigma2[kpsR[r].octave], p);
        if (d > 0.0001f) {
            r2l[r] = i;
            depth[i] = d;
            for (int q = 0; q < 3; ++q) p3d[3 * i + q] = p[q];
        } else {
            l2r[i] = -1;
        }
    }
}

// The triangulated point and its projection into camera 1 (parity hook): out x3D[3] uv1[2].
void oracle_tri_point(const float *cam1, const float *cam2, const omv_kp *kp1, const omv_kp *kp2, const float *R12,
                      const float *t12, float *out) {
    float r1[3], r2[3], R21[9], t2[3], A[16], V[16];
    kb8_unproject_f(cam1, kp1->x, kp1->y, r1);
    kb8_unproject_f(cam2, kp2->x, kp2->y, r2);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R21[3 * i + j] = R12[3 * j + i];
    for (int i = 0; i < 3; ++i) t2[i] = -R21[3 * i] * t12[0] + -R21[3 * i + 1] * t12[1] + -R21[3 * i + 2] * t12[2];
    const float T1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const float T2[12] = {R21[0], R21[1], R21[2], t2[0], R21[3], R21[4], R21[5], t2[1], R21[6], R21[7], R21[8], t2[2]};
    for (int j = 0; j < 4; ++j) {
        A[j] = r1[0] * T1[8 + j] - T1[j];
        A[4 + j] = r1[1] * T1[8 + j] - T1[4 + j];
        A[8 + j] = r2[0] * T2[8 + j] - T2[j];
        A[12 + j] = r2[1] * T2[8 + j] - T2[4 + j];
    }
    jacobi_svd4_v(A, V);
    for (int i = 0; i < 3; ++i) out[i] = V[4 * i + 3] / V[15];
    kb8_project_f(cam1, out, out[3], out[4]);
}

// Parity hooks for the camera-model pieces.
void oracle_kb8_unproject(const float *cam, float x, float y, float *ray) { kb8_unproject_f(cam, x, y, ray); }
void oracle_jacobi_svd4_v(const float *A, float *V) { jacobi_svd4_v(A, V); }
void oracle_eigen_inverse3(const float *m, float *r) { eigen_inverse3(m, r); }
int oracle_pinhole_epipolar(const float *k1, const float *k2, const omv_kp *kp1, const omv_kp *kp2, const float *R12,
                            const float *t12, float unc) {
    return pinhole_epipolar(k1, k2, *kp1, *kp2, R12, t12, unc) ? 1 : 0;
}
float oracle_triangulate_matches(const float *cam1, const float *cam2, const omv_kp *kp1, const omv_kp *kp2,
                                 const float *R12, const float *t12, float sigma, float unc) {
    return triangulate_matches(cam1, cam2, *kp1, *kp2, R12, t12, sigma, unc);
}

}  // extern "C"

// LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:395-780), the per-match geometry after SearchForTriangulation,
// written after the reference's loop: sophTcw1 / Ow1 persist across neighbours, pCamera1 / pCamera2 and side 2 reset
// per neighbour; the listed camera pairs reassign them, the others keep the previous match's.  Float arithmetic with
// Eigen's 3-element expressions left to right; LocalMapping.cc sees `using namespace std` (DBoW2's
// TemplatedVocabulary.h), so cos / atan2 of floats are the float functions.
namespace {
float dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
float norm3(const float *a) { return std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }
int cnmp_cam(const omv_kf_view &k, int idx) {
    return k.n_left < 0 ? 0 : idx < k.n_left ? 0 : idx < k.n_left + k.n_right ? 1 : idx < k.n_left + k.n_right + k.n_sideleft ? 2 : 3;
}
// GeometricTools::Triangulate (src/GeometricTools.cc:27-50)
bool triangulate_gt(const float *x1, const float *x2, const float *T1, const float *T2, float *x3D) {
    float A[16], V[16];
    for (int j = 0; j < 4; ++j) {
        A[j] = x1[0] * T1[8 + j] - T1[j];
        A[4 + j] = x1[1] * T1[8 + j] - T1[4 + j];
        A[8 + j] = x2[0] * T2[8 + j] - T2[j];
        A[12 + j] = x2[1] * T2[8 + j] - T2[4 + j];
    }
    jacobi_svd4_v(A, V);
    if (V[15] == 0) return false;
    for (int i = 0; i < 3; ++i) x3D[i] = V[4 * i + 3] / V[15];
    return true;
}
// KeyFrame::UnprojectStereo (src/KeyFrame.cc:840-854)
bool unproject_stereo(const omv_cnmp_kf &K, int i, const float *depth, float *x3D) {
    const float z = depth[i];
    if (!(z > 0)) return false;
    const omv_kp &kp = (K.kps_raw ? K.kps_raw : K.kf.kps)[i];
    const float x = (kp.x - K.cx) * z * K.invfx, y = (kp.y - K.cy) * z * K.invfy;
    const float c[3] = {x, y, z};
    for (int r = 0; r < 3; ++r) x3D[r] = (K.Rwc[3 * r] * c[0] + K.Rwc[3 * r + 1] * c[1] + K.Rwc[3 * r + 2] * c[2]) + K.twc[r];
    return true;
}

// One neighbour of the loop (:443-782): the baseline gate on the persistent Ow1 (:447-454), then every match in idx1
// order with the camera-pair state; p1 (sophTcw1 / Ow1's camera block) persists across neighbours and is updated in
// place; has_mp1 (may be null) receives AddMapPoint(pMP, idx1) (:773).  Returns false when the gate skips it.
bool cnmp_job(const omv_cnmp_kf &K1, const omv_cnmp_job &J, const float *cams, const int32_t *cam_model, int n_cams,
              int inertial, int far_points, float th_far_points, float scale_factor, int check_baseline, int &p1,
              uint8_t *has_mp1) {
    auto model = [&](int c) { return cam_model ? cam_model[c] : OMV_CAM_KB8; };
    const float ratioFactor = 1.5f * scale_factor;
    const omv_cnmp_kf &K2 = J.kf2;
    for (int idx1 = 0; idx1 < K1.kf.n; ++idx1) J.status[idx1] = 0;
    if (check_baseline) {   // vBaseline = Ow2 - Ow1; baseline = vBaseline.norm(); if (baseline < pKF2->mb) continue;
        const float v[3] = {K2.Ow[0][0] - K1.Ow[p1][0], K2.Ow[0][1] - K1.Ow[p1][1], K2.Ow[0][2] - K1.Ow[p1][2]};
        if (norm3(v) < K2.mb) return false;
    }
    int c1 = 0, c2 = 0, p2 = 0;   // pCamera1 / pCamera2 / sophTcw2: reset per neighbour
    {
        for (int idx1 = 0; idx1 < K1.kf.n; ++idx1) {
            const int idx2 = J.match12[idx1];
            if (idx2 < 0 || idx2 >= K2.kf.n) continue;
            const omv_kp &kp1 = K1.kf.kps[idx1], &kp2 = K2.kf.kps[idx2];
            const int cameraId1 = cnmp_cam(K1.kf, idx1), cameraId2 = cnmp_cam(K2.kf, idx2);
            const float kp1_ur = K1.uright ? K1.uright[idx1] : -1.f, kp2_ur = K2.uright ? K2.uright[idx2] : -1.f;
            const bool bStereo1 = n_cams < 2 && kp1_ur >= 0, bStereo2 = n_cams < 2 && kp2_ur >= 0;
            if (n_cams >= 2) {
                const int code = cameraId1 * 4 + cameraId2;
                bool listed = code == 5 || code == 4 || code == 1 || code == 0;
                if (n_cams >= 4) listed = listed || code == 2 || code == 8 || code == 10 || code == 7 || code == 13 || code == 15;
                if (listed) p1 = c1 = cameraId1, p2 = c2 = cameraId2;
            }
            const float *T1 = K1.Tcw[p1], *T2 = K2.Tcw[p2];
            const float Rwc1[9] = {T1[0], T1[4], T1[8], T1[1], T1[5], T1[9], T1[2], T1[6], T1[10]};
            const float Rwc2[9] = {T2[0], T2[4], T2[8], T2[1], T2[5], T2[9], T2[2], T2[6], T2[10]};
            float xn1[3], xn2[3], ray1[3], ray2[3];
            cam_unproject_f(model(c1), cams + 8 * c1, kp1.x, kp1.y, xn1);
            cam_unproject_f(model(c2), cams + 8 * c2, kp2.x, kp2.y, xn2);
            for (int r = 0; r < 3; ++r) ray1[r] = Rwc1[3 * r] * xn1[0] + Rwc1[3 * r + 1] * xn1[1] + Rwc1[3 * r + 2] * xn1[2];
            for (int r = 0; r < 3; ++r) ray2[r] = Rwc2[3 * r] * xn2[0] + Rwc2[3 * r + 1] * xn2[1] + Rwc2[3 * r + 2] * xn2[2];
            const float cosParallaxRays = dot3(ray1, ray2) / (norm3(ray1) * norm3(ray2));
            float cosParallaxStereo = cosParallaxRays + 1;
            float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
            if (bStereo1) cosParallaxStereo1 = std::cos(2 * std::atan2(K1.mb / 2, K1.depth[idx1]));
            else if (bStereo2) cosParallaxStereo2 = std::cos(2 * std::atan2(K2.mb / 2, K2.depth[idx2]));
            cosParallaxStereo = std::min(cosParallaxStereo1, cosParallaxStereo2);
            float x3D[3];
            bool goodProj = false, bPointStereo = false;
            if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
                (bStereo1 || bStereo2 || (cosParallaxRays < 0.9996 && inertial) || (cosParallaxRays < 0.9998 && !inertial))) {
                goodProj = triangulate_gt(xn1, xn2, T1, T2, x3D);
                if (!goodProj) continue;
            } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
                bPointStereo = true;
                goodProj = unproject_stereo(K1, idx1, K1.depth, x3D);
            } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
                bPointStereo = true;
                goodProj = unproject_stereo(K2, idx2, K2.depth, x3D);
            } else {
                continue;
            }
            if (!goodProj) continue;
            const float R1r2[3] = {T1[8], T1[9], T1[10]}, R2r2[3] = {T2[8], T2[9], T2[10]};
            const float z1 = dot3(R1r2, x3D) + T1[11];
            if (z1 <= 0) continue;
            const float z2 = dot3(R2r2, x3D) + T2[11];
            if (z2 <= 0) continue;
            const float sigmaSquare1 = K1.kf.level_sigma2[kp1.octave];
            const float R1r0[3] = {T1[0], T1[1], T1[2]}, R1r1[3] = {T1[4], T1[5], T1[6]};
            const float x1 = dot3(R1r0, x3D) + T1[3], y1 = dot3(R1r1, x3D) + T1[7];
            const float invz1 = 1.0 / z1;
            if (!bStereo1) {
                const float X[3] = {x1, y1, z1};
                float u, v;
                cam_project_f(model(c1), cams + 8 * c1, X, u, v);
                const float errX1 = u - kp1.x, errY1 = v - kp1.y;
                if ((errX1 * errX1 + errY1 * errY1) > 5.991 * sigmaSquare1) continue;
            } else {
                const float u1 = K1.fx * x1 * invz1 + K1.cx, u1_r = u1 - K1.mbf * invz1, v1 = K1.fy * y1 * invz1 + K1.cy;
                const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y, errX1_r = u1_r - kp1_ur;
                if ((errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * sigmaSquare1) continue;
            }
            const float sigmaSquare2 = K2.kf.level_sigma2[kp2.octave];
            const float R2r0[3] = {T2[0], T2[1], T2[2]}, R2r1[3] = {T2[4], T2[5], T2[6]};
            const float x2 = dot3(R2r0, x3D) + T2[3], y2 = dot3(R2r1, x3D) + T2[7];
            const float invz2 = 1.0 / z2;
            if (!bStereo2) {
                const float X[3] = {x2, y2, z2};
                float u, v;
                cam_project_f(model(c2), cams + 8 * c2, X, u, v);
                const float errX2 = u - kp2.x, errY2 = v - kp2.y;
                if ((errX2 * errX2 + errY2 * errY2) > 5.991 * sigmaSquare2) continue;
            } else {
                const float u2 = K2.fx * x2 * invz2 + K2.cx, u2_r = u2 - K1.mbf * invz2, v2 = K2.fy * y2 * invz2 + K2.cy;
                const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y, errX2_r = u2_r - kp2_ur;
                if ((errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * sigmaSquare2) continue;
            }
            const float n1[3] = {x3D[0] - K1.Ow[p1][0], x3D[1] - K1.Ow[p1][1], x3D[2] - K1.Ow[p1][2]};
            const float n2[3] = {x3D[0] - K2.Ow[p2][0], x3D[1] - K2.Ow[p2][1], x3D[2] - K2.Ow[p2][2]};
            const float dist1 = norm3(n1), dist2 = norm3(n2);
            if (dist1 == 0 || dist2 == 0) continue;
            if (far_points && (dist1 >= th_far_points || dist2 >= th_far_points)) continue;
            const float ratioDist = dist2 / dist1;
            const float ratioOctave = K1.scale_factors[kp1.octave] / K2.scale_factors[kp2.octave];
            if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) continue;
            J.status[idx1] = bPointStereo ? 2 : 1;
            for (int q = 0; q < 3; ++q) J.x3D[3 * idx1 + q] = x3D[q];
            if (has_mp1) has_mp1[idx1] = 1;
        }
    }
    return true;
}
}  // namespace

extern "C" {
// omv_create_new_map_points restated: the jobs in order with the state chain (host arrays throughout: match12 / uright
// / depth / x3D / status / has_mp1 host pointers in this restatement).  side1_state: in/out (null: 0).
void oracle_create_new_map_points(int n_jobs, const omv_cnmp_kf *kf1p, const omv_cnmp_job *jobs, const float *cams,
                                  const int32_t *cam_model, int n_cams, int inertial, int far_points,
                                  float th_far_points, float scale_factor, int check_baseline, int32_t *side1_state,
                                  uint8_t *has_mp1) {
    int p1 = side1_state ? *side1_state : 0;   // sophTcw1 / Ow1 (camera block), persists across neighbours
    for (int j = 0; j < n_jobs; ++j)
        cnmp_job(*kf1p, jobs[j], cams, cam_model, n_cams, inertial, far_points, th_far_points, scale_factor,
                 check_baseline, p1, has_mp1);
    if (side1_state) *side1_state = p1;
}

// LocalMapping::CreateNewMapPoints' whole neighbour loop (:439-783): per neighbour the caller's skip (mbMonocular's
// median-depth test), the baseline gate, SearchForTriangulation(mpCurrentKeyFrame, pKF2, vMatchedIndices, false,
// bCoarse) with checkOri off (matcher(0.6, false), :417) against has_mp1 AS THE PREVIOUS NEIGHBOURS LEFT IT, then the
// geometry, whose accepted matches set has_mp1.  pairs[j]: kf1 / kf2 views, T, match12 (host); the kf1 view's has_mp is
// replaced by has_mp1.  n_matches[j]: the search's return value (0 when skipped).
void oracle_local_mapping_create_new_map_points(const omv_cnmp_kf *kf1p, uint8_t *has_mp1, int n_nb,
                                                const omv_tri_pair *pairs, const omv_cnmp_job *jobs, const int32_t *skip,
                                                const float *cams, const int32_t *cam_model, int n_cams, int inertial,
                                                int check_baseline, int coarse, int far_points, float th_far_points,
                                                float scale_factor, int32_t *n_matches, int32_t *side1_state) {
    const omv_cnmp_kf &K1 = *kf1p;
    int p1 = side1_state ? *side1_state : 0;
    for (int j = 0; j < n_nb; ++j) {
        const omv_cnmp_job &J = jobs[j];
        for (int i = 0; i < K1.kf.n; ++i) J.status[i] = 0, pairs[j].match12[i] = -1;
        n_matches[j] = 0;
        if (skip && skip[j]) continue;
        if (check_baseline) {
            const float v[3] = {J.kf2.Ow[0][0] - K1.Ow[p1][0], J.kf2.Ow[0][1] - K1.Ow[p1][1],
                                J.kf2.Ow[0][2] - K1.Ow[p1][2]};
            if (norm3(v) < J.kf2.mb) continue;
        }
        omv_tri_pair P = pairs[j];
        P.kf1.has_mp = has_mp1;
        n_matches[j] = oracle_search_for_triangulation(&P, cams, cam_model, 0, coarse, 0);
        omv_cnmp_job Jm = J;
        Jm.match12 = P.match12;
        cnmp_job(K1, Jm, cams, cam_model, n_cams, inertial, far_points, th_far_points, scale_factor, 0, p1, has_mp1);
    }
    if (side1_state) *side1_state = p1;
}
}  // extern "C"
