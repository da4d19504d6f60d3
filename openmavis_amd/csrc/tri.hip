// MI355X-native ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:1131-1456) for multi-camera
// keyframe pairs, with the camera models' epipolarConstrain dispatched on camera 1's type (:1380-1387):
// KannalaBrandt8::epipolarConstrain / TriangulateMatches / unproject / Triangulate
// (src/CameraModels/KannalaBrandt8.cpp:219-229, 319-395, 96-126, 414-429; Eigen's JacobiSVD<Matrix4f> restated
// in float) or Pinhole::epipolarConstrain (src/CameraModels/Pinhole.cpp:103-132; Eigen's 3x3 inverse restated).
//
// One 256-thread workgroup per keyframe pair (pairs are independent: vbMatched2 is never set, :1204,
// :1261).  The scan is the reference's: shared FeatureVector nodes in ascending id, for each keypoint idx1
// of the node (without a map point) the best candidate idx2 of the other keyframe's node by Hamming
// distance (<= TH_LOW, later equal distances replace earlier ones) among those passing the epipolar test.
// The only sequential coupling is the camera-pair state (R12, t12, pCamera1, pCamera2) that persists from
// one candidate to the next: camera pairs the reference lists assign it, the others reuse it.
//   1. The node intersection (each thread binary-searches one node of keyframe 1) and the candidate
//      space of all (node, idx1, idx2) in scan order are laid out in LDS.
//   2. All threads compute Hamming distances, 4 consecutive candidates each, and compact the few that
//      can matter (no map point on either side, distance <= TH_LOW) in scan order.
//   3. Epipolar tests run as a flat work list over all threads: a listed camera pair is tested with
//      its own transform; an unlisted one with every state it can possibly meet — the state entering
//      the batch plus each listed pair compacted before it (an OR-scan) — so the result the replay needs
//      is always among them.
//   4. Thread 0 replays the scan over the compacted candidates, looking the results up.
// That is tri_kernel (one workgroup per pair).  The default path splits it over the chip: tri_scan_kernel runs steps
// 1-3's scans on S slices of keyframe 1's nodes per pair, tri_epi_kernel runs every epipolar test as one flat list,
// tri_walk_kernel replays each pair on one wavefront (see the block above tri_scan_kernel); tri_kernel remains for a
// pair whose candidates overflow the slices' workspace.
// Float arithmetic without contraction; glibc's atan2f / tanf and correctly rounded sqrtf are restated
// (omv_device.h), so the result is bit-exact to oracle/tri_oracle.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include <cstdio>
#include <cstdlib>
#include <cstring>

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

constexpr int kTriLow = 50;          // ORBmatcher::TH_LOW
constexpr int kHisto = 30;           // HISTO_LENGTH
constexpr int kTriMaxKp = 16384;     // keypoints of keyframe 1 (orientation bins, 1 byte each; < 2^16)
constexpr int kTriThreads = 512;
constexpr int kTriWaves = kTriThreads / 64;
constexpr int kSeg = kTriThreads;    // keyframe-1 nodes intersected per segment
constexpr int kPerThread = 4;        // consecutive candidates per thread per tile
constexpr int kTile = kTriThreads * kPerThread;
constexpr int kVal = 4096;           // compacted candidates per replay batch

// KannalaBrandt8::project(const Eigen::Vector3f&): cos / sin of the promoted float (C double functions)
__device__ void kb8_project_f(const float *k, const float *X, float &u, float &v) {
    const float x2y2 = X[0] * X[0] + X[1] * X[1];
    const float theta = omv::glibc_atan2f(omv::sqrtf_cr(x2y2), X[2]);
    const float psi = omv::glibc_atan2f(X[1], X[0]);
    const float t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
    const float r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9;
    u = (float)((double)(k[0] * r) * cos((double)psi) + (double)k[2]);
    v = (float)((double)(k[1] * r) * sin((double)psi) + (double)k[3]);
}

// KannalaBrandt8::unproject (precision 1e-6, <= 10 Newton steps, scale = std::tan(theta) / theta_d)
__device__ void kb8_unproject_f(const float *k, float px, float py, float *ray) {
    const float pwx = (px - k[2]) / k[0], pwy = (py - k[3]) / k[1];
    float scale = 1.f;
    float theta_d = omv::sqrtf_cr(pwx * pwx + pwy * pwy);
    theta_d = fminf(fmaxf((float)(-3.14159265358979323846 / 2.f), theta_d), (float)(3.14159265358979323846 / 2.f));
    if ((double)theta_d > 1e-8) {
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
        scale = omv::glibc_tanf(theta) / theta_d;
    }
    ray[0] = pwx * scale, ray[1] = pwy * scale, ray[2] = 1.f;
}

// Pinhole::unprojectEig / project(const Eigen::Vector3f&) (Pinhole.cpp:26-32, :40-45): float, left to right
__device__ __forceinline__ void pinhole_unproject_f(const float *k, float px, float py, float *ray) {
    ray[0] = (px - k[2]) / k[0], ray[1] = (py - k[3]) / k[1], ray[2] = 1.f;
}
__device__ __forceinline__ void pinhole_project_f(const float *k, const float *X, float &u, float &v) {
    u = k[0] * X[0] / X[2] + k[2];
    v = k[1] * X[1] / X[2] + k[3];
}
// GeometricCamera::unprojectEig / project, dispatched on the camera type (the virtual calls of
// KannalaBrandt8::TriangulateMatches on pCamera2, KannalaBrandt8.cpp:330, :382)
__device__ __forceinline__ void cam_unproject_f(int model, const float *k, float px, float py, float *ray) {
    if (model == OMV_CAM_PINHOLE) pinhole_unproject_f(k, px, py, ray);
    else kb8_unproject_f(k, px, py, ray);
}
__device__ __forceinline__ void cam_project_f(int model, const float *k, const float *X, float &u, float &v) {
    if (model == OMV_CAM_PINHOLE) pinhole_project_f(k, X, u, v);
    else kb8_project_f(k, X, u, v);
}

// Eigen Matrix3f::inverse() (Eigen/src/LU/InverseImpl.h, compute_inverse<..., 3>): the cofactors of column 0,
// det = their dot product with column 0, result(i, j) = cofactor(j, i) * (1 / det).  Row-major m / r.
__device__ __forceinline__ float cofactor3(const float *m, int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[3 * i1 + j1] * m[3 * i2 + j2] - m[3 * i1 + j2] * m[3 * i2 + j1];
}
__device__ void eigen_inverse3(const float *m, float *r) {
    const float c0 = cofactor3(m, 0, 0), c1 = cofactor3(m, 1, 0), c2 = cofactor3(m, 2, 0);
    const float det = c0 * m[0] + c1 * m[3] + c2 * m[6];
    const float invdet = 1.f / det;
    r[0] = c0 * invdet, r[1] = c1 * invdet, r[2] = c2 * invdet;
    for (int i = 1; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = cofactor3(m, j, i) * invdet;
}
// C = A B (3x3 row-major), each entry a left-to-right 3-term sum
__device__ __forceinline__ void mat3_mul(const float *A, const float *B, float *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
// Pinhole::epipolarConstrain (Pinhole.cpp:103-132): F12 = K1^-T [t12]x R12 K2^-1 (Eigen's products
// evaluated left to right), the epipolar line of kp1 in image 2, dsqr = num^2 / den < 3.84 unc (double).
// K2 = pCamera2->toK_() -- the same fx 0 cx / 0 fy cy / 0 0 1 form for both camera types.
__device__ bool pinhole_epipolar(const float *k1, const float *k2, const omv_kp &kp1, const omv_kp &kp2,
                                 const float *R12, const float *t12, float unc) {
    const float K1t[9] = {k1[0], 0.f, 0.f, 0.f, k1[1], 0.f, k1[2], k1[3], 1.f};   // K1.transpose()
    const float K2[9] = {k2[0], 0.f, k2[2], 0.f, k2[1], k2[3], 0.f, 0.f, 1.f};
    const float tx[9] = {0.f, -t12[2], t12[1], t12[2], 0.f, -t12[0], -t12[1], t12[0], 0.f};   // Sophus::SO3f::hat
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
    return (double)dsqr < 3.84 * (double)unc;
}

// Eigen::JacobiSVD<Matrix4f>(A, ComputeFullV).matrixV() (row-major A, V): square, no QR preconditioner;
// scale by max |a_ij|; cyclic two-sided Jacobi sweeps with threshold max(FLT_MIN, 2 eps maxDiagEntry);
// singular values sorted descending (first max), V's columns with them.
__device__ void jacobi_svd4_v(const float *A, float *V) {
    float W[16];
    float scale = 0.f;
    for (int i = 0; i < 16; ++i) scale = fmaxf(scale, fabsf(A[i]));
    if (scale == 0.f) scale = 1.f;
    for (int i = 0; i < 16; ++i) W[i] = A[i] / scale, V[i] = (i % 5 == 0) ? 1.f : 0.f;
    const float considerAsZero = 1.17549435e-38f, precision = 2.f * 1.1920928955078125e-07f;
    float maxDiag = fabsf(W[0]);
    for (int i = 1; i < 4; ++i) maxDiag = fmaxf(maxDiag, fabsf(W[5 * i]));
    bool finished = false;
    while (!finished) {
        finished = true;
        for (int p = 1; p < 4; ++p)
            for (int q = 0; q < p; ++q) {
                const float threshold = fmaxf(considerAsZero, precision * maxDiag);
                if (!(fabsf(W[4 * p + q]) > threshold || fabsf(W[4 * q + p]) > threshold)) continue;
                finished = false;
                const float m00 = W[4 * p + p], m01 = W[4 * p + q], m10 = W[4 * q + p], m11 = W[4 * q + q];
                float c1, s1;
                const float t = m00 + m11, d = m10 - m01;
                if (fabsf(d) < considerAsZero) {
                    s1 = 0.f, c1 = 1.f;
                } else {
                    const float u = t / d;
                    const float tmp = omv::sqrtf_cr(1.f + u * u);
                    s1 = 1.f / tmp, c1 = u / tmp;
                }
                float n00 = m00, n01 = m01, n11 = m11;
                if (!(c1 == 1.f && s1 == 0.f)) {
                    n00 = c1 * m00 + s1 * m10, n01 = c1 * m01 + s1 * m11;
                    n11 = -s1 * m01 + c1 * m11;
                }
                float cr, sr;
                const float deno = 2.f * fabsf(n01);
                if (deno < considerAsZero) {
                    cr = 1.f, sr = 0.f;
                } else {
                    const float tau = (n00 - n11) / deno;
                    const float w = omv::sqrtf_cr(tau * tau + 1.f);
                    const float tt = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
                    const float sign_t = tt > 0.f ? 1.f : -1.f;
                    const float n = 1.f / omv::sqrtf_cr(tt * tt + 1.f);
                    sr = -sign_t * (n01 / fabsf(n01)) * fabsf(tt) * n;
                    cr = n;
                }
                const float cl = c1 * cr - s1 * -sr, sl = c1 * -sr + s1 * cr;
                if (!(cl == 1.f && sl == 0.f))
                    for (int k = 0; k < 4; ++k) {
                        const float xi = W[4 * p + k], yi = W[4 * q + k];
                        W[4 * p + k] = cl * xi + sl * yi;
                        W[4 * q + k] = -sl * xi + cl * yi;
                    }
                if (!(cr == 1.f && -sr == 0.f))
                    for (int k = 0; k < 4; ++k) {
                        float xi = W[4 * k + p], yi = W[4 * k + q];
                        W[4 * k + p] = cr * xi + -sr * yi;
                        W[4 * k + q] = -(-sr) * xi + cr * yi;
                        xi = V[4 * k + p], yi = V[4 * k + q];
                        V[4 * k + p] = cr * xi + -sr * yi;
                        V[4 * k + q] = -(-sr) * xi + cr * yi;
                    }
                maxDiag = fmaxf(maxDiag, fmaxf(fabsf(W[4 * p + p]), fabsf(W[4 * q + q])));
            }
    }
    float sv[4];
    for (int i = 0; i < 4; ++i) sv[i] = fabsf(W[5 * i]) * scale;
    for (int i = 0; i < 4; ++i) {
        int pos = i;
        for (int j = i + 1; j < 4; ++j)
            if (sv[j] > sv[pos]) pos = j;
        if (sv[pos] == 0.f) break;
        if (pos != i) {
            const float t = sv[i];
            sv[i] = sv[pos], sv[pos] = t;
            for (int k = 0; k < 4; ++k) {
                const float u = V[4 * k + i];
                V[4 * k + i] = V[4 * k + pos], V[4 * k + pos] = u;
            }
        }
    }
}

// KannalaBrandt8::TriangulateMatches (z1 > 0 on success, -1 .. -5 on the reference's rejections); camera 1 is
// the KannalaBrandt8 `this`, camera 2 of type model2 (its unprojectEig / project are virtual calls)
__device__ float triangulate_matches(const float *cam1, const float *cam2, const omv_kp &kp1, const omv_kp &kp2,
                                     const float *R12, const float *t12, float sigmaLevel, float unc,
                                     float *p3D = nullptr, int model2 = OMV_CAM_KB8) {
    float r1[3], r2[3], r21[3];
    kb8_unproject_f(cam1, kp1.x, kp1.y, r1);
    cam_unproject_f(model2, cam2, kp2.x, kp2.y, r2);
    for (int i = 0; i < 3; ++i) r21[i] = R12[3 * i] * r2[0] + R12[3 * i + 1] * r2[1] + R12[3 * i + 2] * r2[2];
    const float dot = r1[0] * r21[0] + r1[1] * r21[1] + r1[2] * r21[2];
    const float n1 = omv::sqrtf_cr(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
    const float n21 = omv::sqrtf_cr(r21[0] * r21[0] + r21[1] * r21[1] + r21[2] * r21[2]);
    const float cosParallaxRays = dot / (n1 * n21);
    if ((double)cosParallaxRays > 0.9998) return -1;
    float R21[9], t2[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R21[3 * i + j] = R12[3 * j + i];
    for (int i = 0; i < 3; ++i) t2[i] = -R21[3 * i] * t12[0] + -R21[3 * i + 1] * t12[1] + -R21[3 * i + 2] * t12[2];
    // Triangulate: A rows p.x T.row(2) - T.row(0), p.y T.row(2) - T.row(1); Tcw1 = [I | 0], Tcw2 = [R21 | t2]
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
    for (int i = 0; i < 3; ++i) x3D[i] = V[4 * i + 3] / V[15];
    const float z1 = x3D[2];
    if (z1 <= 0) return -2;
    const float z2 = R21[6] * x3D[0] + R21[7] * x3D[1] + R21[8] * x3D[2] + t2[2];
    if (z2 <= 0) return -3;
    float u1, v1;
    kb8_project_f(cam1, x3D, u1, v1);
    const float ex1 = u1 - kp1.x, ey1 = v1 - kp1.y;
    if ((double)(ex1 * ex1 + ey1 * ey1) > 5.991 * (double)sigmaLevel) return -4;
    float x3D2[3];
    for (int i = 0; i < 3; ++i) x3D2[i] = R21[3 * i] * x3D[0] + R21[3 * i + 1] * x3D[1] + R21[3 * i + 2] * x3D[2] + t2[i];
    float u2, v2;
    cam_project_f(model2, cam2, x3D2, u2, v2);
    const float ex2 = u2 - kp2.x, ey2 = v2 - kp2.y;
    if ((double)(ex2 * ex2 + ey2 * ey2) > 5.991 * (double)unc) return -5;
    if (p3D) p3D[0] = x3D[0], p3D[1] = x3D[1], p3D[2] = x3D[2];
    return z1;
}

__device__ __forceinline__ int cam_of(const omv_kf_view &k, int idx) {
    return idx < k.n_left ? 0 : idx < k.n_left + k.n_right ? 1 : idx < k.n_left + k.n_right + k.n_sideleft ? 2 : 3;
}
// (cameraId1, cameraId2) -> OMV_TRI_PAIRS index, or -1 where the reference keeps R12 / t12 (:1300-1392)
__device__ __forceinline__ int pair_of(int c1, int c2) {
    const int code = c1 * 4 + c2;
    switch (code) {
        case 0: return 0;    // LL
        case 1: return 1;    // LR
        case 4: return 2;    // RL
        case 5: return 3;    // RR
        case 2: return 4;    // L-SL
        case 8: return 5;    // SL-L
        case 10: return 6;   // SL-SL
        case 7: return 7;    // R-SR
        case 13: return 8;   // SR-R
        case 15: return 9;   // SR-SR
        default: return -1;
    }
}
__device__ __constant__ int kPairCam1[10] = {0, 0, 1, 1, 0, 2, 2, 1, 3, 3};
__device__ __constant__ int kPairCam2[10] = {0, 1, 0, 1, 2, 0, 2, 3, 1, 3};

struct TriCams {
    float cam[4][8];
    int model[4];   // OMV_CAM_KB8 / OMV_CAM_PINHOLE per camera (L, R, SL, SR)
};

// LocalMapping::CreateNewMapPoints' neighbour gate (src/LocalMapping.cc:447-461), evaluated by every kernel of a
// neighbour's search inside omv_local_mapping_create_new_map_points: the caller's skip, or (!mbMonocular) the baseline
// |Ow2 - Ow1| below pKF2->mb with Ow1 the centre of side 1's PERSISTENT camera block (*p1, written by the previous
// neighbour's cnmp_state_kernel; unchanged while this neighbour's search runs).  p1 == nullptr: no gate (the plain
// SearchForTriangulation calls).
struct TriGate {
    const int *p1;
    int skip, check_baseline;
    float Ow1[4][3], Ow2[3], mb2;
};
__device__ __forceinline__ float gate_norm3(float a, float b, float c) { return omv::sqrtf_cr(a * a + b * b + c * c); }
__device__ __forceinline__ bool gate_skip(const TriGate &g) {
    if (!g.p1) return false;
    if (g.skip) return true;
    if (!g.check_baseline) return false;
    const int p = *g.p1;
    const float baseline = gate_norm3(g.Ow2[0] - g.Ow1[p][0], g.Ow2[1] - g.Ow1[p][1], g.Ow2[2] - g.Ow1[p][2]);
    return baseline < g.mb2;
}

// pCamera1->epipolarConstrain(pCamera2, kp1, kp2, R12, t12, sigma2[kp1.octave], sigma2[kp2.octave]) (ORBmatcher.cc:
// 1380-1387), a virtual call on camera 1's type
__device__ bool epipolar_ok(const omv_tri_pair &P, const TriCams &C, int pr, const omv_kp &kp1, const omv_kp &kp2) {
    const int c1 = kPairCam1[pr], c2 = kPairCam2[pr];
    if (C.model[c1] == OMV_CAM_PINHOLE)
        return pinhole_epipolar(C.cam[c1], C.cam[c2], kp1, kp2, P.T[pr], P.T[pr] + 9, P.kf2.level_sigma2[kp2.octave]);
    return triangulate_matches(C.cam[c1], C.cam[c2], kp1, kp2, P.T[pr], P.T[pr] + 9, P.kf1.level_sigma2[kp1.octave],
                               P.kf2.level_sigma2[kp2.octave], nullptr, C.model[c2]) > 0.0001f;
}

// Exclusive block scan (kTriThreads threads, one value each) with associative `op`; `total` = op over all.
template <typename T, typename Op, int NT = kTriThreads>
__device__ __forceinline__ T block_scan_excl(T v, T id, Op op, T *s_w, T &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T o = __shfl_up(inc, d, 64);
        if (lane >= d) inc = op(o, inc);   // o covers the earlier lanes (op need not commute)
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    T pre = id;
    for (int i = 0; i < w; ++i) pre = op(pre, s_w[i]);
    total = pre;
    for (int i = w; i < NT / 64; ++i) total = op(total, s_w[i]);
    T ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = id;
    __syncthreads();
    return op(pre, ex);
}

// compacted candidate code: distance bits 0-5, listed bit 6, camera pair bits 8-11
constexpr uint16_t kCodeListed = 0x40;

// Steps 1-2 over keyframe 1's nodes [a_lo, a_hi): the node intersection segment by segment, then the Hamming
// distances tile by tile, the candidates that can matter compacted in scan order into v_pk / v_code (n_valid of
// them); `flush` empties the staging when the next tile might not fit.  Every thread of the block calls it.
template <typename Flush>
__device__ __forceinline__ void scan_candidates(const omv_kf_view &K1, const omv_kf_view &K2, int a_lo, int a_hi,
                                                int *seg_s1, int *seg_n1, int *seg_s2, int *seg_n2, int *seg_pref,
                                                uint32_t *v_pk, uint16_t *v_code, int *s_wi, int &n_valid,
                                                Flush &flush) {
    const int tid = threadIdx.x;
    auto add = [](int x, int y) { return x + y; };
    for (int a0 = a_lo; a0 < a_hi; a0 += kSeg) {
        // step 1: this segment's node intersection, in ascending node id
        int s1 = 0, n1 = 0, s2 = 0, n2 = 0;
        const int a = a0 + tid;
        if (a < a_hi) {
            const uint32_t id = K1.node_id[a];
            int lo = 0, hi = K2.n_nodes;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (K2.node_id[mid] < id) lo = mid + 1;
                else hi = mid;
            }
            if (lo < K2.n_nodes && K2.node_id[lo] == id) {
                s1 = K1.node_start[a], n1 = K1.node_start[a + 1] - s1;
                s2 = K2.node_start[lo], n2 = K2.node_start[lo + 1] - s2;
            }
        }
        const int has = (n1 > 0 && n2 > 0) ? 1 : 0;
        int n_seg;
        const int pos = block_scan_excl(has, 0, add, s_wi, n_seg);
        int q_seg;
        const int qoff = block_scan_excl(has ? n1 * n2 : 0, 0, add, s_wi, q_seg);
        if (has) seg_s1[pos] = s1, seg_n1[pos] = n1, seg_s2[pos] = s2, seg_n2[pos] = n2, seg_pref[pos] = qoff;
        if (tid == 0) seg_pref[n_seg] = q_seg;
        __syncthreads();
        // step 2: distances and compaction, tile by tile
        for (int t0 = 0; t0 < q_seg; t0 += kTile) {
            if (n_valid + kTile > kVal) flush();
            uint32_t pk[kPerThread];
            uint16_t cd[kPerThread];
            int cnt = 0;
            const int qb = t0 + tid * kPerThread;
            if (qb < q_seg) {
                int lo = 0, hi = n_seg;   // last node with seg_pref <= qb
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (seg_pref[mid] <= qb) lo = mid;
                    else hi = mid;
                }
                // the thread's candidates (LDS walk), then each dependent global step for all of them together:
                // keypoint indices, map-point flags, descriptors -- three memory round trips per tile instead of
                // three per candidate
                int nd = lo, loc = qb - seg_pref[lo];
                int i1 = loc / seg_n2[nd], i2 = loc - i1 * seg_n2[nd];
                int a1[kPerThread], a2[kPerThread];
                const int nj = min(kPerThread, q_seg - qb);
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) {
                    a1[j] = seg_s1[nd] + i1, a2[j] = seg_s2[nd] + i2;
                    if (j + 1 < nj && ++i2 == seg_n2[nd]) {
                        i2 = 0;
                        if (++i1 == seg_n1[nd]) i1 = 0, ++nd;
                    }
                }
                int x1[kPerThread], x2[kPerThread];
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) {
                    const int jj = min(j, nj - 1);   // past the end: the last candidate again (loads stay in range)
#ifdef OMV_TRI_CHECK
                    if (a1[jj] < 0 || a1[jj] >= K1.node_start[K1.n_nodes] || a2[jj] < 0 || a2[jj] >= K2.node_start[K2.n_nodes]) {
                        printf("scan bad a1 %d a2 %d (blk %d,%d tid %d qb %d q_seg %d nd %d n_seg %d)\n", a1[jj], a2[jj], blockIdx.x, blockIdx.y, tid, qb, q_seg, nd, n_seg);
                        a1[jj] = 0, a2[jj] = 0;
                    }
#endif
                    x1[j] = K1.node_idx[a1[jj]], x2[j] = K2.node_idx[a2[jj]];
                }
#ifdef OMV_TRI_CHECK
#pragma unroll
                for (int j = 0; j < kPerThread; ++j)
                    if (x1[j] < 0 || x1[j] >= K1.n || x2[j] < 0 || x2[j] >= K2.n) {
                        printf("scan bad x1 %d x2 %d (n %d %d) blk %d,%d\n", x1[j], x2[j], K1.n, K2.n, blockIdx.x, blockIdx.y);
                        x1[j] = 0, x2[j] = 0;
                    }
#endif
                bool free_[kPerThread];
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) free_[j] = !K1.has_mp[x1[j]] && !K2.has_mp[x2[j]];
                uint4 d1[kPerThread][2], d2[kPerThread][2];
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) {
                    const uint4 *p1 = reinterpret_cast<const uint4 *>(K1.desc + 32 * (size_t)x1[j]);
                    const uint4 *p2 = reinterpret_cast<const uint4 *>(K2.desc + 32 * (size_t)x2[j]);
                    d1[j][0] = p1[0], d1[j][1] = p1[1], d2[j][0] = p2[0], d2[j][1] = p2[1];
                }
#pragma unroll
                for (int j = 0; j < kPerThread; ++j) {
                    if (j >= nj || !free_[j]) continue;
                    const int dist = __popc(d1[j][0].x ^ d2[j][0].x) + __popc(d1[j][0].y ^ d2[j][0].y) +
                                     __popc(d1[j][0].z ^ d2[j][0].z) + __popc(d1[j][0].w ^ d2[j][0].w) +
                                     __popc(d1[j][1].x ^ d2[j][1].x) + __popc(d1[j][1].y ^ d2[j][1].y) +
                                     __popc(d1[j][1].z ^ d2[j][1].z) + __popc(d1[j][1].w ^ d2[j][1].w);
                    if (dist <= kTriLow) {
                        const int pr = pair_of(cam_of(K1, x1[j]), cam_of(K2, x2[j]));
                        pk[cnt] = (uint32_t)x1[j] << 16 | (uint32_t)x2[j];
                        cd[cnt] = (uint16_t)(dist | (pr >= 0 ? kCodeListed | (pr << 8) : 0));
                        ++cnt;
                    }
                }
            }
            int tot;
            const int off = n_valid + block_scan_excl(cnt, 0, add, s_wi, tot);
            for (int j = 0; j < cnt; ++j) v_pk[off + j] = pk[j], v_code[off + j] = cd[j];
            n_valid += tot;
        }
    }
}

__global__ void __launch_bounds__(kTriThreads) tri_kernel(const omv_tri_pair *pairs, TriCams C, int only_stereo,
                                                          int coarse, int check_ori, int32_t *n_matches, int *err,
                                                          const int *only, TriGate gate) {
    __shared__ uint8_t bins[kTriMaxKp];
    __shared__ int seg_s1[kSeg], seg_n1[kSeg], seg_s2[kSeg], seg_n2[kSeg], seg_pref[kSeg + 1];
    __shared__ uint32_t v_pk[kVal];      // idx1 << 16 | idx2
    __shared__ uint16_t v_code[kVal], v_mask[kVal];
    __shared__ uint32_t v_res[kVal];     // epipolar results, one bit per camera-pair state
    __shared__ int v_item[kVal + 1];
    __shared__ int s_wi[kTriWaves];
    __shared__ unsigned s_wu[kTriWaves];
    __shared__ int hist[kHisto];
    __shared__ int s_keep[kHisto];
    __shared__ int s_state, s_row, s_best, s_bidx, s_fin;
    if (only && !only[blockIdx.x]) return;
    if (gate_skip(gate)) return;   // the walk wrote the skipped neighbour's empty result
    const omv_tri_pair &P = pairs[blockIdx.x];
    const omv_kf_view &K1 = P.kf1, &K2 = P.kf2;
    const int tid = threadIdx.x;
    for (int i = tid; i < K1.n; i += kTriThreads) P.match12[i] = -1;
    if (K1.n > kTriMaxKp || K2.n > 65535) {
        if (tid == 0) atomicExch(err, OMV_ERR_CAPACITY), n_matches[blockIdx.x] = 0;
        return;
    }
    for (int i = tid; i < K1.n; i += kTriThreads) bins[i] = 0xff;
    if (tid < kHisto) hist[tid] = 0;
    if (tid == 0) s_state = 0, s_row = -1, s_best = kTriLow, s_bidx = -1;   // camera-pair state: LL before any assignment
    __syncthreads();
    auto add = [](int x, int y) { return x + y; };
    int nmatch = 0;   // thread 0's count
    // the row the walk has open when it ends (its best match, if any, is written like a finished row)
    auto finish_row = [&](int row, int best) {
        if (row < 0 || best < 0) return;
        P.match12[row] = best;
        ++nmatch;
        if (check_ori) {
            float rot = K1.kps[row].angle - K2.kps[best].angle;
            if ((double)rot < 0.0) rot += 360.0f;
            int bin = (int)roundf(rot * (1.0f / kHisto));
            if (bin == kHisto) bin = 0;
            bins[row] = (uint8_t)bin;
        }
    };
    int n_valid = 0;
#ifdef OMV_TRI_PROFILE
    long long tq[5] = {0, 0, 0, 0, 0}, tl = wall_clock64();
    int n_cand = 0, n_tests = 0, n_flush = 0, n_qseg = 0;
#define OMV_TQ(k) (tq[k] += wall_clock64() - tl, tl = wall_clock64())
#else
#define OMV_TQ(k) ((void)0)
#endif
    // epipolar tests of the compacted batch (step 3) and the in-order replay (step 4)
    auto flush = [&]() {
        __syncthreads();   // the last tile's compacted entries
        OMV_TQ(1);
        if (!coarse) {
            // States entry k can meet: the last listed entry before it that is certain to pass the distance
            // test (an anchor: its distance <= every earlier distance of its row, and <= the replay's
            // bestDist when the row continues from the previous batch) fixes the state; listed entries
            // after the anchor may change it.  Two segmented scans per tile: a min-scan of the distances
            // (reset at row starts) finds the anchors, an OR-scan of the listed pairs (reset at anchors)
            // gives the masks.  Bit 8 / bit 16 mark a segment start.
            auto seg_min = [](unsigned x, unsigned y) {
                return ((x | y) & 0x100u) | ((y & 0x100u) ? (y & 0xffu) : min(x & 0xffu, y & 0xffu));
            };
            auto seg_or = [](unsigned x, unsigned y) {
                return ((x | y) & 0x10000u) | ((y & 0x10000u) ? (y & 0xffffu) : ((x | y) & 0xffffu));
            };
            unsigned cmin = (n_valid > 0 && (int)(v_pk[0] >> 16) == s_row) ? (unsigned)s_best : 0xffu;
            unsigned cor = 1u << s_state;
            int icarry = 0;
            for (int t0 = 0; t0 < n_valid; t0 += kTriThreads) {
                const int k = t0 + tid;
                unsigned vmin = 0xffu, vor = 0;
                bool listed = false;
                int dist = 0, pr = 0;
                if (k < n_valid) {
                    const int code = v_code[k];
                    listed = (code & kCodeListed) != 0;
                    dist = code & 0x3f, pr = (code >> 8) & 15;
                    const int row = (int)(v_pk[k] >> 16);
                    const int prev = k > 0 ? (int)(v_pk[k - 1] >> 16) : s_row;
                    vmin = (row != prev ? 0x100u : 0u) | (unsigned)dist;
                }
                unsigned tmin;
                const unsigned bmin = seg_min(cmin, block_scan_excl(vmin, 0xffu, seg_min, s_wu, tmin));
                const bool row_start = (vmin & 0x100u) != 0;
                const bool anchor = listed && (row_start || (unsigned)dist <= (bmin & 0xffu));
                if (listed) vor = (anchor ? 0x10000u : 0u) | (1u << pr);
                unsigned tor;
                const unsigned bor_ = seg_or(cor, block_scan_excl(vor, 0u, seg_or, s_wu, tor));
                const unsigned m = listed ? (1u << pr) : (bor_ & 0x3ffu);
                const int cnt = k < n_valid ? __popc(m) : 0;
                int itot;
                const int off = icarry + block_scan_excl(cnt, 0, add, s_wi, itot);
                if (k < n_valid) v_mask[k] = (uint16_t)m, v_item[k] = off, v_res[k] = 0;
                cmin = seg_min(cmin, tmin);
                cor = seg_or(cor, tor);
                icarry += itot;
            }
            if (tid == 0) v_item[n_valid] = icarry;
            __syncthreads();
            OMV_TQ(2);
#ifdef OMV_TRI_PROFILE
            n_cand += n_valid, n_tests += icarry, ++n_flush;
#endif
            for (int j = tid; j < icarry; j += kTriThreads) {
                int lo = 0, hi = n_valid;   // last k with v_item[k] <= j
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (v_item[mid] <= j) lo = mid;
                    else hi = mid;
                }
                unsigned m = v_mask[lo];
                for (int r = j - v_item[lo]; r > 0; --r) m &= m - 1;
                const int state = __ffs(m) - 1;
                const uint32_t pk = v_pk[lo];
                if (epipolar_ok(P, C, state, K1.kps[pk >> 16], K2.kps[pk & 0xffff])) atomicOr(&v_res[lo], 1u << state);
            }
            __syncthreads();
            OMV_TQ(3);
        }
        // step 4 on wave 0: 64 entries at a time staged in registers (one per lane), walked in order on wave-uniform
        // values (v_readlane), so the dependent chain is scalar ALU work instead of LDS round trips; the rows the walk
        // finishes are listed (row << 16 | idx2, in v_item, free after step 3) and written out by all threads after
        // the walk's state (camera-pair state, open row, its best distance / match) lives in LDS between batches and
        // in scalar registers during one: every value of the walk is wave-uniform (readfirstlane / readlane)
        if (tid < 64) {
            const int lane = tid;
            int state = __builtin_amdgcn_readfirstlane(s_state), cur_row = __builtin_amdgcn_readfirstlane(s_row);
            int bestDist = __builtin_amdgcn_readfirstlane(s_best), bestIdx2 = __builtin_amdgcn_readfirstlane(s_bidx);
            int n_fin = 0;
            const int nv = __builtin_amdgcn_readfirstlane(n_valid);   // uniform (a block-scan total)
            // branch-free: a taken scalar branch costs a fetch redirect, which dominated the walk (~280 cycles per
            // entry with the branches); the tail of the last 64 is padded with no-op entries (the last entry's row,
            // distance 63 > any bestDist, not listed)
            for (int c0 = 0; c0 < nv; c0 += 64) {
                const int k = c0 + lane;
                const bool in = k < nv;
                const uint32_t pk_l = v_pk[in ? k : nv - 1];
                const int code_l = in ? (int)v_code[k] : 0x3f;
                const uint32_t res_l = (in && !coarse) ? v_res[k] : 0xffffffffu;
#pragma unroll
                for (int j = 0; j < 64; ++j) {
                    const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)pk_l, j);
                    const int code = __builtin_amdgcn_readlane(code_l, j);
                    const uint32_t res = (uint32_t)__builtin_amdgcn_readlane((int)res_l, j);
                    const int idx1 = (int)(pk >> 16);
                    const bool newrow = idx1 != cur_row;
                    const bool emit = newrow && cur_row >= 0 && bestIdx2 >= 0;
                    v_item[n_fin] = (cur_row << 16) | (bestIdx2 & 0xffff);   // kept only when emit (n_fin advances)
                    n_fin += emit ? 1 : 0;
                    cur_row = newrow ? idx1 : cur_row;
                    bestDist = newrow ? kTriLow : bestDist;
                    bestIdx2 = newrow ? -1 : bestIdx2;
                    const int dist = code & 0x3f;
                    const bool cand = dist <= bestDist;
                    state = (cand && (code & kCodeListed)) ? (code >> 8) & 15 : state;
                    const bool take = cand && ((res >> state) & 1u);
                    bestIdx2 = take ? (int)(pk & 0xffff) : bestIdx2;
                    bestDist = take ? dist : bestDist;
                }
            }
            if (lane == 0) s_state = state, s_row = cur_row, s_best = bestDist, s_bidx = bestIdx2, s_fin = n_fin;
        }
        __syncthreads();
        OMV_TQ(4);
        const int n_fin = s_fin;
        nmatch += n_fin;   // thread 0's count (the only one read)
        for (int i = tid; i < n_fin; i += kTriThreads) {
            const int row = (int)((uint32_t)v_item[i] >> 16), best = v_item[i] & 0xffff;
            P.match12[row] = best;
            if (check_ori) {
                float rot = K1.kps[row].angle - K2.kps[best].angle;
                if ((double)rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * (1.0f / kHisto));
                if (bin == kHisto) bin = 0;
                bins[row] = (uint8_t)bin;
            }
        }
        __syncthreads();
        OMV_TQ(0);
        n_valid = 0;
    };
    if (!only_stereo)
        scan_candidates(K1, K2, 0, K1.n_nodes, seg_s1, seg_n1, seg_s2, seg_n2, seg_pref, v_pk, v_code, s_wi, n_valid,
                        flush);
    flush();
    if (tid == 0) finish_row(s_row, s_bidx);
    __syncthreads();
    if (check_ori) {   // rotation histogram: keep the three largest bins (ComputeThreeMaxima, :2537-2573)
        for (int i = tid; i < K1.n; i += kTriThreads)
            if (bins[i] != 0xff) atomicAdd(&hist[bins[i]], 1);
        __syncthreads();
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kHisto; i++) {
                const int s = hist[i];
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
            if (max2 < 0.1f * (float)max1) ind2 = -1, ind3 = -1;
            else if (max3 < 0.1f * (float)max1) ind3 = -1;
            for (int i = 0; i < kHisto; ++i) s_keep[i] = (i == ind1 || i == ind2 || i == ind3) ? 1 : 0;
        }
        __syncthreads();
        int removed = 0;
        for (int i = tid; i < K1.n; i += kTriThreads)
            if (bins[i] != 0xff && !s_keep[bins[i]]) P.match12[i] = -1, ++removed;
        int tot;
        block_scan_excl(removed, 0, add, s_wi, tot);
        if (tid == 0) nmatch -= tot;
    }
    if (tid == 0) n_matches[blockIdx.x] = nmatch;
#ifdef OMV_TRI_PROFILE
    OMV_TQ(1);
    if (tid == 0 && blockIdx.x < 4)
        printf("tri pair %d ticks(100MHz): scan+dist %lld scans %lld epipolar %lld replay %lld writeout %lld; candidates %d tests %d flushes %d pairs scanned %d\n",
               blockIdx.x, tq[1], tq[2], tq[3], tq[4], tq[0], n_cand, n_tests, n_flush, n_qseg);
#endif
#undef OMV_TQ
}

// ---- the same search as three launches, the pairs' scans spread over the chip -----------------------------------
// tri_kernel runs one keyframe pair per workgroup: at 2 waves per SIMD its dependent loads, its epipolar tests and the
// one-wave replay leave a pair ~0.7 ms on one CU.  Here
//   tri_scan_kernel  (slice, pair): steps 1-2 over 1/S of keyframe 1's nodes (a row -- one idx1 -- never spans two
//                    slices: a keypoint sits in one node), then the state masks of step 3 with the camera-pair state
//                    entering the slice unknown (all ten states until the slice's first anchor; slice 0 starts in
//                    LL); entries (pk, code word) and the epipolar test list (entry, state) written out;
//   tri_epi_kernel   every test of every slice as one flat work list (one test per thread);
//   tri_walk_kernel  one workgroup per pair: the replay over the slices in order on one wavefront, branch-free on
//                    scalar registers (one 32-bit word per entry), then the finished rows, the rotation histogram.
// Per (pair, slice) the entries and tests fit fixed capacities; a pair that overflows one is flagged and the host
// runs tri_kernel for it alone.
struct TriWs {
    uint32_t *pk;      // [n_pairs * S][ecap] idx1 << 16 | idx2
    uint32_t *w;       // [..][ecap] dist | listed << 6 | pair state << 7 | row start << 11
    uint32_t *res;     // [..][ecap] epipolar results, one bit per camera-pair state (all ones when coarse)
    uint32_t *tests;   // [..][tcap] entry << 4 | state
    int *cnt, *tcnt;   // [n_pairs * S]
    int *over;         // [n_pairs] a capacity was exceeded: the pair is rerun by tri_kernel
    int S, ecap, tcap;
};

__global__ void __launch_bounds__(kTriThreads) tri_scan_kernel(const omv_tri_pair *pairs, int only_stereo, int coarse,
                                                               TriWs ws, TriGate gate) {
    __shared__ int seg_s1[kSeg], seg_n1[kSeg], seg_s2[kSeg], seg_n2[kSeg], seg_pref[kSeg + 1];
    __shared__ uint32_t v_pk[kVal];
    __shared__ uint16_t v_code[kVal];
    __shared__ int s_wi[kTriWaves];
    __shared__ unsigned s_wu[kTriWaves];
    const int sl = blockIdx.x, p = blockIdx.y, S = ws.S, tid = threadIdx.x;
    const omv_tri_pair &P = pairs[p];
    const omv_kf_view &K1 = P.kf1, &K2 = P.kf2;
    const size_t slot = (size_t)p * S + sl, ebase = slot * ws.ecap, tbase = slot * ws.tcap;
    const bool bad = K1.n > kTriMaxKp || K2.n > 65535 || gate_skip(gate);   // reported by the walk
    const int a_lo = (int)((long long)K1.n_nodes * sl / S), a_hi = (int)((long long)K1.n_nodes * (sl + 1) / S);
    auto add = [](int x, int y) { return x + y; };
    auto seg_min = [](unsigned x, unsigned y) {
        return ((x | y) & 0x100u) | ((y & 0x100u) ? (y & 0xffu) : min(x & 0xffu, y & 0xffu));
    };
    auto seg_or = [](unsigned x, unsigned y) {
        return ((x | y) & 0x10000u) | ((y & 0x10000u) ? (y & 0xffffu) : ((x | y) & 0xffffu));
    };
    int n_valid = 0, n_out = 0, t_out = 0, last_row = -1;
    // scan states carried from batch to batch: a continuing row's earlier distances bound bestDist from below
    // (bestDist is one of them or TH_LOW), so an entry at or below their minimum is an anchor; the pair's state
    // is LL entering slice 0 and unknown entering any other
    unsigned cmin = 0xffu, cor = sl == 0 ? 1u : 0x3ffu;
    auto flush = [&]() {
        __syncthreads();   // the last tile's compacted entries
        int icarry = 0;
        for (int t0 = 0; t0 < n_valid; t0 += kTriThreads) {
            const int k = t0 + tid;
            unsigned vmin = 0xffu, vor = 0;
            bool listed = false;
            int dist = 0, pr = 0;
            uint32_t pk = 0;
            if (k < n_valid) {
                const int code = v_code[k];
                listed = (code & kCodeListed) != 0;
                dist = code & 0x3f, pr = (code >> 8) & 15;
                pk = v_pk[k];
                const int prev = k > 0 ? (int)(v_pk[k - 1] >> 16) : last_row;
                vmin = ((int)(pk >> 16) != prev ? 0x100u : 0u) | (unsigned)dist;
            }
            unsigned tmin;
            const unsigned bmin = seg_min(cmin, block_scan_excl(vmin, 0xffu, seg_min, s_wu, tmin));
            const bool row_start = (vmin & 0x100u) != 0;
            const bool anchor = listed && (row_start || (unsigned)dist <= (bmin & 0xffu));
            if (listed) vor = (anchor ? 0x10000u : 0u) | (1u << pr);
            unsigned tor;
            const unsigned bor_ = seg_or(cor, block_scan_excl(vor, 0u, seg_or, s_wu, tor));
            const unsigned m = coarse ? 0u : (listed ? (1u << pr) : (bor_ & 0x3ffu));
            const int cnt = k < n_valid ? __popc(m) : 0;
            int itot;
            const int off = t_out + icarry + block_scan_excl(cnt, 0, add, s_wi, itot);
            const int e = n_out + k;
            if (k < n_valid && e < ws.ecap) {
                ws.pk[ebase + e] = pk;
                ws.w[ebase + e] = (uint32_t)dist | (listed ? 0x40u : 0u) | ((uint32_t)pr << 7) | (row_start ? 0x800u : 0u);
                ws.res[ebase + e] = coarse ? 0x3ffu : 0u;
                unsigned mm = m;
                for (int r = 0; mm; ++r, mm &= mm - 1)
                    if (off + r < ws.tcap) ws.tests[tbase + off + r] = (uint32_t)e << 4 | (uint32_t)(__ffs(mm) - 1);
            }
            cmin = seg_min(cmin, tmin);
            cor = seg_or(cor, tor);
            icarry += itot;
        }
        if (n_valid > 0) last_row = (int)(v_pk[n_valid - 1] >> 16);
        n_out += n_valid, t_out += icarry;
        __syncthreads();   // v_pk is refilled by the next tile
        n_valid = 0;
    };
    if (!only_stereo && !bad)
        scan_candidates(K1, K2, a_lo, a_hi, seg_s1, seg_n1, seg_s2, seg_n2, seg_pref, v_pk, v_code, s_wi, n_valid,
                        flush);
    flush();
    if (tid == 0) {
        ws.cnt[slot] = min(n_out, ws.ecap), ws.tcnt[slot] = min(t_out, ws.tcap);
        if (n_out > ws.ecap || t_out > ws.tcap) atomicOr(&ws.over[p], 1);
    }
}

constexpr int kEpiThreads = 256, kEpiPerSlot = 2;   // workgroups per (pair, slice) of the flat test list
__global__ void __launch_bounds__(kEpiThreads) tri_epi_kernel(const omv_tri_pair *pairs, TriCams C, TriWs ws) {
    const int slot = blockIdx.y, p = slot / ws.S;
    // an overflowed pair's test list has holes (the tests of entries past the capacity are not written): skip it,
    // tri_kernel reruns the pair
    if (ws.over[p]) return;
    const omv_tri_pair &P = pairs[p];
    const size_t ebase = (size_t)slot * ws.ecap, tbase = (size_t)slot * ws.tcap;
    const int nt = ws.tcnt[slot];
    for (int j = blockIdx.x * kEpiThreads + threadIdx.x; j < nt; j += kEpiPerSlot * kEpiThreads) {
        const uint32_t it = ws.tests[tbase + j];
        const int e = (int)(it >> 4), state = (int)(it & 15);
#ifdef OMV_TRI_CHECK
        if (e >= ws.ecap || state > 9) { printf("epi bad slot %d j %d nt %d e %d state %d\n", slot, j, nt, e, state); continue; }
        {
            const uint32_t pk0 = ws.pk[ebase + e];
            if ((int)(pk0 >> 16) >= P.kf1.n || (int)(pk0 & 0xffff) >= P.kf2.n) { printf("epi bad pk slot %d e %d pk %x\n", slot, e, pk0); continue; }
        }
#endif
        const uint32_t pk = ws.pk[ebase + e];
        if (epipolar_ok(P, C, state, P.kf1.kps[pk >> 16], P.kf2.kps[pk & 0xffff]))
            atomicOr(&ws.res[ebase + e], 1u << state);
    }
}

constexpr int kWalkThreads = 256;
constexpr int kWalkRows = 4096;   // rows of the parallel replay (more: the scalar walk)
constexpr uint64_t kIdentityMap = 0x9876543210ull;   // state s -> s, nibble s

// One row's replay from camera-pair state `st` (entries [e0, e1) of the workspace): the state after it and its best
// entry (-1: none) -- the scalar walk's update, restated per row.
__device__ __forceinline__ int walk_row(const TriWs &ws, int e0, int e1, int &st) {
    int bestDist = kTriLow, bestK = -1;
#ifdef OMV_TRI_CHECK
    if (e0 < 0 || e1 < e0 || e1 - e0 > 65536) { printf("walk_row bad %d %d\n", e0, e1); return -1; }
#endif
    for (int e = e0; e < e1; ++e) {
        const uint32_t w = ws.w[e] | (ws.res[e] << 12);
        const int dist = (int)(w & 63u);
        const bool cand = dist <= bestDist;
        st = (cand && ((w >> 6) & 1u)) ? (int)((w >> 7) & 15u) : st;
        const bool take = cand && ((w >> (12 + st)) & 1u);
        bestK = take ? e : bestK;
        bestDist = take ? dist : bestDist;
    }
    return bestK;
}

__global__ void __launch_bounds__(kWalkThreads) tri_walk_kernel(const omv_tri_pair *pairs, int check_ori, TriWs ws,
                                                                int32_t *n_matches, int *err, int par_walk,
                                                                TriGate gate) {
    __shared__ uint8_t bins[kTriMaxKp];
    __shared__ int fin[kTriMaxKp];   // finished rows: the global entry index of the row's best (parallel replay: rows)
    __shared__ uint8_t instate[kWalkRows + 64];
    __shared__ int hist[kHisto], s_keep[kHisto], s_wi[kWalkThreads / 64], s_fin, s_rows;
    const int p = blockIdx.x, tid = threadIdx.x, S = ws.S;
    const omv_tri_pair &P = pairs[p];
    const omv_kf_view &K1 = P.kf1, &K2 = P.kf2;
    if (gate_skip(gate)) {   // a neighbour the reference `continue`s past: no search, no matches
        for (int i = tid; i < K1.n; i += kWalkThreads) P.match12[i] = -1;
        if (tid == 0) n_matches[p] = 0;
        return;
    }
    if (ws.over[p]) return;   // rerun by tri_kernel
    for (int i = tid; i < K1.n; i += kWalkThreads) P.match12[i] = -1;
    if (K1.n > kTriMaxKp || K2.n > 65535) {
        if (tid == 0) atomicExch(err, OMV_ERR_CAPACITY), n_matches[p] = 0;
        return;
    }
    for (int i = tid; i < K1.n; i += kWalkThreads) bins[i] = 0xff;
    if (tid < kHisto) hist[tid] = 0;
    auto add = [](int x, int y) { return x + y; };
    // rows of the pair (entries with the row-start bit)
    int nr = 0;
    for (int sl = 0; sl < S; ++sl) {
        const int slot = p * S + sl, base = slot * ws.ecap, n = ws.cnt[slot];
        for (int k = tid; k < n; k += kWalkThreads) nr += (ws.w[base + k] >> 11) & 1u;
    }
    for (int d = 32; d >= 1; d >>= 1) nr += __shfl_xor(nr, d, 64);
    if ((tid & 63) == 0) s_wi[tid >> 6] = nr;
    __syncthreads();
    const int R = s_wi[0] + s_wi[1] + s_wi[2] + s_wi[3];
    __syncthreads();
    int nmatch = 0;
    if (par_walk && R <= kWalkRows) {
        // Parallel replay.  The walk's only coupling between rows is the camera-pair state (bestDist restarts per
        // row), so each row is a map state -> state (ten nibbles), evaluated per row on its own thread; one
        // wavefront chains the maps from LL (a table lookup per row); then each row is replayed from its entering
        // state for its best.  Rows never span slices, so a row ends at the next row start or its slice's end.
        int *rstart = fin, *rend = fin + kWalkRows;
        uint64_t *rmap = reinterpret_cast<uint64_t *>(fin + 2 * kWalkRows);
        int rbase = 0;
        for (int sl = 0; sl < S; ++sl) {
            const int slot = p * S + sl, base = slot * ws.ecap, n = ws.cnt[slot];
            const int r0 = rbase;
            for (int c0 = 0; c0 < n; c0 += kWalkThreads) {
                const int k = c0 + tid;
                const int f = k < n ? (int)((ws.w[base + k] >> 11) & 1u) : 0;
                int tot;
                const int pos = rbase + block_scan_excl<int, decltype(add), kWalkThreads>(f, 0, add, s_wi, tot);
#ifdef OMV_TRI_CHECK
                if (f && pos >= kWalkRows) printf("rstart overflow pos %d R %d\n", pos, R);
                if (f && pos < kWalkRows)
#else
                if (f)
#endif
                rstart[pos] = base + k;
                rbase += tot;
            }
            __syncthreads();
            for (int r = r0 + tid; r < rbase; r += kWalkThreads) rend[r] = r + 1 < rbase ? rstart[r + 1] : base + n;
        }
        __syncthreads();
        for (int r = tid; r < R; r += kWalkThreads) {
            uint64_t m = 0;
#pragma unroll
            for (int s0 = 0; s0 < 10; ++s0) {
                int st = s0;
                walk_row(ws, rstart[r], rend[r], st);
                m |= (uint64_t)st << (4 * s0);
            }
            rmap[r] = m;
        }
        __syncthreads();
        if (tid < 64) {
            const int lane = tid;
            int st = 0;
            for (int c0 = 0; c0 < R; c0 += 64) {
                const uint64_t m_l = c0 + lane < R ? rmap[c0 + lane] : kIdentityMap;
                const uint32_t lo_l = (uint32_t)m_l, hi_l = (uint32_t)(m_l >> 32);
#pragma unroll
                for (int j = 0; j < 64; ++j) {
                    const uint64_t m = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo_l, j) |
                                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi_l, j) << 32);
                    instate[c0 + j] = (uint8_t)st;
                    st = (int)((m >> (4 * st)) & 15u);
                }
            }
        }
        __syncthreads();
        for (int r = tid; r < R; r += kWalkThreads) {
            int st = instate[r];
            const int bk = walk_row(ws, rstart[r], rend[r], st);
            if (bk < 0) continue;
            const uint32_t pk = ws.pk[bk];
            const int row = (int)(pk >> 16), best = (int)(pk & 0xffff);
#ifdef OMV_TRI_CHECK
            if (row >= K1.n || best >= K2.n) { printf("walk bad row %d best %d bk %d r %d\n", row, best, bk, r); continue; }
#endif
            P.match12[row] = best;
            ++nmatch;
            if (check_ori) {
                float rot = K1.kps[row].angle - K2.kps[best].angle;
                if ((double)rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * (1.0f / kHisto));
                if (bin == kHisto) bin = 0;
                bins[row] = (uint8_t)bin;
            }
        }
        for (int d = 32; d >= 1; d >>= 1) nmatch += __shfl_xor(nmatch, d, 64);
        if ((tid & 63) == 0) s_wi[tid >> 6] = nmatch;
        __syncthreads();
        nmatch = s_wi[0] + s_wi[1] + s_wi[2] + s_wi[3];
        __syncthreads();
    } else {
    if (tid < 64) {
        // one 32-bit word per entry: dist 0-5, listed 6, state 7-10, row start 11, results 12-21; a padding entry
        // (distance 63, no row start) changes nothing
        const int lane = tid;
        int state = 0, bestDist = kTriLow, bestK = -1, n_fin = 0;
        for (int sl = 0; sl < S; ++sl) {
            const int slot = p * S + sl;
            const int base = slot * ws.ecap, n = __builtin_amdgcn_readfirstlane(ws.cnt[slot]);
            auto load = [&](int c0) {
                const int k = c0 + lane;
                return k < n ? (ws.w[base + k] | (ws.res[base + k] << 12)) : 63u;
            };
            uint32_t nxt = n > 0 ? load(0) : 63u;
            for (int c0 = 0; c0 < n; c0 += 64) {
                const uint32_t w_l = nxt;
                if (c0 + 64 < n) nxt = load(c0 + 64);   // the next 64 in flight during this walk
#pragma unroll
                for (int j = 0; j < 64; ++j) {
                    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)w_l, j);
                    const bool rs = (w >> 11) & 1u;
                    fin[n_fin] = bestK;   // kept only when the row ends with a best (n_fin advances)
                    n_fin += (rs && bestK >= 0) ? 1 : 0;
                    bestDist = rs ? kTriLow : bestDist;
                    bestK = rs ? -1 : bestK;
                    const int dist = (int)(w & 63u);
                    const bool cand = dist <= bestDist;
                    state = (cand && ((w >> 6) & 1u)) ? (int)((w >> 7) & 15u) : state;
                    const bool take = cand && ((w >> (12 + state)) & 1u);
                    bestK = take ? base + c0 + j : bestK;
                    bestDist = take ? dist : bestDist;
                }
            }
        }
        fin[n_fin] = bestK;
        n_fin += bestK >= 0 ? 1 : 0;
        if (lane == 0) s_fin = n_fin;
    }
    __syncthreads();
    const int n_fin = s_fin;
    nmatch = n_fin;
    for (int i = tid; i < n_fin; i += kWalkThreads) {
        const uint32_t pk = ws.pk[fin[i]];
        const int row = (int)(pk >> 16), best = (int)(pk & 0xffff);
        P.match12[row] = best;
        if (check_ori) {
            float rot = K1.kps[row].angle - K2.kps[best].angle;
            if ((double)rot < 0.0) rot += 360.0f;
            int bin = (int)roundf(rot * (1.0f / kHisto));
            if (bin == kHisto) bin = 0;
            bins[row] = (uint8_t)bin;
        }
    }
    }
    __syncthreads();
    if (check_ori) {   // rotation histogram: keep the three largest bins (ComputeThreeMaxima, :2537-2573)
        for (int i = tid; i < K1.n; i += kWalkThreads)
            if (bins[i] != 0xff) atomicAdd(&hist[bins[i]], 1);
        __syncthreads();
        if (tid == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kHisto; i++) {
                const int sv = hist[i];
                if (sv > max1) {
                    max3 = max2, max2 = max1, max1 = sv;
                    ind3 = ind2, ind2 = ind1, ind1 = i;
                } else if (sv > max2) {
                    max3 = max2, max2 = sv;
                    ind3 = ind2, ind2 = i;
                } else if (sv > max3) {
                    max3 = sv;
                    ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) ind2 = -1, ind3 = -1;
            else if (max3 < 0.1f * (float)max1) ind3 = -1;
            for (int i = 0; i < kHisto; ++i) s_keep[i] = (i == ind1 || i == ind2 || i == ind3) ? 1 : 0;
        }
        __syncthreads();
        int removed = 0;
        for (int i = tid; i < K1.n; i += kWalkThreads)
            if (bins[i] != 0xff && !s_keep[bins[i]]) P.match12[i] = -1, ++removed;
        for (int d = 32; d >= 1; d >>= 1) removed += __shfl_xor(removed, d, 64);
        if ((tid & 63) == 0) s_wi[tid >> 6] = removed;
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int w2 = 0; w2 < kWalkThreads / 64; ++w2) tot += s_wi[w2];
            nmatch -= tot;
        }
    }
    if (tid == 0) n_matches[p] = nmatch;
}

// Frame::ComputeMultiFishEyeMatches' depth check (src/Frame.cc:1488-1512) on the Lowe-filtered
// lapping knn pairs (omv_matcher_stereo_lapping's l2r): one thread per left keypoint.
struct StereoTriArgs {
    const omv_kp *kps;
    const int *n_kp, *mono;
    int n_cams, kp_cap;
    float camL[8], camR[8], Rlr[9], tlr[3], sigma2[16];
    int32_t *l2r, *r2l;
    float *depth, *p3d;
};
__global__ void stereo_reset_kernel(StereoTriArgs A) {
    const int frame = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.kp_cap) return;
    A.r2l[(size_t)frame * A.kp_cap + i] = -1;
    A.depth[(size_t)frame * A.kp_cap + i] = -1.0f;
}
__global__ void stereo_tri_kernel(StereoTriArgs A) {
    const int frame = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    const int nL = A.n_kp[frame * A.n_cams];
    if (i >= nL) return;
    const size_t slot = (size_t)frame * A.kp_cap + i;
    int32_t *l2r = A.l2r + slot;
    const int r = *l2r;
    if (r < 0) return;
    const size_t base = (size_t)frame * A.n_cams * A.kp_cap;   // keypoints [frame][cam][kp_cap]: L = 0, R = 1
    const omv_kp &kl = A.kps[base + i], &kr = A.kps[base + A.kp_cap + r];
    float p3D[3];
    const float depth = triangulate_matches(A.camL, A.camR, kl, kr, A.Rlr, A.tlr, A.sigma2[kl.octave],
                                            A.sigma2[kr.octave], p3D);
    if (depth > 0.0001f) {
        A.depth[slot] = depth;
        for (int q = 0; q < 3; ++q) A.p3d[slot * 3 + q] = p3D[q];
        atomicMax(&A.r2l[(size_t)frame * A.kp_cap + r], i);   // the later left index wins
    } else {
        *l2r = -1;
    }
}

// Parity hook: the camera-model pieces for one input (out: ray1[3] ray2[3] V[16] z p3D[3]).
__global__ void tri_debug_kernel(TriCams C, omv_kp kp1, omv_kp kp2, const float *Rt, float sigma, float unc, float *out) {
    kb8_unproject_f(C.cam[0], kp1.x, kp1.y, out);
    kb8_unproject_f(C.cam[1], kp2.x, kp2.y, out + 3);
    float A[16];
    for (int i = 0; i < 16; ++i) A[i] = Rt[12 + i];
    jacobi_svd4_v(A, out + 6);
    out[22] = triangulate_matches(C.cam[0], C.cam[1], kp1, kp2, Rt, Rt + 9, sigma, unc, out + 23);
    // intermediates of the triangulation of (kp1, kp2): x3D[3] and its projection uv1[2] -> out[26..30]
    float r1[3], r2[3], R21[9], t2[3], V[16];
    kb8_unproject_f(C.cam[0], kp1.x, kp1.y, r1);
    kb8_unproject_f(C.cam[1], kp2.x, kp2.y, r2);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R21[3 * i + j] = Rt[3 * j + i];
    for (int i = 0; i < 3; ++i) t2[i] = -R21[3 * i] * Rt[9] + -R21[3 * i + 1] * Rt[10] + -R21[3 * i + 2] * Rt[11];
    const float T1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const float T2[12] = {R21[0], R21[1], R21[2], t2[0], R21[3], R21[4], R21[5], t2[1], R21[6], R21[7], R21[8], t2[2]};
    for (int j = 0; j < 4; ++j) {
        A[j] = r1[0] * T1[8 + j] - T1[j];
        A[4 + j] = r1[1] * T1[8 + j] - T1[4 + j];
        A[8 + j] = r2[0] * T2[8 + j] - T2[j];
        A[12 + j] = r2[1] * T2[8 + j] - T2[4 + j];
    }
    jacobi_svd4_v(A, V);
    float x3D[3];
    for (int i = 0; i < 3; ++i) x3D[i] = V[4 * i + 3] / V[15];
    float u1, v1;
    kb8_project_f(C.cam[0], x3D, u1, v1);
    out[26] = x3D[0], out[27] = x3D[1], out[28] = x3D[2], out[29] = u1, out[30] = v1;
}


// ---- LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:395-783): the geometry of each triangulation match ----
// The reference walks the neighbours and their matches in order; the only state one match hands to the next is the
// camera-pair state (sophTcw1 / Ow1 / pCamera1 of side 1, sophTcw2 / Ow2 / pCamera2 of side 2): listed camera pairs
// assign it, the others keep it; side 1's pose persists across neighbours, the cameras and side 2 reset per neighbour.
// So each match's state is that of the last listed match before it -- an inclusive max-scan over the match positions
// -- and the matches are then independent: one thread per match.  Side 1's block also decides the next neighbour's
// baseline gate (:447-454), so the jobs' entering states are a short scalar chain over the jobs.
//   cnmp_last_kernel   one block per job: the side-1 camera block of its last listed match (or -1)
//   cnmp_kernel        one block per job: the state entering it (the chain over the jobs before it: a job the gate
//                      skips changes nothing), the max-scan over its matches, the per-match geometry, has_mp1 marks
//   cnmp_state_kernel  one thread: the state leaving the last job (side1_state out)
// A whole CreateNewMapPoints (omv_local_mapping_create_new_map_points) interleaves these with each neighbour's
// SearchForTriangulation launches on the stream: the search of neighbour j reads has_mp1 after neighbour j-1's marks.
constexpr int kCnmpThreads = 256;
struct CnmpArgs {
    TriCams C;
    int n_cams, inertial, far_points;
    float th_far, ratio_factor;
};
__device__ __forceinline__ int cnmp_cam(const omv_kf_view &k, int idx) { return k.n_left < 0 ? 0 : cam_of(k, idx); }
// the listed camera pair's state code (1 + 4 cameraId1 + cameraId2), 0 when the reference keeps the previous state
__device__ __forceinline__ int cnmp_listed(int n_cams, int c1, int c2) {
    if (n_cams < 2) return 0;
    const int code = 4 * c1 + c2;
    bool l = code == 5 || code == 4 || code == 1 || code == 0;
    if (n_cams >= 4) l = l || code == 2 || code == 8 || code == 10 || code == 7 || code == 13 || code == 15;
    return l ? 1 + code : 0;
}
__global__ void __launch_bounds__(kCnmpThreads) cnmp_last_kernel(const omv_cnmp_kf *kf1, const omv_cnmp_job *jobs,
                                                                 int n_cams, int *last_p1) {
    __shared__ int best;
    const omv_cnmp_job &J = jobs[blockIdx.x];
    const omv_kf_view &K1 = kf1->kf, &K2 = J.kf2.kf;
    if (threadIdx.x == 0) best = -1;
    __syncthreads();
    int mine = -1;
    for (int i = threadIdx.x; i < K1.n; i += blockDim.x) {
        const int i2 = J.match12[i];
        if (i2 >= 0 && i2 < K2.n && cnmp_listed(n_cams, cnmp_cam(K1, i), cnmp_cam(K2, i2))) mine = i;
    }
    atomicMax(&best, mine);
    __syncthreads();
    if (threadIdx.x == 0) last_p1[blockIdx.x] = best >= 0 ? cnmp_cam(K1, best) : -1;
}

// The baseline gate of job q under side-1 block p1 (LocalMapping.cc:447-454; Eigen's norm as sqrt of the left-to-right
// squared sum)
__device__ __forceinline__ bool cnmp_gate(const omv_cnmp_kf &K1, const omv_cnmp_kf &K2, int p1, int check_baseline) {
    if (!check_baseline) return false;
    const float a = K2.Ow[0][0] - K1.Ow[p1][0], b = K2.Ow[0][1] - K1.Ow[p1][1], c = K2.Ow[0][2] - K1.Ow[p1][2];
    return omv::sqrtf_cr(a * a + b * b + c * c) < K2.mb;
}
// The side-1 block entering job j (and whether the gate skips it): the scalar chain over the jobs before it.
__device__ int cnmp_enter(const omv_cnmp_kf &K1, const omv_cnmp_job *jobs, int j, const int *last_p1, int p1,
                          int check_baseline, bool &skipped) {
    for (int q = 0; q < j; ++q)
        if (!cnmp_gate(K1, jobs[q].kf2, p1, check_baseline) && last_p1[q] >= 0) p1 = last_p1[q];
    skipped = cnmp_gate(K1, jobs[j].kf2, p1, check_baseline);
    return p1;
}

__device__ __forceinline__ float cnmp_dot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ float cnmp_norm3(const float *a) { return omv::sqrtf_cr(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }
__device__ __forceinline__ float cosf_glibc(float x) {
    float s, c;
    omv::glibc_sincosf(x, &s, &c);
    return c;
}
__device__ bool cnmp_unproject_stereo(const omv_cnmp_kf &K, int i, float *x3D) {   // KeyFrame::UnprojectStereo
    const float z = K.depth[i];
    if (!(z > 0)) return false;
    const omv_kp kp = (K.kps_raw ? K.kps_raw : K.kf.kps)[i];
    const float x = (kp.x - K.cx) * z * K.invfx, y = (kp.y - K.cy) * z * K.invfy;
    const float c[3] = {x, y, z};
    for (int r = 0; r < 3; ++r) x3D[r] = (K.Rwc[3 * r] * c[0] + K.Rwc[3 * r + 1] * c[1] + K.Rwc[3 * r + 2] * c[2]) + K.twc[r];
    return true;
}
// One match under state (p1, c1, p2, c2): 0 rejected, 1 triangulated, 2 by UnprojectStereo (x3D written).
__device__ int cnmp_match(const CnmpArgs &a, const omv_cnmp_kf &K1, const omv_cnmp_kf &K2, int idx1, int idx2, int p1,
                          int c1, int p2, int c2, float *x3D) {
    const omv_kp kp1 = K1.kf.kps[idx1], kp2 = K2.kf.kps[idx2];
    const float kp1_ur = K1.uright ? K1.uright[idx1] : -1.f, kp2_ur = K2.uright ? K2.uright[idx2] : -1.f;
    const bool bStereo1 = a.n_cams < 2 && kp1_ur >= 0, bStereo2 = a.n_cams < 2 && kp2_ur >= 0;
    const float *T1 = K1.Tcw[p1], *T2 = K2.Tcw[p2];
    const float Rwc1[9] = {T1[0], T1[4], T1[8], T1[1], T1[5], T1[9], T1[2], T1[6], T1[10]};
    const float Rwc2[9] = {T2[0], T2[4], T2[8], T2[1], T2[5], T2[9], T2[2], T2[6], T2[10]};
    float xn1[3], xn2[3], ray1[3], ray2[3];
    cam_unproject_f(a.C.model[c1], a.C.cam[c1], kp1.x, kp1.y, xn1);
    cam_unproject_f(a.C.model[c2], a.C.cam[c2], kp2.x, kp2.y, xn2);
    for (int r = 0; r < 3; ++r) ray1[r] = Rwc1[3 * r] * xn1[0] + Rwc1[3 * r + 1] * xn1[1] + Rwc1[3 * r + 2] * xn1[2];
    for (int r = 0; r < 3; ++r) ray2[r] = Rwc2[3 * r] * xn2[0] + Rwc2[3 * r + 1] * xn2[1] + Rwc2[3 * r + 2] * xn2[2];
    const float cosParallaxRays = cnmp_dot3(ray1, ray2) / (cnmp_norm3(ray1) * cnmp_norm3(ray2));
    float cosParallaxStereo = cosParallaxRays + 1;
    float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
    if (bStereo1) cosParallaxStereo1 = cosf_glibc(2 * omv::glibc_atan2f(K1.mb / 2, K1.depth[idx1]));
    else if (bStereo2) cosParallaxStereo2 = cosf_glibc(2 * omv::glibc_atan2f(K2.mb / 2, K2.depth[idx2]));
    cosParallaxStereo = fminf(cosParallaxStereo1, cosParallaxStereo2);
    bool goodProj = false, bPointStereo = false;
    if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
        (bStereo1 || bStereo2 || ((double)cosParallaxRays < 0.9996 && a.inertial) ||
         ((double)cosParallaxRays < 0.9998 && !a.inertial))) {
        // GeometricTools::Triangulate (src/GeometricTools.cc:27-50)
        float A[16], V[16];
        for (int j = 0; j < 4; ++j) {
            A[j] = xn1[0] * T1[8 + j] - T1[j];
            A[4 + j] = xn1[1] * T1[8 + j] - T1[4 + j];
            A[8 + j] = xn2[0] * T2[8 + j] - T2[j];
            A[12 + j] = xn2[1] * T2[8 + j] - T2[4 + j];
        }
        jacobi_svd4_v(A, V);
        if (V[15] == 0) return 0;
        for (int i = 0; i < 3; ++i) x3D[i] = V[4 * i + 3] / V[15];
        goodProj = true;
    } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
        bPointStereo = true;
        goodProj = cnmp_unproject_stereo(K1, idx1, x3D);
    } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
        bPointStereo = true;
        goodProj = cnmp_unproject_stereo(K2, idx2, x3D);
    } else {
        return 0;
    }
    if (!goodProj) return 0;
    const float R1r2[3] = {T1[8], T1[9], T1[10]}, R2r2[3] = {T2[8], T2[9], T2[10]};
    const float z1 = cnmp_dot3(R1r2, x3D) + T1[11];
    if (z1 <= 0) return 0;
    const float z2 = cnmp_dot3(R2r2, x3D) + T2[11];
    if (z2 <= 0) return 0;
    const float sigmaSquare1 = K1.kf.level_sigma2[kp1.octave];
    const float R1r0[3] = {T1[0], T1[1], T1[2]}, R1r1[3] = {T1[4], T1[5], T1[6]};
    const float x1 = cnmp_dot3(R1r0, x3D) + T1[3], y1 = cnmp_dot3(R1r1, x3D) + T1[7];
    const float invz1 = (float)(1.0 / (double)z1);
    if (!bStereo1) {
        const float X[3] = {x1, y1, z1};
        float u, v;
        cam_project_f(a.C.model[c1], a.C.cam[c1], X, u, v);
        const float errX1 = u - kp1.x, errY1 = v - kp1.y;
        if ((double)(errX1 * errX1 + errY1 * errY1) > 5.991 * (double)sigmaSquare1) return 0;
    } else {
        const float u1 = K1.fx * x1 * invz1 + K1.cx, u1_r = u1 - K1.mbf * invz1, v1 = K1.fy * y1 * invz1 + K1.cy;
        const float errX1 = u1 - kp1.x, errY1 = v1 - kp1.y, errX1_r = u1_r - kp1_ur;
        if ((double)(errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * (double)sigmaSquare1) return 0;
    }
    const float sigmaSquare2 = K2.kf.level_sigma2[kp2.octave];
    const float R2r0[3] = {T2[0], T2[1], T2[2]}, R2r1[3] = {T2[4], T2[5], T2[6]};
    const float x2 = cnmp_dot3(R2r0, x3D) + T2[3], y2 = cnmp_dot3(R2r1, x3D) + T2[7];
    const float invz2 = (float)(1.0 / (double)z2);
    if (!bStereo2) {
        const float X[3] = {x2, y2, z2};
        float u, v;
        cam_project_f(a.C.model[c2], a.C.cam[c2], X, u, v);
        const float errX2 = u - kp2.x, errY2 = v - kp2.y;
        if ((double)(errX2 * errX2 + errY2 * errY2) > 5.991 * (double)sigmaSquare2) return 0;
    } else {
        // the reference's mpCurrentKeyFrame->mbf here (:706)
        const float u2 = K2.fx * x2 * invz2 + K2.cx, u2_r = u2 - K1.mbf * invz2, v2 = K2.fy * y2 * invz2 + K2.cy;
        const float errX2 = u2 - kp2.x, errY2 = v2 - kp2.y, errX2_r = u2_r - kp2_ur;
        if ((double)(errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * (double)sigmaSquare2) return 0;
    }
    const float n1[3] = {x3D[0] - K1.Ow[p1][0], x3D[1] - K1.Ow[p1][1], x3D[2] - K1.Ow[p1][2]};
    const float n2[3] = {x3D[0] - K2.Ow[p2][0], x3D[1] - K2.Ow[p2][1], x3D[2] - K2.Ow[p2][2]};
    const float dist1 = cnmp_norm3(n1), dist2 = cnmp_norm3(n2);
    if (dist1 == 0 || dist2 == 0) return 0;
    if (a.far_points && (dist1 >= a.th_far || dist2 >= a.th_far)) return 0;
    const float ratioDist = dist2 / dist1;
    const float ratioOctave = K1.scale_factors[kp1.octave] / K2.scale_factors[kp2.octave];
    if (ratioDist * a.ratio_factor < ratioOctave || ratioDist > ratioOctave * a.ratio_factor) return 0;
    return bPointStereo ? 2 : 1;
}

__global__ void __launch_bounds__(kCnmpThreads) cnmp_kernel(const omv_cnmp_kf *kf1, const omv_cnmp_job *jobs,
                                                            const int *last_p1, CnmpArgs a, const int *p1_state,
                                                            int check_baseline, uint8_t *has_mp1) {
    __shared__ int s_scan[kCnmpThreads];
    __shared__ int s_p1, s_skip;
    const int j = blockIdx.x, t = threadIdx.x;
    const omv_cnmp_kf &K1 = *kf1;
    const omv_cnmp_job &J = jobs[j];
    const omv_cnmp_kf &K2 = J.kf2;
    const int n = K1.kf.n, n2 = K2.kf.n, chunk = (n + kCnmpThreads - 1) / kCnmpThreads;
    const int i0 = min(n, t * chunk), i1 = min(n, i0 + chunk);
    // side 1 entering this job: the state entering the call, then the last listed match of every earlier job the
    // gate did not skip
    if (t == 0) {
        bool sk = false;
        s_p1 = cnmp_enter(K1, jobs, j, last_p1, p1_state ? *p1_state : 0, check_baseline, sk);
        s_skip = sk ? 1 : 0;
    }
    __syncthreads();
    const int p1_in = s_p1;
    if (s_skip) {   // the reference `continue`s before SearchForTriangulation: nothing created
        for (int i = i0; i < i1; ++i) J.status[i] = 0;
        return;
    }
    // the last listed match of this thread's chunk, then an inclusive max-scan over the chunks (position-ordered codes)
    int last = -1;
    for (int i = i0; i < i1; ++i) {
        const int i2 = J.match12[i];
        if (i2 >= 0 && i2 < n2) {
            const int code = cnmp_listed(a.n_cams, cnmp_cam(K1.kf, i), cnmp_cam(K2.kf, i2));
            if (code) last = (i << 5) | code;
        }
    }
    s_scan[t] = last;
    __syncthreads();
    for (int d = 1; d < kCnmpThreads; d <<= 1) {
        const int v = t >= d ? s_scan[t - d] : -1;
        __syncthreads();
        s_scan[t] = max(s_scan[t], v);
        __syncthreads();
    }
    int state = t > 0 ? s_scan[t - 1] : -1;   // the listed match before this chunk
    for (int i = i0; i < i1; ++i) {
        J.status[i] = 0;
        const int i2 = J.match12[i];
        if (i2 < 0 || i2 >= n2) continue;
        const int code = cnmp_listed(a.n_cams, cnmp_cam(K1.kf, i), cnmp_cam(K2.kf, i2));
        if (code) state = (i << 5) | code;
        int p1 = p1_in, c1 = 0, p2 = 0, c2 = 0;
        if (state >= 0) {
            const int cc = (state & 31) - 1;
            p1 = c1 = cc >> 2, p2 = c2 = cc & 3;
        }
        float x3D[3];
        const int st = cnmp_match(a, K1, K2, i, i2, p1, c1, p2, c2, x3D);
        J.status[i] = st;
        if (st) {
            for (int q = 0; q < 3; ++q) J.x3D[3 * i + q] = x3D[q];
            if (has_mp1) has_mp1[i] = 1;   // mpCurrentKeyFrame->AddMapPoint(pMP, idx1) (:773)
        }
    }
}

// side1_state after the last job (p1_out may alias p1_in: one thread reads, then writes)
__global__ void cnmp_state_kernel(const omv_cnmp_kf *kf1, const omv_cnmp_job *jobs, int n_jobs, const int *last_p1,
                                  const int *p1_in, int check_baseline, int *p1_out) {
    bool sk = false;
    int p1 = cnmp_enter(*kf1, jobs, n_jobs - 1, last_p1, p1_in ? *p1_in : 0, check_baseline, sk);
    if (!sk && last_p1[n_jobs - 1] >= 0) p1 = last_p1[n_jobs - 1];
    *p1_out = p1;
}

}  // namespace

extern "C" {

omv_status omv_tri_debug(const float *cams2, const omv_kp *kp1, const omv_kp *kp2, const float *R12, const float *t12,
                         const float *svd_in, float sigma, float unc, float *out31) {
    if (!cams2 || !kp1 || !kp2 || !R12 || !t12 || !svd_in || !out31) return OMV_ERR_ARG;
    TriCams C{};
    for (int q = 0; q < 16; ++q) C.cam[q / 8][q % 8] = cams2[q];
    float h[28];
    for (int q = 0; q < 9; ++q) h[q] = R12[q];
    for (int q = 0; q < 3; ++q) h[9 + q] = t12[q];
    for (int q = 0; q < 16; ++q) h[12 + q] = svd_in[q];
    float *d = nullptr;
    HIP_OK(hipMalloc(&d, sizeof(float) * (28 + 31)));
    HIP_OK(hipMemcpy(d, h, sizeof(float) * 28, hipMemcpyHostToDevice));
    tri_debug_kernel<<<1, 1>>>(C, *kp1, *kp2, d, sigma, unc, d + 28);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(out31, d + 28, sizeof(float) * 31, hipMemcpyDeviceToHost));
    HIP_OK(hipFree(d));
    return OMV_OK;
}

omv_status omv_matcher_stereo_triangulate(omv_matcher *m, int n_frames, int n_cams, int kp_cap, const omv_kp *kps,
                                          const int *n_kp, const int *mono, const float *cams, const float *Rlr,
                                          const float *tlr, const float *level_sigma2, int nlevels, int32_t *l2r,
                                          int32_t *r2l, float *depth, float *p3d, void *stream) {
    if (!m || n_frames <= 0 || n_cams < 2 || kp_cap <= 0 || !kps || !n_kp || !mono || !cams || !Rlr || !tlr ||
        !level_sigma2 || nlevels <= 0 || nlevels > 16 || !l2r || !r2l || !depth || !p3d)
        return OMV_ERR_ARG;
    StereoTriArgs A{kps, n_kp, mono, n_cams, kp_cap, {}, {}, {}, {}, {}, l2r, r2l, depth, p3d};
    for (int q = 0; q < 8; ++q) A.camL[q] = cams[q], A.camR[q] = cams[8 + q];
    for (int q = 0; q < 9; ++q) A.Rlr[q] = Rlr[q];
    for (int q = 0; q < 3; ++q) A.tlr[q] = tlr[q];
    for (int q = 0; q < nlevels; ++q) A.sigma2[q] = level_sigma2[q];
    hipStream_t st = (hipStream_t)stream;
    const dim3 g((kp_cap + 255) / 256, n_frames);
    stereo_reset_kernel<<<g, 256, 0, st>>>(A);
    stereo_tri_kernel<<<g, 256, 0, st>>>(A);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}


}  // extern "C"

namespace {

// One chunk of pairs through the sliced search (its workspace sized for the chunk; see omv_matcher_search_for_triangulation).
omv_status tri_search_chunk(omv_matcher *m, int n_pairs, const omv_tri_pair *pairs, const TriCams &C, int only_stereo,
                            int coarse, int check_ori, int32_t *n_matches, hipStream_t st) {
    // S slices per pair: about 1,024 scan workgroups in all (at most 16 per pair)
    int S = std::max(1, std::min(16, (1024 + n_pairs - 1) / n_pairs));
    int ecap = std::max(2048, 32768 / S);
    // test knobs: the slice count, and the entry capacity (a small one forces the overflow rerun)
    const omv::MatcherKnobs kn = omv::matcher_knobs(m);   // read once by omv_matcher_create
    if (kn.tri_slices >= 0) S = std::max(1, std::min(64, kn.tri_slices));
    if (kn.tri_ecap >= 0) ecap = std::max(1, kn.tri_ecap);
    const int tcap = 2 * ecap;
    const size_t slots = (size_t)n_pairs * S;
    const size_t bytes = sizeof(omv_tri_pair) * n_pairs + slots * (size_t)ecap * 12 + slots * (size_t)tcap * 4 +
                         (2 * slots + 2 * (size_t)n_pairs + 1) * sizeof(int);
    char *blob = nullptr;
    HIP_OK(hipMallocAsync((void **)&blob, bytes, st));
    omv_tri_pair *d_pairs = reinterpret_cast<omv_tri_pair *>(blob);
    TriWs ws;
    ws.pk = reinterpret_cast<uint32_t *>(d_pairs + n_pairs);
    ws.w = ws.pk + slots * ecap;
    ws.res = ws.w + slots * ecap;
    ws.tests = ws.res + slots * ecap;
    ws.cnt = reinterpret_cast<int *>(ws.tests + slots * tcap);
    ws.tcnt = ws.cnt + slots;
    ws.over = ws.tcnt + slots;
    int *d_err = ws.over + n_pairs;
    ws.S = S, ws.ecap = ecap, ws.tcap = tcap;
    HIP_OK(hipMemcpyAsync(d_pairs, pairs, sizeof(omv_tri_pair) * n_pairs, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(ws.over, 0, sizeof(int) * (n_pairs + 1), st));   // overflow flags and the error word
    tri_scan_kernel<<<dim3(S, n_pairs), kTriThreads, 0, st>>>(d_pairs, only_stereo, coarse, ws, TriGate{});
    if (!coarse && !only_stereo) tri_epi_kernel<<<dim3(kEpiPerSlot, (unsigned)slots), kEpiThreads, 0, st>>>(d_pairs, C, ws);
    tri_walk_kernel<<<n_pairs, kWalkThreads, 0, st>>>(d_pairs, check_ori, ws, n_matches, d_err,
                                                      kn.tri_walk_seq ? 0 : 1, TriGate{});   // knob: the scalar walk
    HIP_OK(hipGetLastError());
    std::vector<int> over(n_pairs + 1);
    HIP_OK(hipMemcpyAsync(over.data(), ws.over, sizeof(int) * (n_pairs + 1), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    int h_err = over[n_pairs];
    if (std::any_of(over.begin(), over.begin() + n_pairs, [](int v) { return v != 0; })) {
        // a pair with more candidates than the workspace holds: the one-workgroup search for it alone
        tri_kernel<<<n_pairs, kTriThreads, 0, st>>>(d_pairs, C, only_stereo, coarse, check_ori, n_matches, d_err,
                                                    ws.over, TriGate{});
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(&h_err, d_err, sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
    }
    HIP_OK(hipFreeAsync(blob, st));
    return h_err ? (omv_status)h_err : OMV_OK;
}

}  // namespace

extern "C" {

// Pairs go through in chunks of at most kTriChunkPairs: the sliced workspace is sized per chunk (~650 KB per pair at
// one slice), so a call's temporary memory stays bounded (~170 MB) whatever its pair count; pairs are independent, so
// the results do not depend on the chunking.
constexpr int kTriChunkPairs = 256;
omv_status omv_matcher_search_for_triangulation(omv_matcher *m, int n_pairs, const omv_tri_pair *pairs,
                                                const float *cams, const int32_t *cam_model, int only_stereo,
                                                int coarse, int check_ori, int32_t *n_matches, void *stream) {
    if (!m || n_pairs < 0 || (n_pairs > 0 && (!pairs || !cams || !n_matches))) return OMV_ERR_ARG;
    if (n_pairs == 0) return OMV_OK;
    for (int i = 0; i < n_pairs; ++i)
        if (!pairs[i].match12 || pairs[i].kf1.n < 0 || pairs[i].kf2.n < 0) return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    TriCams C;
    for (int c = 0; c < 4; ++c) {
        for (int q = 0; q < 8; ++q) C.cam[c][q] = cams[8 * c + q];
        C.model[c] = cam_model ? cam_model[c] : OMV_CAM_KB8;
        if (C.model[c] != OMV_CAM_KB8 && C.model[c] != OMV_CAM_PINHOLE) return OMV_ERR_ARG;
    }
    omv_status first_err = OMV_OK;
    for (int p0 = 0; p0 < n_pairs; p0 += kTriChunkPairs) {
        const int n = std::min(kTriChunkPairs, n_pairs - p0);
        const omv_status r = tri_search_chunk(m, n, pairs + p0, C, only_stereo, coarse, check_ori, n_matches + p0, st);
        if (r == OMV_ERR_HIP || r == OMV_ERR_ARG) return r;
        if (r != OMV_OK && first_err == OMV_OK) first_err = r;   // a device-reported error word: the rest still run
    }
    return first_err;
}


namespace {
omv_status cnmp_args(const float *cams, const int32_t *cam_model, int n_cams, int inertial, int far_points,
                     float th_far_points, float scale_factor, CnmpArgs &a) {
    a = CnmpArgs{};
    for (int c = 0; c < 4; ++c) {
        for (int q = 0; q < 8; ++q) a.C.cam[c][q] = cams[8 * c + q];
        a.C.model[c] = cam_model ? cam_model[c] : OMV_CAM_KB8;
        if (a.C.model[c] != OMV_CAM_KB8 && a.C.model[c] != OMV_CAM_PINHOLE) return OMV_ERR_ARG;
    }
    a.n_cams = n_cams, a.inertial = inertial ? 1 : 0, a.far_points = far_points ? 1 : 0;
    a.th_far = th_far_points, a.ratio_factor = 1.5f * scale_factor;
    return OMV_OK;
}
}  // namespace

omv_status omv_create_new_map_points(int n_jobs, const omv_cnmp_kf *kf1, const omv_cnmp_job *jobs, const float *cams,
                                     const int32_t *cam_model, int n_cams, int inertial, int far_points,
                                     float th_far_points, float scale_factor, int check_baseline,
                                     int32_t *side1_state, uint8_t *has_mp1, void *stream) {
    if (n_jobs < 0 || n_jobs > 64 || (n_jobs > 0 && (!kf1 || !jobs || !cams)) || n_cams < 1 || n_cams > 4) return OMV_ERR_ARG;
    if (n_jobs == 0 || kf1->kf.n <= 0) return OMV_OK;
    if (kf1->kf.n >= (1 << 26) || !kf1->kf.kps) return OMV_ERR_ARG;
    for (int j = 0; j < n_jobs; ++j)
        if (!jobs[j].match12 || !jobs[j].x3D || !jobs[j].status || !jobs[j].kf2.kf.kps || jobs[j].kf2.kf.n < 0)
            return OMV_ERR_ARG;
    CnmpArgs a;
    if (cnmp_args(cams, cam_model, n_cams, inertial, far_points, th_far_points, scale_factor, a) != OMV_OK)
        return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    // the keyframe views and jobs travel as one device blob: [kf1 | jobs | last_p1 | state]
    const size_t bytes = sizeof(omv_cnmp_kf) + sizeof(omv_cnmp_job) * n_jobs + sizeof(int) * (n_jobs + 1);
    void *blob = nullptr;
    HIP_OK(hipMallocAsync(&blob, bytes, st));
    char *b = (char *)blob;
    HIP_OK(hipMemcpyAsync(b, kf1, sizeof(omv_cnmp_kf), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(b + sizeof(omv_cnmp_kf), jobs, sizeof(omv_cnmp_job) * n_jobs, hipMemcpyHostToDevice, st));
    const omv_cnmp_kf *d_kf1 = (const omv_cnmp_kf *)b;
    const omv_cnmp_job *d_jobs = (const omv_cnmp_job *)(b + sizeof(omv_cnmp_kf));
    int *d_last = (int *)(b + sizeof(omv_cnmp_kf) + sizeof(omv_cnmp_job) * n_jobs);
    int *d_state = d_last + n_jobs;   // the entering state, copied so every block reads it before anyone writes
    if (side1_state) HIP_OK(hipMemcpyAsync(d_state, side1_state, sizeof(int), hipMemcpyDeviceToDevice, st));
    else HIP_OK(hipMemsetAsync(d_state, 0, sizeof(int), st));
    cnmp_last_kernel<<<n_jobs, kCnmpThreads, 0, st>>>(d_kf1, d_jobs, n_cams, d_last);
    cnmp_kernel<<<n_jobs, kCnmpThreads, 0, st>>>(d_kf1, d_jobs, d_last, a, d_state, check_baseline, has_mp1);
    if (side1_state) cnmp_state_kernel<<<1, 1, 0, st>>>(d_kf1, d_jobs, n_jobs, d_last, d_state, check_baseline, side1_state);
    HIP_OK(hipGetLastError());
    HIP_OK(hipFreeAsync(blob, st));
    return OMV_OK;
}

// LocalMapping::CreateNewMapPoints' neighbour loop: per neighbour the gated SearchForTriangulation launches (one pair,
// S slices; the workspace is reused neighbour after neighbour in stream order) and the cnmp launches of one job; the
// side-1 state and has_mp1 carry from one neighbour to the next in device memory, so the host never waits inside.
omv_status omv_local_mapping_create_new_map_points(omv_matcher *m, const omv_cnmp_kf *kf1, uint8_t *has_mp1, int n_nb,
                                                   const omv_cnmp_neighbour *nb, const float *cams,
                                                   const int32_t *cam_model, int n_cams, int inertial,
                                                   int check_baseline, int coarse, int far_points, float th_far_points,
                                                   float scale_factor, int32_t *n_matches, int32_t *side1_state,
                                                   void *stream) {
    if (!m || !kf1 || !has_mp1 || n_nb < 0 || n_nb > 64 || (n_nb > 0 && (!nb || !cams || !n_matches)) ||
        (n_cams != 2 && n_cams != 4))
        return OMV_ERR_ARG;
    if (n_nb == 0) return OMV_OK;
    const omv_kf_view &V1 = kf1->kf;
    if (V1.n < 0 || V1.n >= (1 << 26) || (V1.n > 0 && (!V1.kps || !V1.desc)) || V1.n_nodes < 0) return OMV_ERR_ARG;
    for (int j = 0; j < n_nb; ++j) {
        const omv_kf_view &V2 = nb[j].kf2.kf;
        if (!nb[j].match12 || !nb[j].x3D || !nb[j].status || V2.n < 0 || (V2.n > 0 && (!V2.kps || !V2.desc || !V2.has_mp)))
            return OMV_ERR_ARG;
    }
    CnmpArgs a;
    if (cnmp_args(cams, cam_model, n_cams, inertial, far_points, th_far_points, scale_factor, a) != OMV_OK)
        return OMV_ERR_ARG;
    TriCams C;
    for (int c = 0; c < 4; ++c) {
        for (int q = 0; q < 8; ++q) C.cam[c][q] = cams[8 * c + q];
        C.model[c] = a.C.model[c];
    }
    hipStream_t st = (hipStream_t)stream;
    const omv::MatcherKnobs kn = omv::matcher_knobs(m);
    int S = 16, ecap = 2048;
    if (kn.tri_slices >= 0) S = std::max(1, std::min(64, kn.tri_slices));
    if (kn.tri_ecap >= 0) ecap = std::max(1, kn.tri_ecap);
    const int tcap = 2 * ecap;
    // blob: [pairs | kf1 | jobs | last_p1 | state | err | over | cnt | tcnt | ws pk / w / res | tests]
    std::vector<omv_tri_pair> pairs(n_nb);
    std::vector<omv_cnmp_job> jobs(n_nb);
    for (int j = 0; j < n_nb; ++j) {
        pairs[j].kf1 = V1;
        pairs[j].kf1.has_mp = has_mp1;
        pairs[j].kf2 = nb[j].kf2.kf;
        std::memcpy(pairs[j].T, nb[j].T, sizeof(pairs[j].T));
        pairs[j].match12 = nb[j].match12;
        jobs[j].kf2 = nb[j].kf2;
        jobs[j].match12 = nb[j].match12, jobs[j].x3D = nb[j].x3D, jobs[j].status = nb[j].status;
    }
    const size_t head = sizeof(omv_tri_pair) * n_nb + sizeof(omv_cnmp_kf) + sizeof(omv_cnmp_job) * n_nb;
    const size_t bytes = head + sizeof(int) * (4 + 2 * (size_t)S) + (size_t)S * ecap * 12 + (size_t)S * tcap * 4;
    char *blob = nullptr;
    HIP_OK(hipMallocAsync((void **)&blob, bytes, st));
    omv_tri_pair *d_pairs = reinterpret_cast<omv_tri_pair *>(blob);
    omv_cnmp_kf *d_kf1 = reinterpret_cast<omv_cnmp_kf *>(blob + sizeof(omv_tri_pair) * n_nb);
    omv_cnmp_job *d_jobs = reinterpret_cast<omv_cnmp_job *>(d_kf1 + 1);
    int *d_last = reinterpret_cast<int *>(blob + head), *d_state = d_last + 1, *d_err = d_last + 2;
    TriWs ws;
    ws.over = d_last + 3;
    ws.cnt = d_last + 4, ws.tcnt = ws.cnt + S;
    ws.pk = reinterpret_cast<uint32_t *>(ws.tcnt + S);
    ws.w = ws.pk + (size_t)S * ecap;
    ws.res = ws.w + (size_t)S * ecap;
    ws.tests = ws.res + (size_t)S * ecap;
    ws.S = S, ws.ecap = ecap, ws.tcap = tcap;
    HIP_OK(hipMemcpyAsync(d_pairs, pairs.data(), sizeof(omv_tri_pair) * n_nb, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_kf1, kf1, sizeof(omv_cnmp_kf), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_jobs, jobs.data(), sizeof(omv_cnmp_job) * n_nb, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(d_err, 0, sizeof(int), st));
    if (side1_state) HIP_OK(hipMemcpyAsync(d_state, side1_state, sizeof(int), hipMemcpyDeviceToDevice, st));
    else HIP_OK(hipMemsetAsync(d_state, 0, sizeof(int), st));
    for (int j = 0; j < n_nb; ++j) {
        TriGate g{};
        g.p1 = d_state, g.skip = nb[j].skip ? 1 : 0, g.check_baseline = check_baseline ? 1 : 0;
        std::memcpy(g.Ow1, kf1->Ow, sizeof(g.Ow1));
        for (int q = 0; q < 3; ++q) g.Ow2[q] = nb[j].kf2.Ow[0][q];
        g.mb2 = nb[j].kf2.mb;
        HIP_OK(hipMemsetAsync(ws.over, 0, sizeof(int), st));
        tri_scan_kernel<<<dim3(S, 1), kTriThreads, 0, st>>>(d_pairs + j, 0, coarse, ws, g);
        if (!coarse) tri_epi_kernel<<<dim3(kEpiPerSlot, S), kEpiThreads, 0, st>>>(d_pairs + j, C, ws);
        tri_walk_kernel<<<1, kWalkThreads, 0, st>>>(d_pairs + j, 0, ws, n_matches + j, d_err, kn.tri_walk_seq ? 0 : 1, g);
        // a neighbour whose candidates overflowed the slices: the one-workgroup search (gated on the device flag)
        tri_kernel<<<1, kTriThreads, 0, st>>>(d_pairs + j, C, 0, coarse, 0, n_matches + j, d_err, ws.over, g);
        cnmp_last_kernel<<<1, kCnmpThreads, 0, st>>>(d_kf1, d_jobs + j, n_cams, d_last);
        cnmp_kernel<<<1, kCnmpThreads, 0, st>>>(d_kf1, d_jobs + j, d_last, a, d_state, check_baseline, has_mp1);
        cnmp_state_kernel<<<1, 1, 0, st>>>(d_kf1, d_jobs + j, 1, d_last, d_state, check_baseline, d_state);
    }
    HIP_OK(hipGetLastError());
    if (side1_state) HIP_OK(hipMemcpyAsync(side1_state, d_state, sizeof(int), hipMemcpyDeviceToDevice, st));
    int h_err = 0;
    HIP_OK(hipMemcpyAsync(&h_err, d_err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_OK(hipFreeAsync(blob, st));
    HIP_OK(hipStreamSynchronize(st));
    return h_err ? (omv_status)h_err : OMV_OK;
}

}  // extern "C"
