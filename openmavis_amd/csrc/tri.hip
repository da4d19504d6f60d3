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
// Float arithmetic without contraction; glibc's atan2f / tanf and correctly rounded sqrtf are restated
// (omv_device.h), so the result is bit-exact to oracle/tri_oracle.cpp.
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
template <typename T, typename Op>
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
    for (int i = w; i < kTriWaves; ++i) total = op(total, s_w[i]);
    T ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = id;
    __syncthreads();
    return op(pre, ex);
}

// compacted candidate code: distance bits 0-5, listed bit 6, camera pair bits 8-11
constexpr uint16_t kCodeListed = 0x40;

__global__ void __launch_bounds__(kTriThreads) tri_kernel(const omv_tri_pair *pairs, TriCams C, int only_stereo,
                                                          int coarse, int check_ori, int32_t *n_matches, int *err) {
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
    __shared__ int s_state, s_row, s_best, s_fin;
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
    if (tid == 0) s_state = 0, s_row = -1, s_best = kTriLow;   // camera-pair state: LL before any assignment
    __syncthreads();
    auto add = [](int x, int y) { return x + y; };
    // thread 0's replay state, carried across batches
    int nmatch = 0, cur_row = -1, bestDist = kTriLow, bestIdx2 = -1;
    auto finish_row = [&]() {
        if (cur_row < 0 || bestIdx2 < 0) return;
        P.match12[cur_row] = bestIdx2;
        ++nmatch;
        if (check_ori) {
            float rot = K1.kps[cur_row].angle - K2.kps[bestIdx2].angle;
            if ((double)rot < 0.0) rot += 360.0f;
            int bin = (int)roundf(rot * (1.0f / kHisto));
            if (bin == kHisto) bin = 0;
            bins[cur_row] = (uint8_t)bin;
        }
    };
    int n_valid = 0;
    // epipolar tests of the compacted batch (step 3) and the in-order replay (step 4)
    auto flush = [&]() {
        __syncthreads();   // the last tile's compacted entries
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
        }
        // step 4 on wave 0: 64 entries at a time staged in registers (one per lane), walked in order on wave-uniform
        // values (v_readlane), so the dependent chain is scalar ALU work instead of LDS round trips; the rows the walk
        // finishes are listed (row << 16 | idx2, in v_item, free after step 3) and written out by all threads after
        int n_fin = 0;
        if (tid < 64) {
            const int lane = tid;
            int state = s_state;
            for (int c0 = 0; c0 < n_valid; c0 += 64) {
                const int k = c0 + lane;
                const bool in = k < n_valid;
                const uint32_t pk_l = in ? v_pk[k] : 0u;
                const int code_l = in ? (int)v_code[k] : 0;
                const uint32_t res_l = (in && !coarse) ? v_res[k] : 0xffffffffu;
                const int m = min(64, n_valid - c0);
                for (int j = 0; j < m; ++j) {
                    const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)pk_l, j);
                    const int code = __builtin_amdgcn_readlane(code_l, j);
                    const int idx1 = (int)(pk >> 16);
                    if (idx1 != cur_row) {
                        if (cur_row >= 0 && bestIdx2 >= 0) {
                            if (lane == 0) v_item[n_fin] = (cur_row << 16) | bestIdx2;
                            ++n_fin;
                        }
                        cur_row = idx1, bestDist = kTriLow, bestIdx2 = -1;
                    }
                    const int dist = code & 0x3f;
                    if (dist > bestDist) continue;
                    if (code & kCodeListed) state = (code >> 8) & 15;
                    const uint32_t res = (uint32_t)__builtin_amdgcn_readlane((int)res_l, j);
                    if ((res >> state) & 1u) bestIdx2 = (int)(pk & 0xffff), bestDist = dist;
                }
            }
            if (lane == 0) s_state = state, s_row = cur_row, s_best = bestDist, s_fin = n_fin;
        }
        __syncthreads();
        n_fin = s_fin;
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
        n_valid = 0;
    };
    for (int a0 = 0; a0 < K1.n_nodes && !only_stereo; a0 += kSeg) {
        // step 1: this segment's node intersection, in ascending node id
        int s1 = 0, n1 = 0, s2 = 0, n2 = 0;
        const int a = a0 + tid;
        if (a < K1.n_nodes) {
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
                int nd = lo, loc = qb - seg_pref[lo];
                int i1 = loc / seg_n2[nd], i2 = loc - i1 * seg_n2[nd];
                for (int j = 0; j < kPerThread && qb + j < q_seg; ++j) {
                    const int idx1 = K1.node_idx[seg_s1[nd] + i1], idx2 = K2.node_idx[seg_s2[nd] + i2];
                    if (!K1.has_mp[idx1] && !K2.has_mp[idx2]) {
                        const int dist = omv::hamming256((const uint64_t *)(K1.desc + 32 * (size_t)idx1),
                                                         (const uint64_t *)(K2.desc + 32 * (size_t)idx2));
                        if (dist <= kTriLow) {
                            const int pr = pair_of(cam_of(K1, idx1), cam_of(K2, idx2));
                            pk[cnt] = (uint32_t)idx1 << 16 | (uint32_t)idx2;
                            cd[cnt] = (uint16_t)(dist | (pr >= 0 ? kCodeListed | (pr << 8) : 0));
                            ++cnt;
                        }
                    }
                    if (++i2 == seg_n2[nd]) {
                        i2 = 0;
                        if (++i1 == seg_n1[nd]) i1 = 0, ++nd;
                    }
                }
            }
            int tot;
            const int off = n_valid + block_scan_excl(cnt, 0, add, s_wi, tot);
            for (int j = 0; j < cnt; ++j) v_pk[off + j] = pk[j], v_code[off + j] = cd[j];
            n_valid += tot;
        }
    }
    flush();
    if (tid == 0) finish_row();
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
    omv_tri_pair *d_pairs = nullptr;
    int *d_err = nullptr;
    HIP_OK(hipMallocAsync((void **)&d_pairs, sizeof(omv_tri_pair) * n_pairs + sizeof(int), st));
    d_err = (int *)(d_pairs + n_pairs);
    HIP_OK(hipMemcpyAsync(d_pairs, pairs, sizeof(omv_tri_pair) * n_pairs, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(d_err, 0, sizeof(int), st));
    tri_kernel<<<n_pairs, kTriThreads, 0, st>>>(d_pairs, C, only_stereo, coarse, check_ori, n_matches, d_err);
    HIP_OK(hipGetLastError());
    int h_err = 0;
    HIP_OK(hipMemcpyAsync(&h_err, d_err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_OK(hipFreeAsync(d_pairs, st));
    HIP_OK(hipStreamSynchronize(st));
    return h_err ? (omv_status)h_err : OMV_OK;
}

}  // extern "C"
