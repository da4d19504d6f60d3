// MI355X-native pose-inertial optimisation of tracked frames: Optimizer::PoseInertialOptimizationLastKeyFrame
// (src/Optimizer.cc:5021-5578) for a batch of frames, one workgroup per frame.
//
// The reference builds a 4-vertex g2o graph per frame (VertexPose / VertexVelocity / VertexGyroBias /
// VertexAccBias of the frame; the last keyframe's four vertices fixed), one EdgeMonoOnlyPose per matched
// keypoint (plus an EdgeStereoOnlyPose where the keypoint has a right coordinate), one EdgeInertial, one
// EdgeGyroRW and one EdgeAccRW, and runs 4 rounds of optimize(10) with Gauss-Newton and a dense LDLT
// (BlockSolverX + LinearSolverDense), classifying outliers between rounds.  Here, per Gauss-Newton
// iteration (optimization_algorithm_gauss_newton.cpp:50-95):
//   errors + build   every thread walks its share of the frame's active visual edges: residual, chi2
//                    (kept per edge: e->chi2() is the value of the last computeError), Huber weight,
//                    the 2x6 / 3x6 Jacobian and its 21 + 6 normal-equation terms; a fixed-order
//                    wavefront + LDS reduction (deterministic run to run)
//   inertial         thread 0 linearises EdgeInertial (only the frame's pose / velocity columns of the
//                    9x24 Jacobian are free); 81 threads form its 9x9 J^T Omega J block and the gradient
//   solve + update   wavefront 0: 15x15 LDLT with diagonal pivoting (Eigen::LDLT semantics, one row per
//                    lane); thread 0: ImuCamPose::Update and the additive velocity / bias updates
// The edges' information matrices (EdgeInertial's PSD-projected inverse covariance) come from a small
// one-thread-per-frame kernel launched first.
// Between rounds every thread classifies its edges (mono pass, then stereo pass: the keypoint flag is
// shared and the stereo pass sees the mono pass's writes, as in the reference's two loops).
//
// Optimizer::PoseInertialOptimizationLastFrame (src/Optimizer.cc:5580-6170) is the same kernel with
// kLF = true: the previous frame's four vertices are free (30 states), EdgeInertial contributes all
// 24 Jacobian columns (thread 0) while thread 64 linearises the EdgePriorPoseImu (G2oTypes.cc:748-785,
// Huber 5), the random walks couple the two frames' biases, the 30x30 LDLT runs on wavefront 0 and
// lanes 0 / 1 update the two frames.  At the end the 30-state Hessian is marginalised onto the frame
// (Optimizer::Marginalize, Optimizer.cc:3388-3455) with a wavefront Jacobi pseudo-inverse.
// pose_constraint_kernel is the ConstraintPoseImu ctor (G2oTypes.h:639-659) that turns that matrix
// into the next frame's prior.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdio>
#include <mutex>
#include <vector>

#include "../../include/omv.h"
#include "g2o_types.h"
#include "omv_device.h"

namespace {

using namespace omv_g2o;

#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

constexpr int kPoseThreads = 256;
constexpr int kPoseWaves = kPoseThreads / 64;
constexpr int kNormal = 27;   // 21 upper-triangle terms of the 6x6 pose block + 6 gradient terms

struct PoseArgs {
    double *Rwb, *twb, *Rcw, *tcw, *vel, *bg, *ba;
    const double *kRwb, *ktwb, *kvel, *kbg, *kba;
    const float *preint;
    const int32_t *m_start, *m_cam, *m_kp;
    const double *m_obs;
    const float *m_w, *m_xw;
    const uint8_t *m_close;
    const int32_t *s_start, *s_cam, *s_kp;
    const double *s_obs;
    const float *s_w, *s_xw;
    int kp_cap;
    double *chi2_m, *chi2_s;   // e->chi2() of the last computeError, per edge
    uint8_t *act_m, *act_s;    // edge level 0 (active)
    uint8_t *kp_out;           // Frame::mvbOutlier
    int32_t *n_good;
    double *H;
    int rec_init;
    const double *info;   // [F][99] EdgeInertial 9x9 | GyroRW 3x3 | AccRW 3x3 information (pose_info_kernel)
    const float *preint_rw;   // [F][kPF] the random walks' preintegration (the grouped kernel forms `info` itself)
    // PoseInertialOptimizationLastFrame: the previous frame's ConstraintPoseImu (EdgePriorPoseImu)
    const double *pRwb, *ptwb, *pvel, *pbg, *pba, *pH;
};

// The edges' information matrices (EdgeInertial ctor :486-495 from `preint`, InfoG / InfoA :5397-5406 /
// :5960-5971 from `preint_rw`), one wavefront per frame: kept out of the optimisation kernel so its
// Jacobi sweeps do not size that kernel's registers.
__global__ void __launch_bounds__(64) pose_info_kernel(const float *preint, const float *preint_rw, double *info) {
    __shared__ double sm[243 + 10 + 5];
    const int f = blockIdx.x, lane = threadIdx.x;
    const float *pre = preint + (size_t)f * kPF, *prw = preint_rw + (size_t)f * kPF;
    double *o = info + (size_t)f * 99;
    inertial_info9_wave<true>(pre + PreView::C, o, sm, lane);
    if (lane == 0) {
        double g[9], a[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                g[3 * r + c] = prw[PreView::C + (9 + r) * 15 + 9 + c], a[3 * r + c] = prw[PreView::C + (12 + r) * 15 + 12 + c];
        inv3(g, o + 81);
        inv3(a, o + 90);
    }
}

// ConstraintPoseImu ctor (G2oTypes.h:639-659), one wavefront per matrix: (H + H) / 2, eigenvalues < 1e-12
// zeroed, V diag(w) V^T over the lower triangle (Eigen's SelfAdjointEigenSolver); a positive definite matrix with
// every eigenvalue above the cut passes unchanged.
__global__ void __launch_bounds__(64) pose_constraint_kernel(const double *Hin, double *Hout) {
    __shared__ double A[225], V[225], cs[16];
    __shared__ int pq[16];
    const int f = blockIdx.x, lane = threadIdx.x;
    const double *hi = Hin + (size_t)f * 225;
    // SelfAdjointEigenSolver reads the lower triangle only: a (rounding-)asymmetric H enters as its lower half mirrored
    for (int q = lane; q < 225; q += 64) {
        const int r = q / 15, c = q % 15;
        const double v = r >= c ? hi[q] : hi[c * 15 + r];
        A[q] = (v + v) / 2;
    }
    wave_lds_sync();
    // Every eigenvalue above 1e-12 (A - tau I factors with positive pivots, tau = 1e-12 plus a margin for the
    // factorisation's rounding): the projection is A itself (V diag(w) V^T = A up to rounding)
    const double tau = 1e-12 + 1e-12 * max_abs_diag<15>(A, lane);
    if (ldl_nopiv_wave<15>(A, tau, nullptr, lane)) {
        for (int q = lane; q < 225; q += 64) Hout[(size_t)f * 225 + q] = A[q];
        return;
    }
    sym_eig_wave_par<15>(A, V, cs, pq, lane);
    double out[4];
    for (int q = lane, i = 0; q < 225; q += 64, ++i) {
        const int r = q / 15, c = q % 15;
        double s = 0;
        for (int k = 0; k < 15; ++k) {
            const double w = A[k * 16] < 1e-12 ? 0.0 : A[k * 16];
            s += V[r * 15 + k] * w * V[c * 15 + k];
        }
        out[i] = s;
    }
    for (int q = lane, i = 0; q < 225; q += 64, ++i) Hout[(size_t)f * 225 + q] = out[i];
}

// One visual edge of the frame (EdgeMonoOnlyPose or EdgeStereoOnlyPose).
struct VEdge {
    int cam, kp;
    bool stereo;
    double obs[3];
    double w;
    double X[3];
};

__device__ __forceinline__ VEdge load_edge(const PoseArgs &A, bool stereo, int e) {
    VEdge v;
    v.stereo = stereo;
    if (!stereo) {
        v.cam = A.m_cam[e], v.kp = A.m_kp[e];
        v.obs[0] = A.m_obs[2 * e], v.obs[1] = A.m_obs[2 * e + 1], v.obs[2] = 0;
        v.w = (double)A.m_w[e];
        for (int q = 0; q < 3; ++q) v.X[q] = (double)A.m_xw[3 * e + q];
    } else {
        v.cam = A.s_cam[e], v.kp = A.s_kp[e];
        for (int q = 0; q < 3; ++q) v.obs[q] = A.s_obs[3 * e + q];
        v.w = (double)A.s_w[e];
        for (int q = 0; q < 3; ++q) v.X[q] = (double)A.s_xw[3 * e + q];
    }
    return v;
}

// computeError: obs - ImuCamPose::Project / ProjectStereo (G2oTypes.cc:192-205); returns chi2
__device__ __forceinline__ double edge_error(const Rig &rig, const double *Rcw, const double *tcw, const VEdge &v,
                                             double *r, double *Xc) {
    const double *R = Rcw + 9 * v.cam, *t = tcw + 3 * v.cam;
    mv3(R, v.X, Xc);
    for (int q = 0; q < 3; ++q) Xc[q] += t[q];
    double u, vv;
    cam_project(rig, v.cam, Xc, u, vv);
    r[0] = v.obs[0] - u, r[1] = v.obs[1] - vv, r[2] = 0;
    double c = r[0] * v.w * r[0] + r[1] * v.w * r[1];
    if (v.stereo) {
        r[2] = v.obs[2] - stereo_ur(u, rig.bf, Xc[2]);
        c += r[2] * v.w * r[2];
    }
    return c;
}

// linearizeOplus of EdgeMonoOnlyPose (G2oTypes.cc:382-400) / EdgeStereoOnlyPose (:433-456):
// J = proj_jac Rcb SE3deriv (2 or 3 rows)
// (pj: the camera's 2x3 projection Jacobian at Xc in its first six entries)
__device__ __forceinline__ void edge_jac_pj(const Rig &rig, const VEdge &v, const double *Xc, double *pj, double *JP) {
    const int c = v.cam;
    double Xb[3];
    mv3(rig.Rbc[c], Xc, Xb);
    for (int q = 0; q < 3; ++q) Xb[q] += rig.tbc[c][q];
    // the stereo row always (zero for a mono edge, never read then): constant trip counts keep pr / JP in registers
    // (a row count only known at run time put both on the private stack)
    if (v.stereo) {
        const double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
        pj[6] = pj[0], pj[7] = pj[1], pj[8] = pj[2] + rig.bf * inv_z2;
    } else {
        pj[6] = pj[7] = pj[8] = 0.0;
    }
    double pr[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q)
            pr[3 * r + q] = pj[3 * r] * rig.Rcb[c][q] + pj[3 * r + 1] * rig.Rcb[c][3 + q] + pj[3 * r + 2] * rig.Rcb[c][6 + q];
    const double x = Xb[0], y = Xb[1], z = Xb[2];
    const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 6; ++q)
            JP[6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
}
__device__ __forceinline__ void edge_jac(const Rig &rig, const VEdge &v, const double *Xc, double *JP) {
    double pj[9];
    cam_jac(rig, v.cam, Xc, pj);
    edge_jac_pj(rig, v, Xc, pj, JP);
}

// computeError and linearizeOplus of one visual edge together (edge_error + edge_jac, the same arithmetic): the
// camera's projection and its Jacobian are evaluated side by side in one branch of the camera type -- independent
// chains given Xc (the projection's float atan2f, the Jacobian's double atan2), which the wave interleaves instead of
// running one after the other.
__device__ __forceinline__ double edge_error_jac(const Rig &rig, const double *Rcw, const double *tcw, const VEdge &v,
                                                 double *r, double *Xc, double *JP) {
    const double *R = Rcw + 9 * v.cam, *t = tcw + 3 * v.cam;
    mv3(R, v.X, Xc);
    for (int q = 0; q < 3; ++q) Xc[q] += t[q];
    double u, vv, pj[9];
    if (rig.model[v.cam] == OMV_CAM_PINHOLE) {
        pinhole_project(rig.cam[v.cam], Xc, u, vv);
        pinhole_jac(rig.cam[v.cam], Xc, pj);
    } else {
        kb8_project(rig.cam[v.cam], Xc, u, vv);
        kb8_jac(rig.cam[v.cam], Xc, pj);
    }
    r[0] = v.obs[0] - u, r[1] = v.obs[1] - vv, r[2] = 0;
    double c = r[0] * v.w * r[0] + r[1] * v.w * r[1];
    if (v.stereo) {
        r[2] = v.obs[2] - stereo_ur(u, rig.bf, Xc[2]);
        c += r[2] * v.w * r[2];
    }
    edge_jac_pj(rig, v, Xc, pj, JP);
    return c;
}

// Per-thread normal-equation terms of one edge: acc[0..20] upper 6x6 (row-major i <= j), acc[21..26] b.
__device__ __forceinline__ void edge_normal(const double *JP, bool stereo, double w, const double *om, double *acc) {
    int q = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j, ++q) {
            double h = JP[i] * JP[j] + JP[6 + i] * JP[6 + j];
            if (stereo) h += JP[12 + i] * JP[12 + j];
            acc[q] += w * h;
        }
    for (int i = 0; i < 6; ++i) {
        double t = JP[i] * om[0] + JP[6 + i] * om[1];
        if (stereo) t += JP[12 + i] * om[2];
        acc[21 + i] += t;
    }
}

// Fixed-order workgroup sum of kNormal doubles per thread into out (valid in every thread after the call).
__device__ __forceinline__ void reduce_normal(double *acc, double (*red)[kNormal], double *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int q = 0; q < kNormal; ++q) {
        double v = acc[q];
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        acc[q] = v;
    }
    if (lane == 0)
        for (int q = 0; q < kNormal; ++q) red[wave][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < kNormal) {
        double t = 0;
        for (int w = 0; w < kPoseWaves; ++w) t += red[w][threadIdx.x];
        out[threadIdx.x] = t;
    }
    __syncthreads();
}

template <int W = kPoseWaves>
__device__ __forceinline__ int block_count(int v, int *sh) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wave] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < W; ++w) t += sh[w];
    __syncthreads();
    return t;
}

// State index (LastFrame's 30-vector: frame pose 0-5, v 6-8, bg 9-11, ba 12-14, previous frame 15-29) ->
// column of EdgeInertial's 9x24 Jacobian [P1 V1 G1 A1 P2 V2]; -1 for the frame's biases.
__device__ __forceinline__ int ei_col(int s) { return s < 9 ? 15 + s : (s < 15 ? -1 : s - 15); }

// EdgeGyroRW (`acc` false) / EdgeAccRW Hessian entry between LastFrame states i and j: [[O, -O], [-O, O]]
// over (frame bias, previous frame bias); 0 off the bias blocks.
__device__ __forceinline__ double rw_entry(int i, int j, bool acc, const double *O) {
    const int o = acc ? 12 : 9;
    const int gi = (i >= o && i < o + 3) ? i - o : ((i >= o + 15 && i < o + 18) ? i - o - 15 : -1);
    const int gj = (j >= o && j < o + 3) ? j - o : ((j >= o + 15 && j < o + 18) ? j - o - 15 : -1);
    if (gi < 0 || gj < 0) return 0.0;
    return ((i < 15) == (j < 15)) ? O[3 * gi + gj] : -O[3 * gi + gj];
}

// kLF = false: PoseInertialOptimizationLastKeyFrame (15 free states, the keyframe's vertices fixed);
// kLF = true: PoseInertialOptimizationLastFrame (30 free states, EdgePriorPoseImu on the previous frame).
template <bool kLF>
// Two waves per SIMD (<= 256 VGPRs + AGPRs per lane, a few spills): at one wave per SIMD (318 registers) only one
// frame's workgroup fits a CU and a 1024-frame batch ran in four rounds; two halve that (1.6x per batch, r03i).
__global__ void __launch_bounds__(kPoseThreads, 2) pose_opt_kernel(Rig rig, PoseArgs A) {
    constexpr int N = kLF ? 30 : 15;
    constexpr int NP = kLF ? 225 : 1;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int C = rig.n_cams;
    // vertex states: index 0 = last keyframe (fixed) / previous frame (free), 1 = frame
    __shared__ double sRwb[18], stwb[6], svel[6], sbg[6], sba[6];
    __shared__ double sRcw[kMaxCams * 9], stcw[kMaxCams * 3];
    __shared__ double red[kPoseWaves][kNormal];
    __shared__ double nrm[kNormal];
    __shared__ double J[216], WJ[216], om9[9], info9[81], infoG[9], infoA[9], e9[9];
    __shared__ double Hs[N * N], bs[N], xs[N], xt[N], lt[2 * N];
    __shared__ int s_ok, cnt[kPoseWaves], ltr[N];
    __shared__ int k1s, k2s;
    // EdgePriorPoseImu: ConstraintPoseImu state / information, error, Jacobian, H_prior J, H_prior e
    __shared__ double sPr[kLF ? 21 : 1], pH[NP], JPr[NP], PJ[NP], eP[kLF ? 15 : 1], OeP[kLF ? 15 : 1];
    __shared__ double Am[NP], Vm[NP], ecs[16];   // Marginalize's eigen-decomposition
    __shared__ int epq[16];
    if (tid == 0) {
        for (int q = 0; q < 9; ++q) sRwb[q] = A.kRwb[9 * f + q], sRwb[9 + q] = A.Rwb[9 * f + q];
        for (int q = 0; q < 3; ++q) {
            stwb[q] = A.ktwb[3 * f + q], stwb[3 + q] = A.twb[3 * f + q];
            svel[q] = A.kvel[3 * f + q], svel[3 + q] = A.vel[3 * f + q];
            sbg[q] = A.kbg[3 * f + q], sbg[3 + q] = A.bg[3 * f + q];
            sba[q] = A.kba[3 * f + q], sba[3 + q] = A.ba[3 * f + q];
        }
        k1s = 0, k2s = 1;
    }
    if constexpr (kLF) {
        for (int q = tid; q < 225; q += kPoseThreads) pH[q] = A.pH[(size_t)f * 225 + q];
        if (tid < 21) {
            double v;
            if (tid < 9) v = A.pRwb[9 * f + tid];
            else if (tid < 12) v = A.ptwb[3 * f + tid - 9];
            else if (tid < 15) v = A.pvel[3 * f + tid - 12];
            else if (tid < 18) v = A.pbg[3 * f + tid - 15];
            else v = A.pba[3 * f + tid - 18];
            sPr[tid] = v;
        }
    }
    for (int q = tid; q < C * 9; q += kPoseThreads) sRcw[q] = A.Rcw[(size_t)f * C * 9 + q];
    for (int q = tid; q < C * 3; q += kPoseThreads) stcw[q] = A.tcw[(size_t)f * C * 3 + q];
    for (int q = tid; q < N; q += kPoseThreads) xs[q] = 0.0;
    for (int q = tid; q < 216; q += kPoseThreads) J[q] = 0.0;   // LastKeyFrame writes only the free columns 15-23
    const float *pre = A.preint + (size_t)f * kPF;
    for (int q = tid; q < 99; q += kPoseThreads) {
        const double v = A.info[(size_t)f * 99 + q];
        if (q < 81) info9[q] = v;
        else if (q < 90) infoG[q - 81] = v;
        else infoA[q - 90] = v;
    }
    const int m0 = A.m_start[f], nm = A.m_start[f + 1] - m0;
    const int s0 = A.s_start[f], ns = A.s_start[f + 1] - s0;
    const int ne = nm + ns;
    uint8_t *kpo = A.kp_out + (size_t)f * A.kp_cap;
    for (int q = tid; q < ne; q += kPoseThreads) {   // mvbOutlier[i] = false; level 0
        if (q < nm) kpo[A.m_kp[m0 + q]] = 0, A.act_m[m0 + q] = 1;
        else kpo[A.s_kp[s0 + q - nm]] = 0, A.act_s[s0 + q - nm] = 1;
    }
    __syncthreads();
    State st{sRwb, stwb, nullptr, nullptr, svel, sbg, sba, nullptr};
    Imu imu{};
    imu.n = 1, imu.kf1 = &k1s, imu.kf2 = &k2s, imu.pre = pre;
    const double dmono = (double)(float)sqrt(5.991), dst = (double)(float)sqrt(7.815);
    const float chi2Mono[4] = {kLF ? 5.991f : 12.f, kLF ? 5.991f : 7.5f, 5.991f, 5.991f};   // :5992 / :5432
    const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
    int nBad = 0, nIn = 0;
    // ImuCamPose::its of the pose vertex this thread updates (thread 0 the frame, thread 1 the previous frame): 0 at
    // the vertex's creation (G2oTypes.cc:74), Rwb normalised after every third Update (:220-225)
    int its_v = 0;
    for (int it = 0; it < 4; ++it) {
        const bool robust = it < 3;   // setRobustKernel(0) after the third classification
        for (int gi = 0; gi < 10; ++gi) {
            // computeActiveErrors + the visual part of buildSystem
            double acc[kNormal];
            for (int q = 0; q < kNormal; ++q) acc[q] = 0;
            for (int q = tid; q < ne; q += kPoseThreads) {
                const bool stq = q >= nm;
                const int e = stq ? s0 + q - nm : m0 + q;
                if (!(stq ? A.act_s[e] : A.act_m[e])) continue;
                const VEdge v = load_edge(A, stq, e);
                double r[3], Xc[3], JP[18];
                const double c2 = edge_error_jac(rig, sRcw, stcw, v, r, Xc, JP);
                (stq ? A.chi2_s : A.chi2_m)[e] = c2;
                double w1 = 1.0;
                if (robust) {
                    double r0;
                    if (stq) huber(c2, dst, dst * dst, r0, w1);
                    else huber(c2, dmono, dmono * dmono, r0, w1);
                }
                const double om[3] = {-v.w * r[0] * w1, -v.w * r[1] * w1, stq ? -v.w * r[2] * w1 : 0.0};
                edge_normal(JP, stq, v.w * w1, om, acc);
            }
            if constexpr (kLF) {   // EdgeInertial (all six vertex blocks) and EdgePriorPoseImu, in parallel
                if (tid == 0) {
                    imu_error(st, imu, 0, e9);
                    imu_jacobian(st, imu, 0, J);
                }
                if (tid == 64) prior_error_jac(sPr, sRwb, stwb, svel, sbg, sba, eP, JPr);
            } else {
                if (tid == 0) imu_error_jac_p2v2(st, imu, 0, e9, J);   // EdgeInertial at the current state
            }
            reduce_normal(acc, red, nrm);   // (its barriers also publish J / e9 / eP / JPr)
            if constexpr (kLF) {
                for (int q = tid; q < 216; q += kPoseThreads) {   // Info J over all 24 columns
                    const int r = q / 24, c = q % 24;
                    double t = 0;
                    for (int k = 0; k < 9; ++k) t += info9[r * 9 + k] * J[k * 24 + c];
                    WJ[q] = t;
                }
                for (int q = tid; q < 225; q += kPoseThreads) {   // H_prior J
                    const int k = q / 15, j = q % 15;
                    double t = 0;
                    for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * JPr[l * 15 + j];
                    PJ[q] = t;
                }
                if (tid >= 64 && tid < 79) {   // H_prior e
                    const int k = tid - 64;
                    double t = 0;
                    for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * eP[l];
                    OeP[k] = t;
                }
            } else {
                // EdgeInertial: free columns 15-20 (frame pose) and 21-23 (frame velocity) -> state 0..8
                for (int q = tid; q < 81; q += kPoseThreads) {
                    const int r = q / 9, c = q % 9;
                    double t = 0;
                    for (int k = 0; k < 9; ++k) t += info9[r * 9 + k] * J[k * 24 + 15 + c];
                    WJ[q] = t;
                }
            }
            if (tid < 9) {
                double t = 0;
                for (int k = 0; k < 9; ++k) t += info9[tid * 9 + k] * e9[k];
                om9[tid] = -t;
            }
            __syncthreads();
            if constexpr (kLF) {
                // EdgePriorPoseImu's Huber weight: chi2 = e^T H_prior e (every thread, same order)
                double chi2p = 0, r0, w1p;
                for (int k = 0; k < 15; ++k) chi2p += eP[k] * OeP[k];
                huber(chi2p, 5.0, 25.0, r0, w1p);
                // lower triangle in the oracle's per-element order (visual, inertial, random walks, prior), mirrored
                for (int q = tid; q < N * N; q += kPoseThreads) {
                    const int i = q / N, j = q % N;
                    if (j > i) continue;
                    double h = 0;
                    if (i < 6) h = nrm[j * 6 - j * (j - 1) / 2 + (i - j)];
                    const int ci = ei_col(i), cj = ei_col(j);
                    if (ci >= 0 && cj >= 0) {
                        double t = 0;
                        for (int k = 0; k < 9; ++k) t += J[k * 24 + ci] * WJ[k * 24 + cj];
                        h += t;
                    }
                    h += rw_entry(i, j, false, infoG);
                    h += rw_entry(i, j, true, infoA);
                    if (i >= 15 && j >= 15) {
                        double t = 0;
                        for (int k = 0; k < 15; ++k) t += JPr[k * 15 + i - 15] * (w1p * PJ[k * 15 + j - 15]);
                        h += t;
                    }
                    Hs[i * N + j] = h;
                    Hs[j * N + i] = h;
                }
                if (tid < N) {
                    const int i = tid;
                    double t = i < 6 ? nrm[21 + i] : 0.0;
                    const int ci = ei_col(i);
                    if (ci >= 0) {
                        double u = 0;
                        for (int k = 0; k < 9; ++k) u += J[k * 24 + ci] * om9[k];
                        t += u;
                    }
                    // EdgeGyroRW / EdgeAccRW: e = b_frame - b_prev, J_frame = I, J_prev = -I
                    const int bi = i % 15;
                    if (bi >= 9) {
                        const bool acc_rw = bi >= 12;
                        const int r = (bi - 9) % 3;
                        const double *Iw = acc_rw ? infoA : infoG;
                        const double *bv = acc_rw ? sba : sbg;
                        double ee[3];
                        for (int k = 0; k < 3; ++k) ee[k] = bv[3 + k] - bv[k];
                        const double oe = Iw[3 * r] * ee[0] + Iw[3 * r + 1] * ee[1] + Iw[3 * r + 2] * ee[2];
                        t += i < 15 ? -oe : oe;
                    }
                    if (i >= 15) {   // b -= rho' J^T H_prior e
                        double u = 0;
                        for (int k = 0; k < 15; ++k) u += JPr[k * 15 + i - 15] * (-OeP[k] * w1p);
                        t += u;
                    }
                    bs[i] = t;
                }
            } else {
                for (int q = tid; q < 225; q += kPoseThreads) {
                    const int i = q / 15, j = q % 15;
                    double h = 0;
                    if (i < 6 && j < 6) {   // visual 6x6 (symmetric from the upper triangle)
                        const int a = min(i, j), b = max(i, j);
                        h = nrm[a * 6 - a * (a - 1) / 2 + (b - a)];
                    }
                    if (i < 9 && j < 9) {
                        double t = 0;
                        for (int k = 0; k < 9; ++k) t += J[k * 24 + 15 + i] * WJ[k * 9 + j];
                        h += t;
                    }
                    if (i >= 9 && j >= 9 && (i < 12) == (j < 12)) h += (i < 12 ? infoG : infoA)[3 * ((i - 9) % 3) + (j - 9) % 3];
                    Hs[q] = h;
                }
                if (tid < 15) {
                    double t = tid < 6 ? nrm[21 + tid] : 0.0;
                    if (tid < 9) {
                        double u = 0;
                        for (int k = 0; k < 9; ++k) u += J[k * 24 + 15 + tid] * om9[k];
                        t += u;
                    }
                    if (tid >= 9) {   // EdgeGyroRW / EdgeAccRW: e = b - b_kf, J = I
                        const bool acc_rw = tid >= 12;
                        const int r = (tid - 9) % 3;
                        const double *Iw = acc_rw ? infoA : infoG;
                        const double *bv = acc_rw ? sba : sbg;
                        double ee[3];
                        for (int k = 0; k < 3; ++k) ee[k] = bv[3 + k] - bv[k];
                        t -= Iw[3 * r] * ee[0] + Iw[3 * r + 1] * ee[1] + Iw[3 * r + 2] * ee[2];
                    }
                    bs[tid] = t;
                }
            }   // LastKeyFrame system
            __syncthreads();
            if (tid < 64) {
                const bool ok = ldlt_pivot_solve_wave<N>(Hs, bs, xt, lt, ltr, tid);
                if (tid == 0) {
                    if (ok)   // a failed solve leaves the solver's previous x in place
                        for (int q = 0; q < N; ++q) xs[q] = xt[q];
                    s_ok = ok ? 1 : 0;
                }
                wave_lds_sync();
                // VertexPose::oplusImpl -> ImuCamPose::Update (G2oTypes.cc:211-235): lane 0 the frame (with its
                // cameras), lane 1 the previous frame (LastFrame; its cameras are not read)
                if (tid == 0 || (kLF && tid == 1)) {
                    const int v = tid == 0 ? 1 : 0;
                    const double *xv = xs + (tid == 0 ? 0 : 15);
                    double *Rw = sRwb + 9 * v, *tw = stwb + 3 * v;
                    double t[3], dR[9], Rn[9];
                    mv3(Rw, xv + 3, t);
                    for (int q = 0; q < 3; ++q) tw[q] += t[q];
                    exp_so3(xv, dR);
                    mm3(Rw, dR, Rn);
                    if (++its_v >= 3) polar3(Rn), its_v = 0;   // NormalizeRotation after every third update
                    for (int q = 0; q < 9; ++q) Rw[q] = Rn[q];
                    if (tid == 0) {
                        double Rbw[9], tbw[3];
                        tr3(Rn, Rbw);
                        mv3(Rbw, tw, tbw);
                        for (int q = 0; q < 3; ++q) tbw[q] = -tbw[q];
                        for (int c = 0; c < C; ++c) {
                            double Rc[9], tc[3];
                            mm3(rig.Rcb[c], Rbw, Rc);
                            mv3(rig.Rcb[c], tbw, tc);
                            for (int q = 0; q < 9; ++q) sRcw[9 * c + q] = Rc[q];
                            for (int q = 0; q < 3; ++q) stcw[3 * c + q] = tc[q] + rig.tcb[c][q];
                        }
                    }
                    for (int q = 0; q < 3; ++q)
                        svel[3 * v + q] += xv[6 + q], sbg[3 * v + q] += xv[9 + q], sba[3 * v + q] += xv[12 + q];
                }
            }
            __syncthreads();
            if (!s_ok) break;   // optimize() stops after a failed iteration
        }
        // classification (:5436-5490): the mono pass, then the stereo pass
        int bad = 0, in = 0;
        const float chi2close = 1.5f * chi2Mono[it];
        for (int pass = 0; pass < 2; ++pass) {
            const int n = pass ? ns : nm;
            for (int q = tid; q < n; q += kPoseThreads) {
                const bool stq = pass == 1;
                const int e = stq ? s0 + q : m0 + q;
                const VEdge v = load_edge(A, stq, e);
                double *c2p = stq ? A.chi2_s + e : A.chi2_m + e;
                double Xc[3];
                if (kpo[v.kp]) {   // outliers of the last round: computeError at the current state
                    double r[3];
                    *c2p = edge_error(rig, sRcw, stcw, v, r, Xc);
                }
                const float chi2 = (float)*c2p;
                bool out;
                if (!stq) {
                    const bool close = A.m_close[e] != 0;
                    const double *R = sRcw + 9 * v.cam;
                    const bool depth_pos = (R[6] * v.X[0] + R[7] * v.X[1] + R[8] * v.X[2] + stcw[3 * v.cam + 2]) > 0.0;
                    out = (chi2 > chi2Mono[it] && !close) || (close && chi2 > chi2close) || !depth_pos;
                } else {
                    out = chi2 > chi2Stereo[it];
                }
                kpo[v.kp] = out ? 1 : 0;
                (stq ? A.act_s : A.act_m)[e] = out ? 0 : 1;
                bad += out ? 1 : 0;
                in += out ? 0 : 1;
            }
            __threadfence_block();
            __syncthreads();
        }
        nBad = block_count(bad, cnt);
        nIn = block_count(in, cnt);
        if (ne + (kLF ? 4 : 3) < 10) break;   // optimizer.edges().size() < 10
    }
    if (nIn < 30 && !A.rec_init) {   // recover not too bad points (:5503-5526)
        int bad = 0;
        for (int q = tid; q < ne; q += kPoseThreads) {
            const bool stq = q >= nm;
            const int e = stq ? s0 + q - nm : m0 + q;
            const VEdge v = load_edge(A, stq, e);
            double r[3], Xc[3];
            const double c2 = edge_error(rig, sRcw, stcw, v, r, Xc);
            (stq ? A.chi2_s : A.chi2_m)[e] = c2;
            if (c2 < (stq ? 24.f : 18.f)) kpo[v.kp] = 0;
            else ++bad;
        }
        nBad = block_count(bad, cnt);
    }
    __threadfence_block();
    __syncthreads();
    if constexpr (kLF) {
        // :6112-6156: the 30-state Hessian without robust weights (EdgeInertial, the random walks, the prior,
        // inlier visual edges) at the final state, then Marginalize(H, 0, 14) of the previous frame
        // (:3388-3455): H_ff - H_fp pinv(H_pp) H_pf, JacobiSVD's pseudo-inverse of the symmetric H_pp as
        // V diag(1/w) V^T over |w| > 1e-6.  Hs in this kernel's state order (frame 0-14, previous 15-29).
        if (A.H) {
            double acc[kNormal];
            for (int q = 0; q < kNormal; ++q) acc[q] = 0;
            for (int q = tid; q < ne; q += kPoseThreads) {
                const bool stq = q >= nm;
                const int e = stq ? s0 + q - nm : m0 + q;
                const VEdge v = load_edge(A, stq, e);
                if (kpo[v.kp]) continue;
                double r[3], Xc[3], JP[18];
                edge_error_jac(rig, sRcw, stcw, v, r, Xc, JP);
                const double om[3] = {0, 0, 0};
                edge_normal(JP, stq, v.w, om, acc);
            }
            if (tid == 0) imu_jacobian(st, imu, 0, J);
            if (tid == 64) prior_error_jac(sPr, sRwb, stwb, svel, sbg, sba, eP, JPr);
            reduce_normal(acc, red, nrm);
            for (int q = tid; q < 216; q += kPoseThreads) {
                const int r = q / 24, c = q % 24;
                double t = 0;
                for (int k = 0; k < 9; ++k) t += info9[r * 9 + k] * J[k * 24 + c];
                WJ[q] = t;
            }
            for (int q = tid; q < 225; q += kPoseThreads) {
                const int k = q / 15, j = q % 15;
                double t = 0;
                for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * JPr[l * 15 + j];
                PJ[q] = t;
            }
            __syncthreads();
            for (int q = tid; q < N * N; q += kPoseThreads) {   // the reference's order: ei, egr, ear, ep, visual
                const int i = q / N, j = q % N;
                double h = 0;
                const int ci = ei_col(i), cj = ei_col(j);
                if (ci >= 0 && cj >= 0) {
                    double t = 0;
                    for (int k = 0; k < 9; ++k) t += J[k * 24 + ci] * WJ[k * 24 + cj];
                    h += t;
                }
                h += rw_entry(i, j, false, infoG);
                h += rw_entry(i, j, true, infoA);
                if (i >= 15 && j >= 15) {
                    double t = 0;
                    for (int k = 0; k < 15; ++k) t += JPr[k * 15 + i - 15] * PJ[k * 15 + j - 15];
                    h += t;
                }
                if (i < 6 && j < 6) {
                    const int a = min(i, j), b = max(i, j);
                    h += nrm[a * 6 - a * (a - 1) / 2 + (b - a)];
                }
                Hs[q] = h;
            }
            __syncthreads();
            for (int q = tid; q < 225; q += kPoseThreads) Am[q] = Hs[(15 + q / 15) * N + 15 + q % 15];
            __syncthreads();
            if (tid < 64) pinv15_wave(Am, Vm, PJ, ecs, epq, tid);   // pinv(H_pp) -> PJ
            __syncthreads();
            for (int q = tid; q < 225; q += kPoseThreads) {   // T = H_fp pinv(H_pp) -> JPr
                const int i = q / 15, j = q % 15;
                double s = 0;
                for (int k = 0; k < 15; ++k) s += Hs[i * N + 15 + k] * PJ[k * 15 + j];
                JPr[q] = s;
            }
            __syncthreads();
            for (int q = tid; q < 225; q += kPoseThreads) {
                const int i = q / 15, j = q % 15;
                double s = 0;
                for (int k = 0; k < 15; ++k) s += JPr[i * 15 + k] * Hs[(15 + k) * N + j];
                A.H[(size_t)f * 225 + q] = Hs[i * N + j] - s;
            }
        }
    } else if (A.H) {
        // ConstraintPoseImu's Hessian (:5529-5571): information without robust weights, inlier edges only
        double acc[kNormal];
        for (int q = 0; q < kNormal; ++q) acc[q] = 0;
        for (int q = tid; q < ne; q += kPoseThreads) {
            const bool stq = q >= nm;
            const int e = stq ? s0 + q - nm : m0 + q;
            const VEdge v = load_edge(A, stq, e);
            if (kpo[v.kp]) continue;
            double r[3], Xc[3], JP[18];
            edge_error_jac(rig, sRcw, stcw, v, r, Xc, JP);
            const double om[3] = {0, 0, 0};
            edge_normal(JP, stq, v.w, om, acc);
        }
        if (tid == 0) imu_error_jac_p2v2(st, imu, 0, e9, J);
        reduce_normal(acc, red, nrm);
        for (int q = tid; q < 81; q += kPoseThreads) {
            const int r = q / 9, c = q % 9;
            double t = 0;
            for (int k = 0; k < 9; ++k) t += info9[r * 9 + k] * J[k * 24 + 15 + c];
            WJ[q] = t;
        }
        __syncthreads();
        for (int q = tid; q < 225; q += kPoseThreads) {
            const int i = q / 15, j = q % 15;
            double h = 0;
            if (i < 6 && j < 6) {
                const int a = min(i, j), b = max(i, j);
                h = nrm[a * 6 - a * (a - 1) / 2 + (b - a)];
            }
            if (i < 9 && j < 9) {
                double t = 0;
                for (int k = 0; k < 9; ++k) t += J[k * 24 + 15 + i] * WJ[k * 9 + j];
                h += t;
            }
            if (i >= 9 && j >= 9 && (i < 12) == (j < 12)) h += (i < 12 ? infoG : infoA)[3 * ((i - 9) % 3) + (j - 9) % 3];
            A.H[(size_t)f * 225 + q] = h;
        }
    }
    // state back
    if (tid == 0) {
        for (int q = 0; q < 9; ++q) A.Rwb[9 * f + q] = sRwb[9 + q];
        for (int q = 0; q < 3; ++q) {
            A.twb[3 * f + q] = stwb[3 + q], A.vel[3 * f + q] = svel[3 + q];
            A.bg[3 * f + q] = sbg[3 + q], A.ba[3 * f + q] = sba[3 + q];
        }
        A.n_good[f] = ne - nBad;
    }
    for (int q = tid; q < C * 9; q += kPoseThreads) A.Rcw[(size_t)f * C * 9 + q] = sRcw[q];
    for (int q = tid; q < C * 3; q += kPoseThreads) A.tcw[(size_t)f * C * 3 + q] = stcw[q];
}


// =====================================================================================================================
// Latency path: one frame over G workgroups (Tracking's call pattern is ONE frame whose pose the next frame waits for,
// Tracking.cc:2904-2942).  The frame's visual edges are split by keypoint range over the G workgroups (both edges of a
// keypoint that carries a mono and a stereo edge land in one workgroup, so mvbOutlier stays workgroup-local) and held
// in LDS for the whole call.  Per Gauss-Newton iteration every workgroup evaluates its edges (waves 0-3, one edge per
// thread at <= 256 edges per workgroup), while wave 4 linearises EdgeInertial and wave 5 (LastFrame) EdgePriorPoseImu at
// the same state; the 27 visual normal-equation sums of the G workgroups are exchanged through write-through (`sc1`)
// payload rows and one flag per part (MI355X_MICROARCH.md hand-off R1: drained stores, flag poll, `sc1` loads) and
// summed in part order,
// so every workgroup holds the identical system and runs the identical solve and update -- no second hop to broadcast
// the state.  The 15x15 / 30x30 system is solved by one wavefront with the rows in registers (pivot order first,
// Eigen's transpositions replayed on the original diagonal; right-looking LDL^T with v_readlane row broadcasts).
// =====================================================================================================================
constexpr int kLatThreads = 256;        // one wave per SIMD (512 registers): visual edges on 3 (LastFrame 2) waves, then
                                        // EdgeInertial, then (LastFrame) EdgePriorPoseImu on a wave of its own
__host__ __device__ constexpr int lat_edge_threads(bool lf) { return lf ? 128 : 192; }
constexpr int kLatMaxParts = 48;        // workgroups per frame
constexpr int kLatCap = 1024;           // visual edges per workgroup (LDS)
constexpr int kLatFlagCap = 16384;      // keypoints per frame (mvbOutlier staged in LDS)
constexpr int kLatRow = 32;             // payload words per (frame, slot, part): the 27 normal-equation sums
constexpr int kLatAutoFrames = 16;      // OMV_POSE_AUTO: the grouped kernel up to this many frames per call
constexpr size_t kLatFrameGran = 2 * kLatMaxParts * (kLatRow + 1);   // 8-byte words per frame: two slots (phase parity)
                                                                      // of payload rows + flags
typedef __attribute__((address_space(1))) unsigned long long gu64;
#ifdef OMV_POSE_PROFILE   // phase times of the grouped kernel (wall_clock64 = 100 MHz), printed by part 0
__device__ unsigned long long g_lat_pub[48][48];   // per part, per Gauss-Newton iteration: the hand-off's start
__device__ unsigned long long g_lat_x[4];          // part 0's exchanges: publish -> flags seen -> payload in -> summed, count
#define LAT_T(var) const unsigned long long var = wall_clock64()
#define LAT_ACC(slot, a, b) prof[slot] += (b) - (a)
#else
#define LAT_T(var)
#define LAT_ACC(slot, a, b)
#endif

// Sum over the frame's G workgroups of n <= 32 doubles (lane q of wave 0 holds value q) into out[0..n) (LDS), every
// part getting the identical sums.  MI355X_MICROARCH.md's R1 hand-off: the part's n values go out as write-through
// (`sc1`) 8-byte stores to its payload row of slot (phase & 1), the wave drains them (vmcnt(0)), then ONE lane stores
// the part's flag = salt | phase; the consumer polls the G flags with one load per spin (lane p: part p's flag), then
// reads the payload with `sc1` loads (every load of them: no acquire needed).  The read is laid out for the sum:
// lane (h, q) = (lane >> 5, lane & 31) loads word q of parts h * ceil(G / 2) .. (all in flight, in registers) and
// adds them in part order; the two halves' sums meet by one shuffle (a + b == b + a exactly, so every part's lanes
// get the identical total).  A sum read back from LDS one part at a time was a 47-long chain of LDS round trips
// (~2 us per exchange).  One wavefront; false on a bounded-spin timeout (a missing sibling workgroup).
// Out of line (five call sites; inlined they were a sixth of the kernel's code, whose per-iteration code must stay
// within the CU's instruction cache).
__device__ __attribute__((noinline)) bool lat_exchange(gu64 *fb, int phase, uint32_t salt, int g, int G, double v, int n,
                                                       double *out, int lane) {
    constexpr int L = kLatMaxParts / 2;   // parts per half
    const uint32_t tag = salt | (uint32_t)phase;
    const int sl = phase & 1;
#ifdef OMV_POSE_PROFILE
    const unsigned long long tx0 = wall_clock64();
#endif
    gu64 *pay = fb + (size_t)sl * kLatMaxParts * kLatRow;                                // [part][kLatRow]
    gu64 *flg = fb + (size_t)2 * kLatMaxParts * kLatRow + (size_t)sl * kLatMaxParts;     // [part]
    if (lane < n)
        __hip_atomic_store(pay + g * kLatRow + lane, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the payload has left this CU before the flag (R1)
    if (lane == 0) __hip_atomic_store(flg + g, (unsigned long long)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spins = 0;; ++spins) {
        const unsigned long long x =
            lane < G ? __hip_atomic_load(flg + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (unsigned long long)tag;
        if (__all((uint32_t)x == tag)) break;
        if (spins > (1u << 22)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
#ifdef OMV_POSE_PROFILE
    const unsigned long long tx1 = wall_clock64();
#endif
    const int q = lane & 31, h = lane >> 5, Gh = (G + 1) >> 1, p0 = h * Gh;
    const int np = q < n ? min(Gh, G - p0) : 0;   // parts this lane adds
    double val[L];
#pragma unroll
    for (int m = 0; m < L; ++m)
        val[m] = m < np ? __builtin_bit_cast(double, __hip_atomic_load(pay + (p0 + m) * kLatRow + q, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT))
                        : 0.0;
    double s = 0;
#pragma unroll
    for (int m = 0; m < L; ++m) s = m < np ? s + val[m] : s;
    s += __shfl_xor(s, 32, 64);
    if (h == 0 && q < n) out[q] = s;
    wave_lds_sync();
#ifdef OMV_POSE_PROFILE
    if (g == 0 && lane == 0) {
        const unsigned long long tx2 = wall_clock64();
        atomicAdd(&g_lat_x[0], tx1 - tx0), atomicAdd(&g_lat_x[1], tx2 - tx1);
        atomicAdd(&g_lat_x[3], 1ull);
    }
#endif
    return true;
}

// Eigen::LDLT<MatrixXd> (ldlt_inplace::unblocked's pivot order, isPositive(), _solve_impl's D pseudo-inverse below
// DBL_MIN) of the N x N symmetric H (LDS, row-major) on one wavefront, lane i = pivot position i:
//   pick order  Eigen swaps the largest |diagonal| of the trailing corner to position k, first position on ties; that
//               diagonal is never updated before it is picked, so the order follows from the original diagonal alone:
//               by rank when the magnitudes are distinct, else replayed step by step (one ballot per step)
//   factor      rows of P H P^T in registers; step k: D_k by v_readlane, column k below scaled by 1 / D_k, trailing
//               update from row k (v_readlane broadcasts, FMA); a zero pivot leaves its column unscaled and no update
//               (its terms D_k l l^T vanish in Eigen's left-looking form)
//   solve       y = P b, L y' = y, y'' = D^+ y', L^T x = y'', x = P^T (same per-element subtraction order as Eigen's
//               triangular solves; the factor differs from Eigen's by rounding: right-looking, fused multiply-adds)
// x: LDS out (written only on success); pick / Lm: LDS scratch [N] / [N * N].  Returns isPositive().
// 1 / x by v_rcp_f64 and two Newton steps (the LBA's reciprocal: exact on sampled arguments, a few ulp at worst).
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}

// Eigen's pick order of the N x N symmetric H into pick[] (one wavefront); false on a NaN diagonal.
template <int N>
__device__ __forceinline__ bool ldlt_pick_order(const double *H, int *pick, int lane) {
    static_assert(N <= 32, "rows on lanes 0..31");
    const bool in = lane < N;
    const double dv = in ? fabs(H[lane * (N + 1)]) : 0.0;
    int gt = 0, eq = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double o = fabs(H[j * (N + 1)]);
        gt += o > dv ? 1 : 0;
        eq += o == dv ? 1 : 0;
    }
    if (__ballot(in && !(dv == dv))) return false;
    if (!__ballot(in && eq > 1)) {
        if (in) pick[gt] = lane;
    } else {
        int pos = lane;
        bool picked = false;
        for (int k = 0; k < N; ++k) {
            uint64_t cand = __ballot(in && !picked && gt <= k && k < gt + eq);
            int e = __builtin_ctzll(cand);
            if (cand & (cand - 1)) {
                int bp = __builtin_amdgcn_readlane(pos, e);
                for (uint64_t m = cand & (cand - 1); m; m &= m - 1) {
                    const int c = __builtin_ctzll(m), pc = __builtin_amdgcn_readlane(pos, c);
                    if (pc < bp) bp = pc, e = c;
                }
            }
            const int xk = __builtin_ctzll(__ballot(in && pos == k));
            const int pe = __builtin_amdgcn_readlane(pos, e);
            if (lane == xk) pos = pe;
            if (lane == e) pos = k, picked = true;
            if (lane == 0) pick[k] = e;
        }
    }
    return true;
}

template <int N>
__device__ __forceinline__ bool ldlt_pick_solve(const double *H, const double *b, double *x, int *pick, double *Lm, int lane) {
    static_assert(N <= 32, "rows on lanes 0..31");
    const bool in = lane < N;
    const double dv = in ? fabs(H[lane * (N + 1)]) : 0.0;
    int gt = 0, eq = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double o = fabs(H[j * (N + 1)]);
        gt += o > dv ? 1 : 0;
        eq += o == dv ? 1 : 0;
    }
    if (__ballot(in && !(dv == dv))) return false;   // a NaN diagonal: no factorisation
    if (!__ballot(in && eq > 1)) {
        if (in) pick[gt] = lane;
    } else {   // selection with positional swaps, lanes = elements (pos = current position)
        int pos = lane;
        bool picked = false;
        for (int k = 0; k < N; ++k) {
            uint64_t cand = __ballot(in && !picked && gt <= k && k < gt + eq);
            int e = __builtin_ctzll(cand);
            if (cand & (cand - 1)) {   // several equal magnitudes: the lowest current position
                int bp = __builtin_amdgcn_readlane(pos, e);
                for (uint64_t m = cand & (cand - 1); m; m &= m - 1) {
                    const int c = __builtin_ctzll(m), pc = __builtin_amdgcn_readlane(pos, c);
                    if (pc < bp) bp = pc, e = c;
                }
            }
            const int xk = __builtin_ctzll(__ballot(in && pos == k));
            const int pe = __builtin_amdgcn_readlane(pos, e);
            if (lane == xk) pos = pe;
            if (lane == e) pos = k, picked = true;
            if (lane == 0) pick[k] = e;
        }
    }
    wave_lds_sync();
    const int pi = in ? pick[lane] : 0;
    int pj[N];   // the pick order in registers first, then every row read back to back (H symmetric: column pi of row pj)
#pragma unroll
    for (int j = 0; j < N; ++j) pj[j] = pick[j];
    double r[N];
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? H[pj[j] * N + pi] : 0.0;
    if (!(lane_f64(r[0], 0) != 0.0)) {   // largest |diagonal| zero: Eigen stops with ZeroSign; the solve gives x = 0
        if (in) x[lane] = 0.0;
        wave_lds_sync();
        return true;
    }
    // One basic block for the whole factorisation (no data-dependent branches) so the pivot chain of step k + 1 can
    // issue while step k's trailing update is still in flight: a zero pivot gives inv = 0, hence l = 0 (no update,
    // column k left unscaled), sign bits 1 (a positive D) / 2 (a negative D): Eigen's isPositive() = no bit 2.
    int sign = 0;
    double dmine = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double d = lane_f64(r[k], k);
        dmine = lane == k ? d : dmine;
        const bool nz = fabs(d) > 0.0;
        const double inv = nz ? rcp_nr(d) : 0.0;
        const bool below = lane > k;
        const double l = below ? r[k] * inv : 0.0;
#pragma unroll
        for (int j = k + 1; j < N; ++j) r[j] = __builtin_fma(-l, lane_f64(r[j], k), r[j]);
        r[k] = (below && nz) ? l : r[k];
        sign |= (d > 0 ? 1 : 0) | (d < 0 ? 2 : 0);
    }
    if (sign & 2) return false;
    double y = in ? b[pi] : 0.0;
#pragma unroll
    for (int k = 0; k + 1 < N; ++k) {
        const double yk = lane_f64(y, k);
        if (lane > k) y = __builtin_fma(-r[k], yk, y);
    }
    y = fabs(dmine) > 2.2250738585072014e-308 ? y / dmine : 0.0;
    if (in)
#pragma unroll
        for (int j = 0; j < N; ++j) Lm[lane * N + j] = r[j];
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? Lm[j * N + lane] : 0.0;   // r[j] = L_j,lane
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        const double xj = lane_f64(y, j);
        if (lane < j) y = __builtin_fma(-r[j], xj, y);
    }
    if (in) x[pi] = y;
    wave_lds_sync();
    return true;
}

// The same solve by the whole workgroup (NT threads), for the latency kernel where the other waves would idle: the
// pick order on wave 0 as ldlt_pick_solve; the factorisation of P H P^T element-parallel on its lower triangle (thread
// t owns elements t, t + NT, ... in registers), one workgroup barrier per pivot step: the owners of column k publish
// it to LDS (two buffers by step parity, so a step needs no second barrier), every thread reads D_k and its rows'
// entries and applies a_ij -= (a_ik / D_k) a_jk (a zero pivot: no update, column left unscaled, as ldlt_pick_solve);
// then the triangular solves on wave 0 from the factor staged in Lm.  isPositive() = no negative pivot.  The
// factor's rounding differs from ldlt_pick_solve's in the update's operand (lower-triangle column entries for both
// factors) only.  Called by all NT threads; x written on success.  col: LDS scratch [2 * N]; flag: LDS int.
template <int N, int NT>
__device__ __forceinline__ bool ldlt_elem_solve(const double *H, const double *b, double *x, int *pick, double *Lm,
                                                double *col, int *flag, int tid) {
    constexpr int T = N * (N + 1) / 2, PER = (T + NT - 1) / NT;
    const int lane = tid & 63;
    if (tid < 64) {
        const bool okp = ldlt_pick_order<N>(H, pick, lane);
        if (lane == 0) *flag = okp ? 0 : 1;
    }
    __syncthreads();
    if (*flag) return false;   // a NaN diagonal (uniform)
    int ei[PER], ej[PER];
    double a[PER];
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        const int e = tid + p * NT;
        // row i of the packed lower triangle: i (i + 1) / 2 <= e
        int i = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
        i += (i + 1) * (i + 2) / 2 <= e ? 1 : 0;
        i -= i * (i + 1) / 2 > e ? 1 : 0;
        const int j = e - i * (i + 1) / 2;
        ei[p] = e < T ? i : N, ej[p] = e < T ? j : N;
        a[p] = e < T ? H[pick[i] * N + pick[j]] : 0.0;
    }
    if (!(H[pick[0] * (N + 1)] != 0.0)) {   // largest |diagonal| zero: x = 0
        if (tid < N) x[tid] = 0.0;
        __syncthreads();
        return true;
    }
    int sign = 0;
    for (int k = 0; k < N; ++k) {
        double *c = col + (k & 1) * N;
#pragma unroll
        for (int p = 0; p < PER; ++p)
            if (ej[p] == k) c[ei[p]] = a[p];
        __syncthreads();
        const double d = c[k];
        const bool nz = fabs(d) > 0.0;
        const double inv = nz ? rcp_nr(d) : 0.0;
        sign |= (d > 0 ? 1 : 0) | (d < 0 ? 2 : 0);
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            if (ej[p] > k && ej[p] < N) a[p] = __builtin_fma(-(c[ei[p]] * inv), c[ej[p]], a[p]);
            else if (ej[p] == k && ei[p] > k && nz) a[p] = a[p] * inv;
        }
    }
    if (sign & 2) return false;   // uniform: every thread saw every pivot
#pragma unroll
    for (int p = 0; p < PER; ++p)
        if (ei[p] < N) Lm[ei[p] * N + ej[p]] = a[p];
    __syncthreads();
    if (tid < 64) {
        const bool in = lane < N;
        const int pi = in ? pick[lane] : 0;
        double r[N];
#pragma unroll
        for (int j = 0; j < N; ++j) r[j] = (in && j <= lane) ? Lm[lane * N + j] : 0.0;   // row lane of L, D on the diagonal
        const double dmine = in ? Lm[lane * (N + 1)] : 0.0;
        double y = in ? b[pi] : 0.0;
#pragma unroll
        for (int k = 0; k + 1 < N; ++k) {
            const double yk = lane_f64(y, k);
            if (lane > k) y = __builtin_fma(-r[k], yk, y);
        }
        y = fabs(dmine) > 2.2250738585072014e-308 ? y / dmine : 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) r[j] = (in && j > lane) ? Lm[j * N + lane] : 0.0;   // r[j] = L_j,lane
#pragma unroll
        for (int j = N - 1; j >= 1; --j) {
            const double xj = lane_f64(y, j);
            if (lane < j) y = __builtin_fma(-r[j], xj, y);
        }
        if (in) x[pi] = y;
    }
    __syncthreads();
    return true;
}

// The same solve with the factorisation spread over the whole wavefront: the NP x NP padded matrix (NP = 16 or 32) is
// held P = 64 / NP lanes per row (lane = row + NP * s holds columns s, s + P, ...: R = NP / P registers), so a step's
// trailing update is R FMAs per lane instead of N.  Step k: the lanes holding column k publish it to LDS (one store),
// every lane reads its row's entry (the multiplier) and the entries of its own columns (the pivot row, by symmetry the
// pivot column) and updates; the triangular solves run row-per-lane from the factor staged in LDS.  Pick order, zero
// pivots, isPositive() and the D pseudo-inverse as ldlt_pick_solve.  cb: LDS scratch [NP].
template <int N>
__device__ __forceinline__ bool ldlt_pick_solve_wide(const double *H, const double *b, double *x, int *pick, double *Lm,
                                                     double *cb, int lane) {
    constexpr int NP = N <= 16 ? 16 : 32, P = 64 / NP, R = NP / P;
    static_assert(N <= 32, "at most 32 states");
    const bool in = lane < N;
    const double dv = in ? fabs(H[lane * (N + 1)]) : 0.0;
    int gt = 0, eq = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const double o = fabs(H[j * (N + 1)]);
        gt += o > dv ? 1 : 0;
        eq += o == dv ? 1 : 0;
    }
    if (__ballot(in && !(dv == dv))) return false;   // a NaN diagonal: no factorisation
    if (!__ballot(in && eq > 1)) {
        if (in) pick[gt] = lane;
    } else {   // selection with positional swaps, lanes = elements (pos = current position)
        int pos = lane;
        bool picked = false;
        for (int k = 0; k < N; ++k) {
            uint64_t cand = __ballot(in && !picked && gt <= k && k < gt + eq);
            int e = __builtin_ctzll(cand);
            if (cand & (cand - 1)) {   // several equal magnitudes: the lowest current position
                int bp = __builtin_amdgcn_readlane(pos, e);
                for (uint64_t m = cand & (cand - 1); m; m &= m - 1) {
                    const int c = __builtin_ctzll(m), pc = __builtin_amdgcn_readlane(pos, c);
                    if (pc < bp) bp = pc, e = c;
                }
            }
            const int xk = __builtin_ctzll(__ballot(in && pos == k));
            const int pe = __builtin_amdgcn_readlane(pos, e);
            if (lane == xk) pos = pe;
            if (lane == e) pos = k, picked = true;
            if (lane == 0) pick[k] = e;
        }
    }
    wave_lds_sync();
    const int row = lane & (NP - 1), sub = lane / NP;
    const bool rin = row < N;
    const int pr = rin ? pick[row] : 0;
    double r[R];
#pragma unroll
    for (int m = 0; m < R; ++m) {
        const int j = sub + P * m;
        r[m] = (rin && j < N) ? H[pr * N + pick[j < N ? j : 0]] : 0.0;
    }
    if (!(lane_f64(r[0], 0) != 0.0)) {   // largest |diagonal| zero: Eigen stops with ZeroSign; the solve gives x = 0
        if (in) x[lane] = 0.0;
        wave_lds_sync();
        return true;
    }
    int sign = 0;   // 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
    double dmine = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        constexpr int dummy = 0;
        (void)dummy;
        const int ck = k % P, mk = k / P;
        if (sub == ck) cb[row] = r[mk];   // column k (= row k) of the current matrix, rows >= N publish 0
        wave_lds_sync();
        const double d = cb[k];
        if (row == k) dmine = d;
        if (fabs(d) > 0.0) {
            const double inv = 1.0 / d;
            const double l = row > k ? cb[row] * inv : 0.0;
            const int m0 = (k + 1) / P;
#pragma unroll
            for (int m = m0; m < R; ++m) {
                const int j = sub + P * m;
                const double lj = (m == m0 && j <= k) ? 0.0 : l;   // the boundary register: columns <= k are L's
                r[m] = __builtin_fma(-lj, cb[j], r[m]);
            }
            if (sub == ck && row > k) r[mk] = l;
        }
        wave_lds_sync();   // cb is rewritten by the next step
        if (sign == 1) {
            if (d < 0) sign = 3;
        } else if (sign == 2) {
            if (d > 0) sign = 3;
        } else if (sign == 0) {
            if (d > 0) sign = 1;
            else if (d < 0) sign = 2;
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    if (rin)
#pragma unroll
        for (int m = 0; m < R; ++m) {
            const int j = sub + P * m;
            if (j < N) Lm[row * N + j] = r[m];
        }
    wave_lds_sync();
    // row-per-lane triangular solves (lane = position i < N)
    double Lr[N];
#pragma unroll
    for (int j = 0; j < N; ++j) Lr[j] = in ? Lm[lane * N + j] : 0.0;   // row i of L (j < i)
    const int pi = in ? pick[lane] : 0;
    double y = in ? b[pi] : 0.0;
#pragma unroll
    for (int k = 0; k + 1 < N; ++k) {
        const double yk = lane_f64(y, k);
        y = __builtin_fma(-(lane > k ? Lr[k] : 0.0), yk, y);
    }
    y = fabs(dmine) > 2.2250738585072014e-308 ? y / dmine : 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) Lr[j] = in ? Lm[j * N + lane] : 0.0;   // column i of L: L_j,i (j > i)
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        const double xj = lane_f64(y, j);
        y = __builtin_fma(-(lane < j ? Lr[j] : 0.0), xj, y);
    }
    if (in) x[pi] = y;
    wave_lds_sync();
    return true;
}

// EdgeInertial computeError + linearizeOplus (G2oTypes.cc:502-599) for LastFrame on one wavefront with uniform
// control flow: every lane evaluates the same values -- the error's rotation chain (delta_rot, LogSO3, the inverse right
// Jacobian and the products behind it) and the blocks that do not depend on it (the right Jacobian of the bias
// correction, the velocity / position blocks) are independent instruction streams the wave interleaves -- and single
// lanes store the blocks.  (Lane-role branches on one wavefront serialise: the previous form's nine roles added up to
// ~3.9 us per iteration.)  The arithmetic is imu_error's and imu_jacobian's, operation for operation.  J [9][24]
// (LDS) must be zeroed by the caller.
__device__ __forceinline__ void imu_error_jac_uniform(const State &s, const Imu &I, double *e9o, double *J, int lane) {
    const int k1 = I.kf1[0], k2 = I.kf2[0];
    const float *p = I.pre;
    const double *Rwb1 = s.Rwb + 9 * k1, *Rwb2 = s.Rwb + 9 * k2;
    auto put = [&](int r0, int c0, const double *B, double sgn) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) J[(r0 + r) * 24 + c0 + c] = sgn * B[3 * r + c];
    };
    double e[9], eR[9];
    imu_error(s, I, 0, e, eR);
    const double dt = (double)p[PreView::dT];
    const double g[3] = {0, 0, -(double)9.81f};
    double Rbw1[9];
    tr3(Rwb1, Rbw1);
    // the right Jacobian of the gyro-bias correction (independent of the error)
    double RJ[9], JRg[9];
    {
        float b1[6];
        for (int q = 0; q < 3; ++q) b1[q] = (float)s.ba[3 * k1 + q], b1[3 + q] = (float)s.bg[3 * k1 + q];
        const float dbgf[3] = {b1[3] - p[PreView::b + 3], b1[4] - p[PreView::b + 4], b1[5] - p[PreView::b + 5]};
        const double dbg[3] = {(double)dbgf[0], (double)dbgf[1], (double)dbgf[2]};
        double w3[3];
        for (int q = 0; q < 9; ++q) JRg[q] = p[PreView::JRg + q];
        mv3(JRg, dbg, w3);
        right_jac(w3, RJ);
    }
    {   // velocity / position rows (independent of the error)
        double v[3], w[3], W[9];
        for (int q = 0; q < 3; ++q) v[q] = s.vel[3 * k2 + q] - s.vel[3 * k1 + q] - g[q] * dt;
        mv3(Rbw1, v, w);
        hat3(w, W);
        if (lane == 2) put(3, 0, W, 1.0);
        for (int q = 0; q < 3; ++q)
            v[q] = s.twb[3 * k2 + q] - s.twb[3 * k1 + q] - s.vel[3 * k1 + q] * dt - 0.5 * g[q] * dt * dt;
        mv3(Rbw1, v, w);
        hat3(w, W);
        if (lane == 3) put(6, 0, W, 1.0);
        double A8[9];
        mm3(Rbw1, Rwb2, A8);
        if (lane == 8) put(6, 18, A8, 1.0);
    }
    if (lane == 4) {
        for (int q = 0; q < 3; ++q) J[(6 + q) * 24 + 3 + q] = -1.0;
        put(3, 6, Rbw1, -1.0);
        put(3, 21, Rbw1, 1.0);
    } else if (lane == 5) {
        put(6, 6, Rbw1, -dt);
    } else if (lane == 6) {
        double B[9];
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JVg + q];
        put(3, 9, B, -1.0);
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JVa + q];
        put(3, 12, B, -1.0);
    } else if (lane == 7) {
        double B[9];
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JPg + q];
        put(6, 9, B, -1.0);
        for (int q = 0; q < 9; ++q) B[q] = p[PreView::JPa + q];
        put(6, 12, B, -1.0);
    }
    // the rotation rows (on the error's chain)
    double invJr[9];
    inv_right_jac(e, invJr);
    {
        double R2t[9], A[9], B[9];
        tr3(Rwb2, R2t);
        mm3(invJr, R2t, A);
        mm3(A, Rwb1, B);
        if (lane == 0) {
            put(0, 0, B, -1.0);
            put(0, 15, invJr, 1.0);
        }
    }
    {
        double eRt[9], A[9], B[9], Jg[9];
        tr3(eR, eRt);
        mm3(invJr, eRt, A);
        mm3(A, RJ, B);
        mm3(B, JRg, Jg);
        if (lane == 1) put(0, 9, Jg, -1.0);
    }
    if (lane == 0)
        for (int q = 0; q < 9; ++q) e9o[q] = e[q];
    wave_lds_sync();
}

// Fixed-order sum of the edge waves' partials (wave 0 first).
__device__ __forceinline__ double wave_parts_sum(const double (*red)[kNormal], int q, int n) {
    double v = red[0][q];
    for (int w = 1; w < n; ++w) v += red[w][q];
    return v;
}

// LDS of the grouped kernel beyond its static arrays: the workgroup's visual edges (SoA) and the frame's mvbOutlier.
struct LatEdges {
    double *ob0, *ob1, *ob2, *c2;   // observation (u, v, u_R), e->chi2() of the last computeError
    float *x0, *x1, *x2, *w;        // MapPoint world position, invSigma2
    int32_t *kp;
    uint8_t *cam, *fl;              // camera; flags: 1 stereo, 2 bClose, 4 active (level 0)
    uint8_t *kpo;                   // [kp_cap] mvbOutlier of the keypoints this workgroup owns
};
__host__ __device__ inline size_t lat_lds_bytes(int kp_cap) {
    return (size_t)kLatCap * (4 * 8 + 4 * 4 + 4 + 2) + (((size_t)kp_cap + 15) / 16) * 16;
}
__device__ __forceinline__ LatEdges lat_carve(char *base) {
    LatEdges E;
    E.ob0 = (double *)base, E.ob1 = E.ob0 + kLatCap, E.ob2 = E.ob1 + kLatCap, E.c2 = E.ob2 + kLatCap;
    E.x0 = (float *)(E.c2 + kLatCap), E.x1 = E.x0 + kLatCap, E.x2 = E.x1 + kLatCap, E.w = E.x2 + kLatCap;
    E.kp = (int32_t *)(E.w + kLatCap);
    E.cam = (uint8_t *)(E.kp + kLatCap), E.fl = E.cam + kLatCap, E.kpo = E.fl + kLatCap;
    return E;
}
__device__ __forceinline__ VEdge lat_edge(const LatEdges &E, int q) {
    VEdge v;
    v.cam = E.cam[q], v.kp = E.kp[q], v.stereo = (E.fl[q] & 1) != 0;
    v.obs[0] = E.ob0[q], v.obs[1] = E.ob1[q], v.obs[2] = v.stereo ? E.ob2[q] : 0.0;
    v.w = (double)E.w[q];
    v.X[0] = (double)E.x0[q], v.X[1] = (double)E.x1[q], v.X[2] = (double)E.x2[q];
    return v;
}

// Workgroup-ordered compaction of this part's edges (keypoint in [lo, hi)): the mono list's, then the stereo list's,
// each in list order, into the LDS edge arrays; *nm_loc / *n_loc = mono / all edges taken.  Two phases: every thread
// takes kSel consecutive keypoint indices per chunk (all loads in flight), a workgroup prefix sum of the taken counts
// places them, and the taken edges' source indices are staged in LDS (the chi2 array, unused until the iterations);
// then one thread per taken edge loads its record.  (A chunk of kLatThreads edges per workgroup step was ~19 dependent
// global round trips per frame of ~5,800 edges: most of the call's setup.)  False (uniformly) past kLatCap.
constexpr int kSel = 16;
__device__ bool lat_select(const PoseArgs &A, int m0, int nm, int s0, int ns, int lo, int hi, const LatEdges &E,
                           int *wcnt, int *nm_loc, int *n_loc) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = kLatThreads / 64;
    int *src = reinterpret_cast<int *>(E.c2);   // [kLatCap] (list << 31) | edge
    int total = 0;
    for (int list = 0; list < 2; ++list) {
        const bool stereo = list == 1;
        const int e0 = stereo ? s0 : m0, n = stereo ? ns : nm;
        const int32_t *K = (stereo ? A.s_kp : A.m_kp) + e0;
        for (int base = 0; base < n; base += kLatThreads * kSel) {
            const int q0 = base + tid * kSel;
            int kv[kSel];
#pragma unroll
            for (int u = 0; u < kSel; ++u) kv[u] = q0 + u < n ? K[q0 + u] : 0;
            uint32_t take = 0;   // (part 0's lo is INT_MIN: the bound alone does not exclude the padding)
#pragma unroll
            for (int u = 0; u < kSel; ++u) take |= (q0 + u < n && kv[u] >= lo && kv[u] < hi ? 1u : 0u) << u;
            const int cnt = __builtin_popcount(take);
            int incl = cnt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int t = __shfl_up(incl, d, 64);
                if (lane >= d) incl += t;
            }
            if (lane == 63) wcnt[wave] = incl;
            __syncthreads();
            int off = total + incl - cnt, tot = 0;
#pragma unroll
            for (int w2 = 0; w2 < kW; ++w2) {
                off += w2 < wave ? wcnt[w2] : 0;
                tot += wcnt[w2];
            }
            if (total + tot > kLatCap) return false;
            for (uint32_t b = take; b; b &= b - 1) {
                const int u = __builtin_ctz(b);
                src[off++] = (stereo ? (int)0x80000000 : 0) | (e0 + q0 + u);
            }
            total += tot;
            __syncthreads();   // wcnt is reused
        }
        if (!stereo) *nm_loc = total;
    }
    *n_loc = total;
    for (int d = tid; d < total; d += kLatThreads) {
        const int sv = src[d];
        const bool stereo = sv < 0;
        const int e = sv & 0x7fffffff;
        const int kp = stereo ? A.s_kp[e] : A.m_kp[e];
        E.kp[d] = kp;
        if (!stereo) {
            E.cam[d] = (uint8_t)A.m_cam[e];
            E.ob0[d] = A.m_obs[2 * e], E.ob1[d] = A.m_obs[2 * e + 1], E.ob2[d] = 0.0;
            E.w[d] = A.m_w[e];
            E.x0[d] = A.m_xw[3 * e], E.x1[d] = A.m_xw[3 * e + 1], E.x2[d] = A.m_xw[3 * e + 2];
            E.fl[d] = (uint8_t)(4 | (A.m_close[e] ? 2 : 0));
        } else {
            E.cam[d] = (uint8_t)A.s_cam[e];
            E.ob0[d] = A.s_obs[3 * e], E.ob1[d] = A.s_obs[3 * e + 1], E.ob2[d] = A.s_obs[3 * e + 2];
            E.w[d] = A.s_w[e];
            E.x0[d] = A.s_xw[3 * e], E.x1[d] = A.s_xw[3 * e + 1], E.x2[d] = A.s_xw[3 * e + 2];
            E.fl[d] = 4 | 1;
        }
        E.kpo[kp] = 0;
    }
    __syncthreads();
    return true;
}

// Keypoint-range boundary p of G: the mono list's (else the stereo list's) keypoint at its p/G quantile, made monotone
// over p (the reference creates edges in keypoint order, so the parts balance; any order partitions correctly).
// The keypoint threshold of part boundary p: the keypoint of element d = ne p / G of the frame's mono and stereo
// edges merged in keypoint order (both lists ascend by keypoint; a keypoint's edges go to one part), so every part
// holds ne / G edges up to one keypoint's two.  Merge path by a 64-ary search on one wavefront: lane k tests the
// k-th of 64 candidate mono counts i (B(i): the d - i stereo edges before the split all precede mono edge i), the
// first true lane narrows the range; three rounds for 262,144 edges.  All lanes return the same value.
__device__ int lat_bound_wave(const PoseArgs &A, int p, int G, int m0, int nm, int s0, int ns, int lane) {
    if (p <= 0) return INT_MIN;
    if (p >= G) return INT_MAX;
    const int ne = nm + ns;
    if (ne == 0) return INT_MIN;
    const int d = (int)((int64_t)ne * p / G);
    const int32_t *M = A.m_kp + m0, *S = A.s_kp + s0;
    int lo = max(0, d - ns), hi = min(d, nm);   // the mono count of the first d merged edges lies in [lo, hi]
    while (hi > lo) {
        const int i = lo + (int)(((int64_t)(hi - lo) * lane) / 63);   // lane 63 tests hi
        const int j = d - i;
        const bool b = j == 0 || i == nm || S[j - 1] < M[i];
        const uint64_t bal = __ballot(b);
        const int k = __builtin_ctzll(bal | (1ull << 63));
        const int ik = __shfl(i, k, 64), ik1 = k > 0 ? __shfl(i, k - 1, 64) : lo - 1;
        hi = ik, lo = ik1 + 1;
    }
    const int i = lo, j = d - i;
    if (i < nm && (j >= ns || M[i] <= S[j])) return M[i];
    return j < ns ? S[j] : INT_MAX;
}

template <bool kLF>
__global__ void __launch_bounds__(kLatThreads) pose_lat_kernel(Rig rig_in, PoseArgs A, int G, gu64 *xbuf, uint32_t salt,
                                                              int32_t *err_word) {
    constexpr int N = kLF ? 30 : 15;
    constexpr int NR = kLF ? 24 : 9;   // the system without the frame's bias vertices (see the assembly)
    // reduced index -> state index: the frame's pose + velocity (0-8), then (LastFrame) the previous frame's 15-29
    auto red_full = [](int r) __attribute__((always_inline)) { return r < 9 ? r : r + 6; };
    constexpr int NJ = kLF ? 216 : 81;   // EdgeInertial Jacobian entries kept: 9 x 24 (LastFrame), 9 x 9 (columns 15-23)
    constexpr int NI = kLF ? 24 : 9;
    constexpr int NP = kLF ? 225 : 1;
    // waves: 0 .. kEW-1 visual edges (one per thread), kIW EdgeInertial, kPW EdgePriorPoseImu (LastFrame)
    constexpr int kEW = kLF ? 2 : 3, kIW = kEW, kPW = 3, kET = 64 * kEW;
    const int f = blockIdx.x / G, g = blockIdx.x - f * G, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    gu64 *fb = xbuf + (size_t)f * kLatFrameGran;
    extern __shared__ __attribute__((aligned(16))) char lat_dyn[];
    const LatEdges E = lat_carve(lat_dyn);
    __shared__ Rig rig;
    __shared__ double sRwb[18], stwb[6], svel[6], sbg[6], sba[6];
    __shared__ double sRcw[kMaxCams * 9], stcw[kMaxCams * 3];
    __shared__ double red[3][kNormal], nrm[32];
    __shared__ double Hs[N * N], bs[N], xs[N], xt[N], Lm[N * N], ism[kLF ? 1 : 258];
    __shared__ double info9[81], infoG[9], infoA[9];
    __shared__ double J[NJ], WJ[NJ], e9[9], om9[9], bI[NI], s_w1p;
    __shared__ double cA1[9], cdV[3], cdP[3];
    __shared__ double sPr[kLF ? 21 : 1], pH[NP], JPr[NP], PJ[NP], eP[kLF ? 15 : 1], OeP[kLF ? 15 : 1],
        bP[kLF ? 15 : 1];
    __shared__ double Am[NP], Vm[NP], ecs[16];
    __shared__ int epq[16];
    __shared__ int s_ok, s_abort, wcnt[kLatThreads / 64], pick[N], s_lohi[2];
    __shared__ int k1s, k2s;
    __shared__ double s_cnt[2];
    __shared__ float spre[kPF];   // the frame's IMU::Preintegrated record (read every iteration: kept out of HBM)
    const int C = rig_in.n_cams;
#ifdef OMV_POSE_PROFILE
    unsigned long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __shared__ unsigned long long prof_inert, t2s[48], prof_iw[4];
    if (tid == 0) prof_inert = 0;
    if (tid < 4) prof_iw[tid] = 0;
    if (tid < 48) t2s[tid] = 0;
    LAT_T(t_start);
#endif
    for (int q = tid; q < (int)(sizeof(Rig) / 4); q += kLatThreads)
        reinterpret_cast<uint32_t *>(&rig)[q] = reinterpret_cast<const uint32_t *>(&rig_in)[q];
    if (tid == 0) {
        for (int q = 0; q < 9; ++q) sRwb[q] = A.kRwb[9 * f + q], sRwb[9 + q] = A.Rwb[9 * f + q];
        for (int q = 0; q < 3; ++q) {
            stwb[q] = A.ktwb[3 * f + q], stwb[3 + q] = A.twb[3 * f + q];
            svel[q] = A.kvel[3 * f + q], svel[3 + q] = A.vel[3 * f + q];
            sbg[q] = A.kbg[3 * f + q], sbg[3 + q] = A.bg[3 * f + q];
            sba[q] = A.kba[3 * f + q], sba[3 + q] = A.ba[3 * f + q];
        }
        k1s = 0, k2s = 1;
        s_abort = 0;
    }
    if constexpr (kLF) {
        for (int q = tid; q < 225; q += kLatThreads) pH[q] = A.pH[(size_t)f * 225 + q];
        if (tid < 21) {
            double v;
            if (tid < 9) v = A.pRwb[9 * f + tid];
            else if (tid < 12) v = A.ptwb[3 * f + tid - 9];
            else if (tid < 15) v = A.pvel[3 * f + tid - 12];
            else if (tid < 18) v = A.pbg[3 * f + tid - 15];
            else v = A.pba[3 * f + tid - 18];
            sPr[tid] = v;
        }
    }
    for (int q = tid; q < C * 9; q += kLatThreads) sRcw[q] = A.Rcw[(size_t)f * C * 9 + q];
    for (int q = tid; q < C * 3; q += kLatThreads) stcw[q] = A.tcw[(size_t)f * C * 3 + q];
    for (int q = tid; q < N; q += kLatThreads) xs[q] = 0.0;
    for (int q = tid; q < NJ; q += kLatThreads) J[q] = 0.0;
    for (int q = tid; q < kPF; q += kLatThreads) spre[q] = A.preint[(size_t)f * kPF + q];
    const int m0 = A.m_start[f], nm = A.m_start[f + 1] - m0;
    const int s0 = A.s_start[f], ns = A.s_start[f + 1] - s0;
    const int ne = nm + ns;
    if (wave == 0) {
        const int b0 = lat_bound_wave(A, g, G, m0, nm, s0, ns, lane), b1 = lat_bound_wave(A, g + 1, G, m0, nm, s0, ns, lane);
        if (lane == 0) s_lohi[0] = b0, s_lohi[1] = b1;
    }
    __syncthreads();
    const int lo = s_lohi[0], hi = s_lohi[1];
    int nm_loc = 0, nloc = 0;
    const bool fit = lat_select(A, m0, nm, s0, ns, lo, hi, E, wcnt, &nm_loc, &nloc);
    int phase = 1;
    // setup exchange: every part learns whether some part overflowed its LDS edge capacity
    if (wave == 0) {
        if (!lat_exchange(fb, phase, salt, g, G, fit ? 0.0 : 1.0, 1, s_cnt, lane)) s_abort = 1;
        else if (lane == 0 && s_cnt[0] != 0.0) s_abort = 2;
    } else if (wave == kIW) {
        // the edges' information matrices (pose_info_kernel's work, here beside the setup exchange: no extra launch)
        inertial_info9_wave<true>(spre + PreView::C, info9, kLF ? Lm : ism, lane);   // 258 doubles of scratch
        if (lane == 0) {
            const float *prw = A.preint_rw + (size_t)f * kPF;
            double gq[9], aq[9];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    gq[3 * r + c] = prw[PreView::C + (9 + r) * 15 + 9 + c], aq[3 * r + c] = prw[PreView::C + (12 + r) * 15 + 12 + c];
            inv3(gq, infoG);
            inv3(aq, infoA);
        }
    }
    State st{sRwb, stwb, nullptr, nullptr, svel, sbg, sba, nullptr};
    Imu imu{};
    imu.n = 1, imu.kf1 = &k1s, imu.kf2 = &k2s, imu.pre = spre;
    // LastKeyFrame: the keyframe's vertices are fixed, so IMU::Preintegrated's bias-corrected deltas and dR^T Rbw1
    // are constants of the call (imu_error computes them the same way at every iteration)
    if (!kLF && wave == kIW && lane == 0) {
        const float *p = imu.pre;
        float b1[6];
        for (int q = 0; q < 3; ++q) b1[q] = (float)sba[q], b1[3 + q] = (float)sbg[q];
        double dR[9], dRt[9], R1t[9];
        delta_rot(p, b1, dR);
        delta_vp(p, PreView::dV, PreView::JVg, PreView::JVa, b1, cdV);
        delta_vp(p, PreView::dP, PreView::JPg, PreView::JPa, b1, cdP);
        tr3(sRwb, R1t);
        tr3(dR, dRt);
        mm3(dRt, R1t, cA1);
        for (int r = 0; r < 3; ++r)   // EdgeInertial d(e_v)/d(v2) = Rbw1, constant here
            for (int c = 0; c < 3; ++c) J[(3 + r) * 9 + 6 + c] = R1t[3 * r + c];
    }
    // EdgeInertial's Jacobian / error at the current state on wave 4 (J, e9, WJ = Info J; with `sys` also om9 and
    // bI = J^T om9), the arithmetic of imu_error + imu_jacobian / imu_error_jac_p2v2.  `part` 1: the error and the
    // Jacobian only, 2: the products with the information only (LastFrame's iterations run them beside the visual edges
    // and beside the exchange respectively: the wave's two halves each fit under the other waves' work), 3: both.
    auto inertial_wave = [&](bool sys, int part) __attribute__((always_inline)) {
        if (part & 1) {
        if constexpr (!kLF) {
            const double *R1 = sRwb, *R2 = sRwb + 9;
            const double dt = (double)imu.pre[PreView::dT];
            const double gz[3] = {0, 0, -(double)9.81f};
            if (lane == 0) {   // LogSO3(dR^T Rbw1 Rwb2), InverseRightJacobianSO3 of it
                double B[9], er[3], iJ[9];
                mm3(cA1, R2, B);
                log_so3(B, er);
                for (int q = 0; q < 3; ++q) e9[q] = er[q];
                inv_right_jac(er, iJ);
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) J[r * 9 + c] = iJ[3 * r + c];
            } else if (lane == 1) {
                double t[3], ev[3];
                for (int q = 0; q < 3; ++q) t[q] = svel[3 + q] - svel[q] - gz[q] * dt;
                mtv3(R1, t, ev);
                for (int q = 0; q < 3; ++q) e9[3 + q] = ev[q] - cdV[q];
            } else if (lane == 2) {
                double t[3], ev[3];
                for (int q = 0; q < 3; ++q) t[q] = stwb[3 + q] - stwb[q] - svel[q] * dt - gz[q] * dt * dt / 2;
                mtv3(R1, t, ev);
                for (int q = 0; q < 3; ++q) e9[6 + q] = ev[q] - cdP[q];
            } else if (lane == 3) {   // Rbw1 Rwb2
                double R1t[9], Aq[9];
                tr3(R1, R1t);
                mm3(R1t, R2, Aq);
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) J[(6 + r) * 9 + 3 + c] = Aq[3 * r + c];
            }
        } else {
#ifdef OMV_POSE_PROFILE
            LAT_T(ti0);
#endif
            for (int q = lane; q < 216; q += 64) J[q] = 0.0;
            wave_lds_sync();
#ifdef OMV_POSE_PROFILE
            LAT_T(ti1);
            if (lane == 0) prof_iw[0] += ti1 - ti0;
#endif
            imu_error_jac_uniform(st, imu, e9, J, lane);
#ifdef OMV_POSE_PROFILE
            LAT_T(ti2);
            if (lane == 0) prof_iw[1] += ti2 - ti1;
#endif
        }
        wave_lds_sync();
        }
        if (!(part & 2)) return;
#ifdef OMV_POSE_PROFILE
        LAT_T(ti3);
#endif
        for (int q = lane; q < NJ + 9; q += 64) {
            if (q < NJ) {
                const int r = q / NI, c = q - (q / NI) * NI;
                double t = 0;
                for (int k = 0; k < 9; ++k) t += info9[r * 9 + k] * J[k * NI + c];
                WJ[q] = t;
            } else if (sys) {
                const int r = q - NJ;
                double t = 0;
                for (int k = 0; k < 9; ++k) t += info9[r * 9 + k] * e9[k];
                om9[r] = -t;
            }
        }
#ifdef OMV_POSE_PROFILE
        LAT_T(ti4);
        if (kLF && lane == 0) prof_iw[2] += ti4 - ti3;
#endif
        if (!sys) return;
        wave_lds_sync();
        // bI = J^T om9 here; the quadratic form J^T Info J is summed entry by entry where the system is assembled
        // (all waves), off this wave's path
        if (lane < NI) {
            double u = 0;
            for (int k = 0; k < 9; ++k) u += J[k * NI + lane] * om9[k];
            bI[lane] = u;
        }
    };
    // EdgePriorPoseImu (LastFrame) on wave 5: eP, JPr, PJ = H_prior JPr; with `sys` OeP, the Huber weight w (s_w1p)
    // and bP = -JPr^T w H_prior eP
    auto prior_wave = [&](bool sys) __attribute__((always_inline)) {
        if constexpr (kLF) {
            if (lane == 0) prior_error_jac(sPr, sRwb, stwb, svel, sbg, sba, eP, JPr);
            wave_lds_sync();
            for (int q = lane; q < 240; q += 64) {
                if (q < 225) {
                    const int k = q / 15, j = q % 15;
                    double t = 0;
                    for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * JPr[l * 15 + j];
                    PJ[q] = t;
                } else if (sys) {
                    const int k = q - 225;
                    double t = 0;
                    for (int l = 0; l < 15; ++l) t += pH[k * 15 + l] * eP[l];
                    OeP[k] = t;
                }
            }
            if (!sys) return;
            wave_lds_sync();
            double chi2p = 0, r0, w1p;
            for (int k = 0; k < 15; ++k) chi2p += eP[k] * OeP[k];
            huber(chi2p, 5.0, 25.0, r0, w1p);
            if (lane == 0) s_w1p = w1p;   // JPr^T w PJ is summed where the system is assembled
            if (lane < 15) {
                double u = 0;
                for (int k = 0; k < 15; ++k) u += JPr[k * 15 + lane] * (-OeP[k] * w1p);
                bP[lane] = u;
            }
        }
    };
    __syncthreads();
    if (s_abort) goto fail;
    {
        const double dmono = (double)(float)sqrt(5.991), dst = (double)(float)sqrt(7.815);
        const float chi2Mono[4] = {kLF ? 5.991f : 12.f, kLF ? 5.991f : 7.5f, 5.991f, 5.991f};   // :5992 / :5432
        const float chi2Stereo[4] = {15.6f, 9.8f, 7.815f, 7.815f};
        double nBad = 0, nIn = 0;
        // ImuCamPose::its of the pose vertex this lane updates (lane 0 the frame, lane 1 the previous frame): 0 at the
        // vertex's creation (G2oTypes.cc:74), Rwb normalised after every third Update (:220-225)
        int its_v = 0;
#ifdef OMV_POSE_PROFILE
        unsigned long long t_cls = 0;   // classification passes + their exchanges
        LAT_T(t_loop0);
#endif
        for (int it = 0; it < 4; ++it) {
            const bool robust = it < 3;   // setRobustKernel(0) after the third classification
            for (int gi = 0; gi < 10; ++gi) {
                ++phase;
                // LDS is re-read every iteration: a compiler barrier keeps the loop-invariant LDS reads (information
                // matrices, the prior, the rig) from being hoisted into registers across the whole loop, whose
                // live ranges spanned every wave role's code and spilled
                asm volatile("" ::: "memory");
                LAT_T(t0);
                if (wave < kEW) {   // computeActiveErrors + the visual part of buildSystem
                    double acc[kNormal];
#pragma unroll
                    for (int q = 0; q < kNormal; ++q) acc[q] = 0;
                    for (int q = tid; q < nloc; q += kET) {
                        if (!(E.fl[q] & 4)) continue;
                        const VEdge v = lat_edge(E, q);
                        double r[3], Xc[3], JP[18];
                        const double c2 = edge_error_jac(rig, sRcw, stcw, v, r, Xc, JP);
                        E.c2[q] = c2;
                        double w1 = 1.0;
                        if (robust) {
                            double r0;
                            if (v.stereo) huber(c2, dst, dst * dst, r0, w1);
                            else huber(c2, dmono, dmono * dmono, r0, w1);
                        }
                        const double om[3] = {-v.w * r[0] * w1, -v.w * r[1] * w1, v.stereo ? -v.w * r[2] * w1 : 0.0};
                        edge_normal(JP, v.stereo, v.w * w1, om, acc);
                    }
                    LAT_T(t0e);
                    LAT_ACC(0, t0, t0e);
                    const double mine = wave_transpose_sum(acc, lane);
                    if (lane < kNormal) red[wave][lane] = mine;
                    LAT_T(t0r);
                    LAT_ACC(1, t0e, t0r);
                } else if (wave == kIW) {   // EdgeInertial at the iteration's state
                    inertial_wave(true, kLF ? 1 : 3);
#ifdef OMV_POSE_PROFILE
                    LAT_T(t0i);
                    if (lane == 0) prof_inert += t0i - t0;
#endif
                } else if (kLF && wave == kPW) {   // EdgePriorPoseImu on the previous frame (vertex 0)
                    prior_wave(true);
                }
                __syncthreads();
                LAT_T(t1);
#ifdef OMV_POSE_PROFILE
                if (tid == 0 && f == 0 && it * 10 + gi < 48) {
                    __hip_atomic_store(&g_lat_pub[g][it * 10 + gi], t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (g == 0) t2s[it * 10 + gi] = 0;
                }
#endif
                if (wave == 0) {
                    const double v = lane < kNormal ? wave_parts_sum(red, lane, kEW) : 0.0;
                    if (!lat_exchange(fb, phase, salt, g, G, v, kNormal, nrm, lane) && lane == 0) s_abort = 1;
                } else if (kLF && wave == kIW) {   // EdgeInertial's products with its information, beside the exchange
                    inertial_wave(true, 2);
                }
                __syncthreads();
                LAT_T(t2);
#ifdef OMV_POSE_PROFILE
                if (tid == 0 && f == 0 && g == 0 && it * 10 + gi < 48) t2s[it * 10 + gi] = t2;
#endif
                LAT_ACC(2, t0, t1);
                LAT_ACC(3, t1, t2);
                if (s_abort) goto fail;
                // The system without the frame's bias vertices.  Their only edges are EdgeGyroRW / EdgeAccRW (e = b_frame -
                // b_other, J = +-I, information InfoG / InfoA), so eliminating them is exact: the Schur complement drops the
                // random walks' terms from the other vertex's block and right-hand side, and the eliminated update is
                // x_b = x_other - e (LastFrame: the previous frame's bias update; LastKeyFrame, keyframe fixed: -e).  The
                // reduced system (LastKeyFrame: pose + velocity, 9; LastFrame: the frame's pose + velocity and all 15 of the
                // previous frame's, 24) is positive (semi)definite iff the full one is (InfoG / InfoA are positive
                // definite), so isPositive() and the update agree with the full solve up to rounding.
                for (int q = tid; q < NR * (NR + 1) / 2; q += kLatThreads) {   // the lower triangle, q = i (i + 1) / 2 + j
                    int i = (int)((sqrtf(8.f * (float)q + 1.f) - 1.f) * 0.5f);
                    i += (i + 1) * (i + 2) / 2 <= q ? 1 : 0;
                    i -= i * (i + 1) / 2 > q ? 1 : 0;
                    const int j = q - i * (i + 1) / 2;
                    const int fi = red_full(i), fj = red_full(j);
                    double h = 0;
                    if (fi < 6) h = nrm[fj * 6 - fj * (fj - 1) / 2 + (fi - fj)];
                    if constexpr (kLF) {
                        const int ci = ei_col(fi), cj = ei_col(fj);
                        if (ci >= 0 && cj >= 0) {   // (J^T Info J)_ci,cj
                            double t = 0;
                            for (int k = 0; k < 9; ++k) t += J[k * 24 + ci] * WJ[k * 24 + cj];
                            h += t;
                        }
                        if (fi >= 15 && fj >= 15) {   // (JPr^T w H_prior JPr)_i,j
                            const double w1p = s_w1p;
                            double t = 0;
                            for (int k = 0; k < 15; ++k) t += JPr[k * 15 + fi - 15] * (w1p * PJ[k * 15 + fj - 15]);
                            h += t;
                        }
                    } else {
                        double t = 0;
                        for (int k = 0; k < 9; ++k) t += J[k * 9 + fi] * WJ[k * 9 + fj];
                        h += t;
                    }
                    Hs[i * NR + j] = h;
                    Hs[j * NR + i] = h;
                }
                if (tid < NR) {
                    const int fi = red_full(tid);
                    double t = fi < 6 ? nrm[21 + fi] : 0.0;
                    if constexpr (kLF) {
                        const int ci = ei_col(fi);
                        if (ci >= 0) t += bI[ci];
                        if (fi >= 15) t += bP[fi - 15];
                    } else {
                        t += bI[fi];
                    }
                    bs[tid] = t;
                }
                __syncthreads();
                LAT_T(t3);
                LAT_ACC(4, t2, t3);
                if (wave == 0) {
                    const bool ok = ldlt_pick_solve<NR>(Hs, bs, xt, pick, Lm, lane);
                    LAT_T(t3l);
                    LAT_ACC(5, t3, t3l);
                    if (ok) {   // a failed solve leaves the previous x in place
                        if (lane < NR) xs[red_full(lane)] = xt[lane];
                        if (lane < 3) {   // the eliminated bias updates
                            const double xg = kLF ? xt[18 + lane] : 0.0, xa = kLF ? xt[21 + lane] : 0.0;
                            xs[9 + lane] = xg - (sbg[3 + lane] - sbg[lane]);
                            xs[12 + lane] = xa - (sba[3 + lane] - sba[lane]);
                        }
                    }
                    if (lane == 0) s_ok = ok ? 1 : 0;
                    wave_lds_sync();
                    // VertexPose::oplusImpl -> ImuCamPose::Update (G2oTypes.cc:211-235): lane 0 the frame, lane 1 the
                    // previous frame (LastFrame); then lane c the frame's camera c
                    if (lane == 0 || (kLF && lane == 1)) {
                        const int v = lane == 0 ? 1 : 0;
                        const double *xv = xs + (lane == 0 ? 0 : 15);
                        double *Rw = sRwb + 9 * v, *tw = stwb + 3 * v;
                        double t[3], dR[9], Rn[9];
                        mv3(Rw, xv + 3, t);
                        for (int q = 0; q < 3; ++q) tw[q] += t[q];
                        exp_so3(xv, dR);
                        mm3(Rw, dR, Rn);
                        if (++its_v >= 3) polar3(Rn), its_v = 0;   // NormalizeRotation after every third update
                        for (int q = 0; q < 9; ++q) Rw[q] = Rn[q];
                        for (int q = 0; q < 3; ++q)
                            svel[3 * v + q] += xv[6 + q], sbg[3 * v + q] += xv[9 + q], sba[3 * v + q] += xv[12 + q];
                    }
                    wave_lds_sync();
                    if (lane < C) {
                        const int c = lane;
                        double Rbw[9], tbw[3], Rc[9], tc[3];
                        tr3(sRwb + 9, Rbw);
                        mv3(Rbw, stwb + 3, tbw);
                        for (int q = 0; q < 3; ++q) tbw[q] = -tbw[q];
                        mm3(rig.Rcb[c], Rbw, Rc);
                        mv3(rig.Rcb[c], tbw, tc);
                        for (int q = 0; q < 9; ++q) sRcw[9 * c + q] = Rc[q];
                        for (int q = 0; q < 3; ++q) stcw[3 * c + q] = tc[q] + rig.tcb[c][q];
                    }
                }
                __syncthreads();
                LAT_T(t4);
                LAT_ACC(6, t3, t4);
                if (!s_ok) break;   // optimize() stops after a failed iteration
            }
            // classification (:5436-5490): the mono pass, then the stereo pass; counts summed over the parts
#ifdef OMV_POSE_PROFILE
            LAT_T(t_c0);
#endif
            double bad = 0, in = 0;
            const float chi2close = 1.5f * chi2Mono[it];
            for (int pass = 0; pass < 2; ++pass) {
                if (wave < kEW)
                    for (int q = (pass ? nm_loc : 0) + tid; q < (pass ? nloc : nm_loc); q += kET) {
                        const VEdge v = lat_edge(E, q);
                        double Xc[3];
                        if (E.kpo[v.kp]) {   // outliers of the last round: computeError at the current state
                            double r[3];
                            E.c2[q] = edge_error(rig, sRcw, stcw, v, r, Xc);
                        }
                        const float chi2 = (float)E.c2[q];
                        bool out;
                        if (!v.stereo) {
                            const bool close = (E.fl[q] & 2) != 0;
                            const double *R = sRcw + 9 * v.cam;
                            const bool depth_pos =
                                (R[6] * v.X[0] + R[7] * v.X[1] + R[8] * v.X[2] + stcw[3 * v.cam + 2]) > 0.0;
                            out = (chi2 > chi2Mono[it] && !close) || (close && chi2 > chi2close) || !depth_pos;
                        } else {
                            out = chi2 > chi2Stereo[it];
                        }
                        E.kpo[v.kp] = out ? 1 : 0;
                        E.fl[q] = (uint8_t)((E.fl[q] & 3) | (out ? 0 : 4));
                        bad += out ? 1 : 0;
                        in += out ? 0 : 1;
                    }
                __syncthreads();
            }
            {
                double cnt2[2] = {bad, in};
                const double sb = wave < kEW ? wave_transpose_sum(cnt2, lane) : 0.0;
                if (wave < kEW && lane < 2) red[wave][lane] = sb;
                __syncthreads();
                ++phase;
                if (wave == 0) {
                    const double v = lane < 2 ? wave_parts_sum(red, lane, kEW) : 0.0;
                    if (!lat_exchange(fb, phase, salt, g, G, v, 2, s_cnt, lane) && lane == 0) s_abort = 1;
                }
                __syncthreads();
                if (s_abort) goto fail;
                nBad = s_cnt[0], nIn = s_cnt[1];
            }
#ifdef OMV_POSE_PROFILE
            {
                LAT_T(t_c1);
                t_cls += t_c1 - t_c0;
            }
#endif
            if (ne + (kLF ? 4 : 3) < 10) break;   // optimizer.edges().size() < 10
        }
#ifdef OMV_POSE_PROFILE
        LAT_T(t_loop1);
#endif
        if (nIn < 30 && !A.rec_init) {   // recover not too bad points (:5503-5526)
            double bad = 0;
            if (wave < kEW)
                for (int q = tid; q < nloc; q += kET) {
                    const VEdge v = lat_edge(E, q);
                    double r[3], Xc[3];
                    const double c2 = edge_error(rig, sRcw, stcw, v, r, Xc);
                    E.c2[q] = c2;
                    if (c2 < (v.stereo ? 24.f : 18.f)) E.kpo[v.kp] = 0;
                    else bad += 1;
                }
            double cnt1[1] = {bad};
            const double sb = wave < kEW ? wave_transpose_sum(cnt1, lane) : 0.0;
            if (wave < kEW && lane == 0) red[wave][0] = sb;
            __syncthreads();
            ++phase;
            if (wave == 0) {
                const double v = lane < 1 ? wave_parts_sum(red, 0, kEW) : 0.0;
                if (!lat_exchange(fb, phase, salt, g, G, v, 1, s_cnt, lane) && lane == 0) s_abort = 1;
            }
            __syncthreads();
            if (s_abort) goto fail;
            nBad = s_cnt[0];
        }
#ifdef OMV_POSE_PROFILE
        LAT_T(t_rec);
#endif
        // mvbOutlier of this part's keypoints
        if (wave < kEW)
            for (int q = tid; q < nloc; q += kET) A.kp_out[(size_t)f * A.kp_cap + E.kp[q]] = E.kpo[E.kp[q]];
#ifdef OMV_POSE_PROFILE
        LAT_T(t_h0);
#endif
        if (A.H) {
            // the Hessian without robust weights at the final state (inlier visual edges): visual sums exchanged,
            // EdgeInertial / EdgePriorPoseImu linearised by waves 4 / 5, the matrix formed by part 0
            if (wave < kEW) {
                double acc[kNormal];
#pragma unroll
                for (int q = 0; q < kNormal; ++q) acc[q] = 0;
                for (int q = tid; q < nloc; q += kET) {
                    const VEdge v = lat_edge(E, q);
                    if (E.kpo[v.kp]) continue;
                    double r[3], Xc[3], JP[18];
                    edge_error(rig, sRcw, stcw, v, r, Xc);
                    edge_jac(rig, v, Xc, JP);
                    const double om[3] = {0, 0, 0};
                    edge_normal(JP, v.stereo, v.w, om, acc);
                }
                const double mine = wave_transpose_sum(acc, lane);
                if (lane < kNormal) red[wave][lane] = mine;
            } else if (wave == kIW) {
                inertial_wave(false, 3);
            } else if (kLF && wave == kPW) {
                prior_wave(false);
            }
            __syncthreads();
            ++phase;
            if (wave == 0) {
                const double v = lane < kNormal ? wave_parts_sum(red, lane, kEW) : 0.0;
                if (!lat_exchange(fb, phase, salt, g, G, v, kNormal, nrm, lane) && lane == 0) s_abort = 1;
            }
            __syncthreads();
            if (s_abort) goto fail;
            if (g == 0) {
                if constexpr (kLF) {
                    for (int q = tid; q < N * N; q += kLatThreads) {   // the reference's order: ei, egr, ear, ep, visual
                        const int i = q / N, j = q % N;
                        double h = 0;
                        const int ci = ei_col(i), cj = ei_col(j);
                        if (ci >= 0 && cj >= 0) {
                            double t = 0;
                            for (int k = 0; k < 9; ++k) t += J[k * 24 + ci] * WJ[k * 24 + cj];
                            h += t;
                        }
                        h += rw_entry(i, j, false, infoG);
                        h += rw_entry(i, j, true, infoA);
                        if (i >= 15 && j >= 15) {
                            double t = 0;
                            for (int k = 0; k < 15; ++k) t += JPr[k * 15 + i - 15] * PJ[k * 15 + j - 15];
                            h += t;
                        }
                        if (i < 6 && j < 6) {
                            const int a = min(i, j), b = max(i, j);
                            h += nrm[a * 6 - a * (a - 1) / 2 + (b - a)];
                        }
                        Hs[q] = h;
                    }
                    __syncthreads();
                    // Marginalize(H, 0, 14) (:3388-3455) of the previous frame: H_ff - H_fp pinv(H_pp) H_pf
                    for (int q = tid; q < 225; q += kLatThreads) Am[q] = Hs[(15 + q / 15) * N + 15 + q % 15];
                    __syncthreads();
                    if (wave == 0) pinv15_wave(Am, Vm, PJ, ecs, epq, lane);   // pinv(H_pp) -> PJ
                    __syncthreads();
                    for (int q = tid; q < 225; q += kLatThreads) {   // T = H_fp pinv(H_pp) -> JPr
                        const int i = q / 15, j = q % 15;
                        double s = 0;
                        for (int k = 0; k < 15; ++k) s += Hs[i * N + 15 + k] * PJ[k * 15 + j];
                        JPr[q] = s;
                    }
                    __syncthreads();
                    for (int q = tid; q < 225; q += kLatThreads) {
                        const int i = q / 15, j = q % 15;
                        double s = 0;
                        for (int k = 0; k < 15; ++k) s += JPr[i * 15 + k] * Hs[(15 + k) * N + j];
                        A.H[(size_t)f * 225 + q] = Hs[i * N + j] - s;
                    }
                } else {
                    for (int q = tid; q < 225; q += kLatThreads) {
                        const int i = q / 15, j = q % 15;
                        double h = 0;
                        if (i < 6 && j < 6) {
                            const int a = min(i, j), b = max(i, j);
                            h = nrm[a * 6 - a * (a - 1) / 2 + (b - a)];
                        }
                        if (i < 9 && j < 9) {
                            double t = 0;
                            for (int k = 0; k < 9; ++k) t += J[k * 9 + i] * WJ[k * 9 + j];
                            h += t;
                        }
                        if (i >= 9 && j >= 9 && (i < 12) == (j < 12))
                            h += (i < 12 ? infoG : infoA)[3 * ((i - 9) % 3) + (j - 9) % 3];
                        A.H[(size_t)f * 225 + q] = h;
                    }
                }
            }
        }
#ifdef OMV_POSE_PROFILE
        LAT_T(t_h1);
        if (g == 0 && tid == 0) printf("pose_lat<%d> outlier write + hessian/marginalize %.1f us\n", (int)kLF, (t_h1 - t_h0) / 100.0);
        if (g == 0 && tid == 0 && f == 0) {   // hand-off skew: over the iterations, max - min publish time over the parts,
                                              // and part 0's completion after the last publish
            double skew = 0, post = 0;
            int n_it = 0;
            for (int i = 0; i < 48; ++i) {
                if (t2s[i] == 0) continue;
                unsigned long long mx = 0, mn = ~0ull;
                for (int p = 0; p < G; ++p) {
                    const unsigned long long t = __hip_atomic_load(&g_lat_pub[p][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    mx = t > mx ? t : mx, mn = t < mn ? t : mn;
                }
                skew += (double)(mx - mn), post += (double)t2s[i] - (double)mx, ++n_it;
            }
            printf("pose_lat<%d> hand-off per iteration (%d): publish skew %.2f us, last publish -> part 0 done %.2f us\n",
                   (int)kLF, n_it, skew / n_it / 100.0, post / n_it / 100.0);
        }
        if (g == 0 && tid == 0) {
            LAT_T(t_end);
            printf("pose_lat<%d> exchanges %llu: publish->flags %.2f flags->summed %.2f us each\n", (int)kLF, g_lat_x[3],
                   g_lat_x[0] / 100.0 / g_lat_x[3], g_lat_x[1] / 100.0 / g_lat_x[3]);
            printf("pose_lat<%d> setup %.1f loop %.1f (classification %.1f) recover %.1f hessian+rest %.1f us\n", (int)kLF,
                   (t_loop0 - t_start) / 100.0, (t_loop1 - t_loop0) / 100.0, t_cls / 100.0, (t_rec - t_loop1) / 100.0,
                   (t_end - t_rec) / 100.0);
            printf("pose_lat<%d> G %d edges(w0) %.1f reduce %.1f edges+inertial(barrier) %.1f exchange %.1f build %.1f "
                   "ldlt %.1f ldlt+update %.1f inertial(w4) %.1f total %.1f us\n", (int)kLF, G, prof[0] / 100.0,
                   prof[1] / 100.0, prof[2] / 100.0, prof[3] / 100.0, prof[4] / 100.0, prof[5] / 100.0, prof[6] / 100.0,
                   prof_inert / 100.0, (t_end - t_start) / 100.0);
            printf("pose_lat<%d> inertial wave: error %.1f jacobian %.1f info*J %.1f us\n", (int)kLF, prof_iw[0] / 100.0,
                   prof_iw[1] / 100.0, prof_iw[2] / 100.0);
        }
#endif
        if (g == 0) {   // state back
            if (tid == 0) {
                for (int q = 0; q < 9; ++q) A.Rwb[9 * f + q] = sRwb[9 + q];
                for (int q = 0; q < 3; ++q) {
                    A.twb[3 * f + q] = stwb[3 + q], A.vel[3 * f + q] = svel[3 + q];
                    A.bg[3 * f + q] = sbg[3 + q], A.ba[3 * f + q] = sba[3 + q];
                }
                A.n_good[f] = ne - (int)nBad;
            }
            for (int q = tid; q < C * 9; q += kLatThreads) A.Rcw[(size_t)f * C * 9 + q] = sRcw[q];
            for (int q = tid; q < C * 3; q += kLatThreads) A.tcw[(size_t)f * C * 3 + q] = stcw[q];
        }
        return;
    }
fail:
    // a part overflowed its LDS edge capacity (s_abort 2) or a sibling workgroup never arrived (1): the frame is
    // reported (n_good -1, OMV_ERR_CAPACITY in the handle's error word) and left unoptimised
    if (tid == 0) {
        if (g == 0) A.n_good[f] = -1;
        atomicOr(err_word, s_abort == 2 ? OMV_ERR_CAPACITY : OMV_ERR_HIP);
    }
}


struct EdgeLevels {
    float inv_sigma2[16];
};
struct EdgeOut {
    int32_t *m_start, *m_cam, *m_kp;
    double *m_obs;
    float *m_w, *m_xw;
    uint8_t *m_close;
    int32_t *s_start, *s_cam, *s_kp;
    double *s_obs;
    float *s_w, *s_xw;
    int32_t *err;
};

// The pose graph's visual edges from the frame's map-point assignment, on the device (the edge-creation loop of
// PoseInertialOptimizationLastKeyFrame / LastFrame, Optimizer.cc:5079-5330 / :5640-5800, multi-camera frame, bRight):
// per keypoint i of the concatenated [L | R | SL | SR] order with mvpMapPoints[i] an EdgeMonoOnlyPose of its block
// (obs = the raw keypoint, invSigma2 = mvInvLevelSigma2[octave] / uncertainty2 = 1), and with mvuRight[i] > 0 also
// an EdgeStereoOnlyPose of that block (obs (x, y, u_R)); both lists in keypoint order.  One workgroup,
// 8 consecutive slots (slot = cam * kp_cap + idx) per thread, an ordered scan of the per-thread edge counts per pass.
constexpr int kEdgeBuildThreads = 512, kEdgeSlots = 8;   // 8 consecutive slots per thread: 4096 slots per pass (512: the
                                                          // slot registers fit without spills)
__global__ void __launch_bounds__(kEdgeBuildThreads) pose_edges_kernel(int C, int cap, const omv_kp *kps, const int *n_kp,
                                                                      const int32_t *kp_to_mp, const float *mp_pos,
                                                                      const float *track_depth, EdgeLevels lv,
                                                                      const float *uright, int max_edges, EdgeOut o) {
    __shared__ int wc[kEdgeBuildThreads / 64][2], base[2], snk[kMaxCams];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 2) base[tid] = 0;
    if (tid < C) snk[tid] = n_kp[tid];
    __syncthreads();
    const int S = C * cap;
    for (int b0 = 0; b0 < S; b0 += kEdgeBuildThreads * kEdgeSlots) {
        const int s0 = b0 + tid * kEdgeSlots;
        int mp[kEdgeSlots];
        float ur[kEdgeSlots];
#pragma unroll
        for (int j = 0; j < kEdgeSlots; ++j) {
            const int s = s0 + j, c = s / cap, i = s - c * cap;
            mp[j] = s < S && i < snk[min(c, C - 1)] ? kp_to_mp[s] : -1;
        }
        int cm = 0, cst = 0;
#pragma unroll
        for (int j = 0; j < kEdgeSlots; ++j) {
            ur[j] = (mp[j] >= 0 && uright) ? uright[s0 + j] : -1.0f;
            cm += mp[j] >= 0 ? 1 : 0;
            cst += (mp[j] >= 0 && ur[j] > 0.0f) ? 1 : 0;   // kp_ur > 0 && bRight, every block (:5151, :5207, :5265, ...)
        }
        // exclusive scan of (cm, cst) over the workgroup in slot order
        int im = cm, is = cst;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int um = __shfl_up(im, d, 64), us = __shfl_up(is, d, 64);
            if (lane >= d) im += um, is += us;
        }
        if (lane == 63) wc[wave][0] = im, wc[wave][1] = is;
        __syncthreads();
        int om = base[0], os = base[1], tm = base[0], ts = base[1];
        for (int w = 0; w < kEdgeBuildThreads / 64; ++w) {
            if (w < wave) om += wc[w][0], os += wc[w][1];
            tm += wc[w][0], ts += wc[w][1];
        }
        om += im - cm, os += is - cst;
        // every gather first (all in flight together), then the stores
        float kx[kEdgeSlots], ky[kEdgeSlots], kw[kEdgeSlots], X0[kEdgeSlots], X1[kEdgeSlots], X2[kEdgeSlots], td[kEdgeSlots];
#pragma unroll
        for (int j = 0; j < kEdgeSlots; ++j) {
            kx[j] = ky[j] = kw[j] = X0[j] = X1[j] = X2[j] = td[j] = 0.f;
            if (mp[j] >= 0) {
                const size_t m = (size_t)mp[j];
                const omv_kp k = kps[s0 + j];
                kx[j] = k.x, ky[j] = k.y, kw[j] = lv.inv_sigma2[k.octave & 15];
                X0[j] = mp_pos[3 * m], X1[j] = mp_pos[3 * m + 1], X2[j] = mp_pos[3 * m + 2];
                td[j] = track_depth[m];
            }
        }
#pragma unroll
        for (int j = 0; j < kEdgeSlots; ++j) {
            if (mp[j] < 0) continue;
            const int s = s0 + j, c = s / cap;
            if (om < max_edges) {
                const int e = om;
                o.m_cam[e] = c, o.m_kp[e] = s;
                o.m_obs[2 * e] = (double)kx[j], o.m_obs[2 * e + 1] = (double)ky[j];
                o.m_w[e] = kw[j];
                o.m_xw[3 * e] = X0[j], o.m_xw[3 * e + 1] = X1[j], o.m_xw[3 * e + 2] = X2[j];
                o.m_close[e] = td[j] < 10.f ? 1 : 0;
            }
            ++om;
            if (ur[j] > 0.0f) {
                if (os < max_edges) {
                    const int e = os;
                    o.s_cam[e] = c, o.s_kp[e] = s;
                    o.s_obs[3 * e] = (double)kx[j], o.s_obs[3 * e + 1] = (double)ky[j], o.s_obs[3 * e + 2] = (double)ur[j];
                    o.s_w[e] = kw[j];
                    o.s_xw[3 * e] = X0[j], o.s_xw[3 * e + 1] = X1[j], o.s_xw[3 * e + 2] = X2[j];
                }
                ++os;
            }
        }
        __syncthreads();
        if (tid == 0) base[0] = tm, base[1] = ts;
        __syncthreads();
    }
    if (tid == 0) {
        o.m_start[0] = 0, o.m_start[1] = min(base[0], max_edges);
        o.s_start[0] = 0, o.s_start[1] = min(base[1], max_edges);
        if (base[0] > max_edges || base[1] > max_edges) atomicOr(o.err, OMV_ERR_CAPACITY);
    }
}

// ---- Optimizer::PoseOptimization (src/Optimizer.cc:855-1278) ------------------------------------------------------
// The visual-only pose optimisation: one VertexSE3Expmap (SE3Quat Tcw of camera 0, oplus = exp(dx) * T) with one unary
// edge per matched keypoint — EdgeSE3ProjectXYZOnlyPose(ToBody / SLPoseToBody / SRPoseToBody) through the rig's T_c0
// (OptimizableTypes.cpp:30-171) or EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.cpp:339-404) — optimised by
// Levenberg-Marquardt (optimization_algorithm_levenberg.cpp:61-169: tau 1e-5, 10 trials, Raul's stop) over the 6x6
// Hessian (BlockSolver_6_3 without landmarks + LinearSolverDense = Eigen::LDLT), 4 rounds of optimize(10) each from the
// frame's initial pose, outliers re-classified between rounds.  One workgroup per frame: thread t owns edges t,
// t + 256, ... in every pass, so an edge's chi2 (e->chi2(): the last computeError, a rejected trial's included) and
// level stay thread-private; per pass a fixed-order wavefront + LDS reduction (deterministic run to run); the solve on
// wavefront 0 (ldlt_pick_solve<6>), the LM bookkeeping and the SE3Quat update on thread 0.
struct PoseOnlyArgs {
    const int32_t *m_start, *m_cam, *m_kp;
    const double *m_obs;
    const float *m_w, *m_xw;
    const int32_t *s_start, *s_kp;
    const double *s_obs;
    const float *s_w, *s_xw;
    double *chi2_m, *chi2_s;
    uint8_t *act_m, *act_s;
    uint8_t *kp_out;
    int kp_cap;
    int32_t *n_good;
    double *pose_q, *pose_t;   // [F][4] (x y z w) / [F][3] in/out
};
struct PoseOnlyRig {
    Rig rig;                                          // cameras (project / projectJac by type)
    double q[kMaxCams][4], t[kMaxCams][3], R[kMaxCams][9];   // T_c0 (mTrl / mTsll / mTsrl) and its rotation matrix
    double fx, fy, cx, cy, bf;                        // EdgeStereoSE3ProjectXYZOnlyPose
};

// Eigen's quaternion ops on (x y z w): product, v' = q v q^-1 (_transformVector), Quaternion(Matrix3) and
// SE3Quat::normalizeRotation.
__device__ __forceinline__ void q_mul(const double *a, const double *b, double *r) {
    r[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    r[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    r[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    r[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
}
__device__ __forceinline__ void q_rot(const double *q, const double *v, double *o) {
    double u0 = q[1] * v[2] - q[2] * v[1], u1 = q[2] * v[0] - q[0] * v[2], u2 = q[0] * v[1] - q[1] * v[0];
    u0 += u0, u1 += u1, u2 += u2;
    o[0] = v[0] + q[3] * u0 + (q[1] * u2 - q[2] * u1);
    o[1] = v[1] + q[3] * u1 + (q[2] * u0 - q[0] * u2);
    o[2] = v[2] + q[3] * u2 + (q[0] * u1 - q[1] * u0);
}
__device__ void q_from_mat(const double *m, double *q) {
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t, q[1] = (m[2] - m[6]) * t, q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    }
}
__device__ __forceinline__ void q_normalize_pos(double *q) {
    if (q[3] < 0) q[0] = -q[0], q[1] = -q[1], q[2] = -q[2], q[3] = -q[3];
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; ++i) q[i] /= n;
}
// VertexSE3Expmap::oplusImpl: SE3Quat::exp(dx) * (q, t) (se3quat.h:104-110, :223-257) into (qo, to)
__device__ void se3_oplus(const double *dx, const double *q, const double *t, double *qo, double *to) {
    const double w0 = dx[0], w1 = dx[1], w2 = dx[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9], R[9], V[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    if (theta < 0.00001) {
        for (int k = 0; k < 9; ++k) R[k] = ((k % 4 == 0) ? 1.0 : 0.0) + O[k] + O2[k], V[k] = R[k];
    } else {
        double sn, cs;
        sincos_d(theta, sn, cs);
        const double a = sn / theta, b = (1 - cs) / (theta * theta), c = (theta - sn) / (theta * theta * theta);
        for (int k = 0; k < 9; ++k) {
            const double I = (k % 4 == 0) ? 1.0 : 0.0;
            R[k] = I + a * O[k] + b * O2[k];
            V[k] = I + b * O[k] + c * O2[k];
        }
    }
    double eq[4], et[3];
    q_from_mat(R, eq);
    q_normalize_pos(eq);
    mv3(V, dx + 3, et);
    double rt[3];
    q_rot(eq, t, rt);
    for (int i = 0; i < 3; ++i) to[i] = et[i] + rt[i];
    q_mul(eq, q, qo);
    q_normalize_pos(qo);
}

struct PoseOnlyEdge {
    bool stereo;
    int cam;
    double obs[3], w, X[3];
};
__device__ __forceinline__ PoseOnlyEdge po_edge(const PoseOnlyArgs &A, int m0, int nm, int s0, int e) {
    PoseOnlyEdge v;
    if (e < nm) {
        const int i = m0 + e;
        v.stereo = false, v.cam = A.m_cam[i];
        v.obs[0] = A.m_obs[2 * i], v.obs[1] = A.m_obs[2 * i + 1], v.obs[2] = 0;
        v.w = (double)A.m_w[i];
        for (int q = 0; q < 3; ++q) v.X[q] = (double)A.m_xw[3 * i + q];
    } else {
        const int i = s0 + e - nm;
        v.stereo = true, v.cam = 0;
        for (int q = 0; q < 3; ++q) v.obs[q] = A.s_obs[3 * i + q], v.X[q] = (double)A.s_xw[3 * i + q];
        v.w = (double)A.s_w[i];
    }
    return v;
}
// computeError at (q, t): residual r, chi2 returned; Xl = T Xw (camera 0), Xc = T_c0 Xl
__device__ __forceinline__ double po_error(const PoseOnlyRig &P, const double *q, const double *t, const PoseOnlyEdge &v,
                                           double *r, double *Xl, double *Xc) {
    q_rot(q, v.X, Xl);
    for (int i = 0; i < 3; ++i) Xl[i] += t[i];
    r[2] = 0;
    if (v.stereo) {   // cam_project with a float invz (types_six_dof_expmap.cpp:339-346)
        const float invz = (float)(1.0f / Xl[2]);
        const double u = Xl[0] * invz * P.fx + P.cx;
        r[0] = v.obs[0] - u;
        r[1] = v.obs[1] - (Xl[1] * invz * P.fy + P.cy);
        r[2] = v.obs[2] - (u - P.bf * invz);
        for (int i = 0; i < 3; ++i) Xc[i] = Xl[i];
        return r[0] * (v.w * r[0]) + r[1] * (v.w * r[1]) + r[2] * (v.w * r[2]);
    }
    if (v.cam) {
        q_rot(P.q[v.cam], Xl, Xc);
        for (int i = 0; i < 3; ++i) Xc[i] += P.t[v.cam][i];
    } else {
        for (int i = 0; i < 3; ++i) Xc[i] = Xl[i];
    }
    double u, vv;
    cam_project(P.rig, v.cam, Xc, u, vv);
    r[0] = v.obs[0] - u, r[1] = v.obs[1] - vv;
    return r[0] * (v.w * r[0]) + r[1] * (v.w * r[1]);
}
// the mono rows of linearizeOplus from the camera's projection Jacobian pj at Xc
__device__ __forceinline__ void po_jac_mono_pj(const PoseOnlyRig &P, const PoseOnlyEdge &v, const double *Xl,
                                               const double *pj, double *J) {
    double pr[6];
    const double *R = P.R[v.cam];
    for (int r = 0; r < 2; ++r)
        for (int q = 0; q < 3; ++q)
            pr[3 * r + q] = v.cam ? (-pj[3 * r]) * R[q] + (-pj[3 * r + 1]) * R[3 + q] + (-pj[3 * r + 2]) * R[6 + q]
                                  : -pj[3 * r + q];
    const double x = Xl[0], y = Xl[1], z = Xl[2];
    const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
    for (int r = 0; r < 2; ++r)
        for (int q = 0; q < 6; ++q)
            J[6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
}
// linearizeOplus: -projectJac(Xc) R_c0 SE3deriv(Xl) (mono) / the explicit stereo Jacobian
__device__ __forceinline__ void po_jac(const PoseOnlyRig &P, const PoseOnlyEdge &v, const double *Xl, const double *Xc,
                                       double *J) {
    if (v.stereo) {
        const double x = Xl[0], y = Xl[1], invz = 1.0 / Xl[2], invz_2 = invz * invz;
        J[0] = x * y * invz_2 * P.fx, J[1] = -(1 + (x * x * invz_2)) * P.fx, J[2] = y * invz * P.fx;
        J[3] = -invz * P.fx, J[4] = 0, J[5] = x * invz_2 * P.fx;
        J[6] = (1 + y * y * invz_2) * P.fy, J[7] = -x * y * invz_2 * P.fy, J[8] = -x * invz * P.fy;
        J[9] = 0, J[10] = -invz * P.fy, J[11] = y * invz_2 * P.fy;
        J[12] = J[0] - P.bf * y * invz_2, J[13] = J[1] + P.bf * x * invz_2, J[14] = J[2];
        J[15] = J[3], J[16] = 0, J[17] = J[5] - P.bf * invz_2;
        return;
    }
    double pj[6];
    cam_jac(P.rig, v.cam, Xc, pj);
    po_jac_mono_pj(P, v, Xl, pj, J);
}
// po_error + po_jac (the same arithmetic) with a mono edge's projection and projection Jacobian side by side in one
// branch of the camera type (independent chains given Xc)
__device__ __forceinline__ double po_error_jac(const PoseOnlyRig &P, const double *q, const double *t,
                                               const PoseOnlyEdge &v, double *r, double *Xl, double *Xc, double *J) {
    if (v.stereo) {
        const double c2 = po_error(P, q, t, v, r, Xl, Xc);
        po_jac(P, v, Xl, Xc, J);
        return c2;
    }
    q_rot(q, v.X, Xl);
    for (int i = 0; i < 3; ++i) Xl[i] += t[i];
    r[2] = 0;
    if (v.cam) {
        q_rot(P.q[v.cam], Xl, Xc);
        for (int i = 0; i < 3; ++i) Xc[i] += P.t[v.cam][i];
    } else {
        for (int i = 0; i < 3; ++i) Xc[i] = Xl[i];
    }
    double u, vv, pj[6];
    if (P.rig.model[v.cam] == OMV_CAM_PINHOLE) {
        pinhole_project(P.rig.cam[v.cam], Xc, u, vv);
        pinhole_jac(P.rig.cam[v.cam], Xc, pj);
    } else {
        kb8_project(P.rig.cam[v.cam], Xc, u, vv);
        kb8_jac(P.rig.cam[v.cam], Xc, pj);
    }
    r[0] = v.obs[0] - u, r[1] = v.obs[1] - vv;
    po_jac_mono_pj(P, v, Xl, pj, J);
    return r[0] * (v.w * r[0]) + r[1] * (v.w * r[1]);
}

constexpr int kPoNormal = 28;   // 21 upper-triangle H terms, 6 b terms, the robust chi2

constexpr int kPoThreads = 512;   // pose-only: one edge per thread up to 512 edges, two waves per SIMD
constexpr int kPoWaves = kPoThreads / 64;

__device__ __forceinline__ void po_reduce(double *acc, int n, double (*red)[kPoNormal], double *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int q = 0; q < n; ++q) {
        double v = acc[q];
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        acc[q] = v;
    }
    if (lane == 0)
        for (int q = 0; q < n; ++q) red[wave][q] = acc[q];
    __syncthreads();
    if (threadIdx.x < n) {
        double t = 0;
        for (int w = 0; w < kPoWaves; ++w) t += red[w][threadIdx.x];
        out[threadIdx.x] = t;
    }
    __syncthreads();
}

// Optimizer::PoseOptimization, one 512-thread workgroup per frame.  Thread t owns edge t (and t + 512, ... past 512
// edges): the edge's data and active flag stay in registers for the whole call (no global loads inside the LM
// loop), the per-edge chi2 goes to the workspace for the outlier classification.  Two waves per SIMD: the edge
// passes are long dependent f64 chains (KB8 projection and Jacobian), which one wave per SIMD could not hide.
__global__ void __launch_bounds__(kPoThreads) pose_only_kernel(PoseOnlyRig Parg, PoseOnlyArgs A) {
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    // the rig in LDS: the edges index it by camera (a per-lane index into the by-value kernel argument made the
    // compiler keep a private copy in scratch, reloaded inside the edge chains)
    __shared__ PoseOnlyRig P;
    {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(&Parg);
        uint32_t *dst = reinterpret_cast<uint32_t *>(&P);
        for (int i = tid; i < (int)(sizeof(PoseOnlyRig) / 4); i += kPoThreads) dst[i] = src[i];
    }
    __syncthreads();
    const int m0 = A.m_start[f], nm = A.m_start[f + 1] - m0, s0 = A.s_start[f], ns = A.s_start[f + 1] - s0;
    const int nE = nm + ns;
    __shared__ double q0[4], t0[3], sq[4], st[3], tq[4], tt[3];
    __shared__ double Hs[36], Ad[36], gs[6], xs[6], Lm[36], sums[kPoNormal];
    __shared__ double red[kPoWaves][kPoNormal];
    __shared__ int pick[8], cnt[kPoWaves];
    __shared__ double lambda_s, ni_s, cur_s, ini_s;
    __shared__ int nb_s, qmax_s, again_s, brk_s, ok_s;
    auto chi2_of = [&](int e) -> double & { return e < nm ? A.chi2_m[m0 + e] : A.chi2_s[s0 + e - nm]; };
    auto act_of = [&](int e) -> uint8_t & { return e < nm ? A.act_m[m0 + e] : A.act_s[s0 + e - nm]; };
    auto kp_of = [&](int e) { return e < nm ? A.m_kp[m0 + e] : A.s_kp[s0 + e - nm]; };
    uint8_t *kpo = A.kp_out + (size_t)f * A.kp_cap;
    for (int e = tid; e < nE; e += kPoThreads) act_of(e) = 1, kpo[kp_of(e)] = 0;   // mvbOutlier[i] = false
    if (nE < 3) {
        if (tid == 0) A.n_good[f] = 0;
        return;
    }
    // the thread's first edge, held for the call; its active flag mirrored in a register
    const bool own = tid < nE;
    const PoseOnlyEdge ev = po_edge(A, m0, nm, s0, own ? tid : 0);
    bool act0 = own;
    if (tid == 0) {
        for (int i = 0; i < 4; ++i) q0[i] = A.pose_q[4 * f + i];
        for (int i = 0; i < 3; ++i) t0[i] = A.pose_t[3 * f + i];
        q_normalize_pos(q0);
    }
    if (tid < 6) xs[tid] = 0.0;   // the dense solver's x: kept when a factorisation is not positive
    const double dmono = (double)(float)sqrt(5.991), dst = (double)(float)sqrt(7.815);
    bool robust = true;
    int nBad = 0;
#ifdef OMV_PO_PROFILE   // phase ticks (wall_clock64, 100 MHz) of frame 0, thread 0's view
    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tl = wall_clock64();
    int n_it = 0, n_trials = 0;
#define PO_T(k) (pt[k] += wall_clock64() - tl, tl = wall_clock64())
#else
#define PO_T(k) ((void)0)
#endif
    // edge e (the thread's own first one from registers, the rest from memory) and whether it is active
    auto edge_at = [&](int e, bool &active) -> PoseOnlyEdge {
        if (e == tid) {
            active = act0;
            return ev;
        }
        active = act_of(e) != 0;
        return po_edge(A, m0, nm, s0, e);
    };
    for (int round = 0; round < 4; ++round) {
        __syncthreads();
        if (tid < 4) sq[tid] = q0[tid];
        if (tid < 3) st[tid] = t0[tid];
        int na = act0 ? 1 : 0;
        for (int e = tid + kPoThreads; e < nE; e += kPoThreads) na += act_of(e);
        na = block_count<kPoWaves>(na, cnt);   // (barriers inside)
        if (na > 0) {   // initializeOptimization(0) found the vertex (otherwise optimize() returns -1)
            for (int it = 0; it < 10; ++it) {
                // computeActiveErrors + buildSystem at the current estimate.  The 28 normal-equation terms are summed
                // per edge pass over the wave (fixed butterfly) into the wave's LDS row, then over the waves in order:
                // no per-thread accumulator array live across the edge chain (it made the kernel spill)
                for (int q = tid; q < kPoWaves * kPoNormal; q += kPoThreads) (&red[0][0])[q] = 0.0;
                __syncthreads();
                for (int e0 = 0; e0 < nE; e0 += kPoThreads) {   // wave-uniform trip count
                    const int e = e0 + tid;
                    double J[18], om[3] = {0.0, 0.0, 0.0}, w = 0.0, r0 = 0.0;
                    for (int q = 0; q < 18; ++q) J[q] = 0.0;
                    if (e < nE) {
                        bool active;
                        const PoseOnlyEdge v = edge_at(e, active);
                        if (active) {
                            double r[3], Xl[3], Xc[3];
                            const double c2 = po_error_jac(P, sq, st, v, r, Xl, Xc, J);   // mono: rows 0-1
                            chi2_of(e) = c2;
                            double r1 = 1.0;
                            r0 = c2;
                            if (robust) {
                                const double d = v.stereo ? dst : dmono;
                                huber(c2, d, d * d, r0, r1);
                            }
                            w = v.w * r1;
                            for (int k = 0; k < (v.stereo ? 3 : 2); ++k) om[k] = -v.w * r[k] * r1;
                        }
                    }
                    auto wsum = [&](double x, int q) {
                        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
                        if (lane == 0) red[tid >> 6][q] += x;
                    };
                    int q = 0;
                    for (int i = 0; i < 6; ++i)
                        for (int j = i; j < 6; ++j, ++q)
                            wsum(w * (J[i] * J[j] + J[6 + i] * J[6 + j] + J[12 + i] * J[12 + j]), q);
                    for (int i = 0; i < 6; ++i) wsum(J[i] * om[0] + J[6 + i] * om[1] + J[12 + i] * om[2], 21 + i);
                    wsum(r0, 27);
                }
                PO_T(0);
                __syncthreads();
                if (tid < kPoNormal) {
                    double t = 0;
                    for (int wv = 0; wv < kPoWaves; ++wv) t += red[wv][tid];
                    sums[tid] = t;
                }
                __syncthreads();
                PO_T(1);
                if (tid == 0) {
                    int k = 0;
                    for (int i = 0; i < 6; ++i)
                        for (int j = i; j < 6; ++j, ++k) Hs[6 * i + j] = Hs[6 * j + i] = sums[k];
                    for (int i = 0; i < 6; ++i) gs[i] = sums[21 + i];
                    cur_s = ini_s = sums[27];
                    if (it == 0) {   // computeLambdaInit: tau * max |H_jj|
                        double md = 0;
                        for (int j = 0; j < 6; ++j) md = fmax(fabs(Hs[7 * j]), md);
                        lambda_s = 1e-5 * md, ni_s = 2, nb_s = 0;
                    }
                    qmax_s = 0;
                }
                __syncthreads();
                PO_T(2);
                double rho = 0;
                do {
                    if (tid < 64) {
                        if (lane < 36) Ad[lane] = Hs[lane] + ((lane % 7 == 0) ? lambda_s : 0.0);
                        wave_lds_sync();
                        const bool ok = ldlt_pick_solve<6>(Ad, gs, xs, pick, Lm, lane);
                        if (lane == 0) {
                            ok_s = ok ? 1 : 0;
                            se3_oplus(xs, sq, st, tq, tt);
                        }
                    }
                    __syncthreads();
                    PO_T(3);
                    // computeActiveErrors at the trial estimate
                    double c = 0.0;
                    for (int e = tid; e < nE; e += kPoThreads) {
                        bool active;
                        const PoseOnlyEdge v = edge_at(e, active);
                        if (!active) continue;
                        double r[3], Xl[3], Xc[3];
                        const double c2 = po_error(P, tq, tt, v, r, Xl, Xc);
                        chi2_of(e) = c2;
                        double r0 = c2, r1;
                        if (robust) {
                            const double d = v.stereo ? dst : dmono;
                            huber(c2, d, d * d, r0, r1);
                        }
                        c += r0;
                    }
                    PO_T(4);
                    po_reduce(&c, 1, red, sums);
                    PO_T(5);
#ifdef OMV_PO_PROFILE
                    ++n_trials;
#endif
                    if (tid == 0) {
                        double tempChi = ok_s ? sums[0] : DBL_MAX;
                        double sc = 0;
                        for (int j = 0; j < 6; ++j) sc += xs[j] * (lambda_s * xs[j] + gs[j]);
                        sc += 1e-3;
                        rho = (cur_s - tempChi) / sc;
                        if (rho > 0 && isfinite(tempChi)) {
                            const double a3 = 2 * rho - 1;
                            double alpha = 1. - a3 * a3 * a3;   // pow(2 rho - 1, 3)
                            alpha = fmin(alpha, 2. / 3.);
                            lambda_s *= fmax(1. / 3., alpha);
                            ni_s = 2;
                            cur_s = tempChi;
                            for (int i = 0; i < 4; ++i) sq[i] = tq[i];
                            for (int i = 0; i < 3; ++i) st[i] = tt[i];
                        } else {   // pop(): the estimate restored, the edges keep the rejected trial's errors
                            lambda_s *= ni_s;
                            ni_s *= 2;
                        }
                        qmax_s++;
                        again_s = (rho < 0 && qmax_s < 10) ? 1 : 0;
                        brk_s = 0;
                        if (!again_s) {
                            if (qmax_s == 10 || rho == 0) brk_s = 1;
                            else {
                                nb_s = (ini_s - cur_s) * 1e3 < ini_s ? nb_s + 1 : 0;
                                brk_s = nb_s >= 3 ? 1 : 0;
                            }
                        }
                    }
                    __syncthreads();
                    PO_T(6);
                } while (again_s);
#ifdef OMV_PO_PROFILE
                ++n_it;
#endif
                if (brk_s) break;
            }
        }
        // outlier classification (:1145-1263): an edge left out of this round is re-evaluated at the final estimate
        int bad = 0;
        for (int e = tid; e < nE; e += kPoThreads) {
            bool active;
            const PoseOnlyEdge v = edge_at(e, active);
            double c2 = chi2_of(e);
            if (!active) {
                double r[3], Xl[3], Xc[3];
                c2 = po_error(P, sq, st, v, r, Xl, Xc);
                chi2_of(e) = c2;
            }
            const bool out = (float)c2 > (e < nm ? 5.991f : 7.815f);
            if (e == tid) act0 = !out;
            else act_of(e) = out ? 0 : 1;
            bad += out ? 1 : 0;
        }
        nBad = block_count<kPoWaves>(bad, cnt);
        if (round == 2) robust = false;
        if (nE < 10) break;   // optimizer.edges().size() < 10
    }
#ifdef OMV_PO_PROFILE
    if (tid == 0 && f == 0)
        printf("pose_only ticks(100MHz): iterations %d trials %d edges %llu reduce %llu Hbuild %llu solve+oplus %llu trial-edges %llu trial-reduce %llu bookkeeping %llu\n",
               n_it, n_trials, pt[0], pt[1], pt[2], pt[3], pt[4], pt[5], pt[6]);
#endif
#undef PO_T
    if (own) act_of(tid) = act0 ? 1 : 0;
    for (int e = tid; e < nE; e += kPoThreads) kpo[kp_of(e)] = (e == tid ? act0 : act_of(e) != 0) ? 0 : 1;
    if (tid == 0) {
        for (int i = 0; i < 4; ++i) A.pose_q[4 * f + i] = sq[i];
        for (int i = 0; i < 3; ++i) A.pose_t[3 * f + i] = st[i];
        A.n_good[f] = nE - nBad;
    }
}
}  // namespace

struct omv_pose {
    int max_frames, max_edges;
    double *chi2 = nullptr;   // [2][max_edges]
    uint8_t *act = nullptr;   // [2][max_edges]
    double *info = nullptr;   // [max_frames][99]
    // grouped (latency) path: per frame two slots x kLatMaxParts x (payload row + flag) exchange words, the call's tag salt,
    // the device error word, the path policy (OMV_POSE_AUTO / _BATCH / _GROUPED) and the parts per frame (0: auto)
    unsigned long long *xbuf = nullptr;
    uint32_t call = 0;
    int32_t *err = nullptr;
    int mode = OMV_POSE_AUTO, parts = 0;
};

extern "C" {

omv_status omv_pose_create(int max_frames, int max_edges, omv_pose **out) {
    if (!out || max_frames <= 0 || max_edges < 0) return OMV_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return OMV_ERR_NO_DEVICE;
    omv_pose *h = new omv_pose();
    h->max_frames = max_frames, h->max_edges = max_edges;
    const size_t n = 2 * (size_t)std::max(1, max_edges);
    const size_t xb = (size_t)max_frames * kLatFrameGran * sizeof(unsigned long long);
    if (hipMalloc(&h->chi2, n * sizeof(double)) != hipSuccess || hipMalloc(&h->act, n) != hipSuccess ||
        hipMalloc(&h->info, (size_t)max_frames * 99 * sizeof(double)) != hipSuccess ||
        hipMalloc(&h->xbuf, xb) != hipSuccess || hipMemset(h->xbuf, 0, xb) != hipSuccess ||
        hipMalloc(&h->err, sizeof(int32_t)) != hipSuccess || hipMemset(h->err, 0, sizeof(int32_t)) != hipSuccess) {
        (void)hipFree(h->chi2);
        (void)hipFree(h->act);
        (void)hipFree(h->info);
        (void)hipFree(h->xbuf);
        (void)hipFree(h->err);
        delete h;
        return OMV_ERR_HIP;
    }
    *out = h;
    return OMV_OK;
}

omv_status omv_pose_destroy(omv_pose *h) {
    if (!h) return OMV_ERR_ARG;
    (void)hipFree(h->chi2);
    (void)hipFree(h->act);
    (void)hipFree(h->info);
    (void)hipFree(h->xbuf);
    (void)hipFree(h->err);
    delete h;
    return OMV_OK;
}

omv_status omv_pose_set_mode(omv_pose *h, int mode, int parts) {
    if (!h || mode < OMV_POSE_AUTO || mode > OMV_POSE_GROUPED || parts < 0 || parts > kLatMaxParts) return OMV_ERR_ARG;
    h->mode = mode, h->parts = parts;
    return OMV_OK;
}

omv_status omv_pose_last_error(omv_pose *h, int32_t *err, void *stream) {
    if (!h || !err) return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    HIP_OK(hipMemcpyAsync(err, h->err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemsetAsync(h->err, 0, sizeof(int32_t), st));
    HIP_OK(hipStreamSynchronize(st));
    return OMV_OK;
}

}  // extern "C"

namespace {

// Both optimisations: validate, fill the kernel arguments, launch the information kernel and the
// one-workgroup-per-frame optimisation.  prior == nullptr: LastKeyFrame.
omv_status launch_pose(omv_pose *h, const omv_pose_batch *b, const omv_pose_prior *prior, int rec_init,
                       uint8_t *kp_outlier, int32_t *n_good, double *H, void *stream) {
    if (!h || !b || !kp_outlier || !n_good) return OMV_ERR_ARG;
    if (b->n_frames <= 0 || b->n_frames > h->max_frames || b->n_cams <= 0 || b->n_cams > kMaxCams ||
        b->n_mono < 0 || b->n_stereo < 0 || b->n_mono > h->max_edges || b->n_stereo > h->max_edges || b->kp_cap <= 0)
        return OMV_ERR_ARG;
    if (prior && (!prior->Rwb || !prior->twb || !prior->vel || !prior->bg || !prior->ba || !prior->H ||
                  !prior->preint_kf))
        return OMV_ERR_ARG;
    if (!b->cam || !b->Rcb || !b->tcb || !b->Rbc || !b->tbc || !b->Rwb || !b->twb || !b->Rcw || !b->tcw || !b->vel ||
        !b->bg || !b->ba || !b->kf_Rwb || !b->kf_twb || !b->kf_vel || !b->kf_bg || !b->kf_ba || !b->preint ||
        !b->mono_start || !b->stereo_start)
        return OMV_ERR_ARG;
    if (b->n_mono > 0 && (!b->mono_cam || !b->mono_kp || !b->mono_obs || !b->mono_inv_sigma2 || !b->mono_xw ||
                          !b->mono_close))
        return OMV_ERR_ARG;
    if (b->n_stereo > 0 && (!b->stereo_cam || !b->stereo_kp || !b->stereo_obs || !b->stereo_inv_sigma2 ||
                            !b->stereo_xw))
        return OMV_ERR_ARG;
    Rig rig{};
    rig.n_cams = b->n_cams;
    for (int c = 0; c < b->n_cams; ++c) {
        for (int q = 0; q < 8; ++q) rig.cam[c][q] = b->cam[8 * c + q];
        rig.model[c] = b->cam_model ? b->cam_model[c] : OMV_CAM_KB8;
        if (rig.model[c] != OMV_CAM_KB8 && rig.model[c] != OMV_CAM_PINHOLE) return OMV_ERR_ARG;
        for (int q = 0; q < 9; ++q) rig.Rcb[c][q] = b->Rcb[9 * c + q], rig.Rbc[c][q] = b->Rbc[9 * c + q];
        for (int q = 0; q < 3; ++q) rig.tcb[c][q] = b->tcb[3 * c + q], rig.tbc[c][q] = b->tbc[3 * c + q];
    }
    rig.bf = (double)b->bf;
    PoseArgs A{b->Rwb, b->twb, b->Rcw, b->tcw, b->vel, b->bg, b->ba, b->kf_Rwb, b->kf_twb, b->kf_vel, b->kf_bg,
               b->kf_ba, b->preint, b->mono_start, b->mono_cam, b->mono_kp, b->mono_obs, b->mono_inv_sigma2,
               b->mono_xw, b->mono_close, b->stereo_start, b->stereo_cam, b->stereo_kp, b->stereo_obs,
               b->stereo_inv_sigma2, b->stereo_xw, b->kp_cap, h->chi2, h->chi2 + h->max_edges, h->act,
               h->act + h->max_edges, kp_outlier, n_good, H, rec_init, h->info, prior ? prior->preint_kf : b->preint};
    hipStream_t st = (hipStream_t)stream;
    if (prior) {
        A.pRwb = prior->Rwb, A.ptwb = prior->twb, A.pvel = prior->vel, A.pbg = prior->bg, A.pba = prior->ba;
        A.pH = prior->H;
    }
    // Path: the grouped kernel (G workgroups per frame, latency) for a few frames, the one-workgroup-per-frame kernel
    // for batches.  G from the mean edge count: one visual edge per edge-wave thread.
    const int F = b->n_frames;
    const long long ne_tot = (long long)b->n_mono + b->n_stereo;
    // A part holds at most kLatCap edges and a frame's edges are split over its G parts, so G is sized from the largest
    // frame the batch can hold: no frame has more than ne_tot edges (the per-frame counts live on the device).  AUTO
    // takes the grouped kernel only when that bound fits kLatMaxParts parts.
    const long long g_need = (ne_tot + kLatCap - 3) / (kLatCap - 2);
    const bool grouped_ok = b->kp_cap <= kLatFlagCap;
    bool grouped = h->mode == OMV_POSE_GROUPED ||
                   (h->mode == OMV_POSE_AUTO && F <= kLatAutoFrames && grouped_ok && g_need <= kLatMaxParts);
    if (h->mode == OMV_POSE_GROUPED && !grouped_ok) return OMV_ERR_ARG;
    int G = h->parts;
    const int et = lat_edge_threads(prior != nullptr);
    // one edge per edge-wave thread: parts hold ne / G edges up to one keypoint's two (lat_bound_wave)
    if (G == 0) {
        G = (int)std::min<long long>(kLatMaxParts, std::max<long long>(1, (ne_tot / F + et - 3) / (et - 2)));
        G = (int)std::min<long long>(kLatMaxParts, std::max<long long>(G, g_need));
    }
    if (!grouped) pose_info_kernel<<<F, 64, 0, st>>>(b->preint, prior ? prior->preint_kf : b->preint, h->info);
    if (grouped) {
        h->call = (h->call + 1) & 0xFFFFFu;
        if (h->call == 0) {   // tags repeat after 2^20 calls: clear the granules once
            HIP_OK(hipMemsetAsync(h->xbuf, 0, (size_t)h->max_frames * kLatFrameGran * sizeof(unsigned long long), st));
            h->call = 1;
        }
        const uint32_t salt = h->call << 12;
        const size_t lds = lat_lds_bytes(b->kp_cap);
        gu64 *xb = (gu64 *)h->xbuf;
        // The dynamic-LDS attribute belongs to the kernel, not the handle (hipFuncSetAttribute is process-wide): one
        // grow-only bound per kernel, raised under a lock, so a handle with a smaller kp_cap never lowers the limit
        // another handle's launches rely on.
        {
            static std::mutex mu;
            static size_t lat_lds_max[2] = {0, 0};
            const int pi = prior ? 1 : 0;
            std::lock_guard<std::mutex> lk(mu);
            if (lat_lds_max[pi] < lds) {
                HIP_OK(hipFuncSetAttribute(prior ? (const void *)pose_lat_kernel<true> : (const void *)pose_lat_kernel<false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                lat_lds_max[pi] = lds;
            }
        }
        if (prior) pose_lat_kernel<true><<<F * G, kLatThreads, lds, st>>>(rig, A, G, xb, salt, h->err);
        else pose_lat_kernel<false><<<F * G, kLatThreads, lds, st>>>(rig, A, G, xb, salt, h->err);
    } else if (prior) {
        pose_opt_kernel<true><<<F, kPoseThreads, 0, st>>>(rig, A);
    } else {
        pose_opt_kernel<false><<<F, kPoseThreads, 0, st>>>(rig, A);
    }
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

}  // namespace

extern "C" {

omv_status omv_pose_inertial_last_kf(omv_pose *h, const omv_pose_batch *b, int rec_init, uint8_t *kp_outlier,
                                     int32_t *n_good, double *H, void *stream) {
    return launch_pose(h, b, nullptr, rec_init, kp_outlier, n_good, H, stream);
}

omv_status omv_pose_inertial_last_frame(omv_pose *h, const omv_pose_batch *b, const omv_pose_prior *prior,
                                        int rec_init, uint8_t *kp_outlier, int32_t *n_good, double *H, void *stream) {
    if (!prior) return OMV_ERR_ARG;
    return launch_pose(h, b, prior, rec_init, kp_outlier, n_good, H, stream);
}

omv_status omv_pose_optimization(omv_pose *h, const omv_pose_batch *b, const double *rig_q, const double *rig_t,
                                 double *pose_q, double *pose_t, uint8_t *kp_outlier, int32_t *n_good, void *stream) {
    if (!h || !b || !rig_q || !rig_t || !pose_q || !pose_t || !kp_outlier || !n_good) return OMV_ERR_ARG;
    if (b->n_frames <= 0 || b->n_frames > h->max_frames || b->n_cams <= 0 || b->n_cams > kMaxCams || b->n_mono < 0 ||
        b->n_stereo < 0 || b->n_mono > h->max_edges || b->n_stereo > h->max_edges || b->kp_cap <= 0 || !b->cam ||
        !b->mono_start || !b->stereo_start)
        return OMV_ERR_ARG;
    // every edge array the kernel reads must be present when its kind has edges (the Python binding leaves absent
    // keys NULL): an error here instead of a fault on the device
    if (b->n_mono > 0 && (!b->mono_kp || !b->mono_obs || !b->mono_inv_sigma2 || !b->mono_xw || !b->mono_cam))
        return OMV_ERR_ARG;
    if (b->n_stereo > 0 && (!b->stereo_kp || !b->stereo_obs || !b->stereo_inv_sigma2 || !b->stereo_xw))
        return OMV_ERR_ARG;
    PoseOnlyRig P{};
    P.rig.n_cams = b->n_cams;
    for (int c = 0; c < b->n_cams; ++c) {
        for (int q = 0; q < 8; ++q) P.rig.cam[c][q] = b->cam[8 * c + q];
        P.rig.model[c] = b->cam_model ? b->cam_model[c] : OMV_CAM_KB8;
        if (P.rig.model[c] != OMV_CAM_KB8 && P.rig.model[c] != OMV_CAM_PINHOLE) return OMV_ERR_ARG;
        // SE3Quat(q, t): normalised, w >= 0; toRotationMatrix for the Jacobian
        double q[4] = {rig_q[4 * c], rig_q[4 * c + 1], rig_q[4 * c + 2], rig_q[4 * c + 3]};
        if (q[3] < 0) q[0] = -q[0], q[1] = -q[1], q[2] = -q[2], q[3] = -q[3];
        const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        if (!(n > 0)) return OMV_ERR_ARG;
        for (int i = 0; i < 4; ++i) P.q[c][i] = q[i] / n;
        for (int i = 0; i < 3; ++i) P.t[c][i] = rig_t[3 * c + i];
        const double x = P.q[c][0], y = P.q[c][1], z = P.q[c][2], w = P.q[c][3];
        const double tx = 2 * x, ty = 2 * y, tz = 2 * z, twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x,
                     txy = ty * x, txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
        const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                             txz - twy, tyz + twx, 1 - (txx + tyy)};
        for (int i = 0; i < 9; ++i) P.R[c][i] = R[i];
    }
    P.fx = b->cam[0], P.fy = b->cam[1], P.cx = b->cam[2], P.cy = b->cam[3], P.bf = (double)b->bf;
    const PoseOnlyArgs A{b->mono_start, b->mono_cam, b->mono_kp, b->mono_obs, b->mono_inv_sigma2, b->mono_xw,
                         b->stereo_start, b->stereo_kp, b->stereo_obs, b->stereo_inv_sigma2, b->stereo_xw, h->chi2,
                         h->chi2 + h->max_edges, h->act, h->act + h->max_edges, kp_outlier, b->kp_cap, n_good, pose_q,
                         pose_t};
    static_assert(sizeof(PoseOnlyRig) % 4 == 0, "PoseOnlyRig is copied to LDS by dwords");
    pose_only_kernel<<<b->n_frames, kPoThreads, 0, (hipStream_t)stream>>>(P, A);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_pose_edges_from_matches(omv_pose *h, int n_cams, int kp_cap, const omv_kp *kps, const int *n_kp,
                                       const int32_t *kp_to_mp, const float *mp_pos, const float *mp_track_depth,
                                       const float *inv_level_sigma2, int n_levels, const float *uright, int max_edges,
                                       int32_t *mono_start, int32_t *mono_cam, int32_t *mono_kp, double *mono_obs,
                                       float *mono_inv_sigma2, float *mono_xw, uint8_t *mono_close, int32_t *stereo_start,
                                       int32_t *stereo_cam, int32_t *stereo_kp, double *stereo_obs,
                                       float *stereo_inv_sigma2, float *stereo_xw, void *stream) {
    if (!h || n_cams <= 0 || n_cams > kMaxCams || kp_cap <= 0 || !kps || !n_kp || !kp_to_mp || !mp_pos ||
        !mp_track_depth || !inv_level_sigma2 || n_levels <= 0 || n_levels > 16 || max_edges <= 0 || !mono_start ||
        !mono_cam || !mono_kp || !mono_obs || !mono_inv_sigma2 || !mono_xw || !mono_close || !stereo_start ||
        !stereo_cam || !stereo_kp || !stereo_obs || !stereo_inv_sigma2 || !stereo_xw)
        return OMV_ERR_ARG;
    EdgeLevels lv{};
    for (int l = 0; l < 16; ++l) lv.inv_sigma2[l] = inv_level_sigma2[l < n_levels ? l : n_levels - 1];
    const EdgeOut o{mono_start, mono_cam, mono_kp, mono_obs, mono_inv_sigma2, mono_xw, mono_close, stereo_start,
                    stereo_cam, stereo_kp, stereo_obs, stereo_inv_sigma2, stereo_xw, h->err};
    pose_edges_kernel<<<1, kEdgeBuildThreads, 0, (hipStream_t)stream>>>(n_cams, kp_cap, kps, n_kp, kp_to_mp, mp_pos,
                                                                         mp_track_depth, lv, uright, max_edges, o);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_pose_constraint(int n, const double *H_in, double *H_out, void *stream) {
    if (n < 0 || (n > 0 && (!H_in || !H_out))) return OMV_ERR_ARG;
    if (n == 0) return OMV_OK;
    pose_constraint_kernel<<<n, 64, 0, (hipStream_t)stream>>>(H_in, H_out);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

}  // extern "C"
