// MI355X-native LocalInertialBA inner loop (Optimizer::LocalInertialBA's optimize(),
// src/Optimizer.cc:3270-3321): g2o's Levenberg-Marquardt over EdgeMono / EdgeInertial / EdgeGyroRW /
// EdgeAccRW with the landmark Schur complement, as batched gfx950 kernels on device-resident state.
//
// Per LM iteration (optimization_algorithm_levenberg.cpp:61-169):
//   errors   1 thread / visual edge (+1 thread / inertial edge): residual, chi2, Huber rho; deterministic
//            two-level chi2 reduction (computeActiveErrors + activeRobustChi2)
//   build    1 thread / landmark (edges sorted landmark-major): EdgeMono / EdgeStereo Jacobians, the
//            landmark's Hll / bl and per-keyframe Hpl blocks in registers; 1 workgroup / optimisable
//            keyframe gathers its edges for the pose-diagonal JpT W Jp and JpT W e (fixed-order reduction);
//            1 wavefront / inertial edge writes its 30x30 quadratic form (EdgeInertial + random walks),
//            added into the reduced system colour by colour (no two edges of a colour share a keyframe)
//   per trial (lambda):
//     schur    1 thread / landmark: Dinv = (Hll + lambda I)^-1, BD = Hpl Dinv and Hpl Dinv bl per slot;
//              1 workgroup / reduced-system block gathers its (slot a, slot b) terms BD_a Hpl_b^T and, on the
//              diagonal, the keyframe's coefficients — fixed-order sums throughout, no float atomics, so a
//              solve is bitwise identical run to run
//     ldlt     1 workgroup: block LDL^T of the reduced system (keyframe blocks of 15 / 6) on the
//              symbolic block pattern (host-computed fill-in), the nonzero blocks staged in LDS,
//              then block forward / backward substitution (SimplicialLDLT semantics: no pivoting,
//              failure on a zero or non-finite pivot)
//     update   1 thread / landmark: back-substitution xl = Dinv (bl - Hpl^T xp) and the point update;
//              1 thread / keyframe: ImuCamPose::Update (body-frame SE3 with ExpSO3) + v, bg, ba;
//              the step's computeScale term; errors of the trial state
//   The accept / reject decision (rho, lambda schedule, push/pop) runs on the device (finish_trial_kernel,
//   LmCtl) with one read-back per optimize(); a host-driven loop with the same decisions is kept for
//   sharded solves and parity checks.  Push/pop is a double-buffered state.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <numeric>
#include <set>
#include <type_traits>
#include <vector>

#include "../../include/omv.h"
#include "g2o_types.h"
#include "omv_device.h"

namespace {

using namespace omv_g2o;

constexpr int kGrpEdges = 256;   // edges per buildSystem landmark group / pose chunk (one per thread)

#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)




// Device-resident Levenberg-Marquardt control (optimization_algorithm_levenberg.cpp:61-169), for the
// single-rank path: the accept / reject decision, the lambda schedule and the iteration / stop logic run in
// finish_trial_kernel, so one LM trial is a fixed kernel sequence (captured once as a hipGraph) whose kernels
// read lambda and their gate from here, and the host reads the outcome back once per optimize().
struct LmCtl {
    double lambda, ni, currentChi, iniChi, errors_chi, err0, rho, lambda_init;
    int it, qmax, nBad, trials, its, opt_it, max_trials;
    int done;                // the optimisation has ended
    int errors_of_current;   // the last computed errors belong to the current state (A)
    int need_build;          // the next step starts a new iteration (buildSystem)
    int accepted;            // the last trial was accepted: the trial state becomes current
    int n_acc;               // accepted updates since optimize()'s start: ImuCamPose::its of every optimisable
                             // keyframe (created with its 0, popped with a rejected trial), Rwb normalised after every
                             // third Update (G2oTypes.cc:220-225) -- a trial normalises iff n_acc % 3 == 2
    // double-buffered state and errors (device driver): buffer `cur` holds the current state and its errors, the
    // trial writes buffer cur ^ 1 and an accepted trial flips `cur` -- no copy, and no recomputation of the
    // current errors after a rejected trial (they are still in their buffer); `last` = the buffer of the last
    // computed errors (the reference reports those: g2o keeps a rejected trial's errors after the pop)
    int cur, last;
    int init_pending;        // optimize()'s initial chi not summed yet (the first step's bookkeeping does it)
    double cur_chi;          // activeRobustChi2 of the current state
    int g_active, g_errA, g_build;   // gates of the next step (set by ctl_init / finish_trial)
};
enum { kGateAlways = 0, kGateErrA = 1, kGateBuild = 2, kGateTrial = 3 };
__device__ __forceinline__ bool gate_open(const LmCtl *c, int g) {
    if (!c || g == kGateAlways) return true;
    if (g == kGateErrA) return c->g_errA != 0;
    if (g == kGateBuild) return c->g_build != 0;
    return c->g_active != 0;
}
__device__ __forceinline__ double lm_lambda(const LmCtl *c, double lambda) { return c ? c->lambda : lambda; }

struct ErrBufs {   // per-edge errors of one state: visual [2E], stereo row [E], chi2 [E], inertial [19 NI]
    double *err, *err3, *chi2, *err9;
};
// Buffer of a role (0 = current, 1 = trial): by the control block's `cur` on the device driver, the role itself
// without one (the host driver passes the state it means as the first of the pair).
__device__ __forceinline__ int role_buf(const LmCtl *c, int role) { return c ? ((c->cur ^ role) & 1) : role; }

// EdgeMono / EdgeStereo error of edge e at point X (G2oTypes.h:293-299, :364-402): residual, chi2 into the error
// buffers; returns the robust chi2 (Huber rho_0) for activeRobustChi2.
__device__ __forceinline__ double mono_err_edge(const Rig &rig, const double *R, const double *t, const Edges &E, int e,
                                                const double *X, double delta, double dsqr, double delta_st,
                                                double dsqr_st, double *err, double *err3, double *chi2) {
    const int c = E.cam[e];
    double Xc[3];
    mv3(R, X, Xc);
    Xc[0] += t[0], Xc[1] += t[1], Xc[2] += t[2];
    double u, v;
    cam_project(rig, c, Xc, u, v);
    const double e0 = E.obs[2 * e] - u, e1 = E.obs[2 * e + 1] - v;
    const double w = (double)E.w[e];
    double c2 = e0 * w * e0 + e1 * w * e1;
    err[2 * e] = e0, err[2 * e + 1] = e1;
    const float ur = E.ur[e];
    if (ur >= 0.f) {   // EdgeStereo
        const double e2 = (double)ur - stereo_ur(u, rig.bf, Xc[2]);
        err3[e] = e2;
        c2 += e2 * w * e2;
    }
    chi2[e] = c2;
    double r0, r1;
    if (ur >= 0.f) huber(c2, delta_st, dsqr_st, r0, r1);
    else huber(c2, delta, dsqr, r0, r1);
    return r0;
}

// EdgeInertial + random-walk errors, one block (threads >= I.n contribute 0 to the fixed-order sum).
__device__ __forceinline__ void imu_err_block(double *sh, State s, Imu I, double delta, double dsqr, double *err9,
                                              double *partial) {
    const int i = threadIdx.x;
    double r0 = 0;
    if (i < I.n) {
        double e[9];
        imu_error(s, I, i, e, err9 + (size_t)10 * I.n + 9 * (size_t)i);   // + the rotation error for buildSystem
        const double *W = I.info9 + (size_t)i * 81;
        double c2 = 0;
        for (int r = 0; r < 9; ++r) {
            double t = 0;
            for (int c = 0; c < 9; ++c) t += W[r * 9 + c] * e[c];
            c2 += e[r] * t;
        }
        for (int q = 0; q < 9; ++q) err9[9 * i + q] = e[q];
        err9[(size_t)9 * I.n + i] = c2;   // chi2 after the errors
        if (I.robust[i]) {
            double r1;
            huber(c2, delta, dsqr, r0, r1);
        } else {
            r0 = c2;
        }
        const int k1 = I.kf1[i], k2 = I.kf2[i];
        double eg[3], ea[3];
        for (int q = 0; q < 3; ++q) eg[q] = s.bg[3 * k2 + q] - s.bg[3 * k1 + q], ea[q] = s.ba[3 * k2 + q] - s.ba[3 * k1 + q];
        double tg[3], ta[3];
        mv3(I.infoG + 9 * i, eg, tg);
        mv3(I.infoA + 9 * i, ea, ta);
        r0 += eg[0] * tg[0] + eg[1] * tg[1] + eg[2] * tg[2];
        r0 += ea[0] * ta[0] + ea[1] * ta[1] + ea[2] * ta[2];
    }
    const double t = block_reduce_sum(r0, sh);
    if (threadIdx.x == 0) partial[0] = t;
}

// activeRobustChi2: inertial partial + visual partials in a fixed order (one block of 256).
__device__ __forceinline__ double sum_chi(const double *mono_partial, int n_mono_blocks, const double *imu_partial,
                                          double *sh) {
    double v = 0;
    for (int i = threadIdx.x; i < n_mono_blocks; i += blockDim.x) v += mono_partial[i];
    const double t = block_reduce_sum(v, sh);
    return imu_partial[0] + t;
}

// The next step's gates from the LM state: a trial runs unless the optimisation ended; it starts a new
// iteration (buildSystem) after an iteration ended, and first recomputes the current state's errors when the
// last computed errors were a rejected trial's.
__device__ __forceinline__ void set_gates(LmCtl *c) {
    c->g_active = !c->done;
    c->g_build = !c->done && c->need_build;
    c->g_errA = 0;   // the current errors stay in their buffer (double-buffered): never recomputed
}

// The LM state reset of optimize()'s start (iteration 0's lambda = lambda_init, ni = 2, nBad = 0,
// optimization_algorithm_levenberg.cpp:103-108), without the initial chi.
struct LmReset {
    LmCtl *c;   // null: no reset
    int opt_it, max_trials;
    double lambda_init;
};
__device__ __forceinline__ void ctl_reset(const LmReset &r) {
    LmCtl *c = r.c;
    c->errors_of_current = 1;
    c->cur = c->last = 0;
    c->need_build = 1;
    c->it = c->qmax = c->nBad = c->trials = c->its = 0;
    c->opt_it = r.opt_it, c->max_trials = r.max_trials, c->lambda_init = r.lambda_init;
    c->lambda = r.lambda_init, c->ni = 2, c->rho = 0, c->accepted = 0, c->n_acc = 0;
    c->done = r.opt_it <= 0;
    set_gates(c);
}

// optimize()'s start: err = activeRobustChi2 of the initial state (Optimizer.cc:3273-3274), LM state reset
// (used when no step follows, opt_it <= 0; otherwise the initial error launch resets the control block and the
// first step's bookkeeping sums the initial chi -- one launch less per optimize()).
__global__ void __launch_bounds__(256) ctl_init_kernel(LmCtl *c, const double *mono_partial, int n_mono_blocks,
                                                       const double *imu_partial, int opt_it, int max_trials,
                                                       double lambda_init, const double *pre) {
    __shared__ double sh[8];
    const double chi = pre ? pre[1] : sum_chi(mono_partial, n_mono_blocks, imu_partial, sh);
    if (threadIdx.x == 0) {
        ctl_reset(LmReset{c, opt_it, max_trials, lambda_init});
        c->err0 = c->errors_chi = c->cur_chi = chi;
        c->init_pending = 0;
    }
}

// One step's LM bookkeeping (optimization_algorithm_levenberg.cpp:61-169), after the trial's errors:
//   a step that started an iteration: ++its, currentChi = iniChi = activeRobustChi2 of the current state (kept with
//   its buffer: after a rejected trial the reference recomputes the same errors and gets the same sum), qmax = 0;
//   the trial: rho, accept (the trial state becomes current) or reject (lambda *= ni), then the do-while /
//   iteration / nBad stop tests in the reference's order, and the next step's gates.
__device__ void finish_trial_body(double *sh, LmCtl *c, const double *mono_partial, int n_mono_blocks,
                                  const double *imu_partial, const double *scale_partial, int n_scale, const int *fail,
                                  const double *pre, const double *mono_partial0, const double *imu_partial0) {
    if (!c->g_active) return;
    const bool initp = c->init_pending != 0;
    double chi, ssum, chi0 = 0;
    if (pre) {   // a sharded solve: [initial chi (first step), chi, computeScale] summed over the ranks
        chi0 = pre[0], chi = pre[1], ssum = pre[2];
    } else {
        if (initp) {   // optimize()'s initial errors (their own partial buffers)
            chi0 = sum_chi(mono_partial0, n_mono_blocks, imu_partial0, sh);
            __syncthreads();
        }
        chi = sum_chi(mono_partial, n_mono_blocks, imu_partial, sh);
        double sc = 0;
        for (int i = threadIdx.x; i < n_scale; i += blockDim.x) sc += scale_partial[i];
        __syncthreads();
        ssum = block_reduce_sum(sc, sh);
    }
    if (threadIdx.x != 0) return;
    if (initp) c->err0 = c->errors_chi = c->cur_chi = chi0, c->init_pending = 0;
    if (c->g_build) {   // iteration start: the current state's activeRobustChi2 (its errors are in buffer cur)
        ++c->its;
        c->currentChi = c->iniChi = c->cur_chi;
        c->qmax = 0;
    }
    const int trial_buf = c->cur ^ 1;
    c->last = trial_buf;
    const bool ok = *fail == 0;
    double tempChi = chi;
    c->errors_chi = chi;
    c->errors_of_current = 0;   // the last computed errors belong to the trial state
    if (!ok) tempChi = DBL_MAX;
    double scale = ok ? ssum : 0.0;
    scale += 1e-3;
    const double rho = (c->currentChi - tempChi) / scale;
    c->rho = rho;
    ++c->trials;
    c->accepted = 0;
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3.0);
        alpha = fmin(alpha, 2. / 3.);
        c->lambda *= fmax(1. / 3., alpha);
        c->ni = 2;
        c->currentChi = tempChi;
        c->accepted = 1;
        ++c->n_acc;
        c->errors_of_current = 1;
        c->cur = trial_buf, c->cur_chi = chi;   // the trial's buffers become current
    } else {
        c->lambda *= c->ni;
        c->ni *= 2;
    }
    ++c->qmax;
    if (rho < 0 && c->qmax < c->max_trials) {
        c->need_build = 0;   // another trial of this iteration
    } else {
        c->need_build = 1;
        if (c->qmax == c->max_trials || rho == 0) {
            c->done = 1;
        } else {
            if ((c->iniChi - c->currentChi) * 1e3 < c->iniChi) ++c->nBad;
            else c->nBad = 0;
            if (c->nBad >= 3) c->done = 1;
        }
        if (++c->it >= c->opt_it) c->done = 1;
    }
    set_gates(c);
}

// The current state into buffer 0 at optimize()'s end, when the last accepted trial left it in buffer 1 (one
// contiguous copy of the state block; idempotent).
__global__ void cur_copy_kernel(const LmCtl *c, const double *B, double *A, size_t n) {
    if (!c->cur) return;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (size_t)gridDim.x * blockDim.x) A[q] = B[q];
}

// One LM step's bookkeeping after the trial's errors (one block of 256).
__global__ void __launch_bounds__(256) finish_trial_kernel(LmCtl *c, const double *mono_partial, int n_mono_blocks,
                                                           const double *imu_partial, const double *scale_partial,
                                                           int n_scale, const int *fail, const double *pre,
                                                           const double *mono_partial0, const double *imu_partial0) {
    __shared__ double sh[8];
    finish_trial_body(sh, c, mono_partial, n_mono_blocks, imu_partial, scale_partial, n_scale, fail, pre,
                      mono_partial0, imu_partial0);
}

// A sharded solve's per-rank scalars, all-reduced before the LM bookkeeping: out = [0 (unused), chi of the trial,
// this rank's computeScale terms] (ctl == nullptr: out[1] = chi of the errors just computed, optimize()'s initial
// err).  Gated like the trial.
__global__ void __launch_bounds__(256) trial_scalars_kernel(const LmCtl *c, const double *mono_partial, int n_mono_blocks,
                                                            const double *imu_partial, const double *scale_partial,
                                                            int n_scale, double *out, const double *mono_partial0,
                                                            const double *imu_partial0) {
    __shared__ double sh[8];
    if (c && !c->g_active) return;
    double chiA = 0;   // the initial chi while the first step's bookkeeping still has to take it
    if (c && c->init_pending) {
        chiA = sum_chi(mono_partial0, n_mono_blocks, imu_partial0, sh);
        __syncthreads();
    }
    const double chi = sum_chi(mono_partial, n_mono_blocks, imu_partial, sh);
    double sc = 0;
    if (c)
        for (int i = threadIdx.x; i < n_scale; i += blockDim.x) sc += scale_partial[i];
    __syncthreads();
    const double ssum = block_reduce_sum(sc, sh);
    if (threadIdx.x == 0) out[0] = chiA, out[1] = chi, out[2] = ssum;
}

// Final chi2 = imu partial + visual partials (fixed order); also finishes the computeScale sums.
__global__ void __launch_bounds__(256) finish_kernel(const double *mono_partial, int n_mono_blocks, const double *imu_partial,
                                                     const double *scale_partial, int n_scale, const int *fail,
                                                     double *out) {
    __shared__ double sh[8];
    double v = 0;
    for (int i = threadIdx.x; i < n_mono_blocks; i += blockDim.x) v += mono_partial[i];
    double t = block_reduce_sum(v, sh);
    double s = 0;
    for (int i = threadIdx.x; i < n_scale; i += blockDim.x) s += scale_partial[i];
    __syncthreads();
    const double st = block_reduce_sum(s, sh);
    if (threadIdx.x == 0) {
        out[0] = imu_partial[0] + t;   // activeRobustChi2
        out[1] = st;                   // computeScale
        out[2] = fail ? (double)*fail : 0.0;   // the linear solve of this trial failed
    }
}

// ---- build: landmark groups with the Schur complement on f64 MFMA ---------------------------------------
// buildSystem (block_solver.hpp:381-432) and the landmark Schur complement (:353-486) of one trial in one pass over the
// edges.  A landmark group is a run of whole landmarks (<= 256 edges, <= 128 landmarks, <= 128 slots, <= 32 distinct
// optimisable keyframes; a slot = one landmark's edges on one keyframe).  Per group, on one workgroup:
//   1. one thread per edge: EdgeMono / EdgeStereo Jacobians (JX 3x3, JP 3x6, the robust weight, -W e) into LDS;
//   2. one thread per landmark: Hll = sum w JX^T JX and bl = sum JX^T (-W e) in edge order, the Cholesky factor
//      R R^T = Hll + lambda I and y = R^-1 bl; beside it one thread per slot: Hpl_s = sum w JP^T JX over the slot's
//      edges (in order), then M_s = Hpl_s R^-T, so that Hpl Dinv Hpl^T = M M^T and Hpl Dinv bl = M y;
//   3. the group's share of the reduced system as ONE zero-routed product on v_mfma_f64_16x16x4f64: rows / columns are
//      the group's keyframes in elimination order, 8 per keyframe (6 pose rows, then a Schur right-hand-side column and
//      a gradient column), and the K dimension is [3 per landmark: M routed to its slots' rows, -M to the columns,
//      y to the rhs column] ++ [each residual row of each edge: JP to its keyframe's rows, w JP to the columns, -W e
//      to the gradient column] -- so one accumulation gives  sum JP^T W JP - sum Hpl Dinv Hpl^T  per keyframe pair, the
//      keyframe gradients and the Schur right-hand side, with the cross-landmark and cross-edge sums done by the
//      matrix core in its fixed order (no float atomics: bitwise identical run to run);
//   4. the group's blocks (keyframe pairs it co-observes) and per-keyframe [b | Schur rhs] rows into its own record;
//      assemble_kernel sums the records of a reduced-system block in group order.
// The per-landmark (R^-1, y, bl) and per-slot M_s stay for the back-substitution xl = R^-T (y - sum M_s^T xp_s).
// lambda enters through R, so the build runs every trial (a rejected trial rebuilds at the same linearisation point:
// the current state and its errors are untouched, so the Jacobians are the same numbers; g2o rebuilds only the Schur).
struct Land {
    const int *edge_start;   // [P+1]
    const int *slot_start;   // [P+1]
    const int *slot_kf;      // [nslots]
    const int *slot_edge;    // [nslots+1] first edge of each slot (slots are the keyframe runs of the landmark-major edges)
    const int16_t *slot_lkf; // [nslots] the slot keyframe's index in its group's keyframe list, -1 for a fixed keyframe
    double *lnd;             // [P][12]: R^-1 (lower: 00 10 11 20 21 22) | y = R^-1 bl | bl
    double *M;               // [nslots][18]: M_s = Hpl_s R^-T (6 x 3, row-major), optimisable slots only
    int n;
    const int *grp_pt;       // [n_grp+1] landmarks of each group
    const int *grp_w;        // [n_grp] optimisable keyframes of the group (w); -w - 1: a one-landmark group past the
                             //   LDS limits, built by the scalar path
    const int *grp_tp;       // [n_grp+1] the group's 16x16 output tiles (ti >= tj), as pairs in `tp`
    const uint8_t *tp;       // [2 per tile]
    const int *grp_blk;      // [n_grp] index in blkoff of the group's w(w+1)/2 keyframe pairs (a >= b)
    const int *blkoff;       //   the pair's record in `rec` (36 doubles), -1 if the group's landmarks do not co-observe it
    const int *grp_kf;       // [n_grp] index in rhsoff of the group's w keyframes
    const int *rhsoff;       //   the keyframe's record in `rec_rhs` (12 doubles: gradient 6 | Schur rhs 6)
    double *rec;             // per reduced-system block its groups' 6x6 records, contiguous in group order
    double *rec_rhs;         // per optimisable keyframe its groups' [gradient | Schur rhs] records, in group order
};

// Inertial work lists (host-built once per problem, ascending): per reduced-system block its inertial edges.
struct Gather {
    const int *blk_start;    // [n_slots+1] per reduced-system block: its run of group records in Land::rec
    const int *rhs_start;    // [nb+1] per optimisable keyframe: its run of [gradient | Schur rhs] in Land::rec_rhs
    const int4 *imu_blk;     // per block: inertial edges (edge, side of the block row, side of the column)
    const int *ib_start;     // [n_slots+1]
    const int2 *imu_vec;     // per keyframe: inertial edges (edge, side)
    const int *iv_start;     // [nb+1]
    const double *contrib;   // [n_imu][30 x 30 + 30] per-edge inertial quadratic forms
};

struct Red {   // reduced (non-marginalised) system: 16 rows per optimisable keyframe
    int n;
    const int *offP;   // per keyframe, -1 for fixed
    int n_kf;
};

// One visual edge at the current errors (EdgeMono, or EdgeStereo when ur >= 0): the point Jacobian JX (nr x 3),
// the pose Jacobian JP (nr x 6, ImuCamPose order), the robust weight w = invSigma2 * rho' and the weighted
// residual om = -invSigma2 * rho' * e (constructQuadraticForm, base_binary_edge.hpp:55-116).  Row 2 is zero on an
// EdgeMono.
__device__ __forceinline__ int edge_jacobians(const Rig &rig, const State &s, const Edges &E, int e, double delta,
                                              double dsqr, double delta_st, double dsqr_st, const double *err,
                                              const double *err3, const double *chi2, double JX[9], double JP[18],
                                              double &w, double om[3]) {
    const int k = E.kf[e], c = E.cam[e], C = rig.n_cams;
    const double *Rcw = s.Rcw + ((size_t)k * C + c) * 9, *tcw = s.tcw + ((size_t)k * C + c) * 3;
    const double *X = s.pts + (size_t)E.pt[e] * 3;
    double Xc[3], Xb[3];
    mv3(Rcw, X, Xc);
    for (int q = 0; q < 3; ++q) Xc[q] += tcw[q];
    mv3(rig.Rbc[c], Xc, Xb);
    for (int q = 0; q < 3; ++q) Xb[q] += rig.tbc[c][q];
    const bool st = E.ur[e] >= 0.f;   // EdgeStereo: proj_jac row 2 = row 0, (2,2) += bf / z^2
    double pj[9];
    cam_jac(rig, c, Xc, pj);
    const int nr = st ? 3 : 2;
    if (st) {
        const double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
        pj[6] = pj[0], pj[7] = pj[1], pj[8] = pj[2] + rig.bf * inv_z2;
    } else {
        pj[6] = pj[7] = pj[8] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int q = 0; q < 3; ++q)
            JX[3 * r + q] = -(pj[3 * r] * Rcw[q] + pj[3 * r + 1] * Rcw[3 + q] + pj[3 * r + 2] * Rcw[6 + q]);
    {
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
    double r0, r1;
    if (st) huber(chi2[e], delta_st, dsqr_st, r0, r1);
    else huber(chi2[e], delta, dsqr, r0, r1);
    const double wi = (double)E.w[e];
    w = wi * r1;
    om[0] = -wi * err[2 * e] * r1, om[1] = -wi * err[2 * e + 1] * r1;
    om[2] = st ? -wi * err3[e] * r1 : 0.0;
    return nr;
}

// sum over the residual rows r of A[r][ia] B[r][ib] (row-major, row strides lda / ldb): the EdgeStereo row last
// (zero on an EdgeMono, where the sum is the two-row sum exactly)
__device__ __forceinline__ double rows3(const double *A, int ia, int lda, const double *B, int ib, int ldb) {
    return A[ia] * B[ib] + A[lda + ia] * B[ldb + ib] + A[2 * lda + ia] * B[2 * ldb + ib];
}

// Cholesky factor of D = Hll + lambda I (lower, R R^T = D) inverted: Ri = R^-1 as (00 10 11 20 21 22); y = R^-1 bl.
// Then Dinv = R^-T R^-1, so Hpl Dinv Hpl^T = (Hpl R^-T)(Hpl R^-T)^T and Hpl Dinv bl = (Hpl R^-T) y.  A non-positive
// pivot (D not positive definite, e.g. lambda = 0 on a two-edge-free landmark) gives NaN and the trial's solve fails,
// as the explicit inverse's infinities did.
__device__ __forceinline__ void chol3_inv(const double *H, double lambda, const double *bl, double Ri[6], double y[3]) {
    const double d00 = H[0] + lambda, d10 = H[3], d11 = H[4] + lambda, d20 = H[6], d21 = H[7], d22 = H[8] + lambda;
    const double l00 = sqrt(d00), i00 = 1.0 / l00;
    const double l10 = d10 * i00, l20 = d20 * i00;
    const double l11 = sqrt(d11 - l10 * l10), i11 = 1.0 / l11;
    const double l21 = (d21 - l20 * l10) * i11;
    const double l22 = sqrt(d22 - l20 * l20 - l21 * l21), i22 = 1.0 / l22;
    const double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22, i20 = -(l20 * i00 + l21 * i10) * i22;
    Ri[0] = i00, Ri[1] = i10, Ri[2] = i11, Ri[3] = i20, Ri[4] = i21, Ri[5] = i22;
    y[0] = i00 * bl[0];
    y[1] = i10 * bl[0] + i11 * bl[1];
    y[2] = i20 * bl[0] + i21 * bl[1] + i22 * bl[2];
}
// M = Hpl R^-T (6 x 3): M[r][c] = sum_{q <= c} Hpl[r][q] Ri[c][q]
__device__ __forceinline__ void m_of(const double *Hpl, const double Ri[6], double M[18]) {
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const double h0 = Hpl[3 * r], h1 = Hpl[3 * r + 1], h2 = Hpl[3 * r + 2];
        M[3 * r] = h0 * Ri[0];
        M[3 * r + 1] = h0 * Ri[1] + h1 * Ri[2];
        M[3 * r + 2] = h0 * Ri[3] + h1 * Ri[4] + h2 * Ri[5];
    }
}

constexpr int kGrpLand = 128;    // landmarks per group (one thread each, threads 0..127)
constexpr int kGrpSlots = 128;   // slots per group (one thread each, threads 128..255)
constexpr int kGrpW = 32;        // optimisable keyframes per group (rows of the Schur product: 8 each)
// LDS of one landmark group (doubles, edge / slot / landmark-major rows)
constexpr int kSE = 22;                   // per edge: JP (3 x 6) | w | -W e (3)
constexpr int kLdsE = kSE * kGrpEdges;    // edges; then per slot its 27 diagonal terms; then the MFMA operand panels
constexpr int kLdsX = 9 * kGrpEdges;      // per edge JX (3 x 3)
constexpr int kLdsL = 3 * kGrpLand + 27 * kGrpW;   // per landmark y (3); per landmark R^-1 (6), then per keyframe
                                                   //   the group's 27 diagonal terms
constexpr int kPanel = kLdsE / 16;        // operand panels: ceil(w / 2) * kpad <= kPanel (a group-planning bound)
constexpr size_t kBuildLds = (size_t)(kLdsE + kLdsX + kLdsL) * 8 + kGrpLand * kGrpW;
static_assert(6 * kGrpLand <= 27 * kGrpW, "R^-1 rows fit under the diagonal terms");
static_assert(27 * kGrpSlots <= kLdsE, "the slots' diagonal terms fit the edge region");

typedef double v4d __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void land_group(int g, double *sm, const Rig &rig, const State &s, const Edges &E,
                                           const Land &L, double lambda, double delta, double dsqr, double delta_st,
                                           double dsqr_st, const double *err, const double *err3, const double *chi2) {
    double *SE = sm, *SX = sm + kLdsE, *SY = SX + kLdsX, *SR = SY + 3 * kGrpLand;
    uint8_t *map = (uint8_t *)(SY + kLdsL);
    const int tid = threadIdx.x;
#ifdef OMV_BUILD_PROFILE
    long long tp0 = wall_clock64(), tp1 = 0, tp2 = 0, tp3 = 0, tq[4] = {0, 0, 0, 0};
#define OMV_TQ(k) tq[k] = wall_clock64()
#else
#define OMV_TQ(k)
#endif
    const int p0 = L.grp_pt[g], p1 = L.grp_pt[g + 1], np = p1 - p0;
    const int e0 = L.edge_start[p0], ne = L.edge_start[p1] - e0;
    const int s0 = L.slot_start[p0], ns = L.slot_start[p1] - s0;
    const int w = L.grp_w[g], ntile = (w + 1) >> 1, kpad = (3 * np + 3) & ~3;
    for (int q = tid; q < np * kGrpW; q += blockDim.x) map[q] = 0xFF;
    // phase 1: one thread per edge: Jacobians, weight, -W e into LDS (edge-major rows)
    if (tid < ne) {
        double JX[9], JP[18], wt, om[3];
        edge_jacobians(rig, s, E, e0 + tid, delta, dsqr, delta_st, dsqr_st, err, err3, chi2, JX, JP, wt, om);
        double *o = SE + kSE * tid;
#pragma unroll
        for (int q = 0; q < 18; ++q) o[q] = JP[q];
        o[18] = wt;
#pragma unroll
        for (int q = 0; q < 3; ++q) o[19 + q] = om[q];
#pragma unroll
        for (int q = 0; q < 9; ++q) SX[9 * tid + q] = JX[q];
    }
    __syncthreads();
#ifdef OMV_BUILD_PROFILE
    tp1 = wall_clock64();
#endif
    // phase 2a: threads 0..127 one landmark each (Hll, bl in edge order; Cholesky), 128..255 one slot each (Hpl and the
    // slot's keyframe-diagonal terms: 21 of sum w JP^T JP and 6 of sum JP^T (-W e), in edge order)
    double Hpl[18], Ps[27];
    int my_slot = -1, my_pl = 0;
    if (tid < kGrpLand) {
        if (tid < np) {
            const int p = p0 + tid;
            double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
            for (int f = L.edge_start[p] - e0, f1 = L.edge_start[p + 1] - e0; f < f1; ++f) {
                double jx[9], om[3];
#pragma unroll
                for (int q = 0; q < 9; ++q) jx[q] = SX[9 * f + q];
#pragma unroll
                for (int q = 0; q < 3; ++q) om[q] = SE[kSE * f + 19 + q];
                const double wt = SE[kSE * f + 18];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    bl[r] += rows3(jx, r, 3, om, 0, 1);
#pragma unroll
                    for (int q = 0; q < 3; ++q) H[3 * r + q] += wt * rows3(jx, r, 3, jx, q, 3);
                }
            }
            double Ri[6], y[3];
            chol3_inv(H, lambda, bl, Ri, y);
#pragma unroll
            for (int q = 0; q < 6; ++q) SR[6 * tid + q] = Ri[q];
#pragma unroll
            for (int q = 0; q < 3; ++q) SY[3 * tid + q] = y[q];
            double *o = L.lnd + (size_t)p * 12;
#pragma unroll
            for (int q = 0; q < 6; ++q) o[q] = Ri[q];
#pragma unroll
            for (int q = 0; q < 3; ++q) o[6 + q] = y[q], o[9 + q] = bl[q];
            for (int sl = L.slot_start[p], s1 = L.slot_start[p + 1]; sl < s1; ++sl) {
                const int a = L.slot_lkf[sl];
                if (a >= 0) map[tid * kGrpW + a] = (uint8_t)(sl - s0);
            }
        }
    } else if (tid - kGrpLand < ns) {
        my_slot = s0 + tid - kGrpLand;
        if (L.slot_lkf[my_slot] >= 0) {
#pragma unroll
            for (int q = 0; q < 18; ++q) Hpl[q] = 0;
#pragma unroll
            for (int q = 0; q < 27; ++q) Ps[q] = 0;
            for (int f = L.slot_edge[my_slot] - e0, f1 = L.slot_edge[my_slot + 1] - e0; f < f1; ++f) {
                double jx[9], jp[18], om[3];
#pragma unroll
                for (int q = 0; q < 9; ++q) jx[q] = SX[9 * f + q];
#pragma unroll
                for (int q = 0; q < 18; ++q) jp[q] = SE[kSE * f + q];
#pragma unroll
                for (int q = 0; q < 3; ++q) om[q] = SE[kSE * f + 19 + q];
                const double wt = SE[kSE * f + 18];
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int q = 0; q < 3; ++q) Hpl[3 * r + q] += wt * rows3(jp, r, 6, jx, q, 3);
                int q = 0;
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int c = 0; c <= r; ++c) Ps[q++] += wt * rows3(jp, r, 6, jp, c, 6);
#pragma unroll
                for (int r = 0; r < 6; ++r) Ps[21 + r] += rows3(jp, r, 6, om, 0, 1);
            }
            my_pl = E.pt[L.slot_edge[my_slot]] - p0;   // the slot's landmark
        } else {
            my_slot = -1;
        }
    }
    __syncthreads();
    OMV_TQ(0);
    // phase 2b: M_s = Hpl_s R^-T (kept in registers for the panels); the slot's diagonal terms into LDS (slot-major)
    double M[18];
    if (my_slot >= 0) {
        double Ri[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) Ri[q] = SR[6 * my_pl + q];
        m_of(Hpl, Ri, M);
        double *o = L.M + (size_t)my_slot * 18;
#pragma unroll
        for (int q = 0; q < 18; ++q) o[q] = M[q];
        const int sl = tid - kGrpLand;
#pragma unroll
        for (int q = 0; q < 27; ++q) SE[27 * sl + q] = Ps[q];
    }
    __syncthreads();
    OMV_TQ(1);
    // phase 2c: the keyframe-diagonal terms of the group, per keyframe a the slots' terms in landmark order
    // (SR's R^-1 rows are dead: the sums take their place)
    double *SP = SR;
    for (int q = tid; q < w * 27; q += blockDim.x) {
        const int a = q / 27, e = q - 27 * a;
        double v = 0;
        int pl = 0;
        for (; pl + 4 <= np; pl += 4) {
            int sl[4];
            double x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) sl[u] = map[(pl + u) * kGrpW + a];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = SE[27 * (sl[u] & 127) + e];
#pragma unroll
            for (int u = 0; u < 4; ++u) v += sl[u] != 0xFF ? x[u] : 0.0;
        }
        for (; pl < np; ++pl) {
            const int sl = map[pl * kGrpW + a];
            const double x = SE[27 * (sl & 127) + e];
            v += sl != 0xFF ? x : 0.0;
        }
        SP[q] = v;
    }
    __syncthreads();
    OMV_TQ(2);
    // phase 3a: the MFMA operand panels, one per 16-row tile (keyframes 2t, 2t + 1): panel t holds for K = 3 pl + c
    // the 16 values of rows 16 t .. 16 t + 15: M_{pl, a}[r][c] at row 8 a + r, y_pl[c] at row 8 a + 6 (where landmark pl
    // has a slot on keyframe a), zero elsewhere -- zero-filled, then scattered by the slot threads
    double *PN = SE;
    const int npan = ntile * kpad * 16;
    for (int q = tid; q < npan; q += blockDim.x) PN[q] = 0.0;
    __syncthreads();
    if (my_slot >= 0) {
        const int a = L.slot_lkf[my_slot];
        double *o = PN + ((size_t)(a >> 1) * kpad + 3 * my_pl) * 16 + 8 * (a & 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
#pragma unroll
            for (int r = 0; r < 6; ++r) o[16 * c + r] = M[3 * r + c];
            o[16 * c + 6] = SY[3 * my_pl + c];
        }
    }
    __syncthreads();
#ifdef OMV_BUILD_PROFILE
    tp2 = wall_clock64();
#endif
    // phase 3b: Out(tile ti, tj) = init + sum_K A[.][K] B[K][.] on v_mfma_f64_16x16x4f64, A = panel ti (pose rows only),
    // B = -panel tj on the pose columns, +panel tj on the Schur rhs column, 0 on the gradient column; a diagonal tile
    // starts from the keyframes' diagonal terms, so each block comes out as sum JP^T W JP - sum Hpl Dinv Hpl^T and the
    // gradient / Schur rhs columns as b / sum Hpl Dinv bl.  Operand loads are affine in the step: no dependent chains.
    const int lane = tid & 63, wave = tid >> 6, li = lane & 15, kk = lane >> 4;
    const int t0 = L.grp_tp[g], nt = L.grp_tp[g + 1] - t0;
    const int nsteps = kpad >> 2;
    const int *blkoff = L.blkoff + L.grp_blk[g], *rhsoff = L.rhsoff + L.grp_kf[g];
    for (int it = wave; it < nt; it += (int)(blockDim.x >> 6)) {
        const int ti = L.tp[2 * (t0 + it)], tj = L.tp[2 * (t0 + it) + 1];
        const int ar = li & 7, bc = li & 7;
        const double amask = ar < 6 ? 1.0 : 0.0, bsign = bc < 6 ? -1.0 : (bc == 6 ? 1.0 : 0.0);
        const int b_kf = 2 * tj + (li >> 3);
        v4d acc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // rows 16 ti + kk + 4 j of column 16 tj + li
            const int R = 16 * ti + kk + 4 * j, a = R >> 3, r = R & 7;
            double v = 0;
            if (a == b_kf && a < w && r < 6) {
                if (bc < 6) v = SP[27 * a + (r >= bc ? r * (r + 1) / 2 + bc : bc * (bc + 1) / 2 + r)];
                else if (bc == 7) v = SP[27 * a + 21 + r];
            }
            acc[j] = v;
        }
        const double *pa = PN + (size_t)ti * kpad * 16 + 16 * kk + li, *pb = PN + (size_t)tj * kpad * 16 + 16 * kk + li;
        for (int st = 0; st < nsteps; st += 4) {
            double av[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int o = st + u < nsteps ? 64 * (st + u) : 0;
                av[u] = pa[o], bv[u] = pb[o];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double m = st + u < nsteps ? 1.0 : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u] * amask * m, bv[u] * bsign, acc, 0, 0, 0);
            }
        }
        // out: each block / keyframe row to its place in the block's (keyframe's) contiguous record run
        if (b_kf >= w) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int R = 16 * ti + kk + 4 * j, a = R >> 3, r = R & 7;
            if (r >= 6 || a >= w) continue;
            if (bc < 6) {
                if (a >= b_kf) {
                    const int o = blkoff[a * (a + 1) / 2 + b_kf];
                    if (o >= 0) L.rec[(size_t)o * 36 + 6 * r + bc] = acc[j];
                }
            } else if (a == b_kf) {
                L.rec_rhs[(size_t)rhsoff[a] * 12 + (bc == 7 ? 0 : 6) + r] = acc[j];
            }
        }
    }
#ifdef OMV_BUILD_PROFILE
    __syncthreads();
    tp3 = wall_clock64();
    if (tid == 0 && ((g & 63) == 0 || tp3 - tp0 > 2000))
        printf("build group %d: edges %d landmarks %d slots %d w %d tiles %d | ticks(100MHz) jac %lld land %lld (2a %lld 2b %lld 2c %lld 3a %lld) mfma %lld\n",
               g, ne, np, ns, w, nt, tp1 - tp0, tp2 - tp1, tq[0] - tp1, tq[1] - tq[0], tq[2] - tq[1], tp2 - tq[2], tp3 - tp2);
#endif
#undef OMV_TQ
}

// A one-landmark group past the LDS limits (> 256 edges, > 128 slots or > 32 optimisable keyframes): the same
// quantities by the scalar path.  Windows of 64 edges: per edge its 30 landmark terms and 27 pose terms in LDS,
// thread 0 walks them in edge order (Hll, bl, per slot Hpl and the pose terms), then one thread per slot forms M_s,
// one thread per keyframe pair the block.
constexpr int kBigWin = 64;
__device__ __forceinline__ void land_group_big(int g, double *sm, const Rig &rig, const State &s, const Edges &E,
                                            const Land &L, double lambda, double delta, double dsqr, double delta_st,
                                            double dsqr_st, const double *err, const double *err3, const double *chi2) {
    double *T = sm;                       // [57][kBigWin]
    double *SL = sm + kLdsE + kLdsX;      // R^-1 | y of the landmark
    int *inv = (int *)(sm + kLdsE);       // keyframe index -> slot (the JX region as ints)
    const int tid = threadIdx.x;
    const int p = L.grp_pt[g], w = -L.grp_w[g] - 1, nblk = w * (w + 1) / 2;
    const int e0 = L.edge_start[p], e1 = L.edge_start[p + 1];
    const int *blkoff = L.blkoff + L.grp_blk[g], *rhsoff = L.rhsoff + L.grp_kf[g];
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0}, Hp[18], P[27];
    int cur = -1;
    auto flush = [&]() {   // thread 0: the finished slot `cur`
        const int a = L.slot_lkf[cur];
        if (a < 0) return;
        double *o = L.M + (size_t)cur * 18;
        for (int q = 0; q < 18; ++q) o[q] = Hp[q];
        double *B = L.rec + (size_t)blkoff[a * (a + 1) / 2 + a] * 36;
        int q = 0;
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c <= r; ++c, ++q) B[6 * r + c] = B[6 * c + r] = P[q];
        for (int r = 0; r < 6; ++r) L.rec_rhs[(size_t)rhsoff[a] * 12 + r] = P[21 + r];
    };
    for (int base = e0; base < e1; base += kBigWin) {
        if (tid < kBigWin && base + tid < e1) {
            double JX[9], JP[18], wt, om[3];
            edge_jacobians(rig, s, E, base + tid, delta, dsqr, delta_st, dsqr_st, err, err3, chi2, JX, JP, wt, om);
            for (int r = 0; r < 3; ++r) {
                T[(9 + r) * kBigWin + tid] = rows3(JX, r, 3, om, 0, 1);
                for (int q = 0; q < 3; ++q) T[(3 * r + q) * kBigWin + tid] = wt * rows3(JX, r, 3, JX, q, 3);
            }
            for (int r = 0; r < 6; ++r)
                for (int q = 0; q < 3; ++q) T[(12 + 3 * r + q) * kBigWin + tid] = wt * rows3(JP, r, 6, JX, q, 3);
            int q = 0;
            for (int r = 0; r < 6; ++r)
                for (int c = 0; c <= r; ++c, ++q) T[(30 + q) * kBigWin + tid] = wt * rows3(JP, r, 6, JP, c, 6);
            for (int r = 0; r < 6; ++r) T[(51 + r) * kBigWin + tid] = rows3(JP, r, 6, om, 0, 1);
        }
        __syncthreads();
        if (tid == 0)
            for (int f = base; f < min(base + kBigWin, e1); ++f) {
                const int le = f - base;
                for (int q = 0; q < 3; ++q) bl[q] += T[(9 + q) * kBigWin + le];
                for (int q = 0; q < 9; ++q) H[q] += T[q * kBigWin + le];
                const int sl = E.slot[f];
                if (sl != cur) {
                    if (cur >= 0) flush();
                    for (int q = 0; q < 18; ++q) Hp[q] = 0;
                    for (int q = 0; q < 27; ++q) P[q] = 0;
                    cur = sl;
                }
                for (int q = 0; q < 18; ++q) Hp[q] += T[(12 + q) * kBigWin + le];
                for (int q = 0; q < 27; ++q) P[q] += T[(30 + q) * kBigWin + le];
            }
        __syncthreads();
    }
    if (tid == 0) {
        if (cur >= 0) flush();
        double Ri[6], y[3];
        chol3_inv(H, lambda, bl, Ri, y);
        double *o = L.lnd + (size_t)p * 12;
        for (int q = 0; q < 6; ++q) o[q] = Ri[q], SL[q] = Ri[q];
        for (int q = 0; q < 3; ++q) o[6 + q] = y[q], o[9 + q] = bl[q], SL[6 + q] = y[q];
    }
    for (int sl = L.slot_start[p] + tid; sl < L.slot_start[p + 1]; sl += blockDim.x)
        if (L.slot_lkf[sl] >= 0) inv[L.slot_lkf[sl]] = sl;
    __threadfence_block();
    __syncthreads();
    for (int sl = L.slot_start[p] + tid; sl < L.slot_start[p + 1]; sl += blockDim.x) {
        if (L.slot_lkf[sl] < 0) continue;
        double h[18], M[18], Ri[6];
        double *o = L.M + (size_t)sl * 18;
        for (int q = 0; q < 18; ++q) h[q] = o[q];
        for (int q = 0; q < 6; ++q) Ri[q] = SL[q];
        m_of(h, Ri, M);
        for (int q = 0; q < 18; ++q) o[q] = M[q];
    }
    __threadfence_block();
    __syncthreads();
    for (int q = tid; q < nblk; q += blockDim.x) {
        int a = 0;
        while ((a + 1) * (a + 2) / 2 <= q) ++a;
        const int b = q - a * (a + 1) / 2;
        const double *Ma = L.M + (size_t)inv[a] * 18, *Mb = L.M + (size_t)inv[b] * 18;
        double *B = L.rec + (size_t)blkoff[q] * 36;
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c < 6; ++c) {
                const double t = Ma[3 * r] * Mb[3 * c] + Ma[3 * r + 1] * Mb[3 * c + 1] + Ma[3 * r + 2] * Mb[3 * c + 2];
                B[6 * r + c] = (a == b ? B[6 * r + c] : 0.0) - t;
            }
    }
    for (int a = tid; a < w; a += blockDim.x) {
        const double *Ma = L.M + (size_t)inv[a] * 18;
        for (int r = 0; r < 6; ++r)
            L.rec_rhs[(size_t)rhsoff[a] * 12 + 6 + r] = Ma[3 * r] * SL[6] + Ma[3 * r + 1] * SL[7] + Ma[3 * r + 2] * SL[8];
    }
}

// ---- build: inertial + random-walk edges, one wavefront each -------------------------------------

// Inertial + random-walk edges of one EdgeInertial i (one wavefront): the 30 x 30 quadratic form and 30 gradient
// over the edge's local variables [P1 V1 G1 A1 P2 V2 G2 A2] (EdgeInertial over the first 24, EdgeGyroRW on
// G1 / G2, EdgeAccRW on A1 / A2), written to its own slot; assemble_kernel adds the slots into the reduced system.
constexpr int kImuLoc = 30, kImuContrib = kImuLoc * kImuLoc + kImuLoc;
__device__ __forceinline__ void imu_contrib_block(int i, double *sm, State s, Imu I, double delta, double dsqr,
                                                  const double *err9, double *contrib) {
    double *J = sm, *WJ = sm + 216, *om = sm + 432;   // J (9 x 24), Omega' J (9 x 24), -Omega' e
    const int lane = threadIdx.x, nt = blockDim.x;
    for (int q = lane; q < 216; q += nt) J[q] = 0;
    __syncthreads();
    imu_jacobian_par(s, I, i, err9 + (size_t)10 * I.n + 9 * (size_t)i, err9 + 9 * (size_t)i, J, WJ);   // WJ: RJ scratch
    __syncthreads();
    const double *e = err9 + 9 * i;
    const double c2 = err9[(size_t)9 * I.n + i];
    double r0, r1 = 1.0;
    if (I.robust[i]) huber(c2, delta, dsqr, r0, r1);
    const double *W = I.info9 + (size_t)i * 81;
    for (int q = lane; q < 216; q += nt) {
        const int r = q / 24, c = q % 24;
        double t = 0;
        for (int k = 0; k < 9; ++k) t += W[r * 9 + k] * J[k * 24 + c];
        WJ[q] = t * r1;
    }
    if (lane < 9) {
        double t = 0;
        for (int k = 0; k < 9; ++k) t += W[lane * 9 + k] * e[k];
        om[lane] = -t * r1;
    }
    __syncthreads();
    const int k1 = I.kf1[i], k2 = I.kf2[i];
    double *Hc = contrib + (size_t)i * kImuContrib, *bc = Hc + kImuLoc * kImuLoc;
    const double *Ig = I.infoG + 9 * i, *Ia = I.infoA + 9 * i;
    for (int q = lane; q < kImuLoc * kImuLoc; q += nt) {
        const int a = q / kImuLoc, b = q % kImuLoc;
        double t = 0;
        if (a < 24 && b < 24)
            for (int k = 0; k < 9; ++k) t += J[k * 24 + a] * WJ[k * 24 + b];
        // random walks: H += J^T Info J with J1 = -I (G1 / A1), J2 = I (G2 / A2)
        const int ga = a >= 9 && a < 12 ? 0 : (a >= 24 && a < 27 ? 1 : -1), gb = b >= 9 && b < 12 ? 0 : (b >= 24 && b < 27 ? 1 : -1);
        const int aa = a >= 12 && a < 15 ? 0 : (a >= 27 ? 1 : -1), ab = b >= 12 && b < 15 ? 0 : (b >= 27 ? 1 : -1);
        if (ga >= 0 && gb >= 0) {
            const int r = a - (ga ? 24 : 9), c = b - (gb ? 24 : 9);
            t += (ga == gb ? 1.0 : -1.0) * Ig[3 * r + c];
        }
        if (aa >= 0 && ab >= 0) {
            const int r = a - (aa ? 27 : 12), c = b - (ab ? 27 : 12);
            t += (aa == ab ? 1.0 : -1.0) * Ia[3 * r + c];
        }
        Hc[q] = t;
    }
    if (lane < kImuLoc) {
        double t = 0;
        if (lane < 24)
            for (int k = 0; k < 9; ++k) t += J[k * 24 + lane] * om[k];
        // random walks: b -= J^T Info e, e = b2 - b1 (+ on the first keyframe's bias, - on the second's)
        int which = -1, r = 0;   // 0 gyro, 1 acc
        if (lane >= 9 && lane < 15) which = lane >= 12, r = lane - (lane >= 12 ? 12 : 9);
        else if (lane >= 24) which = lane >= 27, r = lane - (lane >= 27 ? 27 : 24);
        if (which >= 0) {
            const double *bv = which ? s.ba : s.bg, *Iw = which ? Ia : Ig;
            double ee[3];
            for (int q = 0; q < 3; ++q) ee[q] = bv[3 * k2 + q] - bv[3 * k1 + q];
            const double Oe = Iw[3 * r] * ee[0] + Iw[3 * r + 1] * ee[1] + Iw[3 * r + 2] * ee[2];
            t += lane < 24 ? Oe : -Oe;
        }
        bc[lane] = t;
    }
}

// The whole build in one launch: blocks [0, n_imu) the inertial edges' quadratic forms, blocks from n_imu_pad (n_imu
// rounded up to 8, so the landmark groups keep their XCD-aware order) the landmark groups.  Independent halves, side by
// side.  Dynamic LDS: kBuildLds.
__global__ void __launch_bounds__(kGrpEdges) build_all_kernel(Rig rig, State s0, State s1, Edges E, Land L, int n_grp,
                                                              Imu I, int n_imu, int n_imu_pad, double lambda,
                                                              double delta, double dsqr, double delta_st, double dsqr_st,
                                                              double delta_imu, double dsqr_imu, ErrBufs e0, ErrBufs e1,
                                                              double *contrib, const LmCtl *ctl) {
    extern __shared__ double sm[];
    if (!gate_open(ctl, kGateTrial)) return;
    lambda = lm_lambda(ctl, lambda);
    const int bi = role_buf(ctl, 0);   // the current state and its errors
    const State s = bi ? s1 : s0;
    const ErrBufs eb = bi ? e1 : e0;
    const int b = blockIdx.x;
    if (b < n_imu_pad) {
#ifdef OMV_BUILD_PROFILE
        const long long ti0 = wall_clock64();
#endif
        if (b < n_imu) imu_contrib_block(b, sm, s, I, delta_imu, dsqr_imu, eb.err9, contrib);
#ifdef OMV_BUILD_PROFILE
        __syncthreads();
        if (threadIdx.x == 0 && b == 0) printf("build imu block 0: ticks(100MHz) %lld\n", wall_clock64() - ti0);
#endif
        return;
    }
    const int bl = b - n_imu_pad, chunk = (n_grp + 7) >> 3;
    const int g = (bl & 7) * chunk + (bl >> 3);
    if (g >= n_grp) return;
    if (L.grp_w[g] < 0) return;   // build_big_kernel's
    land_group(g, sm, rig, s, E, L, lambda, delta, dsqr, delta_st, dsqr_st, eb.err, eb.err3, eb.chi2);
}

// The one-landmark groups past the LDS limits (rare: a landmark with > 256 edges, > 128 slots or > 32 optimisable
// keyframes), one workgroup each, launched only when the problem has any.
__global__ void __launch_bounds__(kGrpEdges) build_big_kernel(Rig rig, State s0, State s1, Edges E, Land L,
                                                              const int *big, int n_big, double lambda, double delta,
                                                              double dsqr, double delta_st, double dsqr_st, ErrBufs e0,
                                                              ErrBufs e1, const LmCtl *ctl) {
    extern __shared__ double sm[];
    if (!gate_open(ctl, kGateTrial) || (int)blockIdx.x >= n_big) return;
    lambda = lm_lambda(ctl, lambda);
    const int bi = role_buf(ctl, 0);
    const State s = bi ? s1 : s0;
    const ErrBufs eb = bi ? e1 : e0;
    land_group_big(big[blockIdx.x], sm, rig, s, E, L, lambda, delta, dsqr, delta_st, dsqr_st, eb.err, eb.err3, eb.chi2);
}

// ---- trial: the reduced system, assembled per block -------------------------------------------------------
// The reduced system is stored as 16x16 blocks (keyframe block = pose 6 | v 3 | bg 3 | ba 3 | pad 1,
// padded to one f64 MFMA tile) on the symbolic LDL^T pattern (fill-in included) of the elimination order
// `perm` (position -> keyframe, host-chosen, see plan_order): slot(pi, pj) for block row pi >= block column
// pj, row-major 16x16 each, holding H's block (perm[pi], perm[pj]).  Padding rows have zero gradient and
// lambda on the diagonal, so they solve to exactly zero and add nothing to computeScale.  b and the Schur
// right-hand side stay in keyframe order (16 k + r).
// Entry (r, c) of a 16x16 block sits at 16 r + (c ^ r): a column read by 16 lanes (one per row), as the MFMA
// A operands and the pivot columns are, touches 16 distinct LDS banks instead of two (rows are 32 banks apart).
__host__ __device__ __forceinline__ int sw16(int r, int c) { return 16 * r + (c ^ r); }

struct BlockPat {
    int nb, n_slots, n_lev;
    int n_lds;                       // hybrid solver (G = 2): slots 0 .. n_lds-1 in LDS, the rest in global scratch
    const int *perm;                 // [nb] position -> keyframe
    const int *slot_kr, *slot_kc;    // [n_slots] keyframes of the block's row / column
    const int *dslot;                // [nb] diagonal slot per position
    const int *lev_start, *lev_col;  // elimination-tree levels: the positions of level l
    const int *ug_start;             // [n_lev+1] update groups of a level (one target block each)
    const int *ug_split;             // [n_lev] groups ug_start[l] .. ug_split[l]: the diagonal blocks of level l + 1
    const int *crit_grp;             // [nb] per position: the group updating its diagonal from the level below, or -1
    const int *ug_task_start;        // [n_groups+1]
    const int4 *ug;                  //   (slot(i, j), slot(i, k), slot(j, k), dslot(k)), ascending k
    const int4 *inv_rec;             // [2 nb] per lev_col entry: (dslot, crit group's first / end update, -), its first
                                     // update (the inverse task in two reads instead of five dependent ones)
    const int *rs_start;             // [nb+1] row structure of position i: (slot(i, k), k), k < i
    const int2 *rs;
    const int *cs_start;             // [nb+1] column structure of position k: (slot(i, k), i), i > k
    const int2 *cs;
    // every array above but slot_kr / slot_kc lives in one contiguous device blob; when blob_ints > 0 the solver stages
    // it into LDS after the blocks, so the per-level schedule reads on its critical path are LDS reads, not dependent
    // global loads
    const int *blob;
    int blob_ints;
};

// One block per reduced-system block: the group records of the block in group order (each sum JP^T W JP - sum
// Hpl Dinv Hpl^T over the group's edges / landmarks), the inertial edges touching it, + lambda on the diagonal; on a
// diagonal block the keyframe's b and Schur right-hand side from the records' rows.  `pose_lambda` is 0 on the ranks
// > 0 of a sharded solve (lambda enters once).
// sum of n runs of `stride` doubles (entry `off` of each), in run order; eight loads in flight, the same order of adds
__device__ __forceinline__ double run_sum(const double *base, int n, int stride, int off) {
    double v = 0;
    int q = 0;
    for (; q + 8 <= n; q += 8) {
        double a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = base[(size_t)(q + u) * stride + off];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += a[u];
    }
    for (; q < n; ++q) v += base[(size_t)q * stride + off];
    return v;
}

// One block per reduced-system block: its run of group records in group order (each sum JP^T W JP - sum
// Hpl Dinv Hpl^T over one group's edges / landmarks), the inertial edges touching it, + lambda on the diagonal; on a
// diagonal block the keyframe's b and Schur right-hand side from its run of [gradient | Schur rhs] records.
// `pose_lambda` is 0 on the ranks > 0 of a sharded solve (lambda enters once).
// The record runs are long (a block's records come from every landmark group touching it): each of the 36 entries'
// runs (and, on a diagonal block, the 12 right-hand-side runs) is cut into kAsmSplit fixed contiguous pieces summed by
// separate threads, the pieces then added in piece order -- a fixed order, so the result is the same run to run.
constexpr int kAsmSplit = 7;
__global__ void __launch_bounds__(256) assemble_kernel(Gather G, Imu I, BlockPat P, const double *rec,
                                                       const double *rec_rhs, double lambda, int pose_lambda, double *S,
                                                       double *bvec, double *coef, const LmCtl *ctl) {
    if (!gate_open(ctl, kGateTrial)) return;
    __shared__ double part[kAsmSplit][36], rpart[kAsmSplit][12];
    lambda = lm_lambda(ctl, lambda);
    const int t = blockIdx.x, tid = threadIdx.x;
    const int kr = P.slot_kr[t], kc = P.slot_kc[t];
    const bool diag = kr == kc;
    if (tid < 36 * kAsmSplit) {
        const int pair = tid % 36, piece = tid / 36;
        const int g0 = G.blk_start[t], n = G.blk_start[t + 1] - g0, chunk = (n + kAsmSplit - 1) / kAsmSplit;
        const int q0 = min(n, piece * chunk), q1 = min(n, q0 + chunk);
        const bool need = !diag || (pair % 6) <= (pair / 6);
        part[piece][pair] = need ? run_sum(rec + (size_t)(g0 + q0) * 36, q1 - q0, 36, pair) : 0.0;
    }
    if (diag) {   // (block-uniform) the right-hand-side pieces on threads 0..83 once their record pieces are done
        __syncthreads();
        if (tid < 12 * kAsmSplit) {
            const int col = tid % 12, piece = tid / 12;
            const int k0 = G.rhs_start[kr], n = G.rhs_start[kr + 1] - k0, chunk = (n + kAsmSplit - 1) / kAsmSplit;
            const int q0 = min(n, piece * chunk), q1 = min(n, q0 + chunk);
            rpart[piece][col] = run_sum(rec_rhs + (size_t)(k0 + q0) * 12, q1 - q0, 12, col);
        }
    }
    __syncthreads();
    const int r = tid >> 4, c = tid & 15;
    double v = 0;
    if (!diag || c <= r) {
        if (r < 6 && c < 6)
            for (int piece = 0; piece < kAsmSplit; ++piece) v += part[piece][6 * r + c];
        if (r < 15 && c < 15) {   // inertial edges touching the block (variable groups present in the system)
            const bool rows_ok = r < 6 || I.offV[kr] >= 0, cols_ok = c < 6 || I.offV[kc] >= 0;
            if (rows_ok && cols_ok)
                for (int q = G.ib_start[t]; q < G.ib_start[t + 1]; ++q) {
                    const int4 e = G.imu_blk[q];
                    v += G.contrib[(size_t)e.x * kImuContrib + (15 * e.y + r) * kImuLoc + 15 * e.z + c];
                }
        }
        if (diag && r == c && pose_lambda) v += lambda;
    }
    S[(size_t)t * 256 + sw16(r, c)] = v;
    if (diag && tid < 16) {   // b and the Schur right-hand side of keyframe kr
        double bv = 0, cf = 0;
        if (tid < 6)
            for (int piece = 0; piece < kAsmSplit; ++piece) bv += rpart[piece][tid], cf += rpart[piece][6 + tid];
        if (tid < 15 && (tid < 6 || I.offV[kr] >= 0))
            for (int q = G.iv_start[kr]; q < G.iv_start[kr + 1]; ++q) {
                const int2 e = G.imu_vec[q];
                bv += G.contrib[(size_t)e.x * kImuContrib + kImuLoc * kImuLoc + 15 * e.y + tid];
            }
        bvec[16 * kr + tid] = bv;
        coef[16 * kr + tid] = cf;
    }
}

// ---- trial: keyframe update (in the errors kernel) -----------------------------------------------------------
// ImuCamPose::Update (G2oTypes.cc:211-235): the new body pose of optimisable keyframe k from the current state a and the
// solution xp (keyframe order), and camera c's Rcw / tcw of it.
__device__ __forceinline__ void kf_trial_pose(const Rig &rig, const State &a, const double *u, int k, int c, bool norm,
                                              double Rn[9], double twb[3], double Rc[9], double tc[3]) {
    double Rwb[9], dRw[9], tt[3];
    for (int q = 0; q < 9; ++q) Rwb[q] = a.Rwb[9 * k + q];
    mv3(Rwb, u + 3, tt);
    for (int q = 0; q < 3; ++q) twb[q] = a.twb[3 * k + q] + tt[q];
    exp_so3(u, dRw);
    mm3(Rwb, dRw, Rn);
    if (norm) polar3(Rn);   // NormalizeRotation after every third update (:220-225)
    double Rbw[9], tbw[3];
    tr3(Rn, Rbw);
    mv3(Rbw, twb, tbw);
    for (int q = 0; q < 3; ++q) tbw[q] = -tbw[q];
    mm3(rig.Rcb[c], Rbw, Rc);
    mv3(rig.Rcb[c], tbw, tc);
    for (int q = 0; q < 3; ++q) tc[q] += rig.tcb[c][q];
}

// ---- trial: block LDL^T of the reduced system (one workgroup, 16x16 f64 MFMA tiles) -------------

// Wave-synchronous step: LDS operations of one wavefront complete in order, so the fence only has
// to stop the compiler (wavefront scope); the global-memory fallback needs workgroup scope.
template <int G>
__device__ __forceinline__ void wave_sync() {
    if (G) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// 1 / x by v_rcp_f64 and two Newton steps (within an ulp of the IEEE quotient; the pivots are normal
// numbers -- a zero / non-finite pivot is flagged by the caller)
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// The reduced system is factored as a block LDL^T with 16x16 block pivots: A = L D L^T, L_ik = S_ik D_k^-1, D_k = S_kk
// (each S the block as it stands when column k is eliminated).  Nothing but the blocks themselves and D_k^-1 is kept:
// the diagonal slot of column k is overwritten by D_k^-1, the panels S_ik stay unscaled in place, and
//   trailing update   S_ij -= S_ik D_k^-1 S_jk^T             (two f64 MFMA products, the inner one in registers)
//   forward           z_k = D_k^-1 (y_k - sum_{j < k} S_kj z_j)
//   backward          x_k = z_k - D_k^-1 sum_{i > k} S_ik^T x_i
// so a level is one diagonal-inverse phase and one phase of updates + forward columns.  The solution is that of the
// damped system (SimplicialLDLT's scalar LDL^T on its own AMD order, linear_solver_eigen.h:94-120, differs only in
// rounding).

// One wavefront: D (16x16 symmetric, lower triangle read) -> D^-1 in place (full), by sixteen 1x1 sweeps held in
// registers (the sweep operator): with pivot p = M_kk, r = 1 / p,
//   i, j != k : M_ij - M_ik (M_kj r)      row k : M_kj r      column k : M_ik r      M_kk : -r
// after all sixteen M = -D^-1 (no pivoting: D is the damped, positive definite Hessian block).  Lane l owns column
// j = l & 15, rows q + 4t (q = l >> 4).  Per pass the pivot is a uniform read (v_readlane), the row M_k. a cross-row
// ds_bpermute issued ahead of the reciprocal, and the column M_.k a DPP row broadcast of lane k of each 16-lane row --
// no LDS store / load round trip between passes (a v_permlane16/32_swap row broadcast measured slower: more
// instructions on an issue-bound pass; so did 2x2 pivot blocks, 4,200 vs 3,760 cycles).  A zero / non-finite
// pivot flags the solve (through the non-finite entries it leaves).
__device__ __forceinline__ double readlane_f64(double x, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int K>
__device__ __forceinline__ double row_bcast_f64(double x) {   // lane K of each 16-lane row, to the whole row
    const long long b = __builtin_bit_cast(long long, x);
    const long long r = __builtin_amdgcn_update_dpp(b, b, 0x150 + K, 0xf, 0xf, false);   // all lanes written
    return __builtin_bit_cast(double, r);
}
template <int K>
__device__ __forceinline__ void sweep_pass(double cur[4], int q, int j) {
    constexpr int tk = K >> 2, qk = K & 3;
    const double p = readlane_f64(cur[tk], 16 * qk + K);
    const double mkj = __shfl(cur[tk], 16 * qk + j, 64);   // issued early: its latency hides behind the reciprocal
    const double r = rcp_nr(p);
    const double f = mkj * r;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const double mik = row_bcast_f64<K>(cur[t]);
        double v = j == K ? mik * r : __builtin_fma(-mik, f, cur[t]);
        if (t == tk) v = q == qk ? (j == K ? -r : f) : v;
        cur[t] = v;
    }
}
template <int K>
__device__ __forceinline__ void sweep_all(double cur[4], int q, int j) {
    if constexpr (K < 16) {
        sweep_pass<K>(cur, q, j);
        sweep_all<K + 1>(cur, q, j);
    }
}

template <int G>
__device__ __forceinline__ void inv16(double *D, int lane, int *bad) {
    const int q = lane >> 4, j = lane & 15;
    double cur[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int i = q + 4 * t;
        cur[t] = D[i >= j ? sw16(i, j) : sw16(j, i)];
    }
    sweep_all<0>(cur, q, j);
#pragma unroll
    for (int t = 0; t < 4; ++t) D[sw16(q + 4 * t, j)] = -cur[t];
    // a zero or non-finite pivot leaves an infinite or NaN entry (1 / 0 = inf spreads through its row and column):
    // one check of the result instead of one per pass
    const bool fin = isfinite(cur[0]) && isfinite(cur[1]) && isfinite(cur[2]) && isfinite(cur[3]);
    if (__ballot(!fin) && lane == 0) *bad = 1;
    wave_sync<G>();
}

// One wavefront: S_ij -= S_ik Dinv_k S_jk^T.  Q = Dinv_k S_jk^T by four 16x16x4 f64 MFMAs leaves Q[kq + 4s][rc] in
// accumulator s of lane (rc, kq) -- exactly the B operand of step s of the second product -- so Q never leaves the
// registers.  A/B operand lane maps: A[l&15][4s + (l>>4)], B[4s + (l>>4)][l&15]; D: col l&15, row (l>>4) + 4i.
__device__ __forceinline__ void update16(double *Sij, const double *Sik, const double *Sjk, const double *Dinv, int lane) {
    const int rc = lane & 15, kq = lane >> 4;
    v4d Q = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int kk = 4 * s + kq;
        Q = __builtin_amdgcn_mfma_f64_16x16x4f64(Dinv[sw16(rc, kk)], Sjk[sw16(rc, kk)], Q, 0, 0, 0);
    }
    v4d acc;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = Sij[sw16(kq + 4 * i, rc)];
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-Sik[sw16(rc, 4 * s + kq)], Q[s], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) Sij[sw16(kq + 4 * i, rc)] = acc[i];
}

constexpr int kLdltThreads = 512;
constexpr size_t kLdltLds = 160 * 1024 - 512;   // dynamic LDS of the solver (the static part is one int)

// Forward substitution of one column (one wavefront): z_i = Dinv_i (y_i - sum_k S_ik z_k) over the row structure
// (descendants, final by then); lane group grp takes the terms m = 4 grp .. 4 grp + 3 of every block (four loads of
// S and four of z per lane and block, all lanes busy whatever the block count).
// Block s of the solver's storage: LDS, or (hybrid, s >= n_lds) global scratch.  A value type: a reference-capturing
// lambda here put the kernel's locals on the private stack (144 B of scratch per lane, ~9 us more per solve).
template <int G>
struct BlkAt {
    double *pk, *gs;
    int n_lds;
    __device__ __forceinline__ double *operator()(int s) const {
        return G == 2 && s >= n_lds ? gs + (size_t)s * 256 : pk + (size_t)s * 256;
    }
};

template <typename Blk>
__device__ __forceinline__ void forward_col(const Blk blk, double *y, const BlockPat &P, int i, int lane) {
    const int r16 = lane & 15, grp = lane >> 4;
    double acc[4] = {0, 0, 0, 0};   // four chains (the sum is latency-bound)
    for (int q = P.rs_start[i]; q < P.rs_start[i + 1]; ++q) {
        const int2 e = P.rs[q];
        const double *Sik = blk(e.x);
        const double *zk = y + 16 * e.y + 4 * grp;
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m] = __builtin_fma(Sik[sw16(r16, 4 * grp + m)], zk[m], acc[m]);
    }
    double a = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    a += __shfl_xor(a, 16, 64);
    a += __shfl_xor(a, 32, 64);
    const double v = y[16 * i + r16] - a;
    // Dinv_i v: lane group grp takes columns 4 grp .. 4 grp + 3, then the four partial sums
    const double *Di = blk(P.dslot[i]);
    double out = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) out = __builtin_fma(Di[sw16(r16, 4 * grp + m)], __shfl(v, 4 * grp + m, 16), out);
    out += __shfl_xor(out, 16, 64);
    out += __shfl_xor(out, 32, 64);
    if (lane < 16) y[16 * i + lane] = out;
}

// Block LDL^T on the host-planned elimination order, level by level of its elimination tree: the columns of one level
// are independent (their trailing updates only reach ancestors, at higher levels), so a level's diagonal inverses run
// on separate wavefronts, then its trailing updates -- grouped by target block, each group on one wavefront in
// ascending column order (no two wavefronts write a block) -- beside its columns' forward substitutions.  Backward
// substitution gathers each column's structure (ancestors) level by level downwards.
// G: 0 blocks in LDS, 1 blocks in global scratch (pattern too large for LDS), 2 the first P.n_lds blocks in LDS and
// the rest in global scratch
template <int G>
__global__ void __launch_bounds__(kLdltThreads) ldlt_kernel(const double *Sp, BlockPat Pg, const double *b,
                                                            const double *coef, double *x, double *gscratch,
                                                            int *fail, const LmCtl *ctl) {
    extern __shared__ __attribute__((aligned(16))) double lsm[];
    __shared__ int bad;
    if (!gate_open(ctl, kGateTrial)) return;
    const int nb = Pg.nb, nv = 16 * nb;
    double *pk = G == 1 ? gscratch : lsm;
    const int n_lds = G == 2 ? Pg.n_lds : Pg.n_slots;
    double *y = pk + (size_t)n_lds * 256;
    double *xs = y + nv;
    const BlkAt<G> blk{pk, gscratch, n_lds};
    BlockPat P = Pg;   // the schedule, rebased onto its LDS copy when staged
    if (G != 1 && Pg.blob_ints > 0) {
        int *sched = reinterpret_cast<int *>(xs + nv);
        for (int q = threadIdx.x; q < Pg.blob_ints; q += blockDim.x) sched[q] = Pg.blob[q];
        auto rb = [&](auto *p) { return reinterpret_cast<decltype(p)>(sched + (reinterpret_cast<const int *>(p) - Pg.blob)); };
        P.perm = rb(Pg.perm), P.dslot = rb(Pg.dslot), P.lev_start = rb(Pg.lev_start), P.lev_col = rb(Pg.lev_col);
        P.ug_start = rb(Pg.ug_start), P.ug_split = rb(Pg.ug_split), P.crit_grp = rb(Pg.crit_grp);
        P.ug_task_start = rb(Pg.ug_task_start), P.ug = rb(Pg.ug), P.rs_start = rb(Pg.rs_start), P.rs = rb(Pg.rs);
        P.cs_start = rb(Pg.cs_start), P.cs = rb(Pg.cs), P.inv_rec = rb(Pg.inv_rec);
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    if (tid == 0) bad = 0;
#ifdef OMV_LDLT_PROFILE
    const long long t_0 = wall_clock64();
    long long t_1 = 0, t_3 = 0;
    __shared__ int pf_task[4];   // inverse ticks, forward ticks, inverse count, forward count
    __shared__ int pf_lev[16][4];   // per level: phase ticks, max inverse task ticks, inverses, other tasks (the
                                    // static LDS must stay under the 512 B beside kLdltLds, or the plan changes)
    if (tid < 4) pf_task[tid] = 0;
    if (tid < 64) pf_lev[tid >> 2][tid & 3] = 0;
#endif
    {
        const double2 *src = (const double2 *)Sp;
        double2 *dst = (double2 *)pk;
        // eight loads in flight per thread (a dependent load-store loop waits one memory latency per 8 KB)
        const int n2 = n_lds * 128, T = blockDim.x;
        for (int q0 = tid; q0 < n2; q0 += 8 * T) {
            double2 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = src[min(q0 + k * T, n2 - 1)];   // unconditional: all eight in flight
#pragma unroll
            for (int k = 0; k < 8; ++k) dst[min(q0 + k * T, n2 - 1)] = v[k];   // past the end: the last entry again
        }
        if (G == 2) {   // the global part, at its own offsets of the scratch
            double2 *gd = (double2 *)gscratch;
            for (int q = n2 + tid; q < P.n_slots * 128; q += T) gd[q] = src[q];
        }
        for (int q = tid; q < nv; q += blockDim.x) {
            const int g = 16 * Pg.perm[q >> 4] + (q & 15);   // (the LDS copy is not complete before the barrier)
            y[q] = b[g] - coef[g];
        }
    }
    __syncthreads();
#ifdef OMV_LDLT_PROFILE
    long long pf_fac = 0, pf_upd = 0, tp = wall_clock64();
#define OMV_LDLT_TICK(acc)                       \
    {                                            \
        const long long tn = wall_clock64();     \
        acc += tn - tp;                          \
        tp = tn;                                 \
    }
#else
#define OMV_LDLT_TICK(acc)
#endif
    // One phase per level l: level l's diagonal inverses -- each preceded, on its wavefront, by the updates of its
    // diagonal block from level l - 1 (the only trailing updates an inverse of level l waits for) -- beside level
    // l - 1's forward columns (their inverses and all their descendants' z are final) and level l - 1's other trailing
    // updates (no block of these is touched by an inverse of level l), so the bulk of each level's updates runs beside
    // the next level's inverses.  Each target block's updates come in ascending column order on one wavefront.
    // Wavefronts 0 .. ni-1 start on the inverses; with fewer than four inverses the wavefronts sharing their SIMDs
    // (w + 4) stay idle so the inverses -- the critical path -- issue alone; every other wavefront (and an inverse
    // wavefront once done) claims tasks from an LDS counter.  A phase advances the counter by its claimed tasks plus
    // one final failed claim per participating wavefront, so phase bases need no reset.
    __shared__ int claim;
    if (tid == 0) claim = 0;
    __syncthreads();
    int base = 0;
    for (int lev = 0; lev <= P.n_lev; ++lev) {
        const int c0 = P.lev_start[min(lev, P.n_lev)], c1 = lev < P.n_lev ? P.lev_start[lev + 1] : c0;
        const int f0 = lev > 0 ? P.lev_start[lev - 1] : 0, f1 = lev > 0 ? P.lev_start[lev] : 0;
        const int r0 = lev > 0 ? P.ug_split[lev - 1] : 0, r1 = lev > 0 ? P.ug_start[lev] : 0;
        const int ni = c1 - c0, nf = f1 - f0, na = ni + nf + (r1 - r0);
        const int ns = min(ni, nw);   // statically placed inverses
        const int n_idle = ni < 4 ? max(0, min(ni, nw - 4)) : 0;
        const bool idle = ni < 4 && wave >= 4 && wave - 4 < ni;
        if (!idle) {
            int q = wave < ns ? wave : -1;
            for (;;) {
                if (q < 0) {
                    int qn = 0;
                    if (lane == 0) qn = atomicAdd(&claim, 1);
                    q = ns + __shfl(qn, 0, 64) - base;
                    if (q >= na) break;
                }
#ifdef OMV_LDLT_PROFILE
                const long long tq = wall_clock64();
#endif
                if (q < ni) {
                    const int4 ir = P.inv_rec[2 * (c0 + q)], t0 = P.inv_rec[2 * (c0 + q) + 1];
                    if (ir.y < ir.z) {
                        for (int u = ir.y; u < ir.z; ++u) {
                            const int4 t = u == ir.y ? t0 : P.ug[u];
                            update16(blk(t.x), blk(t.y), blk(t.z), blk(t.w), lane);
                        }
                        wave_sync<G>();
                    }
                    inv16<G>(blk(ir.x), lane, &bad);
                } else if (q < ni + nf) {
                    forward_col(blk, y, P, P.lev_col[f0 + q - ni], lane);
                } else {
                    const int g = r0 + q - ni - nf;
                    for (int u = P.ug_task_start[g]; u < P.ug_task_start[g + 1]; ++u) {
                        const int4 t = P.ug[u];
                        update16(blk(t.x), blk(t.y), blk(t.z), blk(t.w), lane);
                    }
                }
#ifdef OMV_LDLT_PROFILE
                if (lane == 0 && q < ni + nf) atomicAdd(q < ni ? &pf_task[0] : &pf_task[1], (int)(wall_clock64() - tq));
                if (lane == 0 && q < ni + nf) atomicAdd(q < ni ? &pf_task[2] : &pf_task[3], 1);
                if (lane == 0 && lev < 16 && q < ni) atomicMax(&pf_lev[lev][1], (int)(wall_clock64() - tq));
#endif
                q = -1;
            }
        }
        base += (na - ns) + (nw - n_idle);
        __syncthreads();
#ifdef OMV_LDLT_PROFILE
        if (tid == 0 && lev < 16) pf_lev[lev][0] = (int)(wall_clock64() - tp), pf_lev[lev][2] = ni, pf_lev[lev][3] = na - ni;
#endif
        OMV_LDLT_TICK(pf_fac)
    }
#undef OMV_LDLT_TICK
#ifdef OMV_LDLT_PROFILE
    t_1 = wall_clock64();
#endif
    const int r16 = lane & 15, grp = lane >> 4;
    // backward: x_k = z_k - Dinv_k sum_i S_ik^T x_i
    for (int lev = P.n_lev - 1; lev >= 0; --lev) {
        for (int c = P.lev_start[lev] + wave; c < P.lev_start[lev + 1]; c += nw) {
            const int k = P.lev_col[c];
            double acc4[4] = {0, 0, 0, 0};   // lane group grp: rows 4 grp .. 4 grp + 3 of every block
            for (int q = P.cs_start[k]; q < P.cs_start[k + 1]; ++q) {
                const int2 e = P.cs[q];
                const double *Sik = blk(e.x);
                const double *xi = xs + 16 * e.y + 4 * grp;
#pragma unroll
                for (int r = 0; r < 4; ++r) acc4[r] = __builtin_fma(Sik[sw16(4 * grp + r, r16)], xi[r], acc4[r]);
            }
            double acc = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
            acc += __shfl_xor(acc, 16, 64);
            acc += __shfl_xor(acc, 32, 64);
            const double *Dk = blk(P.dslot[k]);
            double out = 0;
#pragma unroll
            for (int m = 0; m < 4; ++m) out = __builtin_fma(Dk[sw16(r16, 4 * grp + m)], __shfl(acc, 4 * grp + m, 16), out);
            out += __shfl_xor(out, 16, 64);
            out += __shfl_xor(out, 32, 64);
            if (lane < 16) xs[16 * k + lane] = y[16 * k + r16] - out;
        }
        __syncthreads();
    }
#ifdef OMV_LDLT_PROFILE
    t_3 = wall_clock64();
    if (tid == 0)
        printf("ldlt ticks(100MHz): factor+fwd %lld (diag inverse+fwd %lld updates %lld) bwd %lld slots %d levels %d; "
               "per inverse %.1f per forward col %.1f\n",
               t_1 - t_0, pf_fac, pf_upd, t_3 - t_1, P.n_slots, P.n_lev, (double)pf_task[0] / max(pf_task[2], 1),
               (double)pf_task[1] / max(pf_task[3], 1));
    if (tid == 0)
        for (int l = 0; l <= min(P.n_lev, 15); ++l)
            printf("  level %d: phase %d max-inverse %d inverses %d other %d\n", l, pf_lev[l][0], pf_lev[l][1],
                   pf_lev[l][2], pf_lev[l][3]);
#endif
    for (int q = tid; q < nv; q += blockDim.x) x[16 * P.perm[q >> 4] + (q & 15)] = xs[q];
    if (tid == 0) *fail = bad;
}

// ---- errors: computeActiveErrors, one workgroup per landmark group --------------------------------------
// Block 0 (when there are inertial edges or a trial): on a trial (xp) the keyframe update of every optimisable keyframe
// into the trial state (one thread per keyframe and camera) and the pose part of computeScale (scale_partial[0]), then
// the inertial / random-walk errors of that state (this block wrote it: a block-scope fence orders it).  Blocks 1..:
// the landmark groups of the build (whole landmarks and their edges), XCD-contiguous.  On a trial a group first
// back-substitutes its landmarks, xl = Dinv (bl - sum_s Hpl_s^T xp_s) = R^-T (y - sum_s M_s^T xp_s) from the build's
// R^-1, y and M_s (the trial point into the trial state and LDS; the landmark part of computeScale into
// scale_partial[1 + g]) while its other threads form the trial Rcw / tcw of the group's keyframes in LDS (the same
// arithmetic as block 0's: no block reads another's writes), then its edges' errors.  Without xp the points and poses
// are the state's.  The state / error buffers are the role's (role_buf); the updates start from the role-0 state.
struct ErrTrial {
    const double *xp;        // the solution (keyframe order), or null: no update
    int norm;                // host driver: this trial normalises the keyframe rotations (the device driver reads it
                             // from the control block)
    const double *b;         // the assembled gradient (keyframe order)
    double lambda;
    const int *offV, *offG, *offA;
    int n_opt;
    const int16_t *e_lkf;    // [E] the edge keyframe's index in its group's list, -1 fixed
    const int *lkf_kf;       // per group (at Land::grp_kf[g]) its keyframes
};
__global__ void __launch_bounds__(256) err_kernel(int n_grp, int lead, int has_imu, Rig rig, State s0, State s1, Edges E,
                                                  Land L, Red R, ErrTrial T, double delta, double dsqr, double delta_st,
                                                  double dsqr_st, ErrBufs e0, ErrBufs e1, double *partial,
                                                  double *scale_partial, Imu I, double delta_imu, double dsqr_imu,
                                                  double *imu_partial, const LmCtl *ctl, int gate, int role,
                                                  LmReset reset) {
    __shared__ double sh[8];
    extern __shared__ double dyn[];   // 3 per landmark, then 12 per (group keyframe, camera)
    if (reset.c && blockIdx.x == 0 && threadIdx.x == 0) ctl_reset(reset), reset.c->init_pending = 1;
    if (!gate_open(ctl, gate)) return;
    const int bi = role_buf(ctl, role);
    const State s = bi ? s1 : s0;
    const State a = role_buf(ctl, 0) ? s1 : s0;
    const ErrBufs eb = bi ? e1 : e0;
    const bool trial = T.xp != nullptr;
    const bool norm = ctl ? ctl->n_acc % 3 == 2 : T.norm != 0;
    const double lambda = trial ? lm_lambda(ctl, T.lambda) : 0.0;
    const int tid = threadIdx.x, C = rig.n_cams;
    int bid = blockIdx.x;
    if (lead) {
        if (bid == 0) {
            if (trial) {
                for (int t = tid; t < T.n_opt * C; t += blockDim.x) {
                    const int k = t / C, c = t - k * C;
                    double Rn[9], twb[3], Rc[9], tc[3];
                    kf_trial_pose(rig, a, T.xp + R.offP[k], k, c, norm, Rn, twb, Rc, tc);
                    for (int q = 0; q < 9; ++q) s.Rcw[((size_t)k * C + c) * 9 + q] = Rc[q];
                    for (int q = 0; q < 3; ++q) s.tcw[((size_t)k * C + c) * 3 + q] = tc[q];
                    if (c == 0) {
                        for (int q = 0; q < 9; ++q) s.Rwb[9 * k + q] = Rn[q];
                        for (int q = 0; q < 3; ++q) {
                            s.twb[3 * k + q] = twb[q];
                            s.vel[3 * k + q] = a.vel[3 * k + q] + (T.offV[k] >= 0 ? T.xp[T.offV[k] + q] : 0.0);
                            s.bg[3 * k + q] = a.bg[3 * k + q] + (T.offG[k] >= 0 ? T.xp[T.offG[k] + q] : 0.0);
                            s.ba[3 * k + q] = a.ba[3 * k + q] + (T.offA[k] >= 0 ? T.xp[T.offA[k] + q] : 0.0);
                        }
                    }
                }
                double sc = 0;   // pose part of sum_j x_j (lambda x_j + b_j); b is the assembled gradient (bvec)
                for (int q = tid; q < R.n; q += blockDim.x) sc += T.xp[q] * (lambda * T.xp[q] + T.b[q]);
                const double tt = block_reduce_sum(sc, sh);
                if (tid == 0) scale_partial[0] = tt;
                __threadfence_block();
                __syncthreads();
            }
            if (has_imu) imu_err_block(sh, s, I, delta_imu, dsqr_imu, eb.err9, imu_partial);
            return;
        }
        --bid;
    }
    const int chunk = (n_grp + 7) >> 3, g = (bid & 7) * chunk + (bid >> 3);
    if (g >= n_grp) return;
    const int p0 = L.grp_pt[g], np = L.grp_pt[g + 1] - p0;
    const int f0 = L.edge_start[p0], ne = L.edge_start[p0 + np] - f0;
    const int w = L.grp_w[g];   // < 0: a one-landmark group past the LDS limits (its poses per edge)
    double *X = dyn, *PS = dyn + 3 * kGrpLand;
    double sc = 0;
    if (tid < np) {
        const int p = p0 + tid;
        double Xp[3];
        if (trial) {
            const double *l = L.lnd + (size_t)p * 12;
            double Ri[6], c[3], bl[3];
            for (int q = 0; q < 6; ++q) Ri[q] = l[q];
            for (int q = 0; q < 3; ++q) c[q] = l[6 + q], bl[q] = l[9 + q];
            for (int sl = L.slot_start[p]; sl < L.slot_start[p + 1]; ++sl) {
                const int o = R.offP[L.slot_kf[sl]];
                if (o < 0) continue;
                const double *M = L.M + (size_t)sl * 18;
                for (int q = 0; q < 3; ++q)
                    for (int r = 0; r < 6; ++r) c[q] -= M[3 * r + q] * T.xp[o + r];
            }
            const double xl[3] = {Ri[0] * c[0] + Ri[1] * c[1] + Ri[3] * c[2], Ri[2] * c[1] + Ri[4] * c[2], Ri[5] * c[2]};
            for (int q = 0; q < 3; ++q) {
                Xp[q] = a.pts[(size_t)p * 3 + q] + xl[q];
                s.pts[(size_t)p * 3 + q] = Xp[q];
                sc += xl[q] * (lambda * xl[q] + bl[q]);
            }
        } else {
            for (int q = 0; q < 3; ++q) Xp[q] = s.pts[(size_t)p * 3 + q];
        }
        for (int q = 0; q < 3; ++q) X[3 * tid + q] = Xp[q];
    } else if (tid >= kGrpLand && trial && w > 0) {   // threads 128..: the trial poses of the group's keyframes
        for (int t = tid - kGrpLand; t < w * C; t += blockDim.x - kGrpLand) {
            const int la = t / C, c = t - la * C, k = T.lkf_kf[L.grp_kf[g] + la];
            double Rn[9], twb[3];
            kf_trial_pose(rig, a, T.xp + R.offP[k], k, c, norm, Rn, twb, PS + 12 * t, PS + 12 * t + 9);
        }
    }
    __syncthreads();
    double r0 = 0;
    for (int f = tid; f < ne; f += blockDim.x) {
        const int e = f0 + f, la = trial ? T.e_lkf[e] : -1, cam = E.cam[e];
        double Rc[9], tc[3];   // the edge camera's pose, in registers
        if (la < 0) {          // a fixed keyframe (identical in both buffers), or not a trial
            const size_t o = (size_t)E.kf[e] * C + cam;
            for (int q = 0; q < 9; ++q) Rc[q] = s.Rcw[o * 9 + q];
            for (int q = 0; q < 3; ++q) tc[q] = s.tcw[o * 3 + q];
        } else if (w > 0) {
            const double *o = PS + 12 * (la * C + cam);
            for (int q = 0; q < 9; ++q) Rc[q] = o[q];
            for (int q = 0; q < 3; ++q) tc[q] = o[9 + q];
        } else {   // the scalar group: per edge
            double Rn[9], twb[3];
            kf_trial_pose(rig, a, T.xp + R.offP[E.kf[e]], E.kf[e], cam, norm, Rn, twb, Rc, tc);
        }
        r0 += mono_err_edge(rig, Rc, tc, E, e, X + 3 * (E.pt[e] - p0), delta, dsqr, delta_st, dsqr_st, eb.err, eb.err3,
                            eb.chi2);
    }
    const double t = block_reduce_sum(r0, sh);
    if (tid == 0) partial[g] = t;
    if (trial) {
        __syncthreads();
        const double ts = block_reduce_sum(sc, sh);
        if (tid == 0) scale_partial[1 + g] = ts;
    }
}

// The optimisation's epilogue on the device (single rank): per visual edge the reference's outlier test
// (Optimizer.cc:3282-3311: EdgeMono chi2 > 5.991, or > 1.5 * 5.991 when the point's trackDepth < 10, or a
// non-positive depth; EdgeStereo chi2 > 7.815) at the final state, written in the caller's edge order with
// the chi2, and the points in the caller's order; the host reads one staging block.
__global__ void epilogue_kernel(Rig rig, State s0, State s1, size_t n_state, Edges E, const int *perm_edge,
                                int n_mono_all, const float *track_depth, const int *perm_pt, int n_pts, uint8_t *flags,
                                double *chi2_out, double *pts_out, const double *chi2_0, const double *chi2_1,
                                const LmCtl *ctl, double *head, int n_head) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const double *chi2 = ctl && ctl->last ? chi2_1 : chi2_0;   // the last computed errors (a rejected trial's too)
    // the device driver's current state (double-buffered); buffer 1 is also copied into buffer 0, where the next
    // optimize() starts
    const bool in1 = ctl && ctl->cur;
    const State s = in1 ? s1 : s0;
    if (in1)
        for (size_t k = q; k < n_state; k += (size_t)gridDim.x * blockDim.x) s0.Rwb[k] = s1.Rwb[k];
    if (q < n_head) head[q] = s.Rwb[q];   // the keyframe part of the state (it precedes the points)
    if (q < E.n) {
        const int e = q, o = perm_edge[e];
        const double c2 = chi2[e];
        uint8_t f;
        if (o >= n_mono_all) {
            f = c2 > 7.815f ? 1 : 0;
        } else {
            const int k = E.kf[e], c = E.cam[e], p = E.pt[e], C = rig.n_cams;
            const double *R = s.Rcw + ((size_t)k * C + c) * 9, *t = s.tcw + ((size_t)k * C + c) * 3;
            const double *X = s.pts + 3 * (size_t)p;
            const bool depth_pos = (R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2]) > 0.0;
            const bool close = track_depth[p] < 10.f;
            f = ((c2 > 5.991f && !close) || (c2 > 1.5f * 5.991f && close) || !depth_pos) ? 1 : 0;
        }
        flags[o] = f;
        if (chi2_out) chi2_out[o] = c2;
    }
    if (q < n_pts)
        for (int d = 0; d < 3; ++d) pts_out[3 * (size_t)perm_pt[q] + d] = s.pts[3 * (size_t)q + d];
}

// ---- evaluation helpers for parity ---------------------------------------------------------------
// [9] / [18] per edge: 3 residual rows (the third is zero on an EdgeMono)
__global__ void mono_jac_kernel(Rig rig, State s, Edges E, double *jx, double *jp) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E.n) return;
    const int k = E.kf[e], c = E.cam[e], C = rig.n_cams;
    const double *Rcw = s.Rcw + ((size_t)k * C + c) * 9, *tcw = s.tcw + ((size_t)k * C + c) * 3;
    const double *X = s.pts + (size_t)E.pt[e] * 3;
    double Xc[3], Xb[3];
    mv3(Rcw, X, Xc);
    for (int q = 0; q < 3; ++q) Xc[q] += tcw[q];
    mv3(rig.Rbc[c], Xc, Xb);
    for (int q = 0; q < 3; ++q) Xb[q] += rig.tbc[c][q];
    double pj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    cam_jac(rig, c, Xc, pj);
    if (E.ur[e] >= 0.f) {
        const double inv_z2 = 1.0 / (Xc[2] * Xc[2]);
        pj[6] = pj[0], pj[7] = pj[1], pj[8] = pj[2] + rig.bf * inv_z2;
    }
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            jx[9 * e + 3 * r + q] = -(pj[3 * r] * Rcw[q] + pj[3 * r + 1] * Rcw[3 + q] + pj[3 * r + 2] * Rcw[6 + q]);
    double pr[9];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            pr[3 * r + q] = pj[3 * r] * rig.Rcb[c][q] + pj[3 * r + 1] * rig.Rcb[c][3 + q] + pj[3 * r + 2] * rig.Rcb[c][6 + q];
    const double x = Xb[0], y = Xb[1], z = Xb[2];
    const double se3[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 6; ++q)
            jp[18 * e + 6 * r + q] = pr[3 * r] * se3[q] + pr[3 * r + 1] * se3[6 + q] + pr[3 * r + 2] * se3[12 + q];
}

// ---- host-side analysis ------------------------------------------------------------------------------
void host_inv(std::vector<double> &A, int n) {   // Gauss-Jordan with partial pivoting
    std::vector<double> I(n * n, 0.0);
    for (int i = 0; i < n; ++i) I[i * n + i] = 1;
    for (int c = 0; c < n; ++c) {
        int p = c;
        for (int r = c + 1; r < n; ++r)
            if (std::fabs(A[r * n + c]) > std::fabs(A[p * n + c])) p = r;
        if (p != c)
            for (int k = 0; k < n; ++k) std::swap(A[p * n + k], A[c * n + k]), std::swap(I[p * n + k], I[c * n + k]);
        const double d = A[c * n + c];
        for (int k = 0; k < n; ++k) A[c * n + k] /= d, I[c * n + k] /= d;
        for (int r = 0; r < n; ++r)
            if (r != c && A[r * n + c] != 0) {
                const double f = A[r * n + c];
                for (int k = 0; k < n; ++k) A[r * n + k] -= f * A[c * n + k], I[r * n + k] -= f * I[c * n + k];
            }
    }
    A = I;
}
void host_sym_eig(std::vector<double> A, int n, std::vector<double> &w, std::vector<double> &V) {
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
                    A[k * n + p] = c * akp - s * akq, A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk, A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq, V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
    w.resize(n);
    for (int i = 0; i < n; ++i) w[i] = A[i * n + i];
}

// Symbolic block LDL^T of the keyframe adjacency `adj` (nb x nb, symmetric) in the elimination order `perm`
// (position -> keyframe): the filled lower pattern in positions and each position's elimination-tree level
// (leaves 0, a parent above all its children).  Returns the number of levels (the factorisation's critical
// path in diagonal-block steps) and the number of stored blocks.
int symbolic_ldlt(int nb, const std::vector<uint8_t> &adj, const std::vector<int> &perm, std::vector<uint8_t> &pat,
                  std::vector<int> &level, int &n_slots) {
    pat.assign((size_t)nb * nb, 0);
    for (int i = 0; i < nb; ++i)
        for (int j = 0; j <= i; ++j) pat[(size_t)i * nb + j] = i == j || adj[(size_t)perm[i] * nb + perm[j]];
    for (int k = 0; k < nb; ++k)
        for (int i = k + 1; i < nb; ++i)
            if (pat[(size_t)i * nb + k])
                for (int j = k + 1; j <= i; ++j)
                    if (pat[(size_t)j * nb + k]) pat[(size_t)i * nb + j] = 1;
    level.assign(nb, 0);
    n_slots = 0;
    int top = 0;
    for (int k = 0; k < nb; ++k) {
        for (int i = k; i < nb; ++i) n_slots += pat[(size_t)i * nb + k];
        for (int i = k + 1; i < nb; ++i)
            if (pat[(size_t)i * nb + k]) {   // the parent: the first block below the diagonal
                level[i] = std::max(level[i], level[k] + 1);
                break;
            }
        top = std::max(top, level[k]);
    }
    return nb > 0 ? top + 1 : 0;
}

// The elimination order of the reduced system's keyframe blocks.  Candidates: the keyframe order, and every
// two-way dissection of it -- a cut c, the separator S = the keyframes before c adjacent to one at or after c,
// then [before c minus S, in order] [from c, reversed] [S]: the two sides share no block, so their columns
// factor concurrently, and each side is eliminated away from the separator (no fill beyond it).  The one with
// the fewest elimination-tree levels whose blocks fit `max_slots` wins (ties: fewer blocks, then earlier).
// The solution of the damped system does not depend on the order beyond rounding (SimplicialLDLT's own AMD
// ordering is a different one again, linear_solver_eigen.h:60).
std::vector<int> plan_order(int nb, const std::vector<uint8_t> &adj, int max_slots) {
    std::vector<int> best(nb);
    std::iota(best.begin(), best.end(), 0);
    std::vector<uint8_t> pat;
    std::vector<int> lev;
    int best_slots = 0;
    int best_h = symbolic_ldlt(nb, adj, best, pat, lev, best_slots);
    for (int cut = 1; cut < nb; ++cut) {
        std::vector<int> order, sep;
        for (int v = 0; v < cut; ++v) {
            bool s = false;
            for (int w = cut; w < nb && !s; ++w) s = adj[(size_t)v * nb + w] != 0;
            (s ? sep : order).push_back(v);
        }
        if (sep.size() * 2 > (size_t)nb) continue;
        for (int w = nb - 1; w >= cut; --w) order.push_back(w);
        order.insert(order.end(), sep.begin(), sep.end());
        int ns = 0;
        const int h = symbolic_ldlt(nb, adj, order, pat, lev, ns);
        if (ns > max_slots) continue;
        if (h < best_h || (h == best_h && ns < best_slots)) best = order, best_h = h, best_slots = ns;
    }
    return best;
}

template <typename T>
T *dalloc(std::vector<void *> &owned, size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)) != hipSuccess) return nullptr;
    owned.push_back(p);
    return (T *)p;
}

}  // namespace

// =============================================================================================
struct omv_lba {
    int max_kf, max_cams, max_pts, max_mono, max_imu;
    std::vector<void *> owned;   // device allocations of the current problem
    // problem
    Rig rig{};
    int n_kf = 0, n_opt = 0, n_pts = 0, n_mono = 0, n_imu = 0, n_red = 0, n_slots = 0;
    State st[3]{};   // current / trial (push-pop double buffer) / the uploaded initial state
    int cur = 0;
    Edges E{};
    Land L{};
    Red R{};
    Imu I{};
    BlockPat BP{};
    Gather G{};
    double *d_imu_contrib = nullptr;   // [n_imu][30 x 30 + 30] per-edge inertial contributions
    int n_lgrp = 0;   // landmark groups (build, errors, back-substitution)
    int n_big = 0;             // one-landmark groups of the scalar build path
    const int16_t *d_e_lkf = nullptr;   // per edge: its keyframe's index in the group's list (-1: fixed)
    const int *d_lkf_kf = nullptr;      // per (group, local keyframe): the keyframe
    const int *d_big = nullptr;
    // device epilogue (single rank): perm_edge / perm_pt / trackDepth in device order, one staging block
    // [state without points | points in caller order | chi2 in caller order | outlier flags in caller order]
    int *d_perm_edge = nullptr, *d_perm_pt = nullptr;
    float *d_track_depth = nullptr;
    double *d_stage = nullptr, *h_stage = nullptr;
    size_t stage_bytes = 0;
    bool epi_ready = false;    // the staging block holds this optimize()'s final result
    bool epi_chi2 = false;     //   including the chi2
    int *d_offP = nullptr, *d_offV = nullptr, *d_offG = nullptr, *d_offA = nullptr;
    double *d_err = nullptr, *d_chi2 = nullptr, *d_err9 = nullptr;
    double *d_err_b = nullptr, *d_chi2_b = nullptr, *d_err9_b = nullptr, *d_err3_b = nullptr;   // the second error buffer
    ErrBufs eb(int i) const { return i ? ErrBufs{d_err_b, d_err3_b, d_chi2_b, d_err9_b} : ErrBufs{d_err, d_err3, d_chi2, d_err9}; }
    double *d_partial = nullptr, *d_imu_partial = nullptr, *d_scale_partial = nullptr, *d_out = nullptr;
    double *d_partial0 = nullptr, *d_imu_partial0 = nullptr;   // optimize()'s initial errors (device driver)
    double *h_out = nullptr;   // pinned host copy of d_out: the per-trial 24-byte read-back
    LmCtl *d_ctl = nullptr;    // device-resident LM control (single-rank path)
    LmCtl *h_ctl = nullptr;    // pinned copy: the one read-back per optimize()
    hipGraph_t step_graph = nullptr;
    hipGraphExec_t step_exec = nullptr;   // one LM step (trial, and buildSystem when an iteration starts)
    hipGraph_t step4_graph = nullptr;
    hipGraphExec_t step4_exec = nullptr;  // four LM steps in one launch (no launch gap between them)
    // four LM steps + the speculative epilogue + the staging and control read-backs (index: chi2 read-back or not):
    // the batch that usually ends the optimize() in one launch (a graph -> kernel -> copy transition on the stream
    // costs ~10 us each)
    hipGraph_t step4e_graph[2] = {nullptr, nullptr};
    hipGraphExec_t step4e_exec[2] = {nullptr, nullptr};
    bool timing = false;       // direct launches with per-stage events instead of the captured step
    bool host_lm = false;      // force the host-driven LM loop (parity checks of the device control)
    double *d_S = nullptr, *d_coef = nullptr, *d_x = nullptr, *d_scratch = nullptr;
    int *d_fail = nullptr;
    double *d_bb = nullptr;    // the trial's copy of b (all-reduced with the packed system when sharded)
    size_t n_reduce = 0;
    int rank = 0, world = 1;   // landmark sharding (omv_lba_set_comm)
    omv_allreduce_fn allreduce = nullptr;
    void *ar_ctx = nullptr;
    bool imu_here = false;     // this rank evaluates the inertial edges (rank 0)
    size_t ldlt_lds = 0;
    int use_lds = 0;
    bool lds_ok = false;
    std::vector<int> perm_pt;     // device point index -> caller index
    std::vector<int> perm_edge;   // device edge index -> caller index
    double delta_mono, dsqr_mono, delta_st, dsqr_st, delta_imu, dsqr_imu;
    int n_mono_all = 0, n_stereo_all = 0;   // caller edge counts (perm_edge >= n_mono_all: EdgeStereo)
    double *d_err3 = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev[8];
    double stage_ms[4] = {0, 0, 0, 0};
    int last_trials = 0;
    int host_syncs = 0;        // host waits of the last optimize()'s LM loop (the device driver: one per batch)
    size_t state_doubles() const { return (size_t)n_kf * (24 + 12 * rig.n_cams) + 3 * (size_t)n_pts; }
};

static void free_problem(omv_lba *h) {
    for (void *p : h->owned) (void)hipFree(p);
    h->owned.clear();
    if (h->h_stage) (void)hipHostFree(h->h_stage);
    h->h_stage = nullptr, h->stage_bytes = 0;
    if (h->step_exec) (void)hipGraphExecDestroy(h->step_exec);
    if (h->step_graph) (void)hipGraphDestroy(h->step_graph);
    if (h->step4_exec) (void)hipGraphExecDestroy(h->step4_exec);
    if (h->step4_graph) (void)hipGraphDestroy(h->step4_graph);
    h->step_exec = nullptr, h->step_graph = nullptr;   // the captured step holds the old problem's pointers
    h->step4_exec = nullptr, h->step4_graph = nullptr;
    for (int q = 0; q < 2; ++q) {
        if (h->step4e_exec[q]) (void)hipGraphExecDestroy(h->step4e_exec[q]);
        if (h->step4e_graph[q]) (void)hipGraphDestroy(h->step4e_graph[q]);
        h->step4e_exec[q] = nullptr, h->step4e_graph[q] = nullptr;
    }
}

extern "C" {

omv_status omv_lba_create(int max_kf, int max_cams, int max_pts, int max_mono, int max_imu, omv_lba **out) {
    if (!out || max_kf <= 0 || max_cams <= 0 || max_cams > kMaxCams || max_pts < 0 || max_mono < 0 || max_imu < 0)
        return OMV_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return OMV_ERR_NO_DEVICE;
    omv_lba *h = new omv_lba();
    h->max_kf = max_kf, h->max_cams = max_cams, h->max_pts = max_pts, h->max_mono = max_mono, h->max_imu = max_imu;
    HIP_OK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    for (auto &e : h->ev) HIP_OK(hipEventCreate(&e));
    HIP_OK(hipHostMalloc((void **)&h->h_out, 4 * sizeof(double), hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void **)&h->h_ctl, sizeof(LmCtl), hipHostMallocDefault));
    HIP_OK(hipMalloc((void **)&h->d_ctl, sizeof(LmCtl)));
    // the reduced-system factorisation stages its nonzero blocks in up to 150 KB of LDS
    h->lds_ok = hipFuncSetAttribute((const void *)ldlt_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kLdltLds) == hipSuccess &&
                hipFuncSetAttribute((const void *)ldlt_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kLdltLds) == hipSuccess;
    // the landmark groups of the build take ~77 KB of LDS (two workgroups per CU)
    if (hipFuncSetAttribute((const void *)build_all_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBuildLds) !=
            hipSuccess ||
        hipFuncSetAttribute((const void *)build_big_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBuildLds) !=
            hipSuccess) {
        delete h;
        return OMV_ERR_HIP;
    }
    (void)hipGetLastError();
    *out = h;
    return OMV_OK;
}

omv_status omv_lba_destroy(omv_lba *h) {
    if (!h) return OMV_ERR_ARG;
    free_problem(h);
    for (auto &e : h->ev) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    if (h->h_out) (void)hipHostFree(h->h_out);
    if (h->h_ctl) (void)hipHostFree(h->h_ctl);
    if (h->d_ctl) (void)hipFree(h->d_ctl);
    if (h->step_exec) (void)hipGraphExecDestroy(h->step_exec);
    if (h->step_graph) (void)hipGraphDestroy(h->step_graph);
    if (h->step4_exec) (void)hipGraphExecDestroy(h->step4_exec);
    if (h->step4_graph) (void)hipGraphDestroy(h->step4_graph);
    for (int q = 0; q < 2; ++q) {
        if (h->step4e_exec[q]) (void)hipGraphExecDestroy(h->step4e_exec[q]);
        if (h->step4e_graph[q]) (void)hipGraphDestroy(h->step4e_graph[q]);
    }
    delete h;
    return OMV_OK;
}

omv_status omv_lba_set_problem(omv_lba *h, const omv_lba_problem *p) {
    if (!h || !p) return OMV_ERR_ARG;
    if (p->n_cams <= 0 || p->n_cams > h->max_cams || p->n_kf > h->max_kf || p->n_pts < 0 || p->n_mono < 0 ||
        p->n_imu > h->max_imu || p->n_opt > p->n_kf || p->n_opt < 1)
        return OMV_ERR_ARG;
    free_problem(h);
    const int C = p->n_cams, K = p->n_kf, P_all = p->n_pts, NI = p->n_imu;
    const int EM = p->n_mono, ES = p->n_stereo > 0 ? p->n_stereo : 0, E_all = EM + ES;
    if (ES > 0 && (!p->stereo_pt || !p->stereo_kf || !p->stereo_obs || !p->stereo_inv_sigma2)) return OMV_ERR_ARG;
    for (int e = 0; e < ES; ++e)   // an EdgeStereo exists only where mvuRight >= 0 (Optimizer.cc:3075, :3108)
        if (!(p->stereo_obs[3 * (size_t)e + 2] >= 0.0)) return OMV_ERR_ARG;
    h->n_mono_all = EM, h->n_stereo_all = ES;
    // visual edge e < EM: EdgeMono e; e >= EM: EdgeStereo e - EM (camera 0, EdgeStereo(0) at :3118)
    auto e_pt_of = [&](int e) { return e < EM ? p->mono_pt[e] : p->stereo_pt[e - EM]; };
    auto e_kf_of = [&](int e) { return e < EM ? p->mono_kf[e] : p->stereo_kf[e - EM]; };
    auto e_cam_of = [&](int e) { return e < EM ? p->mono_cam[e] : 0; };
    h->n_kf = K, h->n_opt = p->n_opt, h->n_imu = NI;
    h->imu_here = NI > 0 && h->rank == 0;
    // rig
    Rig &rig = h->rig;
    rig.n_cams = C;
    for (int c = 0; c < C; ++c) {
        for (int q = 0; q < 8; ++q) rig.cam[c][q] = p->cam[8 * c + q];
        rig.model[c] = p->cam_model ? p->cam_model[c] : OMV_CAM_KB8;
        if (rig.model[c] != OMV_CAM_KB8 && rig.model[c] != OMV_CAM_PINHOLE) return OMV_ERR_ARG;
        for (int q = 0; q < 9; ++q) rig.Rcb[c][q] = p->Rcb[9 * c + q], rig.Rbc[c][q] = p->Rbc[9 * c + q];
        for (int q = 0; q < 3; ++q) rig.tcb[c][q] = p->tcb[3 * c + q], rig.tbc[c][q] = p->tbc[3 * c + q];
    }
    // reduced-system layout: per optimisable keyframe pose (6) [+ v bg ba (9)]
    // keyframe block k occupies reduced indices 16k .. 16k+15: pose 0-5, v 6-8, bg 9-11, ba 12-14, pad 15
    std::vector<int> offP(K, -1), offV(K, -1), offG(K, -1), offA(K, -1);
    const int nred = 16 * p->n_opt;
    for (int k = 0; k < p->n_opt; ++k) {
        offP[k] = 16 * k;
        if (p->kf_imu[k]) offV[k] = 16 * k + 6, offG[k] = 16 * k + 9, offA[k] = 16 * k + 12;
    }
    h->n_red = nred;
    // landmark order: by the first optimisable keyframe observing them (workgroup keyframe spans stay small)
    std::vector<std::vector<int>> pe(P_all);
    for (int e = 0; e < E_all; ++e) {
        if (e_pt_of(e) < 0 || e_pt_of(e) >= P_all || e_kf_of(e) < 0 || e_kf_of(e) >= K || e_cam_of(e) < 0 ||
            e_cam_of(e) >= C)
            return OMV_ERR_ARG;
        pe[e_pt_of(e)].push_back(e);
    }
    std::vector<int> key(P_all, 1 << 30);
    for (int q = 0; q < P_all; ++q)
        for (int e : pe[q]) key[q] = std::min(key[q], e_kf_of(e) < p->n_opt ? e_kf_of(e) : (1 << 29) + e_kf_of(e));
    std::vector<int> order(P_all);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[a] < key[b]; });
    // block pattern of the reduced system (keyframe blocks) from ALL landmarks: every rank of a
    // sharded solve lays out the identical packed system
    const int nb = p->n_opt;
    std::vector<uint8_t> adj((size_t)nb * nb, 0);   // keyframe adjacency (symmetric)
    for (int q = 0; q < P_all; ++q)
        for (int a : pe[q])
            for (int b : pe[q]) {
                const int i = e_kf_of(a), j = e_kf_of(b);
                if (i < nb && j < nb && i != j) adj[(size_t)i * nb + j] = 1;
            }
    // this rank's landmarks: a contiguous share of the landmark order
    if (h->world > 1) {
        const size_t lo = (size_t)P_all * h->rank / h->world, hi = (size_t)P_all * (h->rank + 1) / h->world;
        order = std::vector<int>(order.begin() + lo, order.begin() + hi);
    }
    const int P = (int)order.size();
    int E = 0;
    for (int q : order) E += (int)pe[q].size();
    if (P > h->max_pts || E > h->max_mono) return OMV_ERR_ARG;
    h->n_pts = P, h->n_mono = E;
    h->perm_pt = order;
    std::vector<int> e_pt, e_kf, e_cam, e_slot, pt_edge(P + 1, 0), pt_slot(P + 1, 0), slot_kf;
    std::vector<double> e_obs;
    std::vector<float> e_w, e_ur;
    h->perm_edge.clear();
    for (int q = 0; q < P; ++q) {
        std::vector<int> es = pe[order[q]];
        std::stable_sort(es.begin(), es.end(), [&](int a, int b) { return e_kf_of(a) < e_kf_of(b); });
        pt_edge[q] = (int)e_pt.size();
        pt_slot[q] = (int)slot_kf.size();
        int last_kf = -1;
        for (int e : es) {
            const int kf = e_kf_of(e);
            if (kf != last_kf) slot_kf.push_back(kf), last_kf = kf;
            e_pt.push_back(q), e_kf.push_back(kf), e_cam.push_back(e_cam_of(e));
            e_slot.push_back((int)slot_kf.size() - 1);
            if (e < EM) {
                e_obs.push_back(p->mono_obs[2 * e]), e_obs.push_back(p->mono_obs[2 * e + 1]);
                e_w.push_back(p->mono_inv_sigma2[e]);
                e_ur.push_back(-1.f);
            } else {
                const double *o = p->stereo_obs + 3 * (size_t)(e - EM);
                e_obs.push_back(o[0]), e_obs.push_back(o[1]);
                e_w.push_back(p->stereo_inv_sigma2[e - EM]);
                // the reference stores mvuRight (a float >= 0) in the double measurement
                e_ur.push_back((float)o[2]);
            }
            h->perm_edge.push_back(e);
        }
    }
    pt_edge[P] = (int)e_pt.size();
    pt_slot[P] = (int)slot_kf.size();
    h->n_slots = (int)slot_kf.size();
    // inertial edges: ids checked, and their blocks in the keyframe adjacency
    for (int i = 0; i < NI; ++i) {
        if (p->imu_kf1[i] < 0 || p->imu_kf1[i] >= K || p->imu_kf2[i] < 0 || p->imu_kf2[i] >= K ||
            p->imu_kf1[i] == p->imu_kf2[i])
            return OMV_ERR_ARG;
        const int a = p->imu_kf1[i], b = p->imu_kf2[i];
        if (a < nb && b < nb) adj[(size_t)a * nb + b] = adj[(size_t)b * nb + a] = 1;
    }
    // elimination order (every rank of a sharded solve plans from the same full pattern) and its symbolic LDL^T
    const size_t vec_bytes = 2 * (size_t)nred * sizeof(double);
    const int lds_slots = h->lds_ok && kLdltLds > vec_bytes ? (int)((kLdltLds - vec_bytes) / (256 * sizeof(double))) : 0;
    const std::vector<int> perm = plan_order(nb, adj, std::max(lds_slots, 1));
    std::vector<int> ipos(nb);
    for (int q = 0; q < nb; ++q) ipos[perm[q]] = q;
    std::vector<uint8_t> pat;
    std::vector<int> level;
    int n_slots = 0;
    const int n_lev = symbolic_ldlt(nb, adj, perm, pat, level, n_slots);
    std::vector<int> slot((size_t)nb * nb, -1), slot_kr, slot_kc, dslot(nb);
    for (int j = 0; j < nb; ++j)   // column-major in positions: a column's panel blocks sit together
        for (int i = j; i < nb; ++i)
            if (pat[(size_t)i * nb + j]) {
                slot[(size_t)i * nb + j] = (int)slot_kr.size();
                slot_kr.push_back(perm[i]), slot_kc.push_back(perm[j]);
            }
    for (int k = 0; k < nb; ++k) dslot[k] = slot[(size_t)k * nb + k];
    // level schedule: columns per level; trailing updates grouped by target block (ascending k)
    std::vector<int> lev_start(n_lev + 1, 0), lev_col, ug_start(n_lev + 1, 0), ug_split(std::max(n_lev, 1), 0),
        ug_task_start(1, 0), crit_grp(nb, -1);
    std::vector<int> slot_kr_pos(n_slots), slot_kc_pos(n_slots);   // block positions of each slot
    for (int j = 0; j < nb; ++j)
        for (int i = j; i < nb; ++i)
            if (slot[(size_t)i * nb + j] >= 0) slot_kr_pos[slot[(size_t)i * nb + j]] = i, slot_kc_pos[slot[(size_t)i * nb + j]] = j;
    std::vector<int4> ug;
    for (int l = 0; l < n_lev; ++l) {
        lev_start[l] = (int)lev_col.size();
        ug_start[l] = (int)ug_task_start.size() - 1;
        std::map<int, std::vector<int4>> by_target;   // target slot -> updates in ascending k
        for (int k = 0; k < nb; ++k) {
            if (level[k] != l) continue;
            lev_col.push_back(k);
            std::vector<int> col;
            for (int i = k + 1; i < nb; ++i)
                if (pat[(size_t)i * nb + k]) col.push_back(i);
            for (size_t a = 0; a < col.size(); ++a)
                for (size_t c = 0; c <= a; ++c) {
                    const int i = col[a], j = col[c];
                    by_target[slot[(size_t)i * nb + j]].push_back(
                        make_int4(slot[(size_t)i * nb + j], slot[(size_t)i * nb + k], slot[(size_t)j * nb + k], dslot[k]));
                }
        }
        // the diagonal blocks of level l + 1 first: their inverses wait only for these groups, the rest of the level's
        // updates run beside those inverses
        for (int pass = 0; pass < 2; ++pass) {
            for (auto &kv : by_target) {
                const int kr = slot_kr_pos[kv.first], kc = slot_kc_pos[kv.first];
                const bool crit = kr == kc && level[kr] == l + 1;
                if (crit != (pass == 0)) continue;
                if (crit) crit_grp[kr] = (int)ug_task_start.size() - 1;
                ug.insert(ug.end(), kv.second.begin(), kv.second.end());
                ug_task_start.push_back((int)ug.size());
            }
            if (pass == 0) ug_split[l] = (int)ug_task_start.size() - 1;
        }
    }
    lev_start[n_lev] = (int)lev_col.size();
    ug_start[n_lev] = (int)ug_task_start.size() - 1;
    std::vector<int4> inv_rec(2 * (size_t)std::max(nb, 1), make_int4(0, 0, 0, 0));
    for (size_t c = 0; c < lev_col.size(); ++c) {
        const int col = lev_col[c], g = crit_grp[col];
        const int u0 = g >= 0 ? ug_task_start[g] : 0, u1 = g >= 0 ? ug_task_start[g + 1] : 0;
        inv_rec[2 * c] = make_int4(dslot[col], u0, u1, 0);
        if (u0 < u1) inv_rec[2 * c + 1] = ug[u0];
    }
    std::vector<int> rs_start(nb + 1, 0), cs_start(nb + 1, 0);
    std::vector<int2> rs, cs;
    for (int i = 0; i < nb; ++i) {
        rs_start[i] = (int)rs.size();
        for (int k = 0; k < i; ++k)
            if (pat[(size_t)i * nb + k]) rs.push_back(make_int2(slot[(size_t)i * nb + k], k));
    }
    rs_start[nb] = (int)rs.size();
    for (int k = 0; k < nb; ++k) {
        cs_start[k] = (int)cs.size();
        for (int i = k + 1; i < nb; ++i)
            if (pat[(size_t)i * nb + k]) cs.push_back(make_int2(slot[(size_t)i * nb + k], i));
    }
    cs_start[nb] = (int)cs.size();
    // buildSystem landmark groups (land_group): whole landmarks in landmark order, at most kGrpEdges edges, kGrpLand
    // landmarks, kGrpSlots slots and kGrpW optimisable keyframes; a landmark past one of those alone forms a group of
    // its own built by the scalar path (land_group_big).  Per group: its keyframes in elimination order (local index a),
    // its record (w(w+1)/2 blocks a >= b of 36, then w rows of [gradient 6 | Schur rhs 6]), the 16x16 output tiles that
    // hold a co-observed keyframe pair, and per diagonal tile the residual rows of its keyframes' edges.
    std::vector<int> slot_edge(h->n_slots + 1, 0);
    for (int e = E - 1; e >= 0; --e) slot_edge[e_slot[e]] = e;
    slot_edge[h->n_slots] = E;
    std::vector<int16_t> slot_lkf(h->n_slots, -1);
    std::vector<int> grp_pt(1, 0), grp_w, grp_tp(1, 0), grp_blk, blkoff, grp_kf, rhsoff, lkf_kf;
    std::vector<int> blk_start(n_slots + 1, 0), rhs_start(nb + 1, 0);
    std::vector<uint8_t> tp;
    {
        // per reduced-system block / keyframe: the (blkoff / rhsoff index) of each contributing group, in group order
        std::vector<std::vector<int>> by_blk(n_slots), by_kf(nb);
        auto opt_kfs = [&](int q0, int q1) {   // distinct optimisable keyframes of landmarks [q0, q1)
            std::set<int> k;
            for (int q = q0; q < q1; ++q)
                for (int a = pt_slot[q]; a < pt_slot[q + 1]; ++a)
                    if (slot_kf[a] < nb) k.insert(slot_kf[a]);
            return k;
        };
        auto panel_ok = [&](int n_land, int n_kf) {   // the MFMA operand panels fit their LDS region
            return (n_kf + 1) / 2 * ((3 * n_land + 3) & ~3) <= kPanel;
        };
        auto fits = [&](int q0, int q1) {
            const int nk = (int)opt_kfs(q0, q1).size();
            return pt_edge[q1] - pt_edge[q0] <= kGrpEdges && q1 - q0 <= kGrpLand && pt_slot[q1] - pt_slot[q0] <= kGrpSlots &&
                   nk <= kGrpW && panel_ok(q1 - q0, nk);
        };
        for (int q = 0; q < P;) {
            int r = q + 1;
            const bool big = !fits(q, r);
            if (!big) {
                std::set<int> k = opt_kfs(q, r);
                while (r < P && r - q < kGrpLand && pt_edge[r + 1] - pt_edge[q] <= kGrpEdges &&
                       pt_slot[r + 1] - pt_slot[q] <= kGrpSlots) {
                    std::set<int> k2 = k;
                    for (int a = pt_slot[r]; a < pt_slot[r + 1]; ++a)
                        if (slot_kf[a] < nb) k2.insert(slot_kf[a]);
                    if ((int)k2.size() > kGrpW || !panel_ok(r + 1 - q, (int)k2.size())) break;
                    k.swap(k2);
                    ++r;
                }
            }
            // the group's keyframes in elimination order
            std::set<int> ks = opt_kfs(q, r);
            std::vector<int> kl(ks.begin(), ks.end());
            std::sort(kl.begin(), kl.end(), [&](int x, int y) { return ipos[x] < ipos[y]; });
            const int w = (int)kl.size(), nblk = w * (w + 1) / 2;
            std::vector<int> lk(nb, -1);
            for (int a = 0; a < w; ++a) lk[kl[a]] = a;
            for (int a = pt_slot[q]; a < pt_slot[r]; ++a) slot_lkf[a] = (int16_t)(slot_kf[a] < nb ? lk[slot_kf[a]] : -1);
            const int g = (int)grp_w.size();
            grp_w.push_back(big ? -w - 1 : w);
            grp_blk.push_back((int)blkoff.size());
            grp_kf.push_back((int)rhsoff.size());
            blkoff.resize(blkoff.size() + nblk, -1);
            rhsoff.resize(rhsoff.size() + w, -1);
            lkf_kf.insert(lkf_kf.end(), kl.begin(), kl.end());
            // co-observed keyframe pairs (a >= b): the group's blocks
            std::vector<uint8_t> co((size_t)std::max(w, 1) * std::max(w, 1), 0);
            for (int x = q; x < r; ++x) {
                std::vector<int> loc;
                for (int a = pt_slot[x]; a < pt_slot[x + 1]; ++a)
                    if (slot_kf[a] < nb) loc.push_back(lk[slot_kf[a]]);
                for (int u : loc)
                    for (int v : loc)
                        if (u >= v) co[(size_t)u * w + v] = 1;
            }
            for (int u = 0; u < w; ++u) {
                by_kf[kl[u]].push_back(grp_kf[g] + u);
                for (int v = 0; v <= u; ++v)
                    if (co[(size_t)u * w + v])
                        by_blk[slot[(size_t)ipos[kl[u]] * nb + ipos[kl[v]]]].push_back(grp_blk[g] + u * (u + 1) / 2 + v);
            }
            if (!big) {
                const int nt = (w + 1) / 2;
                for (int ti = 0; ti < nt; ++ti)
                    for (int tj = 0; tj <= ti; ++tj) {
                        bool any = false;
                        for (int u = 2 * ti; u < std::min(w, 2 * ti + 2) && !any; ++u)
                            for (int v = 2 * tj; v < std::min(w, 2 * tj + 2) && !any; ++v) any = u >= v && co[(size_t)u * w + v];
                        if (any) tp.push_back((uint8_t)ti), tp.push_back((uint8_t)tj);
                    }
            }
            grp_tp.push_back((int)tp.size() / 2);
            grp_pt.push_back(r);
            (void)g;
            q = r;
        }
        // records contiguous per block (per keyframe), in group order: assemble_kernel reads them as one run
        for (int t = 0; t < n_slots; ++t) {
            blk_start[t + 1] = blk_start[t] + (int)by_blk[t].size();
            for (size_t i = 0; i < by_blk[t].size(); ++i) blkoff[by_blk[t][i]] = blk_start[t] + (int)i;
        }
        for (int k = 0; k < nb; ++k) {
            rhs_start[k + 1] = rhs_start[k] + (int)by_kf[k].size();
            for (size_t i = 0; i < by_kf[k].size(); ++i) rhsoff[by_kf[k][i]] = rhs_start[k] + (int)i;
        }
    }
    h->n_lgrp = (int)grp_w.size();
    std::vector<int> big_grp;
    for (int g = 0; g < h->n_lgrp; ++g)
        if (grp_w[g] < 0) big_grp.push_back(g);
    h->n_big = (int)big_grp.size();
    // inertial edges per block (edge, side of the row keyframe, side of the column keyframe; side 0 = kf1) and per
    // keyframe (edge, side), in edge order; only the rank that evaluates them
    std::vector<int> ib_start(n_slots + 1, 0), iv_start(nb + 1, 0);
    std::vector<int4> imu_blk;
    std::vector<int2> imu_vec;
    {
        std::vector<std::vector<int4>> bl(n_slots);
        std::vector<std::vector<int2>> vl(nb);
        if (h->imu_here)
            for (int i = 0; i < NI; ++i) {
                const int kk[2] = {p->imu_kf1[i], p->imu_kf2[i]};
                for (int sr = 0; sr < 2; ++sr) {
                    if (kk[sr] >= nb) continue;
                    vl[kk[sr]].push_back(make_int2(i, sr));
                    for (int sc = 0; sc < 2; ++sc) {
                        if (kk[sc] >= nb || ipos[kk[sr]] < ipos[kk[sc]]) continue;
                        bl[slot[(size_t)ipos[kk[sr]] * nb + ipos[kk[sc]]]].push_back(make_int4(i, sr, sc, 0));
                    }
                }
            }
        for (int t = 0; t < n_slots; ++t) {
            ib_start[t] = (int)imu_blk.size();
            imu_blk.insert(imu_blk.end(), bl[t].begin(), bl[t].end());
        }
        ib_start[n_slots] = (int)imu_blk.size();
        for (int k = 0; k < nb; ++k) {
            iv_start[k] = (int)imu_vec.size();
            imu_vec.insert(imu_vec.end(), vl[k].begin(), vl[k].end());
        }
        iv_start[nb] = (int)imu_vec.size();
    }
    const size_t ldlt_bytes = ((size_t)n_slots * 256 + 2 * (size_t)nred) * sizeof(double);
    // the solver's storage: 1 every block in LDS; 2 (the pattern does not fit) the vectors, the schedule and the first
    // blocks in LDS, the rest in global scratch; 0 (no LDS attribute, or a test build) every block in global scratch
    h->use_lds = !h->lds_ok ? 0 : ldlt_bytes <= kLdltLds ? 1 : kLdltLds > 2 * (size_t)nred * sizeof(double) + 8 * 256 * sizeof(double) ? 2 : 0;
#ifdef OMV_LBA_FORCE_G
    h->use_lds = 0;
#endif
    h->ldlt_lds = h->use_lds == 1 ? ldlt_bytes : 0;
    // inertial information (EdgeInertial ctor :486-495) and random-walk information
    std::vector<double> info9((size_t)NI * 81), infoG((size_t)NI * 9), infoA((size_t)NI * 9);
    for (int i = 0; i < NI; ++i) {
        const float *pr = p->preint + (size_t)i * kPF + PreView::C;
        std::vector<double> A(81);
        for (int r = 0; r < 9; ++r)
            for (int c = 0; c < 9; ++c) A[r * 9 + c] = (double)pr[r * 15 + c];
        host_inv(A, 9);
        for (int r = 0; r < 9; ++r)
            for (int c = r + 1; c < 9; ++c) A[r * 9 + c] = A[c * 9 + r] = (A[r * 9 + c] + A[c * 9 + r]) / 2;
        std::vector<double> w, V;
        host_sym_eig(A, 9, w, V);
        for (double &x : w)
            if (x < 1e-12) x = 0;
        const double sc = p->imu_info_scale ? (double)p->imu_info_scale[i] : 1.0;
        for (int r = 0; r < 9; ++r)
            for (int c = 0; c < 9; ++c) {
                double s = 0;
                for (int k = 0; k < 9; ++k) s += V[r * 9 + k] * w[k] * V[c * 9 + k];
                info9[(size_t)i * 81 + r * 9 + c] = s * sc;
            }
        double g[9], a[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) g[3 * r + c] = pr[(9 + r) * 15 + 9 + c], a[3 * r + c] = pr[(12 + r) * 15 + 12 + c];
        inv3(g, &infoG[(size_t)9 * i]);
        inv3(a, &infoA[(size_t)9 * i]);
    }
    h->delta_mono = (double)(float)std::sqrt(5.991);   // thHuberMono / thHuberStereo are floats (:3028-3031)
    h->dsqr_mono = h->delta_mono * h->delta_mono;
    h->delta_st = (double)(float)std::sqrt(7.815);
    h->dsqr_st = h->delta_st * h->delta_st;
    rig.bf = (double)p->bf;
    h->delta_imu = std::sqrt(16.92);
    h->dsqr_imu = h->delta_imu * h->delta_imu;
    // ---- device allocations + uploads
    std::vector<void *> &ow = h->owned;
    auto up = [&](auto *dst, const auto *src, size_t n) {
        return hipMemcpy(dst, src, n * sizeof(*src), hipMemcpyHostToDevice);
    };
    for (int b = 0; b < 3; ++b) {
        // one contiguous block per state: Rwb | twb | Rcw | tcw | vel | bg | ba | pts (one copy to read back)
        State &s = h->st[b];
        double *blk = dalloc<double>(ow, h->state_doubles());
        if (!blk) return OMV_ERR_HIP;
        s.Rwb = blk, s.twb = s.Rwb + 9 * K, s.Rcw = s.twb + 3 * K, s.tcw = s.Rcw + 9 * K * C;
        s.vel = s.tcw + 3 * K * C, s.bg = s.vel + 3 * K, s.ba = s.bg + 3 * K, s.pts = s.ba + 3 * K;
        HIP_OK(up(s.Rwb, p->Rwb, 9 * K));
        HIP_OK(up(s.twb, p->twb, 3 * K));
        HIP_OK(up(s.Rcw, p->Rcw, 9 * K * C));
        HIP_OK(up(s.tcw, p->tcw, 3 * K * C));
        HIP_OK(up(s.vel, p->vel, 3 * K));
        HIP_OK(up(s.bg, p->bg, 3 * K));
        HIP_OK(up(s.ba, p->ba, 3 * K));
        std::vector<double> pts((size_t)3 * P);
        for (int q = 0; q < P; ++q)
            for (int d = 0; d < 3; ++d) pts[3 * q + d] = p->pts[3 * (size_t)order[q] + d];
        HIP_OK(up(s.pts, pts.data(), pts.size()));
    }
    h->cur = 0;
    int *d_e_pt = dalloc<int>(ow, E), *d_e_kf = dalloc<int>(ow, E), *d_e_cam = dalloc<int>(ow, E),
        *d_e_slot = dalloc<int>(ow, E);
    double *d_e_obs = dalloc<double>(ow, 2 * (size_t)E);
    float *d_e_w = dalloc<float>(ow, E), *d_e_ur = dalloc<float>(ow, E);
    if (!d_e_w) return OMV_ERR_HIP;
    HIP_OK(up(d_e_pt, e_pt.data(), E));
    HIP_OK(up(d_e_kf, e_kf.data(), E));
    HIP_OK(up(d_e_cam, e_cam.data(), E));
    HIP_OK(up(d_e_slot, e_slot.data(), E));
    HIP_OK(up(d_e_obs, e_obs.data(), 2 * (size_t)E));
    HIP_OK(up(d_e_w, e_w.data(), E));
    if (!d_e_ur) return OMV_ERR_HIP;
    HIP_OK(up(d_e_ur, e_ur.data(), E));
    h->E = Edges{d_e_pt, d_e_kf, d_e_cam, d_e_slot, d_e_obs, d_e_w, d_e_ur, E};
    int *d_pt_edge = dalloc<int>(ow, P + 1), *d_pt_slot = dalloc<int>(ow, P + 1), *d_slot_kf = dalloc<int>(ow, h->n_slots),
        *d_slot_edge = dalloc<int>(ow, h->n_slots + 1);
    int16_t *d_slot_lkf = dalloc<int16_t>(ow, h->n_slots);
    double *d_lnd = dalloc<double>(ow, 12 * (size_t)P), *d_M = dalloc<double>(ow, 18 * (size_t)h->n_slots),
           *d_rec = dalloc<double>(ow, 36 * (size_t)blk_start[n_slots]),
           *d_rec_rhs = dalloc<double>(ow, 12 * (size_t)rhs_start[nb]);
    if (!d_rec || !d_rec_rhs || !d_M || !d_lnd || !d_slot_lkf || !d_slot_edge) return OMV_ERR_HIP;
    HIP_OK(up(d_pt_edge, pt_edge.data(), P + 1));
    HIP_OK(up(d_pt_slot, pt_slot.data(), P + 1));
    HIP_OK(up(d_slot_edge, slot_edge.data(), h->n_slots + 1));
    if (h->n_slots > 0) HIP_OK(up(d_slot_kf, slot_kf.data(), h->n_slots));
    if (h->n_slots > 0) HIP_OK(up(d_slot_lkf, slot_lkf.data(), h->n_slots));
    {
        auto upl = [&](const auto &v) {
            using T = typename std::decay_t<decltype(v)>::value_type;
            T *d = dalloc<T>(ow, v.size());
            if (d && !v.empty() && up(d, v.data(), v.size()) != hipSuccess) d = nullptr;
            return (const T *)d;
        };
        Land &L = h->L;
        L = Land{d_pt_edge, d_pt_slot, d_slot_kf, d_slot_edge, d_slot_lkf, d_lnd, d_M, P,
                 upl(grp_pt), upl(grp_w), upl(grp_tp), upl(tp),
                 upl(grp_blk), upl(blkoff), upl(grp_kf), upl(rhsoff), d_rec, d_rec_rhs};
        if (!L.grp_pt || !L.grp_w || !L.grp_tp || !L.tp || !L.grp_blk || !L.blkoff ||
            !L.grp_kf || !L.rhsoff)
            return OMV_ERR_HIP;
        h->d_big = upl(big_grp);
        std::vector<int16_t> e_lkf(E);
        for (int e = 0; e < E; ++e) e_lkf[e] = slot_lkf[e_slot[e]];
        h->d_e_lkf = upl(e_lkf);
        h->d_lkf_kf = upl(lkf_kf);
        if (!h->d_big || !h->d_e_lkf || !h->d_lkf_kf) return OMV_ERR_HIP;
    }
    h->d_offP = dalloc<int>(ow, K), h->d_offV = dalloc<int>(ow, K), h->d_offG = dalloc<int>(ow, K),
    h->d_offA = dalloc<int>(ow, K);
    HIP_OK(up(h->d_offP, offP.data(), K));
    HIP_OK(up(h->d_offV, offV.data(), K));
    HIP_OK(up(h->d_offG, offG.data(), K));
    HIP_OK(up(h->d_offA, offA.data(), K));
    h->R = Red{nred, h->d_offP, K};
    // inertial
    int *d_k1 = dalloc<int>(ow, NI), *d_k2 = dalloc<int>(ow, NI);
    float *d_pre = dalloc<float>(ow, (size_t)NI * kPF);
    double *d_i9 = dalloc<double>(ow, (size_t)NI * 81), *d_iG = dalloc<double>(ow, (size_t)NI * 9),
           *d_iA = dalloc<double>(ow, (size_t)NI * 9);
    uint8_t *d_rob = dalloc<uint8_t>(ow, NI);
    h->d_imu_contrib = dalloc<double>(ow, (size_t)NI * kImuContrib);
    if (!d_rob || !h->d_imu_contrib) return OMV_ERR_HIP;
    if (NI > 0) {
        HIP_OK(up(d_k1, p->imu_kf1, NI));
        HIP_OK(up(d_k2, p->imu_kf2, NI));
        HIP_OK(up(d_pre, p->preint, (size_t)NI * kPF));
        HIP_OK(up(d_i9, info9.data(), info9.size()));
        HIP_OK(up(d_iG, infoG.data(), infoG.size()));
        HIP_OK(up(d_iA, infoA.data(), infoA.size()));
        std::vector<uint8_t> rob(NI, 0);
        if (p->imu_robust) std::copy(p->imu_robust, p->imu_robust + NI, rob.begin());
        HIP_OK(up(d_rob, rob.data(), NI));
    }
    h->I = Imu{NI, d_k1, d_k2, d_pre, d_i9, d_iG, d_iA, d_rob, h->d_offP, h->d_offV, h->d_offG, h->d_offA};
    // reduction work lists
    auto upv = [&](const auto &v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        T *d = dalloc<T>(ow, v.size());
        if (d && !v.empty() && up(d, v.data(), v.size()) != hipSuccess) d = nullptr;
        return (const T *)d;
    };
    {
        Gather &g = h->G;
        g.blk_start = upv(blk_start), g.rhs_start = upv(rhs_start);
        g.imu_blk = upv(imu_blk), g.ib_start = upv(ib_start), g.imu_vec = upv(imu_vec), g.iv_start = upv(iv_start);
        g.contrib = h->d_imu_contrib;
        if (!g.blk_start || !g.rhs_start || !g.imu_blk || !g.ib_start || !g.imu_vec || !g.iv_start) return OMV_ERR_HIP;
    }
    // block pattern + level schedule
    {
        BlockPat &B = h->BP;
        B.nb = nb, B.n_slots = n_slots, B.n_lev = n_lev;
        B.slot_kr = upv(slot_kr), B.slot_kc = upv(slot_kc);
        std::vector<int> blob;
        auto put = [&](const auto &v) {   // 16-byte aligned sub-array
            const size_t off = blob.size(), n = v.size() * sizeof(v[0]) / sizeof(int);
            blob.resize(off + ((n + 3) & ~(size_t)3));
            if (n) std::memcpy(blob.data() + off, v.data(), n * sizeof(int));
            return off;
        };
        const size_t o_perm = put(perm), o_dslot = put(dslot), o_ls = put(lev_start), o_lc = put(lev_col);
        const size_t o_us = put(ug_start), o_usp = put(ug_split), o_cg = put(crit_grp), o_uts = put(ug_task_start);
        const size_t o_ug = put(ug), o_rss = put(rs_start), o_rs = put(rs), o_css = put(cs_start), o_cs = put(cs);
        const size_t o_ir = put(inv_rec);
        const int *d_blob = upv(blob);
        if (!B.slot_kr || !B.slot_kc || !d_blob) return OMV_ERR_HIP;
        B.blob = d_blob;
        B.perm = d_blob + o_perm, B.dslot = d_blob + o_dslot, B.lev_start = d_blob + o_ls, B.lev_col = d_blob + o_lc;
        B.ug_start = d_blob + o_us, B.ug_split = d_blob + o_usp, B.crit_grp = d_blob + o_cg;
        B.ug_task_start = d_blob + o_uts, B.ug = (const int4 *)(d_blob + o_ug);
        B.rs_start = d_blob + o_rss, B.rs = (const int2 *)(d_blob + o_rs);
        B.cs_start = d_blob + o_css, B.cs = (const int2 *)(d_blob + o_cs);
        B.inv_rec = (const int4 *)(d_blob + o_ir);
        // stage the schedule in LDS when it fits beside the blocks and vectors
        const size_t sched_bytes = blob.size() * sizeof(int);
        B.blob_ints = 0;
        B.n_lds = n_slots;
        if (h->use_lds == 2) {   // hybrid: the vectors and the schedule in LDS, then as many blocks as fit
            const size_t vb = 2 * (size_t)nred * sizeof(double);
            const bool sch = vb + sched_bytes + 8 * 256 * sizeof(double) <= kLdltLds;
            B.n_lds = std::min(n_slots, (int)((kLdltLds - vb - (sch ? sched_bytes : 0)) / (256 * sizeof(double))));
            h->ldlt_lds = (size_t)B.n_lds * 256 * sizeof(double) + vb + (sch ? sched_bytes : 0);
            B.blob_ints = sch ? (int)blob.size() : 0;
        } else if (h->use_lds && h->ldlt_lds + sched_bytes <= kLdltLds) {
            h->ldlt_lds += sched_bytes;
            B.blob_ints = (int)blob.size();
        }
    }
    // work buffers
    h->d_err = dalloc<double>(ow, 2 * (size_t)E);
    h->d_chi2 = dalloc<double>(ow, E);
    h->d_err3 = dalloc<double>(ow, E);
    h->d_err9 = dalloc<double>(ow, 19 * (size_t)NI);   // [9n errors | n chi2 | 9n rotation errors eR]
    h->d_err_b = dalloc<double>(ow, 2 * (size_t)E);       // the device driver's second (double-buffered) set
    h->d_chi2_b = dalloc<double>(ow, E);
    h->d_err3_b = dalloc<double>(ow, E);
    h->d_err9_b = dalloc<double>(ow, 19 * (size_t)NI);
    h->d_partial = dalloc<double>(ow, std::max(1, h->n_lgrp));
    h->d_imu_partial = dalloc<double>(ow, 1);
    h->d_partial0 = dalloc<double>(ow, std::max(1, h->n_lgrp));
    h->d_imu_partial0 = dalloc<double>(ow, 1);
    h->d_scale_partial = dalloc<double>(ow, h->n_lgrp + 1);
    h->d_out = dalloc<double>(ow, 4);
    // [packed blocks | b | coef]: contiguous, the one buffer a sharded solve all-reduces per trial
    h->d_S = dalloc<double>(ow, (size_t)n_slots * 256 + 2 * (size_t)nred);
    h->d_bb = h->d_S + (size_t)n_slots * 256;
    h->d_coef = h->d_bb + nred;
    h->n_reduce = (size_t)n_slots * 256 + 2 * (size_t)nred;
    h->d_x = dalloc<double>(ow, nred);
    h->d_scratch = dalloc<double>(ow, h->use_lds == 1 ? 8 : (size_t)n_slots * 256 + 2 * (size_t)nred + 8);
    h->d_fail = dalloc<int>(ow, 1);
    if (!h->d_fail) return OMV_ERR_HIP;
    HIP_OK(hipMemset(h->d_imu_partial, 0, sizeof(double)));
    HIP_OK(hipMemset(h->d_imu_partial0, 0, sizeof(double)));
    // device epilogue (single rank): caller-order permutations, trackDepth in device order, the staging block
    if (h->world == 1) {
        std::vector<float> td(P, 1e30f);
        if (p->pt_track_depth)
            for (int q = 0; q < P; ++q) td[q] = p->pt_track_depth[order[q]];
        h->d_perm_edge = dalloc<int>(ow, E), h->d_perm_pt = dalloc<int>(ow, P), h->d_track_depth = dalloc<float>(ow, P);
        const size_t head = (size_t)(h->st[0].pts - h->st[0].Rwb);
        h->stage_bytes = (head + 3 * (size_t)P + ((size_t)E + 7) / 8 + (size_t)E) * sizeof(double);
        h->d_stage = dalloc<double>(ow, (h->stage_bytes + 7) / 8);
        if (!h->d_perm_edge || !h->d_perm_pt || !h->d_track_depth || !h->d_stage) return OMV_ERR_HIP;
        if (E > 0) HIP_OK(up(h->d_perm_edge, h->perm_edge.data(), E));
        if (P > 0) HIP_OK(up(h->d_perm_pt, order.data(), P));
        if (P > 0) HIP_OK(up(h->d_track_depth, td.data(), P));
        HIP_OK(hipHostMalloc((void **)&h->h_stage, h->stage_bytes, hipHostMallocDefault));
    }
    return OMV_OK;
}

}  // extern "C"

// ---- the LM driver ---------------------------------------------------------------------------------
// computeActiveErrors: the visual and inertial errors in one launch (err_kernel).
// lba_errors: the errors of state s into the first error buffer (host driver, optimize()'s start, evaluation);
// lba_trial_errors: the device driver's trial state and buffer (role 1 of the control block's `cur`).
// n_grp_err: the partial count of the visual errors (one per landmark group, in the group order).
// launch_errors: s0 / s1 and the error buffers by role (role_buf); `xp` (a trial): the landmarks' back-substitution
// first, from the role-0 state into the role's state.  The host driver keeps one error buffer (both ErrBufs eb(0)).
static omv_status launch_errors(omv_lba *h, const State &s0, const State &s1, const LmCtl *ctl, int gate, int role,
                                LmReset reset = LmReset{}, bool init_partials = false, const double *xp = nullptr,
                                double lambda = 0.0, bool one_buffer = false, int n_acc = 0) {
    const int ng = h->n_mono > 0 || xp ? h->n_lgrp : 0;
    const int lead = xp || h->imu_here ? 1 : 0;
    const int blocks = (ng > 0 ? omv::xcd_grid(ng) : 0) + lead;
    const ErrTrial T{xp, n_acc % 3 == 2 ? 1 : 0, h->d_bb, lambda, h->d_offV, h->d_offG, h->d_offA, h->n_opt, h->d_e_lkf,
                     h->d_lkf_kf};
    const size_t lds = (3 * (size_t)kGrpLand + 12 * (size_t)kGrpW * h->rig.n_cams) * sizeof(double);
    if (blocks > 0)
        err_kernel<<<blocks, 256, lds, h->stream>>>(ng, lead, h->imu_here ? 1 : 0, h->rig, s0, s1, h->E, h->L, h->R, T,
                                                    h->delta_mono, h->dsqr_mono, h->delta_st, h->dsqr_st, h->eb(0),
                                                    one_buffer ? h->eb(0) : h->eb(1),
                                                    init_partials ? h->d_partial0 : h->d_partial, h->d_scale_partial,
                                                    h->I, h->delta_imu, h->dsqr_imu,
                                                    init_partials ? h->d_imu_partial0 : h->d_imu_partial, ctl, gate, role,
                                                    reset);
    return hipGetLastError() == hipSuccess ? OMV_OK : OMV_ERR_HIP;
}
static int n_grp_err(const omv_lba *h) { return h->n_mono > 0 ? h->n_lgrp : 0; }
static omv_status lba_errors(omv_lba *h, const State &s) { return launch_errors(h, s, s, nullptr, kGateAlways, 0); }
// the device driver's trial: back-substitution + errors into the trial buffer (role 1)
static omv_status lba_trial_errors(omv_lba *h, const LmCtl *c) {
    return launch_errors(h, h->st[0], h->st[1], c, kGateTrial, 1, LmReset{}, false, h->d_x, 0.0);
}

// In-place SUM over the ranks of a sharded solve (no-op on one rank).
// The collective path runs whenever a communicator was given (omv_lba_set_comm), a single rank included: one RCCL
// rank exercises exactly the multi-rank call sequence (stream order, in-place buffers, host-sync count).
static bool lba_collective(const omv_lba *h) { return h->allreduce != nullptr; }
static omv_status lba_allreduce(omv_lba *h, double *buf, size_t n) {
    if (!lba_collective(h)) return OMV_OK;
    HIP_OK(hipGetLastError());
    return h->allreduce(h->ar_ctx, buf, n, (void *)h->stream) == 0 ? OMV_OK : OMV_ERR_HIP;
}

// n_scale counts the update's partials (pose part first); only rank 0 contributes the pose part.
static omv_status lba_read_scalars(omv_lba *h, int n_scale, double out[3], bool with_fail) {
    const int s0 = (h->rank > 0 && n_scale > 0) ? 1 : 0;
    finish_kernel<<<1, 256, 0, h->stream>>>(h->d_partial, n_grp_err(h), h->d_imu_partial,
                                           h->d_scale_partial + s0, n_scale - s0, with_fail ? h->d_fail : nullptr,
                                           h->d_out);
    omv_status rs = lba_allreduce(h, h->d_out, 2);
    if (rs != OMV_OK) return rs;
    HIP_OK(hipMemcpyAsync(h->h_out, h->d_out, 3 * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    ++h->host_syncs;
    for (int q = 0; q < 3; ++q) out[q] = h->h_out[q];
    return OMV_OK;
}

// Residuals + Jacobians of the visual edges at the current state, in the caller's order; EdgeMono
// rows go to the mono_* arrays (2 rows), EdgeStereo rows to the stereo_* arrays (3 rows).
static omv_status lba_eval(omv_lba *h, double *mono_err, double *mono_jx, double *mono_jp, double *imu_err,
                           double *st_err, double *st_jx, double *st_jp) {
    if (!h) return OMV_ERR_ARG;
    const State &s = h->st[h->cur];
    omv_status r = lba_errors(h, s);
    if (r != OMV_OK) return r;
    std::vector<double> jx, jp;
    double *d_jx = nullptr, *d_jp = nullptr;
    const int E = h->n_mono;
    const bool jac = mono_jx || mono_jp || st_jx || st_jp;
    if (jac && E > 0) {
        HIP_OK(hipMalloc(&d_jx, sizeof(double) * 9 * E));
        HIP_OK(hipMalloc(&d_jp, sizeof(double) * 18 * E));
        mono_jac_kernel<<<(E + 255) / 256, 256, 0, h->stream>>>(h->rig, s, h->E, d_jx, d_jp);
    }
    HIP_OK(hipStreamSynchronize(h->stream));
    std::vector<double> err(2 * (size_t)E), err3(E), e9(10 * (size_t)h->n_imu);
    if (E > 0) {
        HIP_OK(hipMemcpy(err.data(), h->d_err, err.size() * sizeof(double), hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(err3.data(), h->d_err3, err3.size() * sizeof(double), hipMemcpyDeviceToHost));
    }
    if (h->imu_here) HIP_OK(hipMemcpy(e9.data(), h->d_err9, e9.size() * sizeof(double), hipMemcpyDeviceToHost));
    if (d_jx) {
        jx.resize(9 * (size_t)E), jp.resize(18 * (size_t)E);
        HIP_OK(hipMemcpy(jx.data(), d_jx, jx.size() * sizeof(double), hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(jp.data(), d_jp, jp.size() * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipFree(d_jx);
        (void)hipFree(d_jp);
    }
    const int EM = h->n_mono_all;
    for (int e = 0; e < E; ++e) {   // back to the caller's edge order
        const int o = h->perm_edge[e];
        if (o < EM) {
            if (mono_err) mono_err[2 * o] = err[2 * e], mono_err[2 * o + 1] = err[2 * e + 1];
            if (mono_jx) std::memcpy(mono_jx + 6 * (size_t)o, &jx[9 * (size_t)e], 48);
            if (mono_jp) std::memcpy(mono_jp + 12 * (size_t)o, &jp[18 * (size_t)e], 96);
        } else {
            const size_t q = (size_t)(o - EM);
            if (st_err) st_err[3 * q] = err[2 * e], st_err[3 * q + 1] = err[2 * e + 1], st_err[3 * q + 2] = err3[e];
            if (st_jx) std::memcpy(st_jx + 9 * q, &jx[9 * (size_t)e], 72);
            if (st_jp) std::memcpy(st_jp + 18 * q, &jp[18 * (size_t)e], 144);
        }
    }
    if (imu_err && h->imu_here) std::memcpy(imu_err, e9.data(), 9 * sizeof(double) * h->n_imu);
    return OMV_OK;
}

extern "C" {

omv_status omv_lba_evaluate(omv_lba *h, double *mono_err, double *mono_jx, double *mono_jp, double *imu_err) {
    return lba_eval(h, mono_err, mono_jx, mono_jp, imu_err, nullptr, nullptr, nullptr);
}

omv_status omv_lba_evaluate_stereo(omv_lba *h, double *stereo_err, double *stereo_jx, double *stereo_jp) {
    return lba_eval(h, nullptr, nullptr, nullptr, nullptr, stereo_err, stereo_jx, stereo_jp);
}

static omv_status lba_finish_result(omv_lba *h, const omv_lba_opts *o, omv_lba_problem *p, omv_lba_result *res);
static bool lba_epilogue_ok(const omv_lba *h);
static omv_status lba_enqueue_epilogue(omv_lba *h, bool want_chi2);

// buildSystem + the landmark Schur complement at state A (the current state; B the other buffer, picked by the control
// block's `cur` on the device driver): the landmark groups and the inertial edges' quadratic forms in one launch, side
// by side (build_all_kernel), then the reduced system assembled per block (assemble_kernel).  Every sum is in a fixed
// order: the system is identical run to run.  lambda enters the landmark groups (R R^T = Hll + lambda I), so both run
// every trial; on a sharded solve lambda enters the pose diagonal once (rank 0), every rank damps its own landmarks.
static omv_status launch_build(omv_lba *h, const State &A, const State &B, const LmCtl *c, double lambda) {
    const int n_imu = h->imu_here ? h->n_imu : 0, n_imu_pad = (n_imu + 7) & ~7;
    const int grid = n_imu_pad + (h->n_lgrp > 0 ? omv::xcd_grid(h->n_lgrp) : 0);
    if (grid > 0)
        build_all_kernel<<<grid, kGrpEdges, kBuildLds, h->stream>>>(
            h->rig, A, B, h->E, h->L, h->n_lgrp, h->I, n_imu, n_imu_pad, lambda, h->delta_mono, h->dsqr_mono,
            h->delta_st, h->dsqr_st, h->delta_imu, h->dsqr_imu, h->eb(0), h->eb(1), h->d_imu_contrib, c);
    if (h->n_big > 0)
        build_big_kernel<<<h->n_big, kGrpEdges, kBuildLds, h->stream>>>(h->rig, A, B, h->E, h->L, h->d_big, h->n_big,
                                                                        lambda, h->delta_mono, h->dsqr_mono, h->delta_st,
                                                                        h->dsqr_st, h->eb(0), h->eb(1), c);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

static omv_status launch_assemble(omv_lba *h, double lambda, const LmCtl *c) {
    assemble_kernel<<<h->BP.n_slots, 256, 0, h->stream>>>(h->G, h->I, h->BP, h->L.rec, h->L.rec_rhs, lambda,
                                                          h->rank == 0 ? 1 : 0, h->d_S, h->d_bb, h->d_coef, c);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

static void launch_ldlt(omv_lba *h, const LmCtl *c) {
    if (h->use_lds == 1)
        ldlt_kernel<0><<<1, kLdltThreads, h->ldlt_lds, h->stream>>>(h->d_S, h->BP, h->d_bb, h->d_coef, h->d_x,
                                                                    h->d_scratch, h->d_fail, c);
    else if (h->use_lds == 2)
        ldlt_kernel<2><<<1, kLdltThreads, h->ldlt_lds, h->stream>>>(h->d_S, h->BP, h->d_bb, h->d_coef, h->d_x,
                                                                    h->d_scratch, h->d_fail, c);
    else
        ldlt_kernel<1><<<1, kLdltThreads, 0, h->stream>>>(h->d_S, h->BP, h->d_bb, h->d_coef, h->d_x, h->d_scratch,
                                                          h->d_fail, c);
}

// One LM step of the device driver: the gated kernel sequence (see LmCtl).  The state and error buffers are
// double-buffered: the kernels take both (st[0], st[1]) and pick the current / trial one by the control block's
// `cur`, an accepted trial flips it -- no copy launch, and no recomputation of the current errors after a rejected
// trial.  With `ev`, events bracket the stages (build, Schur, solve, update + errors).
static omv_status lba_step(omv_lba *h, hipEvent_t *ev) {
    hipStream_t st = h->stream;
    LmCtl *c = h->d_ctl;
    const State &A = h->st[0], &B = h->st[1];
    omv_status rs;
    if (ev) HIP_OK(hipEventRecord(ev[0], st));
    if ((rs = launch_build(h, A, B, c, 0.0)) != OMV_OK) return rs;
    if (ev) HIP_OK(hipEventRecord(ev[1], st));
    if ((rs = launch_assemble(h, 0.0, c)) != OMV_OK) return rs;
    // sharded: one in-place SUM of this rank's partial reduced system [blocks | b | Schur rhs], ordered on the stream
    if ((rs = lba_allreduce(h, h->d_S, h->n_reduce)) != OMV_OK) return rs;
    if (ev) HIP_OK(hipEventRecord(ev[2], st));
    launch_ldlt(h, c);
    if (ev) HIP_OK(hipEventRecord(ev[3], st));
    if ((rs = lba_trial_errors(h, c)) != OMV_OK) return rs;
    const int nmb = n_grp_err(h), nsc = 1 + h->n_lgrp;
    const double *pre = nullptr;
    if (lba_collective(h)) {   // [chi(A), chi, computeScale] of this rank's edges / landmarks, summed over the ranks
        const int s0 = h->rank > 0 ? 1 : 0;   // the keyframe part of computeScale enters once (rank 0)
        trial_scalars_kernel<<<1, 256, 0, st>>>(c, h->d_partial, nmb, h->d_imu_partial, h->d_scale_partial + s0,
                                                nsc - s0, h->d_out, h->d_partial0, h->d_imu_partial0);
        if ((rs = lba_allreduce(h, h->d_out, 3)) != OMV_OK) return rs;
        pre = h->d_out;
    }
    finish_trial_kernel<<<1, 256, 0, st>>>(c, h->d_partial, nmb, h->d_imu_partial, h->d_scale_partial, nsc, h->d_fail,
                                           pre, h->d_partial0, h->d_imu_partial0);
    if (ev) HIP_OK(hipEventRecord(ev[4], st));
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

// optimize() with the LM control on the device: the initial errors, then LM steps in batches (opt_it first: every
// iteration takes at least one trial) until the device reports the end; one read-back per batch (host_syncs counts
// them); the last accepted trial's state copied into A.  Identical decisions to the host-driven loop below.  A
// sharded solve (world > 1) runs the same gated steps launched directly (its two all-reduces per step are calls into
// the caller's collective, ordered on the handle's stream): every rank reaches identical decisions from the
// all-reduced system and scalars, so every rank launches the same steps and collectives.
static omv_status lba_optimize_device(omv_lba *h, const omv_lba_opts *o, omv_lba_result *res) {
    const bool want_chi2 = res->mono_chi2 || res->stereo_chi2;
    h->epi_ready = false;
    hipStream_t st = h->stream;
    if (h->cur != 0) {   // the device path keeps the current state in st[0]
        HIP_OK(hipMemcpyAsync(h->st[0].Rwb, h->st[1].Rwb, h->state_doubles() * sizeof(double), hipMemcpyDeviceToDevice,
                              st));
        h->cur = 0;
    }
    omv_status rs;
    h->host_syncs = 0;
    const int nmb = n_grp_err(h);
    const bool sharded = lba_collective(h);
    if (o->opt_it > 0 && nmb + (h->imu_here ? 1 : 0) > 0) {
        // the initial errors into their own partials, the control block reset by the same launch; the first step's
        // bookkeeping sums the initial chi (through the first all-reduce on a sharded solve)
        if ((rs = launch_errors(h, h->st[0], h->st[0], nullptr, kGateAlways, 0,
                                LmReset{h->d_ctl, o->opt_it, o->max_trials, o->lambda_init}, true)) != OMV_OK)
            return rs;
    } else {
        if ((rs = lba_errors(h, h->st[0])) != OMV_OK) return rs;
        if (sharded) {
            trial_scalars_kernel<<<1, 256, 0, st>>>(nullptr, h->d_partial, nmb, h->d_imu_partial, nullptr, 0, h->d_out,
                                                    nullptr, nullptr);
            if ((rs = lba_allreduce(h, h->d_out, 3)) != OMV_OK) return rs;
        }
        ctl_init_kernel<<<1, 256, 0, st>>>(h->d_ctl, h->d_partial, nmb, h->d_imu_partial, o->opt_it, o->max_trials,
                                           o->lambda_init, sharded ? h->d_out : nullptr);
    }
    HIP_OK(hipGetLastError());
    const bool direct = h->timing || sharded;   // a collective call cannot be captured
    if (!direct && !h->step_exec) {   // capture one step and four steps (the problem's pointers are fixed
                                         // until set_problem); a batch is launched as 4-step graphs + single steps
        for (int n : {1, 4}) {
            HIP_OK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            for (int q = 0; q < n && rs == OMV_OK; ++q) rs = lba_step(h, nullptr);
            hipGraph_t g = nullptr;
            const hipError_t ce = hipStreamEndCapture(st, &g);
            if (rs != OMV_OK) return rs;
            if (ce != hipSuccess) {
                fprintf(stderr, "omv: LM step capture failed: %s\n", hipGetErrorString(ce));
                return OMV_ERR_HIP;
            }
            (n == 1 ? h->step_graph : h->step4_graph) = g;
            HIP_OK(hipGraphInstantiate(n == 1 ? &h->step_exec : &h->step4_exec, g, nullptr, nullptr, 0));
        }
    }
    // the fused batch: four steps, the epilogue and the read-backs captured together (once per problem and chi2 mode)
    const bool fuse_epi = !direct && lba_epilogue_ok(h);
    const int wc = want_chi2 ? 1 : 0;
    if (fuse_epi && !h->step4e_exec[wc]) {
        HIP_OK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        rs = OMV_OK;
        for (int q = 0; q < 4 && rs == OMV_OK; ++q) rs = lba_step(h, nullptr);
        if (rs == OMV_OK) rs = lba_enqueue_epilogue(h, want_chi2);
        const hipError_t me = hipMemcpyAsync(h->h_ctl, h->d_ctl, sizeof(LmCtl), hipMemcpyDeviceToHost, st);
        hipGraph_t g = nullptr;
        const hipError_t ce = hipStreamEndCapture(st, &g);
        if (rs != OMV_OK) return rs;
        if (ce != hipSuccess || me != hipSuccess) {
            fprintf(stderr, "omv: LM batch capture failed: %s\n", hipGetErrorString(ce != hipSuccess ? ce : me));
            return OMV_ERR_HIP;
        }
        h->step4e_graph[wc] = g;
        HIP_OK(hipGraphInstantiate(&h->step4e_exec[wc], g, nullptr, nullptr, 0));
        h->epi_ready = false;
    }
    const int max_steps = std::max(0, o->opt_it) * std::max(1, o->max_trials);
    std::vector<std::array<hipEvent_t, 5>> evs;
    int launched = 0, batch = std::min(std::max(0, o->opt_it), max_steps);
    while (true) {
        bool fused = false;   // this batch's last launch carried the epilogue and the control read-back
        for (int i = 0; i < batch;) {
            if (h->timing) {
                std::array<hipEvent_t, 5> e{};
                for (auto &x : e) HIP_OK(hipEventCreate(&x));
                evs.push_back(e);
                if ((rs = lba_step(h, evs.back().data())) != OMV_OK) return rs;
                ++i;
            } else if (direct) {
                if ((rs = lba_step(h, nullptr)) != OMV_OK) return rs;
                ++i;
            } else if (i + 4 <= batch) {
                fused = fuse_epi && i + 4 == batch;
                HIP_OK(hipGraphLaunch(fused ? h->step4e_exec[wc] : h->step4_exec, st));
                i += 4;
            } else {
                HIP_OK(hipGraphLaunch(h->step_exec, st));
                ++i;
            }
        }
        launched += batch;
        // the epilogue rides along with the control read-back (kept when the device reports the end)
        if (fused) {
            h->epi_ready = true, h->epi_chi2 = want_chi2;
        } else {
            const bool spec = lba_epilogue_ok(h);
            if (spec && (rs = lba_enqueue_epilogue(h, want_chi2)) != OMV_OK) return rs;
            HIP_OK(hipMemcpyAsync(h->h_ctl, h->d_ctl, sizeof(LmCtl), hipMemcpyDeviceToHost, st));
        }
        HIP_OK(hipStreamSynchronize(st));
        ++h->host_syncs;
        if (h->h_ctl->done || launched >= max_steps) break;
        h->epi_ready = false;
        batch = std::min(4, max_steps - launched);
    }
    if (!h->epi_ready) {   // the last accepted trial's state into A
        cur_copy_kernel<<<64, 256, 0, st>>>(h->d_ctl, h->st[1].Rwb, h->st[0].Rwb, h->state_doubles());
        HIP_OK(hipGetLastError());
    }
    const LmCtl &c = *h->h_ctl;
    for (double &m : h->stage_ms) m = 0;
    for (auto &e : evs) {
        float ms;
        for (int k = 0; k < 4; ++k) {
            HIP_OK(hipEventElapsedTime(&ms, e[k], e[k + 1]));
            h->stage_ms[k] += ms;
        }
        for (auto &x : e) (void)hipEventDestroy(x);
    }
    h->last_trials = c.trials;
    res->err = (float)c.err0;
    res->err_end = (float)c.errors_chi;
    res->iterations = c.its;
    res->trials = c.trials;
    res->lambda = c.lambda;
    return OMV_OK;
}

omv_status omv_lba_optimize(omv_lba *h, const omv_lba_opts *o, omv_lba_problem *p, omv_lba_result *res) {
    if (!h || !o || !p || !res) return OMV_ERR_ARG;
    hipStream_t st = h->stream;
    double sc[3];
    omv_status rs;
    for (double &m : h->stage_ms) m = 0;
    h->host_syncs = 0;
    if (!h->host_lm) {
        if ((rs = lba_optimize_device(h, o, res)) != OMV_OK) return rs;
        return lba_finish_result(h, o, p, res);
    }
    // err = activeRobustChi2 at the initial state (Optimizer.cc:3273-3274)
    if ((rs = lba_errors(h, h->st[h->cur])) != OMV_OK) return rs;
    if ((rs = lba_read_scalars(h, 0, sc, false)) != OMV_OK) return rs;
    res->err = (float)sc[0];
    double errors_chi = sc[0];
    bool errors_of_current = true;
    double lambda = 0, ni = 2;
    int nBad = 0, trials = 0, its = 0, n_acc = 0;   // n_acc: accepted updates (ImuCamPose::its, see LmCtl)
    for (int it = 0; it < o->opt_it; ++it) {
        ++its;
        State &A = h->st[h->cur];
        State &B = h->st[1 - h->cur];
        if (!errors_of_current) {
            if ((rs = lba_errors(h, A)) != OMV_OK) return rs;
            if ((rs = lba_read_scalars(h, 0, sc, false)) != OMV_OK) return rs;
            errors_chi = sc[0];
            errors_of_current = true;
        }
        double currentChi = errors_chi;
        const double iniChi = currentChi;
        if (it == 0) {
            lambda = o->lambda_init;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        float ms;
        do {
            // buildSystem + the landmark Schur complement at this trial's lambda (a retry rebuilds at the same state; this
            // driver has one error buffer, which the rejected trial overwrote: the current state's errors first)
            if (qmax > 0 && (rs = lba_errors(h, A)) != OMV_OK) return rs;
            HIP_OK(hipEventRecord(h->ev[0], st));
            if ((rs = launch_build(h, A, A, nullptr, lambda)) != OMV_OK) return rs;
            HIP_OK(hipEventRecord(h->ev[1], st));
            HIP_OK(hipEventRecord(h->ev[2], st));
            if ((rs = launch_assemble(h, lambda, nullptr)) != OMV_OK) return rs;
            // one exchange: sum the partial reduced systems [blocks | b | Schur rhs] of the landmark shards
            if ((rs = lba_allreduce(h, h->d_S, h->n_reduce)) != OMV_OK) return rs;
            HIP_OK(hipEventRecord(h->ev[3], st));
            launch_ldlt(h, nullptr);
            HIP_OK(hipEventRecord(h->ev[4], st));
            // the keyframe update and the landmarks' back-substitution A -> B, the trial's errors (one launch, this
            // driver's one error buffer)
            if ((rs = launch_errors(h, A, B, nullptr, kGateAlways, 1, LmReset{}, false, h->d_x, lambda, true, n_acc)) !=
                OMV_OK)
                return rs;
            if ((rs = lba_read_scalars(h, 1 + h->n_lgrp, sc, true)) != OMV_OK) return rs;
            const int fail = sc[2] != 0.0;
            HIP_OK(hipEventRecord(h->ev[5], st));
            HIP_OK(hipEventSynchronize(h->ev[5]));
            HIP_OK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
            h->stage_ms[0] += ms;
            HIP_OK(hipEventElapsedTime(&ms, h->ev[2], h->ev[3]));
            h->stage_ms[1] += ms;
            HIP_OK(hipEventElapsedTime(&ms, h->ev[3], h->ev[4]));
            h->stage_ms[2] += ms;
            HIP_OK(hipEventElapsedTime(&ms, h->ev[4], h->ev[5]));
            h->stage_ms[3] += ms;
            const bool ok = fail == 0;
            double tempChi = sc[0];
            errors_chi = sc[0];
            errors_of_current = false;   // the last computed errors belong to the trial state
            if (!ok) tempChi = std::numeric_limits<double>::max();
            double scale = ok ? sc[1] : 0.0;
            scale += 1e-3;
            rho = (currentChi - tempChi) / scale;
            ++trials;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
                ++n_acc;
                // fixed keyframes are identical in both buffers; make B the current state
                h->cur = 1 - h->cur;
                errors_of_current = true;
                // the next trial rewrites every optimisable keyframe and every point of the other buffer
            } else {
                lambda *= ni;
                ni *= 2;
            }
            qmax++;
        } while (rho < 0 && qmax < o->max_trials);
        if (qmax == o->max_trials || rho == 0) break;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) break;
    }
    h->last_trials = trials;
    res->err_end = (float)errors_chi;
    res->iterations = its;
    res->trials = trials;
    res->lambda = lambda;
    return lba_finish_result(h, o, p, res);
}

// The epilogue shared by both LM drivers: state write-back in the caller's order, per-edge chi2 and the
// reference's outlier / FAIL tests (Optimizer.cc:3282-3321).
// The single-rank device epilogue: state of A (an accepted last trial copied in first), outlier flags, chi2 when
// asked for and the points in the caller's order into the staging block [head | points | flags | chi2], then
// its read-back into pinned memory (not synchronised here).
static bool lba_epilogue_ok(const omv_lba *h) {
    return h->world == 1 && h->d_stage && h->cur == 0 && h->n_mono_all + h->n_stereo_all == h->n_mono;
}
static omv_status lba_enqueue_epilogue(omv_lba *h, bool want_chi2) {
    hipStream_t st = h->stream;
    const State &s = h->st[0];
    const int P = h->n_pts, E = h->n_mono;
    const size_t head = (size_t)(s.pts - s.Rwb), fl = ((size_t)E + 7) / 8;
    double *d_pts = h->d_stage + head;
    uint8_t *d_flags = (uint8_t *)(d_pts + 3 * (size_t)P);
    double *d_chi2 = d_pts + 3 * (size_t)P + fl;
    const int n = std::max(std::max(E, P), (int)head);
    epilogue_kernel<<<(n + 255) / 256, 256, 0, st>>>(h->rig, s, h->st[1], h->state_doubles(), h->E, h->d_perm_edge,
                                                     h->n_mono_all, h->d_track_depth,
                                                     h->d_perm_pt, P, d_flags, want_chi2 ? d_chi2 : nullptr, d_pts,
                                                     h->d_chi2, h->d_chi2_b, h->host_lm ? nullptr : h->d_ctl,
                                                     h->d_stage, (int)head);
    HIP_OK(hipGetLastError());
    const size_t bytes = (head + 3 * (size_t)P + fl + (want_chi2 ? (size_t)E : 0)) * sizeof(double);
    HIP_OK(hipMemcpyAsync(h->h_stage, h->d_stage, bytes, hipMemcpyDeviceToHost, st));
    h->epi_ready = true, h->epi_chi2 = want_chi2;
    return OMV_OK;
}

static omv_status lba_finish_result(omv_lba *h, const omv_lba_opts *o, omv_lba_problem *p, omv_lba_result *res) {
    hipStream_t st = h->stream;
    const State &s = h->st[h->cur];
    const int K = h->n_kf, C = h->rig.n_cams, P = h->n_pts, E = h->n_mono;
    const bool fail = (2 * res->err < res->err_end || std::isnan(res->err) || std::isnan(res->err_end)) && !o->large;
    res->status = fail ? OMV_LBA_FAIL : OMV_LBA_OK;
    auto take_head = [&](const double *q) {
        auto take = [&](double *dst, size_t n) {
            std::memcpy(dst, q, n * sizeof(double));
            q += n;
        };
        take(p->Rwb, 9 * (size_t)K), take(p->twb, 3 * (size_t)K), take(p->Rcw, 9 * (size_t)K * C);
        take(p->tcw, 3 * (size_t)K * C), take(p->vel, 3 * (size_t)K), take(p->bg, 3 * (size_t)K), take(p->ba, 3 * (size_t)K);
    };
    if (lba_epilogue_ok(h)) {
        // device epilogue: outlier flags / chi2 / points in the caller's order, one staging read-back (already in
        // flight with the LM control's last read-back when the device driver ran)
        const bool want_chi2 = res->mono_chi2 || res->stereo_chi2;
        if (!h->epi_ready || (want_chi2 && !h->epi_chi2)) {
            omv_status rs = lba_enqueue_epilogue(h, want_chi2);
            if (rs != OMV_OK) return rs;
            HIP_OK(hipStreamSynchronize(st));
        }
        h->epi_ready = false;
        const size_t head = (size_t)(s.pts - s.Rwb);
        take_head(h->h_stage);
        std::memcpy(p->pts, h->h_stage + head, 3 * sizeof(double) * (size_t)P);
        const uint8_t *hf = (const uint8_t *)(h->h_stage + head + 3 * (size_t)P);
        const double *hc = h->h_stage + head + 3 * (size_t)P + ((size_t)E + 7) / 8;
        const int EM = h->n_mono_all, ES = h->n_stereo_all;
        if (res->mono_chi2) std::memcpy(res->mono_chi2, hc, sizeof(double) * EM);
        if (res->stereo_chi2) std::memcpy(res->stereo_chi2, hc + EM, sizeof(double) * ES);
        if (res->mono_outlier) std::memcpy(res->mono_outlier, hf, EM);
        if (res->stereo_outlier) std::memcpy(res->stereo_outlier, hf + EM, ES);
        return OMV_OK;
    }
    // sharded rank: this rank's landmarks and edges only, on the host
    std::vector<double> stg(h->state_doubles()), chi2(E);
    HIP_OK(hipMemcpyAsync(stg.data(), s.Rwb, stg.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    // the last computed errors: buffer `last` of the device driver's control block (the host driver uses the first)
    const double *d_last_chi2 = (!h->host_lm && h->h_ctl && h->h_ctl->last) ? h->d_chi2_b : h->d_chi2;
    if (E > 0) HIP_OK(hipMemcpyAsync(chi2.data(), d_last_chi2, sizeof(double) * E, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    take_head(stg.data());
    {
        const double *q = stg.data() + (s.pts - s.Rwb);
        for (int i = 0; i < P; ++i)
            for (int d = 0; d < 3; ++d) p->pts[3 * (size_t)h->perm_pt[i] + d] = q[3 * (size_t)i + d];
    }
    for (int e = 0; e < E; ++e) {
        const int oe = h->perm_edge[e];
        if (oe >= h->n_mono_all) {   // EdgeStereo: chi2 > chi2Stereo2 (:3299-3311)
            const int q = oe - h->n_mono_all;
            if (res->stereo_chi2) res->stereo_chi2[q] = chi2[e];
            if (res->stereo_outlier) res->stereo_outlier[q] = chi2[e] > 7.815f ? 1 : 0;
            continue;
        }
        if (res->mono_chi2) res->mono_chi2[oe] = chi2[e];
        if (res->mono_outlier) {
            const int k = p->mono_kf[oe], c = p->mono_cam[oe], pt = p->mono_pt[oe];
            const double *R = p->Rcw + ((size_t)k * C + c) * 9, *t = p->tcw + ((size_t)k * C + c) * 3;
            const double *X = p->pts + 3 * (size_t)pt;
            const bool depth_pos = (R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2]) > 0.0;
            const bool close = p->pt_track_depth[pt] < 10.f;
            const double c2 = chi2[e];
            res->mono_outlier[oe] = ((c2 > 5.991f && !close) || (c2 > 1.5f * 5.991f && close) || !depth_pos) ? 1 : 0;
        }
    }
    return OMV_OK;
}

omv_status omv_lba_reset(omv_lba *h) {
    if (!h || !h->st[2].pts) return OMV_ERR_ARG;
    for (int b = 0; b < 2; ++b)
        HIP_OK(hipMemcpyAsync(h->st[b].Rwb, h->st[2].Rwb, h->state_doubles() * sizeof(double), hipMemcpyDeviceToDevice,
                              h->stream));
    h->cur = 0;
    HIP_OK(hipStreamSynchronize(h->stream));
    return OMV_OK;
}

omv_status omv_lba_set_comm(omv_lba *h, int rank, int world, omv_allreduce_fn allreduce, void *ctx) {
    if (!h || world < 1 || rank < 0 || rank >= world || (world > 1 && !allreduce)) return OMV_ERR_ARG;
    h->rank = rank, h->world = world, h->allreduce = allreduce, h->ar_ctx = ctx;
    return OMV_OK;
}

omv_status omv_lba_shard(omv_lba *h, int32_t *n_pts, int32_t *n_mono, int32_t *pt_index) {
    if (!h) return OMV_ERR_ARG;
    if (n_pts) *n_pts = h->n_pts;
    if (n_mono) *n_mono = h->n_mono;
    if (pt_index) std::copy(h->perm_pt.begin(), h->perm_pt.end(), pt_index);
    return OMV_OK;
}

omv_status omv_lba_enable_timing(omv_lba *h, int on) {
    if (!h) return OMV_ERR_ARG;
    h->timing = on != 0;
    return OMV_OK;
}

omv_status omv_lba_set_driver(omv_lba *h, int host_driven) {
    if (!h) return OMV_ERR_ARG;
    h->host_lm = host_driven != 0;
    return OMV_OK;
}

omv_status omv_lba_host_syncs(omv_lba *h, int *host_syncs, int *trials) {
    if (!h) return OMV_ERR_ARG;
    if (host_syncs) *host_syncs = h->host_syncs;
    if (trials) *trials = h->last_trials;
    return OMV_OK;
}

omv_status omv_lba_stage_ms(omv_lba *h, double *ms4, int *trials) {
    if (!h || !ms4) return OMV_ERR_ARG;
    for (int k = 0; k < 4; ++k) ms4[k] = h->stage_ms[k];
    if (trials) *trials = h->last_trials;
    return OMV_OK;
}

}  // extern "C"
