// Cycle costs of the grouped pose kernel's building blocks in isolation (one workgroup, nothing else on the GPU):
// the one-wave pivoted LDLT solve (15 and 30 states) and one visual edge per thread (error + Jacobian + normal terms).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I include -I openmavis_amd/csrc
//        tools/micro/pose_parts_bench.hip -o tools/micro/pose_parts_bench
#include "../../openmavis_amd/csrc/pose.hip"
#include <cmath>

namespace {

template <int N>
__device__ __forceinline__ bool ldlt_stage(const double *H, const double *b, double *x, int *pick, double *Lm, int lane, int stage) {
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
    if (stage == 1) return true;
    const int pi = in ? pick[lane] : 0;
    double r[N];
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? H[pi * N + pick[j]] : 0.0;
    if (!(lane_f64(r[0], 0) != 0.0)) {   // largest |diagonal| zero: Eigen stops with ZeroSign; the solve gives x = 0
        if (in) x[lane] = 0.0;
        wave_lds_sync();
        return true;
    }
    if (stage == 2) { if (in) x[lane] = r[N - 1]; return true; }
    int sign = 0;   // 0 ZeroSign, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
    double dmine = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double d = lane_f64(r[k], k);
        if (lane == k) dmine = d;
        if (fabs(d) > 0.0) {   // rows above k update with l = 0 (an exact no-op): no exec-mask branches or selects
            const double inv = 1.0 / d;
            const bool below = lane > k;
            const double l = below ? r[k] * inv : 0.0;
#pragma unroll
            for (int j = k + 1; j < N; ++j) r[j] = __builtin_fma(-l, lane_f64(r[j], k), r[j]);
            if (below) r[k] = l;
        }
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
    if (stage == 3) { if (in) x[lane] = r[N - 1] + dmine; return true; }
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


template <int N>
__global__ void __launch_bounds__(64) ldlt_bench(const double *Hin, const double *bin, double *xout, int reps,
                                                 unsigned long long *ticks, int stage) {
    __shared__ double H[N * N], b[N], x[N], Lm[N * N], cb[32];
    __shared__ int pick[N];
    const int lane = threadIdx.x;
    for (int q = lane; q < N * N; q += 64) H[q] = Hin[q];
    if (lane < N) b[lane] = bin[lane];
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        ok &= stage == 9 ? ldlt_pick_solve_wide<N>(H, b, x, pick, Lm, cb, lane) : stage ? ldlt_stage<N>(H, b, x, pick, Lm, lane, stage) : ldlt_pick_solve<N>(H, b, x, pick, Lm, lane);
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = wall_clock64();
    if (lane < N) xout[lane] = ok ? x[lane] : -1.0;
    if (lane == 0) ticks[0] = t1 - t0;
}

template <int N>
__global__ void __launch_bounds__(256) ldlt_elem_bench(const double *Hin, const double *bin, double *xout, int reps,
                                                      unsigned long long *ticks) {
    __shared__ double H[N * N], b[N], x[N], Lm[N * N], col[2 * N];
    __shared__ int pick[N], flag;
    const int tid = threadIdx.x;
    for (int q = tid; q < N * N; q += 256) H[q] = Hin[q];
    if (tid < N) b[tid] = bin[tid];
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        ok &= ldlt_elem_solve<N, 256>(H, b, x, pick, Lm, col, &flag, tid);
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = wall_clock64();
    if (tid < N) xout[tid] = ok ? x[tid] : -1.0;
    if (tid == 0) ticks[0] = t1 - t0;
}

__global__ void __launch_bounds__(256) edge_bench(Rig rig_in, const float *xw, const double *obs, int reps,
                                                  double *out, unsigned long long *ticks) {
    __shared__ Rig rig;
    __shared__ double sRcw[kMaxCams * 9], stcw[kMaxCams * 3];
    const int tid = threadIdx.x;
    for (int q = tid; q < (int)(sizeof(Rig) / 4); q += 256)
        reinterpret_cast<uint32_t *>(&rig)[q] = reinterpret_cast<const uint32_t *>(&rig_in)[q];
    for (int q = tid; q < kMaxCams * 9; q += 256) sRcw[q] = (q % 9 % 4 == 0) ? 1.0 : 0.0;
    for (int q = tid; q < kMaxCams * 3; q += 256) stcw[q] = 0.0;
    __syncthreads();
    VEdge v;
    v.cam = tid % rig.n_cams, v.kp = tid, v.stereo = false;
    v.obs[0] = obs[2 * tid], v.obs[1] = obs[2 * tid + 1], v.obs[2] = 0;
    v.w = 1.0;
    for (int q = 0; q < 3; ++q) v.X[q] = xw[3 * tid + q];
    double acc[kNormal];
    for (int q = 0; q < kNormal; ++q) acc[q] = 0;
    const unsigned long long t0 = wall_clock64();
    for (int r = 0; r < reps; ++r) {
        double rr[3], Xc[3], JP[18];
        const double c2 = edge_error(rig, sRcw, stcw, v, rr, Xc);
        double w1 = 1.0, r0;
        huber(c2, 2.4477, 5.991, r0, w1);
        edge_jac(rig, v, Xc, JP);
        const double om[3] = {-v.w * rr[0] * w1, -v.w * rr[1] * w1, 0.0};
        edge_normal(JP, false, v.w * w1, om, acc);
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = wall_clock64();
    double s = 0;
    for (int q = 0; q < kNormal; ++q) s += acc[q];
    out[tid] = s;
    if (tid == 0) ticks[0] = t1 - t0;
}

}  // namespace

int main() {
    const int reps = 200;
    std::vector<double> H30(900), b30(30), H15(225), b15(15);
    unsigned seed = 7;
    auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return (seed >> 8) / 16777216.0 - 0.5; };
    std::vector<double> M(900);
    for (auto &m : M) m = rnd();
    for (int i = 0; i < 30; ++i)
        for (int j = 0; j < 30; ++j) {
            double s = i == j ? 30.0 : 0.0;
            for (int k = 0; k < 30; ++k) s += M[i * 30 + k] * M[j * 30 + k];
            H30[i * 30 + j] = s;
        }
    for (int i = 0; i < 15; ++i)
        for (int j = 0; j < 15; ++j) H15[i * 15 + j] = H30[i * 30 + j];
    for (auto &v : b30) v = rnd();
    for (int i = 0; i < 15; ++i) b15[i] = b30[i];
    double *dH, *db, *dx;
    unsigned long long *dt, t;
    if (hipMalloc(&dH, 900 * 8) || hipMalloc(&db, 30 * 8) || hipMalloc(&dx, 256 * 8) || hipMalloc(&dt, 8)) return 1;
    for (int pass = 0; pass < 2; ++pass) {
        (void)hipMemcpy(dH, H15.data(), 225 * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b15.data(), 15 * 8, hipMemcpyHostToDevice);
        for (int stg = 1; stg <= 4; ++stg) {
            ldlt_bench<15><<<1, 64>>>(dH, db, dx, reps, dt, stg);
            (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
            if (pass) printf("ldlt<15> up to stage %d (1 pick, 2 gather, 3 factor, 4 solve): %.3f us\n", stg, t / 100.0 / reps);
        }
        ldlt_bench<15><<<1, 64>>>(dH, db, dx, reps, dt, 0);
        (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        if (pass) printf("ldlt_pick_solve<15>: %.3f us per solve\n", t / 100.0 / reps);
        (void)hipMemcpy(dH, H30.data(), 900 * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b30.data(), 30 * 8, hipMemcpyHostToDevice);
        ldlt_bench<30><<<1, 64>>>(dH, db, dx, reps, dt, 0);
        (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        if (pass) printf("ldlt_pick_solve<30>: %.3f us per solve\n", t / 100.0 / reps);
        std::vector<double> xa(30), xb(30);
        (void)hipMemcpy(xa.data(), dx, 30 * 8, hipMemcpyDeviceToHost);
        ldlt_bench<30><<<1, 64>>>(dH, db, dx, reps, dt, 9);
        (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(xb.data(), dx, 30 * 8, hipMemcpyDeviceToHost);
        double md = 0, mx = 0;
        for (int i = 0; i < 30; ++i) md = std::max(md, std::fabs(xa[i] - xb[i])), mx = std::max(mx, std::fabs(xa[i]));
        if (pass) printf("ldlt_pick_solve_wide<30>: %.3f us per solve (max |dx| %.3g of %.3g)\n", t / 100.0 / reps, md, mx);
        (void)hipMemcpy(dH, H15.data(), 225 * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b15.data(), 15 * 8, hipMemcpyHostToDevice);
        ldlt_bench<15><<<1, 64>>>(dH, db, dx, reps, dt, 0);
        (void)hipMemcpy(xa.data(), dx, 15 * 8, hipMemcpyDeviceToHost);
        ldlt_bench<15><<<1, 64>>>(dH, db, dx, reps, dt, 9);
        (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(xb.data(), dx, 15 * 8, hipMemcpyDeviceToHost);
        md = 0, mx = 0;
        for (int i = 0; i < 15; ++i) md = std::max(md, std::fabs(xa[i] - xb[i])), mx = std::max(mx, std::fabs(xa[i]));
        if (pass) printf("ldlt_pick_solve_wide<15>: %.3f us per solve (max |dx| %.3g of %.3g)\n", t / 100.0 / reps, md, mx);
        for (int n : {15, 30}) {
            (void)hipMemcpy(dH, n == 15 ? H15.data() : H30.data(), n * n * 8, hipMemcpyHostToDevice);
            (void)hipMemcpy(db, n == 15 ? b15.data() : b30.data(), n * 8, hipMemcpyHostToDevice);
            if (n == 15) ldlt_bench<15><<<1, 64>>>(dH, db, dx, reps, dt, 0);
            else ldlt_bench<30><<<1, 64>>>(dH, db, dx, reps, dt, 0);
            (void)hipMemcpy(xa.data(), dx, n * 8, hipMemcpyDeviceToHost);
            if (n == 15) ldlt_elem_bench<15><<<1, 256>>>(dH, db, dx, reps, dt);
            else ldlt_elem_bench<30><<<1, 256>>>(dH, db, dx, reps, dt);
            (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(xb.data(), dx, n * 8, hipMemcpyDeviceToHost);
            md = 0, mx = 0;
            for (int i = 0; i < n; ++i) md = std::max(md, std::fabs(xa[i] - xb[i])), mx = std::max(mx, std::fabs(xa[i]));
            if (pass) printf("ldlt_elem_solve<%d, 256>: %.3f us per solve (max |dx| %.3g of %.3g)\n", n, t / 100.0 / reps, md, mx);
        }
        (void)hipMemcpy(dH, H15.data(), 225 * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b15.data(), 15 * 8, hipMemcpyHostToDevice);
        // ties on the diagonal: the replayed pick order
        std::vector<double> Ht = H15;
        for (int i = 9; i < 15; ++i) Ht[i * 15 + i] = 50.0;
        (void)hipMemcpy(dH, Ht.data(), 225 * 8, hipMemcpyHostToDevice);
        ldlt_bench<15><<<1, 64>>>(dH, db, dx, reps, dt, 0);
        (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        if (pass) printf("ldlt_pick_solve<15> with diagonal ties: %.3f us per solve\n", t / 100.0 / reps);
    }
    Rig rig{};
    rig.n_cams = 5;
    for (int c = 0; c < 5; ++c) {
        const float k[8] = {380.f, 380.f, 360.f, 270.f, 0.01f, -0.002f, 0.0005f, -0.0001f};
        for (int q = 0; q < 8; ++q) rig.cam[c][q] = k[q];
        rig.model[c] = OMV_CAM_KB8;
        for (int q = 0; q < 9; ++q) rig.Rcb[c][q] = rig.Rbc[c][q] = (q % 4 == 0) ? 1.0 : 0.0;
    }
    std::vector<float> xw(768);
    std::vector<double> obs(512);
    for (int i = 0; i < 256; ++i) {
        xw[3 * i] = (float)(rnd() * 4), xw[3 * i + 1] = (float)(rnd() * 3), xw[3 * i + 2] = (float)(5 + rnd() * 4);
        obs[2 * i] = 360 + rnd() * 100, obs[2 * i + 1] = 270 + rnd() * 100;
    }
    float *dxw;
    double *dobs;
    if (hipMalloc(&dxw, 768 * 4) || hipMalloc(&dobs, 512 * 8)) return 1;
    (void)hipMemcpy(dxw, xw.data(), 768 * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dobs, obs.data(), 512 * 8, hipMemcpyHostToDevice);
    for (int pass = 0; pass < 2; ++pass) {
        edge_bench<<<1, 256>>>(rig, dxw, dobs, reps, dx, dt);
        (void)hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        if (pass) printf("visual edge (KB8, error + Jacobian + normal terms, 4 waves on one CU): %.3f us per edge pass\n",
                         t / 100.0 / reps);
    }
    return 0;
}
