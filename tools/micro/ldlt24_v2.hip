// Micro-benchmark: ldlt_pick_solve<N> (pose.hip) against a variant whose pivot-row broadcast goes through LDS for all
// entries but the next pivot's (issued at the start of the step, its latency behind the reciprocal chain) and whose
// factor columns are stored transposed as they are formed (no LDS transpose before the backward solve).  Same
// arithmetic, so the solutions must be bit-identical; cycles per solve by clock64.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include tools/micro/ldlt24_v2.hip -o /tmp/ldlt24_v2
#include <cstring>
#include "../../openmavis_amd/csrc/pose.hip"

namespace {
template <int N>
__device__ __forceinline__ bool ldlt_v2(const double *H, const double *b, double *x, int *pick, double *Lm, int lane) {
    constexpr int S = (N + 2) & ~1;   // stride of the transposed factor (even: 16-byte rows)
    double *Lt = Lm, *rowbuf = Lm + S * N;   // Lt[k * S + i] = L_ik (i > k); rowbuf: two pivot-row buffers of S
    const bool in = lane < N;
    if (!ldlt_pick_order<N>(H, pick, lane)) return false;
    wave_lds_sync();
    const int pi = in ? pick[lane] : 0;
    int pj[N];
#pragma unroll
    for (int j = 0; j < N; ++j) pj[j] = pick[j];
    double r[N];
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? H[pj[j] * N + pi] : 0.0;
    if (!(lane_f64(r[0], 0) != 0.0)) {
        if (in) x[lane] = 0.0;
        wave_lds_sync();
        return true;
    }
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
        if (below && in) Lt[k * S + lane] = r[k];
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
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = (in && j > lane) ? Lt[lane * S + j] : 0.0;   // r[j] = L_j,lane
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        const double xj = lane_f64(y, j);
        if (lane < j) y = __builtin_fma(-r[j], xj, y);
    }
    if (in) x[pi] = y;
    wave_lds_sync();
    return true;
}

template <int N, int V>
__global__ void __launch_bounds__(64) bench(const double *Hs, const double *bs, double *xs, long long *cyc, int reps) {
    __shared__ double H[N * N], b[N], x[N], Lm[N * N + 4 * N + 8];
    __shared__ int pick[N];
    const int lane = threadIdx.x;
    for (int q = lane; q < N * N; q += 64) H[q] = Hs[(size_t)blockIdx.x * N * N + q];
    if (lane < N) b[lane] = bs[(size_t)blockIdx.x * N + lane];
    wave_lds_sync();
    long long t0 = clock64();
    for (int r = 0; r < reps; ++r) {
        if (V == 0) ldlt_pick_solve<N>(H, b, x, pick, Lm, lane);
        else ldlt_v2<N>(H, b, x, pick, Lm, lane);
        if (lane < N) b[lane] += 1e-300 * x[lane];
        wave_lds_sync();
    }
    long long t1 = clock64();
    if (lane < N) xs[(size_t)blockIdx.x * N + lane] = x[lane];
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
}  // namespace

template <int N>
static void run() {
    const int F = 8, reps = 200;
    std::vector<double> H(F * N * N), b(F * N);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
    for (int f = 0; f < F; ++f) {
        std::vector<double> A(N * N);
        for (auto &v : A) v = rnd();
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) {
                double t = i == j ? N : 0.0;
                for (int k = 0; k < N; ++k) t += A[i * N + k] * A[j * N + k];
                H[(size_t)f * N * N + i * N + j] = t * (1.0 + 10.0 * (i % 5));
            }
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < i; ++j) H[(size_t)f * N * N + j * N + i] = H[(size_t)f * N * N + i * N + j];
        for (int i = 0; i < N; ++i) b[f * N + i] = rnd();
    }
    double *dH, *db, *dx0, *dx1;
    long long *dc;
    (void)hipMalloc(&dH, H.size() * 8), (void)hipMalloc(&db, b.size() * 8), (void)hipMalloc(&dx0, b.size() * 8);
    (void)hipMalloc(&dx1, b.size() * 8), (void)hipMalloc(&dc, F * 8);
    (void)hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
    std::vector<long long> c(F);
    std::vector<double> x0(F * N), x1(F * N);
    for (int v = 0; v < 2; ++v) {
        (void)hipMemcpy(db, b.data(), b.size() * 8, hipMemcpyHostToDevice);
        if (v == 0) bench<N, 0><<<F, 64>>>(dH, db, dx0, dc, reps);
        else bench<N, 1><<<F, 64>>>(dH, db, dx1, dc, reps);
        (void)hipMemcpy(c.data(), dc, F * 8, hipMemcpyDeviceToHost);
        double m = 0;
        for (auto q : c) m += (double)q / reps;
        printf("N=%d %s: %.0f cycles per solve\n", N, v == 0 ? "current" : "v3 (transposed columns stored in the factor loop)", m / F);
    }
    (void)hipMemcpy(x0.data(), dx0, x0.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(x1.data(), dx1, x1.size() * 8, hipMemcpyDeviceToHost);
    int ndiff = 0;
    for (int q = 0; q < F * N; ++q) ndiff += memcmp(&x0[q], &x1[q], 8) != 0;
    printf("N=%d solutions differing bitwise: %d of %d\n", N, ndiff, F * N);
}

int main() {
    run<6>();
    run<9>();
    run<24>();
    return 0;
}
