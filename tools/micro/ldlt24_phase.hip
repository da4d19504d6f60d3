// Micro-benchmark: where ldlt_pick_solve<24>'s cycles go (pick order, row loads, factorisation, forward, transpose,
// backward), one wavefront, clock64 stamps between the phases (the phases copied from pose.hip's ldlt_pick_solve).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include tools/micro/ldlt24_phase.hip -o /tmp/ldlt24_phase
#include "../../openmavis_amd/csrc/pose.hip"

namespace {
template <int N>
__device__ __forceinline__ void phased(const double *H, const double *b, double *x, int *pick, double *Lm, int lane,
                                       long long *t) {
    const bool in = lane < N;
    t[0] = clock64();
    ldlt_pick_order<N>(H, pick, lane);
    wave_lds_sync();
    t[1] = clock64();
    const int pi = in ? pick[lane] : 0;
    int pj[N];
#pragma unroll
    for (int j = 0; j < N; ++j) pj[j] = pick[j];
    double r[N];
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? H[pj[j] * N + pi] : 0.0;
    if (!(lane_f64(r[0], 0) != 0.0)) return;
    t[2] = clock64();
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
    if (sign & 2) return;
    t[3] = clock64();
    double y = in ? b[pi] : 0.0;
#pragma unroll
    for (int k = 0; k + 1 < N; ++k) {
        const double yk = lane_f64(y, k);
        if (lane > k) y = __builtin_fma(-r[k], yk, y);
    }
    y = fabs(dmine) > 2.2250738585072014e-308 ? y / dmine : 0.0;
    t[4] = clock64();
    if (in)
#pragma unroll
        for (int j = 0; j < N; ++j) Lm[lane * N + j] = r[j];
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < N; ++j) r[j] = in ? Lm[j * N + lane] : 0.0;
    t[5] = clock64();
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        const double xj = lane_f64(y, j);
        if (lane < j) y = __builtin_fma(-r[j], xj, y);
    }
    if (in) x[pi] = y;
    wave_lds_sync();
    t[6] = clock64();
}

template <int N>
__global__ void __launch_bounds__(64) bench(const double *Hs, const double *bs, double *xs, long long *cyc, int reps) {
    __shared__ double H[N * N], b[N], x[N], Lm[N * N];
    __shared__ int pick[N];
    const int lane = threadIdx.x;
    for (int q = lane; q < N * N; q += 64) H[q] = Hs[(size_t)blockIdx.x * N * N + q];
    if (lane < N) b[lane] = bs[(size_t)blockIdx.x * N + lane];
    wave_lds_sync();
    long long acc[6] = {0, 0, 0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        long long t[7];
        phased<N>(H, b, x, pick, Lm, lane, t);
        for (int q = 0; q < 6; ++q) acc[q] += t[q + 1] - t[q];
        if (lane < N) b[lane] += 1e-300 * x[lane];
        wave_lds_sync();
    }
    if (lane < N) xs[(size_t)blockIdx.x * N + lane] = x[lane];
    if (lane == 0)
        for (int q = 0; q < 6; ++q) cyc[blockIdx.x * 6 + q] = acc[q];
}
}  // namespace

int main() {
    constexpr int N = 24, F = 8, reps = 200;
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
    double *dH, *db, *dx;
    long long *dc;
    hipMalloc(&dH, H.size() * 8), hipMalloc(&db, b.size() * 8), hipMalloc(&dx, b.size() * 8), hipMalloc(&dc, F * 6 * 8);
    hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), b.size() * 8, hipMemcpyHostToDevice);
    bench<N><<<F, 64>>>(dH, db, dx, dc, reps);
    std::vector<long long> c(F * 6);
    hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost);
    const char *names[6] = {"pick order", "row loads", "factor", "forward", "transpose", "backward"};
    for (int q = 0; q < 6; ++q) {
        double m = 0;
        for (int f = 0; f < F; ++f) m += (double)c[f * 6 + q] / reps;
        printf("N=%d %-10s %7.0f cycles\n", N, names[q], m / F);
    }
    return 0;
}
