// Microbenchmark: lba.hip's 16x16 diagonal inverse (inv16) and trailing update (update16) on one wavefront,
// alone on the GPU: ns and clock cycles per call (calibrates the LDL^T critical path).
#include "../../openmavis_amd/csrc/lba.hip"

__global__ void __launch_bounds__(64) bench_inv(int n, long long *out, double *res) {
    __shared__ double D[4 * 256];
    __shared__ int bad;
    const int lane = threadIdx.x;
    for (int e = lane; e < 256; e += 64) {
        const int r = e / 16, c = e % 16;
        const double v = r == c ? 20.0 + r : 1.0 / (1 + r + c);
        D[sw16(r, c)] = v, D[256 + sw16(r, c)] = v, D[512 + sw16(r, c)] = 0.5 * v, D[768 + sw16(r, c)] = 0.25 * v;
    }
    if (lane == 0) bad = 0;
    __syncthreads();
    const long long t0 = wall_clock64(), c0 = clock64();
    for (int i = 0; i < n; ++i) inv16<false>(D, lane, &bad);   // the inverse of the inverse: values stay bounded
    const long long t1 = wall_clock64(), c1 = clock64();
    for (int i = 0; i < n; ++i) update16(D + 256, D + 512, D + 768, D, lane);
    const long long t2 = wall_clock64(), c2 = clock64();
    if (lane == 0) out[0] = t1 - t0, out[1] = c1 - c0, out[2] = t2 - t1, out[3] = c2 - c1, out[4] = bad;
    for (int e = lane; e < 256; e += 64) res[e] = D[e];
}

// v_rcp_f64 accuracy: ulps off the IEEE quotient after 0 / 1 / 2 Newton steps, over 2^20 arguments per thread block
__global__ void rcp_acc(unsigned long long *maxulp) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long m0 = 0, m1 = 0, m2 = 0;
    for (unsigned k = 0; k < 64; ++k) {
        const unsigned h = (i * 64 + k) * 2654435761u;
        const double x = ldexp(1.0 + h * (1.0 / 4294967296.0), (int)(h >> 26) - 32);
        const double q = 1.0 / x;
        double r = __builtin_amdgcn_rcp(x);
        auto ulp = [&](double v) {
            const long long a = __builtin_bit_cast(long long, v), b = __builtin_bit_cast(long long, q);
            return (unsigned long long)(a > b ? a - b : b - a);
        };
        m0 = max(m0, ulp(r));
        double e = fma(-x, r, 1.0);
        r = fma(r, e, r);
        m1 = max(m1, ulp(r));
        e = fma(-x, r, 1.0);
        r = fma(r, e, r);
        m2 = max(m2, ulp(r));
    }
    atomicMax(&maxulp[0], m0), atomicMax(&maxulp[1], m1), atomicMax(&maxulp[2], m2);
}

int main() {
    {
        unsigned long long *u, hu[3];
        if (hipMalloc(&u, sizeof(hu)) != hipSuccess || hipMemset(u, 0, sizeof(hu)) != hipSuccess) return 1;
        rcp_acc<<<256, 256>>>(u);
        if (hipMemcpy(hu, u, sizeof(hu), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("v_rcp_f64 max ulp: raw %llu, 1 Newton %llu, 2 Newton %llu\n", hu[0], hu[1], hu[2]);
    }
    long long *d, h[5];
    double *r, hr[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&r, sizeof(hr)) != hipSuccess) return 1;
    const int n = 2000;
    for (int rep = 0; rep < 3; ++rep) {
        bench_inv<<<1, 64>>>(n, d, r);
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        if (hipMemcpy(hr, r, sizeof(hr), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("inv16: %.1f ns %.0f cycles per call; update16: %.1f ns %.0f cycles; clock %.2f GHz; bad %lld; D00 %.6f\n",
               h[0] * 10.0 / n, (double)h[1] / n, h[2] * 10.0 / n, (double)h[3] / n, h[1] / (h[0] * 10.0), h[4], hr[0]);
    }
    return hipFree(d) == hipSuccess && hipFree(r) == hipSuccess ? 0 : 1;
}
