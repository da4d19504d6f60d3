// Micro-benchmark: cycles per v_mfma_f64_16x16x4f64 on gfx950, one wave, dependent accumulator chain vs four
// independent chains; hipcc --offload-arch=gfx950 -O3 tools/micro/mfma64_bench.hip -o tools/micro/mfma64_bench
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void dep(double *out, long long *cyc, int n) {
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    v4d acc = {0, 0, 0, 0};
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    long long t1 = clock64();
    out[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void ind(double *out, long long *cyc, int n) {
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    long long t0 = clock64();
    for (int i = 0; i < n; i += 4) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    long long t1 = clock64();
    out[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double *o;
    long long *c, h;
    hipMalloc(&o, 64 * 8);
    hipMalloc(&c, 8);
    const int n = 4096;
    for (int r = 0; r < 2; ++r) {
        dep<<<1, 64>>>(o, c, n);
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("dependent chain: %.1f cycles per MFMA\n", (double)h / n);
        ind<<<1, 64>>>(o, c, n);
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("4 independent chains: %.1f cycles per MFMA\n", (double)h / n);
    }
    return 0;
}
