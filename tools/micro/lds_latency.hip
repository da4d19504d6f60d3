// Microbenchmark: dependent LDS read chain and clock rates on one wavefront (calibrates the resolve profile).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(64) chain(int n, long long *out) {
    __shared__ int buf[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) buf[i] = (i * 37 + 11) & 4095;
    __syncthreads();
    int p = lane;
    const long long t0 = wall_clock64(), c0 = clock64();
    for (int i = 0; i < n; ++i) p = buf[p];
    const long long t1 = wall_clock64(), c1 = clock64();
    if (lane == 0) out[0] = t1 - t0, out[1] = c1 - c0, out[2] = p;
}
int main() {
    long long *d, h[3];
    hipMalloc(&d, 24);
    for (int rep = 0; rep < 3; ++rep) {
        chain<<<1, 64>>>(10000, d);
        hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        printf("10000 dependent ds_read: %lld ticks(100MHz) = %.1f ns each; %lld clock64 = %.1f cycles each; clock %.2f GHz\n",
               h[0], h[0] * 10.0 / 10000, h[1], h[1] / 10000.0, h[1] / (h[0] * 10.0));
    }
    return 0;
}
