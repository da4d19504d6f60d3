// Prints what v_permlane16_swap / v_permlane32_swap return for a = lane id (the row-broadcast helper of
// lba.hip's inv16 relies on: permlane16_swap(a, a) = {[r0 r0 r2 r2], [r1 r1 r3 r3]},
// permlane32_swap(z, z) = {[lo lo], [hi hi]}).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *out) {
    const unsigned a = threadIdx.x;
    const auto r = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    const auto s = __builtin_amdgcn_permlane32_swap(a, a, false, false);
    out[threadIdx.x] = r[0], out[64 + threadIdx.x] = r[1], out[128 + threadIdx.x] = s[0], out[192 + threadIdx.x] = s[1];
}
int main() {
    unsigned *d, h[256];
    if (hipMalloc(&d, 1024) != hipSuccess) return 1;
    k<<<1, 64>>>(d);
    if (hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *nm[4] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]"};
    for (int v = 0; v < 4; ++v) {
        printf("%s:", nm[v]);
        for (int l = 0; l < 64; l += 8) printf(" %u", h[64 * v + l]);
        printf("\n");
    }
    return hipFree(d) == hipSuccess ? 0 : 1;
}
