// Does ds_read_u8_d16 / ds_read_u8_d16_hi into one register keep the other half on gfx950?  (Tried for the FAST ring
// loads: every strength came out <= 0, as if the second load zeroed the first's half.)  One wave, LDS filled with a
// byte pattern, the two-load pair against plain byte loads.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/d16_check.hip -o /tmp/d16_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int RS>
__device__ __forceinline__ void ring_pairs_d16(const uint8_t *p, uint32_t (&x)[9]) {
    constexpr int s = RS, b = 3 * s + 1;
    const uint32_t a = (uint32_t)(uintptr_t)(p - b);
    asm volatile(
        "ds_read_u8_d16 %0, %9 offset:%10\n\tds_read_u8_d16_hi %0, %9 offset:%11\n\t"
        "ds_read_u8_d16 %1, %9 offset:%12\n\tds_read_u8_d16_hi %1, %9 offset:%13\n\t"
        "ds_read_u8_d16 %2, %9 offset:%14\n\tds_read_u8_d16_hi %2, %9 offset:%15\n\t"
        "ds_read_u8_d16 %3, %9 offset:%16\n\tds_read_u8_d16_hi %3, %9 offset:%17\n\t"
        "ds_read_u8_d16 %4, %9 offset:%18\n\tds_read_u8_d16_hi %4, %9 offset:%19\n\t"
        "ds_read_u8_d16 %5, %9 offset:%20\n\tds_read_u8_d16_hi %5, %9 offset:%21\n\t"
        "ds_read_u8_d16 %6, %9 offset:%22\n\tds_read_u8_d16_hi %6, %9 offset:%23\n\t"
        "ds_read_u8_d16 %7, %9 offset:%24\n\tds_read_u8_d16_hi %7, %9 offset:%25\n\t"
        "ds_read_u8_d16 %8, %9 offset:%26\n\tds_read_u8_d16_hi %8, %9 offset:%26\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7]),
          "=&v"(x[8])
        : "v"(a), "i"(b + 3 * s), "i"(b - 3 * s), "i"(b + 3 * s + 1), "i"(b - 3 * s - 1), "i"(b + 2 * s + 2),
          "i"(b - 2 * s - 2), "i"(b + s + 3), "i"(b - s - 3), "i"(b + 3), "i"(b - 3), "i"(b - s + 3), "i"(b + s - 3),
          "i"(b - 2 * s + 2), "i"(b + 2 * s - 2), "i"(b - 3 * s + 1), "i"(b + 3 * s - 1), "i"(b)
        : "memory");
}

__global__ void check(int *bad, uint32_t *dump) {
    __shared__ uint8_t lds[68 * 16];
    for (int i = threadIdx.x; i < 68 * 16; i += 64) lds[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const int r = 4 + (threadIdx.x & 7), q = 4 + (threadIdx.x >> 3);
    const uint8_t *p = lds + r * 68 + q;
    uint32_t x[9];
    ring_pairs_d16<68>(p, x);
    const int s = 68;
    const int o[16] = {3 * s, 3 * s + 1, 2 * s + 2, s + 3, 3, -s + 3, -2 * s + 2, -3 * s + 1, -3 * s, -3 * s - 1,
                       -2 * s - 2, -s - 3, -3, s - 3, 2 * s - 2, 3 * s - 1};
    int nb = 0;
    for (int k = 0; k < 8; ++k) {
        const uint32_t want = (uint32_t)p[o[k]] | ((uint32_t)p[o[k + 8]] << 16);
        nb += want != x[k];
        if (threadIdx.x == 0) dump[2 * k] = want, dump[2 * k + 1] = x[k];
    }
    nb += x[8] != ((uint32_t)p[0] | ((uint32_t)p[0] << 16));
    if (threadIdx.x == 0) dump[16] = (uint32_t)p[0] | ((uint32_t)p[0] << 16), dump[17] = x[8];
    atomicAdd(bad, nb);
}

int main() {
    int *bad;
    uint32_t *dump;
    (void)hipMalloc(&bad, 4), (void)hipMalloc(&dump, 18 * 4);
    (void)hipMemset(bad, 0, 4);
    check<<<1, 64>>>(bad, dump);
    int h = -1;
    uint32_t d[18];
    (void)hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(d, dump, 72, hipMemcpyDeviceToHost);
    printf("mismatches %d\n", h);
    for (int k = 0; k < 9; ++k) printf("pair %d want %08x got %08x\n", k, d[2 * k], d[2 * k + 1]);
    return 0;
}
