// Device-side arithmetic helpers for the gfx950 kernels.  Every float path here must be compiled
// with -ffp-contract=off: the reference's float expressions are evaluated without fused
// multiply-adds, and bit-exact keypoints/descriptors depend on reproducing their rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace omv {

// cvRound(float): round half to even (x86 cvtss2si under the default MXCSR).
__device__ __forceinline__ int round_even(float v) { return (int)__builtin_rintf(v); }

// cv::fastAtan2 (OpenCV 4.x atan_f32, degrees, float).  Coefficients are the float products
// 0.99978784f*(float)(180/pi) etc., folded exactly as the host compiler folds them.
__device__ __forceinline__ float fast_atan2_deg(float y, float x) {
    const float r2d = (float)(180.0 / 3.14159265358979323846);
    const float k1 = 0.9997878412794807f * r2d;
    const float k3 = -0.3258083974640975f * r2d;
    const float k5 = 0.1555786518463281f * r2d;
    const float k7 = -0.04432655554792128f * r2d;
    const float eps = (float)2.220446049250313080847e-16;   // (float)DBL_EPSILON
    float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((k7 * c2 + k5) * c2 + k3) * c2 + k1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((k7 * c2 + k5) * c2 + k3) * c2 + k1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---- single-precision sin/cos, bit-identical to the host glibc (2.35) cosf/sinf ------------------
// The reference calls cos()/sin() on a float (src/ORBextractor.cc:49), i.e. glibc's cosf/sinf.
// Those evaluate a double-precision polynomial after a one-step pi/2 reduction; we restate that
// published algorithm with the same constants and explicit fma() where the x86-64 FMA build fuses.
// Verified bit-exact against the host libm over every float in [0, 2*pi] (tests/test_oracle.py
// re-checks a sample; tools/check_sincosf.c is the exhaustive sweep).
struct SinCosTab {
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
__device__ __forceinline__ float sincosf_poly(double x, double x2, const SinCosTab &p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = __builtin_fma(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = __builtin_fma(x3, p.s1, x);
        return (float)__builtin_fma(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = __builtin_fma(x2, p.c4, p.c3);
    double c1 = __builtin_fma(x2, p.c1, p.c0);
    double x6 = x4 * x2;
    double c = __builtin_fma(x4, p.c2, c1);
    return (float)__builtin_fma(x6, c2, c);
}
__device__ __forceinline__ uint32_t top12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

// Valid for |y| < 120 (the reduce_fast range), which covers every angle in [0, 2*pi).
__device__ __forceinline__ void glibc_sincosf(float y, float *sinp, float *cosp) {
    const SinCosTab t0 = {0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
                          0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
                          -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};
    const SinCosTab t1 = {0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
                          -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
                          -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};
    double x = y;
    if (top12(y) < top12(0x1.921FB6p-1f)) {
        if (top12(y) < top12(0x1p-12f)) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
        double x2 = x * x;
        *sinp = sincosf_poly(x, x2, t0, 0);
        *cosp = sincosf_poly(x, x2, t0, 1);
        return;
    }
    double r = x * t0.hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    double xr = __builtin_fma(-(double)n, t0.hpi, x);
    const double sgn[4] = {1.0, -1.0, -1.0, 1.0};
    double s = sgn[n & 3];
    const SinCosTab &p = (n & 2) ? t1 : t0;
    *sinp = sincosf_poly(xr * s, xr * xr, p, n);
    *cosp = sincosf_poly(xr * s, xr * xr, p, n ^ 1);
}

__device__ __forceinline__ int reflect101(int p, int n) {
    // single reflection suffices: callers stay within one image width of the border
    p = p < 0 ? -p : p;
    return p >= n ? 2 * n - 2 - p : p;
}

// Hamming distance of two 256-bit descriptors held as 4 x u64.
__device__ __forceinline__ int hamming256(const uint64_t *a, const uint64_t *b) {
    return __popcll(a[0] ^ b[0]) + __popcll(a[1] ^ b[1]) + __popcll(a[2] ^ b[2]) + __popcll(a[3] ^ b[3]);
}


// glibc atan2f (fdlibm e_atan2f.c / s_atanf.c), float, no contraction.  KannalaBrandt8::project
// computes theta / psi with atan2f (KannalaBrandt8.cpp:30-31, :50-51); this restatement is
// bit-identical to the host libm (tools/check_atan2f.c, tests/test_native_cpu.py).
__device__ __forceinline__ uint32_t f32_bits(float f) { return __float_as_uint(f); }
__device__ inline float glibc_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
    const int32_t hx = (int32_t)f32_bits(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) id = 0, x = (2.0f * x - 1.0f) / (2.0f + x);
            else id = 1, x = (x - 1.0f) / (x + 1.0f);
        } else {
            if (ix < 0x401c0000) id = 2, x = (x - 1.5f) / (1.0f + 1.5f * x);
            else id = 3, x = -1.0f / x;
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}
__device__ inline float glibc_atan2f(float y, float x) {
    const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f, tiny = 1.0e-30f;
    const int32_t hx = (int32_t)f32_bits(x), ix = hx & 0x7fffffff, hy = (int32_t)f32_bits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return glibc_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m < 2) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            const float r[4] = {pi_o_4 + tiny, -pi_o_4 - tiny, 3.0f * pi_o_4 + tiny, -3.0f * pi_o_4 - tiny};
            return r[m];
        }
        const float r[4] = {0.0f, -0.0f, pi + tiny, -pi - tiny};
        return r[m];
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = glibc_atanf(fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return __uint_as_float(f32_bits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// Correctly rounded f32 sqrt (libm sqrtf): v_sqrt_f32 alone is 1 ulp; the f64 sqrt is correctly
// rounded and 53 >= 2*24+2 bits make the second rounding innocuous.
__device__ __forceinline__ float sqrtf_cr(float x) { return (float)sqrt((double)x); }

// glibc 2.35 tanf (std::tan(float) in KannalaBrandt8::unproject): fdlibm's __kernel_tanf after a
// double-precision reduction (pi/4 < |x| < 120: n = nearbyint(x 2/pi), r = x - n pi/2).  Bit-identical
// to the host libm on every float with |x| < 120 (tools/check_tanf.c, exhaustive).
__device__ inline float glibc_kernel_tanf(float x, float y, int iy) {
    const float T[] = {3.3333334327e-01f, 1.3333334029e-01f, 5.3968254477e-02f, 2.1869488060e-02f,
                       8.8632395491e-03f, 3.5920790397e-03f, 1.4562094584e-03f, 5.8804126456e-04f,
                       2.4646313977e-04f, 7.8179444245e-05f, 7.1407252108e-05f, -1.8558637748e-05f,
                       2.5907305826e-05f};
    const float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
    float z, r, v, w, s;
    const int32_t hx = (int32_t)f32_bits(x), ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {   // |x| < 2**-13
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return 1.0f / fabsf(x);
            else if (iy == 1) return x;
            else return -1.0f / x;
        }
    }
    if (ix >= 0x3f2ca140) {   // |x| >= 0.6744
        if (hx < 0) x = -x, y = -y;
        z = pio4 - x;
        w = pio4lo - y;
        x = z + w;
        y = 0.0f;
        if (fabsf(x) < 0x1p-13f) return (1 - ((hx >> 30) & 2)) * iy * (1.0f - 2 * iy * x);
    }
    z = x * x;
    w = z * z;
    r = T[1] + w * (T[3] + w * (T[5] + w * (T[7] + w * (T[9] + w * T[11]))));
    v = z * (T[2] + w * (T[4] + w * (T[6] + w * (T[8] + w * (T[10] + w * T[12])))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T[0] * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    float a, t;
    z = __uint_as_float(f32_bits(w) & 0xfffff000u);
    v = r - (z - x);
    t = a = -1.0f / w;
    t = __uint_as_float(f32_bits(t) & 0xfffff000u);
    s = 1.0f + t * z;
    return t + a * (s + t * v);
}
__device__ inline float glibc_tanf(float x) {
    const int32_t ix = (int32_t)(f32_bits(x) & 0x7fffffffu);
    if (ix <= 0x3f490fda) return glibc_kernel_tanf(x, 0.0f, 1);
    const double xd = (double)x, nd = rint(xd * 0.6366197723675814);
    const int n = (int)nd;
    const double r = xd - nd * 1.5707963267948966;
    const float y0 = (float)r, y1 = (float)(r - (double)y0);
    return glibc_kernel_tanf(y0, y1, 1 - ((n & 1) << 1));
}

// XCD-aware block order: the dispatcher deals workgroup b to XCD b % 8, so consecutive logical blocks
// (neighbouring cells / keypoints / map points of one image or frame, which share bytes) are given to one XCD:
// physical b runs logical (b % 8) * ceil(n / 8) + b / 8 and those bytes are fetched into one L2, not eight.
// The grid is padded to a multiple of 8; returns -1 for a padding block.
__device__ __forceinline__ int xcd_block(int n_logical) {
    const int chunk = (n_logical + 7) >> 3;
    const int b = (int)(blockIdx.x & 7) * chunk + (int)(blockIdx.x >> 3);
    return b < n_logical ? b : -1;
}
__host__ inline int xcd_grid(int n_logical) { return (n_logical + 7) & ~7; }

}  // namespace omv
// v_mul_u32_u24 (full rate) for operands the caller knows are < 2^24: HIP's __umul24 masks its operands and the
// backend then emits v_and + v_mul_lo_u32 (quarter rate) unless it can prove the mask redundant.
extern "C" __device__ __attribute__((const)) uint32_t omv_llvm_mul_u24(uint32_t, uint32_t) __asm("llvm.amdgcn.mul.u24.i32");
namespace omv {
__device__ __forceinline__ int mul_u24(int a, int b) { return (int)omv_llvm_mul_u24((uint32_t)a, (uint32_t)b); }

// Test knobs of a matcher handle (OMV_BOW_TOP, OMV_TRI_SLICES, OMV_TRI_ECAP, OMV_TRI_WALK, OMV_CAND, OMV_CAND_PW),
// read once by omv_matcher_create (not per call); -1 / 0: unset.  Defined in match.hip for the other matcher
// translation units.
struct MatcherKnobs {
    int bow_top = -1, tri_slices = -1, tri_ecap = -1, tri_walk_seq = 0;
    int cand_mode = 0;     // OMV_CAND: SearchByProjection candidates 0 by batch size, 1 "global" (no LDS staging), 2 "lds"
    int cand_pw = -1;      // OMV_CAND_PW: map points per wave of the LDS-staged candidate kernel
};
MatcherKnobs matcher_knobs(const struct ::omv_matcher *m);
// omv_matcher_search_kf's entry capacity of a handle (max_frames x n_cams x max_mps)
size_t matcher_kf_entry_cap(const struct ::omv_matcher *m);

}  // namespace omv
