// MI355X-native ORB extractor: the path of ORBextractor::operator() (src/ORBextractor.cc:987-1071)
// as five gfx950 kernels over a batch of device-resident images.
//
//   K1 pyr_resize   one launch per pyramid level l >= 1, level l from level l-1 (ComputePyramid
//                   :1073-1104; cv::resize INTER_LINEAR 8U fixed point), coefficient tables
//                   precomputed on the host in the reference's float/double order.
//   K2 fast_cells   one wavefront per FAST cell (ComputeKeyPointsOctTree :709-794): the cell region
//                   is staged in LDS, each lane evaluates FAST-9 "strength" S for pixels (corner at
//                   threshold t <=> S > t, cornerScore = S - 1), then the cell-local 3x3 NMS at
//                   iniThFAST with the minThFAST fallback; keypoints emitted in row-major order.
//   K3 octree       one workgroup per (image, level): DistributeOctTree (:496-702) as a parallel
//                   list rebuild per subdivision round (prefix scans over the node list, atomics in
//                   LDS for quadrant counts) plus the libstdc++ introsort replica for the
//                   (size, UL.x) refinement ordering; picks max-response key per node; classifies
//                   lapping/non-lapping for the output split (:1045-1067).
//   K4 describe     one wavefront per keypoint: intensity-centroid angle over the un-blurred level
//                   (IC_Angle :19-43, fastAtan2), the GaussianBlur 7x7 (:1035-1036, OpenCV's bit-exact
//                   8U path) evaluated in LDS at the 512 rBRIEF sample points only, 4 ballots
//                   (computeOrbDescriptor :46-90); writes the keypoint and descriptor straight into
//                   its final (mono-front / lapping-back) row.  No blurred pyramid exists.
//
// All float code is compiled with -ffp-contract=off (see omv_device.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <climits>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/omv.h"
#include "omv_device.h"
#include "omv_introsort.h"

namespace {

constexpr int kMaxLevels = 16;
constexpr int kOrbStages = 4;   // pyramid, FAST cells, octree, describe (omv_orb_stage_ms)
constexpr int kEdge = 19;     // EDGE_THRESHOLD
constexpr int kMinB = kEdge - 3;
#define OMV_PATTERN_TABLE_BEGIN
#define OMV_PATTERN_TABLE_END
constexpr int kPattern[256 * 4] = {
#include "orb_pattern_31.inc"
};
// the 256 point pairs (ax, ay, bx, by) as floats (the reference's int x float products convert the pattern
// coordinate first): one 16-byte entry per pair, loaded by each lane once per keypoint before the patch staging
struct FloatPattern {
    float v[256][4];
};
constexpr FloatPattern float_pattern() {
    FloatPattern p{};
    for (int i = 0; i < 256; ++i)
        for (int q = 0; q < 4; ++q) p.v[i][q] = (float)kPattern[4 * i + q];
    return p;
}
__constant__ FloatPattern c_patternf = float_pattern();
__constant__ int c_gauss7[7] = {18, 34, 48, 56, 48, 34, 18};

struct LevelGeom {
    int w, h, pitch;        // level l pixels; pitch of the level in the pyramid buffer
    long long off;          // byte offset of level l inside one image's pyramid block (l >= 1)
    int maxBX, maxBY;       // FAST region bounds (cols - 16, rows - 16)
    int cell_begin, cell_end;
    int quota;              // mnFeaturesPerLevel
    int out_cap;            // max keypoints this level can emit (quota + 2, or 4 * nIni)
    int out_off;            // offset of this level's slots in the per-image level-output block
    long long cand_off;     // offset of this level's compact candidates in the per-image block
    int cand_cap;
    int nIni;
    float hX;
    float scale;            // mvScaleFactor[l]
    float size;             // (float)(int)(PATCH_SIZE * mvScaleFactor[l])
    int xtab_off, ytab_off; // resize tables (l >= 1)
    int xq_off, use_xq;     // quad table (l >= 1; use_xq: every pixel pair's sources fit two dwords)
    // q / d as __umulhi(q, ceil(2^32 / d)) (exact for q < 2^16), host-computed: d = output quads (w + 3) / 4, the
    // 16-byte groups of a staged row (w + 15) / 16, and w (a 64-bit division per launch was ~100 scalar instructions)
    uint32_t m_quads, m_groups, m_w;
};

struct Cell {
    int level, y0, y1, x0, x1;   // region rows [y0,y1), cols [x0,x1) in level coordinates
};

struct Geom {
    int nlevels;
    int W, H;
    int ini_th, min_th;
    int n_cells;            // cells per image
    int cell_cap;           // keypoint slots per cell
    long long pyr_bytes;    // pyramid block per image (levels >= 1)
    long long cand_per_img;
    int out_per_img;        // level-output slots per image
    int n_max;              // output rows per image
    int node_cap;           // octree LDS node capacity
    int ccnt_cap;           // octree child-count region (>= 4 node_cap; also holds the level's cell scan)
    unsigned long long umax_pk;          // IC_Angle's umax[0..15], 4 bits each (the disc half-widths)
    LevelGeom lv[kMaxLevels];
};

struct XTab {
    int sx0, sx1, coef;   // coef = a0 | (a1 << 16)
};

// One output quad (dx = 4q .. 4q+3) of a resize row: pixel pair p = j >> 1 reads the two source dwords at dword
// index a[p] of the staged row; sel[j] is the v_perm selector that lays (src[sx0], src[sx1]) of pixel j out as a
// u16 pair, cf[j] = (a0, a1) as a u16 pair, so h = v_dot2_u32_u16(perm, cf) = src[sx0] a0 + src[sx1] a1 exactly.
struct __attribute__((aligned(16))) XQuad {
    int a[2];
    uint32_t sel[4], cf[4];
    int pad[2];
};
static_assert(sizeof(XQuad) == 48, "XQuad LDS addressing");

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ const uint8_t *level_base(const Geom &g, const uint8_t *images, size_t img_stride,
                                                     size_t pitch0, const uint8_t *pyr, int img, int l,
                                                     int *pitch) {
    if (l == 0) {
        *pitch = (int)pitch0;
        return images + (size_t)img * img_stride;
    }
    *pitch = g.lv[l].pitch;
    return pyr + (size_t)img * g.pyr_bytes + g.lv[l].off;
}

// K1 --------------------------------------------------------------------------------------------
// One workgroup per (block of kPyrBlock output rows, image) of level l: the source rows of level l-1
// the block reads (y.sx0 of its first row .. y.sx1 of its last, ~1.2 kPyrBlock + 2) are staged in LDS
// once with 16-byte loads, together with the level's x table; each thread then computes 4 adjacent
// output pixels per step and stores them as one dword (level pitches are 16-byte aligned).
constexpr int kPyrBlock = 16;

// cv::resize's vertical pass on the horizontal sums: (b0 (h0 >> 4) >> 16) + (b1 (h1 >> 4) >> 16) + 2 >> 2.  The
// coefficients are < 2^12 and h >> 4 < 2^15 (both non-negative), so the products are 24-bit multiplies at full rate
// (an int multiply is v_mul_lo_u32, a quarter-rate instruction: 8 of them per output quad).
__device__ __forceinline__ int vmix(int b0, int b1, int h0, int h1) {
    return ((omv::mul_u24(b0, h0 >> 4) >> 16) + (omv::mul_u24(b1, h1 >> 4) >> 16) + 2) >> 2;
}

__global__ void __launch_bounds__(256) pyr_resize_kernel(Geom g, int l, const uint8_t *images, size_t img_stride,
                                                         size_t pitch0, uint8_t *pyr, const XTab *xt,
                                                         const XTab *yt, const XQuad *xq, int n_images) {
    extern __shared__ __attribute__((aligned(16))) uint32_t pyr_lds[];
    const LevelGeom &L = g.lv[l];
    const int img = blockIdx.y, tid = threadIdx.x;
    const int dy0 = blockIdx.x * kPyrBlock, dy1 = min(dy0 + kPyrBlock, L.h);
    int sp;
    const uint8_t *src = level_base(g, images, img_stride, pitch0, pyr, img, l - 1, &sp);
    const int sw = g.lv[l - 1].w;
    const int ndw = ((sw + 15) >> 4) << 2;   // LDS row: whole 16-byte groups
    const int nq = (L.w + 3) >> 2;
    XTab *xs = reinterpret_cast<XTab *>(pyr_lds);            // [L.w]  (generic path)
    XQuad *xqs = reinterpret_cast<XQuad *>(pyr_lds);         // [nq]   (quad path)
    uint32_t *rows = pyr_lds + 12 * nq;                      // [nr][ndw] (+4 dwords of slack)
    const int sy0 = yt[L.ytab_off + dy0].sx0, sy1 = yt[L.ytab_off + dy1 - 1].sx1;
    const int nr = sy1 - sy0 + 1;
    XTab *ys = reinterpret_cast<XTab *>(rows + nr * ndw + 4);   // [kPyrBlock] the block's y entries
    const bool quad = L.use_xq != 0;
    if (quad)
        for (int i = tid; i < nq; i += 256) xqs[i] = xq[L.xq_off + i];
    else
        for (int i = tid; i < L.w; i += 256) xs[i] = xt[L.xtab_off + i];
    if (tid < dy1 - dy0) ys[tid] = yt[L.ytab_off + dy0 + tid];
    // q / d as __umulhi(q, ceil(2^32 / d)): exact for q < 2^32 / d (q < 2^16 here)
    if ((sp & 15) == 0 && (((uintptr_t)src) & 15) == 0) {   // 16-byte loads (the groups stay inside the pitch)
        const int n4 = ndw >> 2;
        const uint32_t m4 = g.lv[l - 1].m_groups;
        for (int q = tid; q < nr * n4; q += 256) {
            const int r = (int)__umulhi((uint32_t)q, m4), i = q - r * n4;
            reinterpret_cast<uint4 *>(rows)[q] = reinterpret_cast<const uint4 *>(src + (size_t)(sy0 + r) * sp)[i];
        }
    } else {
        uint8_t *b = reinterpret_cast<uint8_t *>(rows);
        const uint32_t mw = g.lv[l - 1].m_w;
        for (int q = tid; q < nr * sw; q += 256) {
            const int r = (int)__umulhi((uint32_t)q, mw), i = q - r * sw;
            b[(size_t)r * ndw * 4 + i] = src[(size_t)(sy0 + r) * sp + i];
        }
    }
    __syncthreads();
    const uint32_t mq = L.m_quads;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    for (int q = tid; q < (dy1 - dy0) * nq; q += 256) {
        // row / column split and LDS row offsets as 24-bit multiplies (r < kPyrBlock, nq and ndw < 2^12)
        const int r = (int)__umulhi((uint32_t)q, mq), qd = q - omv::mul_u24(r, nq), dx0 = qd * 4,
                  dy = dy0 + r;
        const XTab y = ys[r];
        const int b0 = (short)(y.coef & 0xffff), b1 = (short)(y.coef >> 16);
        uint32_t packed = 0;
        if (quad) {
            const XQuad X = *reinterpret_cast<const XQuad *>(reinterpret_cast<const char *>(xqs) + omv::mul_u24(qd, 48u));
            const uint32_t *R0 = rows + omv::mul_u24(y.sx0 - sy0, ndw),
                           *R1 = rows + omv::mul_u24(y.sx1 - sy0, ndw);
            const uint32_t u0[4] = {R0[X.a[0]], R0[X.a[0] + 1], R0[X.a[1]], R0[X.a[1] + 1]};
            const uint32_t u1[4] = {R1[X.a[0]], R1[X.a[0] + 1], R1[X.a[1]], R1[X.a[1] + 1]};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int pp = 2 * (j >> 1);
                const u16x2 cf = __builtin_bit_cast(u16x2, X.cf[j]);
                const int h0 = (int)__builtin_amdgcn_udot2(
                    __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(u0[pp + 1], u0[pp], X.sel[j])), cf, 0u, false);
                const int h1 = (int)__builtin_amdgcn_udot2(
                    __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(u1[pp + 1], u1[pp], X.sel[j])), cf, 0u, false);
                packed |= (uint32_t)vmix(b0, b1, h0, h1) << (8 * j);   // <= 255: the weights sum to <= 2049
            }
        } else {
            const uint8_t *R0 = reinterpret_cast<const uint8_t *>(rows + omv::mul_u24(y.sx0 - sy0, ndw));
            const uint8_t *R1 = reinterpret_cast<const uint8_t *>(rows + omv::mul_u24(y.sx1 - sy0, ndw));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int dx = dx0 + j;
                if (dx < L.w) {
                    const XTab x = xs[dx];
                    const int a0 = (short)(x.coef & 0xffff), a1 = (short)(x.coef >> 16);
                    const int h0 = R0[x.sx0] * a0 + R0[x.sx1] * a1;
                    const int h1 = R1[x.sx0] * a0 + R1[x.sx1] * a1;
                    const int v = vmix(b0, b1, h0, h1);
                    packed |= (uint32_t)min(v, 255) << (8 * j);
                }
            }
        }
        uint8_t *dst = pyr + (size_t)img * g.pyr_bytes + L.off + (size_t)dy * L.pitch;
        if (dx0 + 3 < L.w) {
            *reinterpret_cast<uint32_t *>(dst + dx0) = packed;
        } else {
            for (int j = 0; j < 4 && dx0 + j < L.w; ++j) dst[dx0 + j] = (uint8_t)(packed >> (8 * j));
        }
    }
}


// K1 as one launch: workgroup (band b, image) computes band b of EVERY level.  Level l's rows are split in nb
// contiguous bands; band b also computes the halo rows its next level reads from the neighbouring bands
// (host-planned: need_l = own_l united with the source rows of need_{l+1}), so a level never waits for another
// workgroup.  Level l - 1's needed rows stay in LDS (ping-pong buffers) while level l is formed from them: the
// pyramid is read from memory once (level 0) and written once, with one launch instead of nlevels - 1 dependent
// ones.  Same arithmetic as pyr_resize_kernel, so the same bytes.
struct PyrBand {
    int own_lo, own_hi, need_lo, need_hi;   // rows of one level (level 0: need only)
};
constexpr int kPyrChainMaxImages = 16;   // default: one launch for batches up to this many images (B = 1 latency)
__global__ void __launch_bounds__(256) pyr_chain_kernel(Geom g, const uint8_t *images, size_t img_stride, size_t pitch0,
                                                        uint8_t *pyr, const XTab *xt, const XTab *yt, const XQuad *xq,
                                                        const PyrBand *bands, int buf_dw, int tab_dw) {
    extern __shared__ __attribute__((aligned(16))) uint32_t pyr_lds[];
    const int b = blockIdx.x, img = blockIdx.y, tid = threadIdx.x;
    const PyrBand *B = bands + (size_t)b * kMaxLevels;
    uint32_t *prev = pyr_lds, *cur = pyr_lds + buf_dw;
    // the level's x table (quads or pixels) and the y entries of its needed rows, staged per level: every output
    // quad of the band reads them (from memory that was 48 + 12 bytes of table traffic per 4 output pixels)
    uint32_t *tab = pyr_lds + 2 * (size_t)buf_dw + 4;
    XTab *ys = reinterpret_cast<XTab *>(tab + tab_dw);
    XQuad *xqs = reinterpret_cast<XQuad *>(tab);
    XTab *xs = reinterpret_cast<XTab *>(tab);
    {   // level 0's needed rows from the image
        const PyrBand b0 = B[0];
        const int sw = g.lv[0].w, ndw = ((sw + 15) >> 4) << 2, nr = b0.need_hi - b0.need_lo;
        const uint8_t *src = images + (size_t)img * img_stride;
        if ((pitch0 & 15) == 0 && (((uintptr_t)src) & 15) == 0) {
            const int n4 = ndw >> 2;
            const uint32_t m4 = g.lv[0].m_groups;
            for (int q = tid; q < nr * n4; q += 256) {
                const int r = (int)__umulhi((uint32_t)q, m4), i = q - r * n4;
                reinterpret_cast<uint4 *>(prev)[q] = reinterpret_cast<const uint4 *>(src + (size_t)(b0.need_lo + r) * pitch0)[i];
            }
        } else {
            uint8_t *bb = reinterpret_cast<uint8_t *>(prev);
            const uint32_t mw = g.lv[0].m_w;
            for (int q = tid; q < nr * sw; q += 256) {
                const int r = (int)__umulhi((uint32_t)q, mw), i = q - r * sw;
                bb[(size_t)r * ndw * 4 + i] = src[(size_t)(b0.need_lo + r) * pitch0 + i];
            }
        }
    }
    __syncthreads();
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    for (int l = 1; l < g.nlevels; ++l) {
        const LevelGeom &L = g.lv[l];
        const PyrBand bp = B[l - 1], bc = B[l];
        const int sndw = ((g.lv[l - 1].w + 15) >> 4) << 2, cndw = ((L.w + 15) >> 4) << 2;
        const int nq = (L.w + 3) >> 2, nr = bc.need_hi - bc.need_lo;
        const bool quad = L.use_xq != 0;
        if (quad)
            for (int i = tid; i < nq; i += 256) xqs[i] = xq[L.xq_off + i];
        else
            for (int i = tid; i < L.w; i += 256) xs[i] = xt[L.xtab_off + i];
        for (int i = tid; i < nr; i += 256) ys[i] = yt[L.ytab_off + bc.need_lo + i];
        __syncthreads();
        const uint32_t mq = L.m_quads;
        for (int q = tid; q < nr * nq; q += 256) {
            const int r = (int)__umulhi((uint32_t)q, mq), qd = q - omv::mul_u24(r, nq), dx0 = qd * 4,
                      dy = bc.need_lo + r;
            const XTab y = ys[r];
            const int b0 = (short)(y.coef & 0xffff), b1 = (short)(y.coef >> 16);
            uint32_t packed = 0;
            if (quad) {
                const XQuad X = *reinterpret_cast<const XQuad *>(reinterpret_cast<const char *>(xqs) + omv::mul_u24(qd, 48u));
                const uint32_t *R0 = prev + omv::mul_u24(y.sx0 - bp.need_lo, sndw),
                               *R1 = prev + omv::mul_u24(y.sx1 - bp.need_lo, sndw);
                const uint32_t u0[4] = {R0[X.a[0]], R0[X.a[0] + 1], R0[X.a[1]], R0[X.a[1] + 1]};
                const uint32_t u1[4] = {R1[X.a[0]], R1[X.a[0] + 1], R1[X.a[1]], R1[X.a[1] + 1]};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int pp = 2 * (j >> 1);
                    const u16x2 cf = __builtin_bit_cast(u16x2, X.cf[j]);
                    const int h0 = (int)__builtin_amdgcn_udot2(
                        __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(u0[pp + 1], u0[pp], X.sel[j])), cf, 0u, false);
                    const int h1 = (int)__builtin_amdgcn_udot2(
                        __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(u1[pp + 1], u1[pp], X.sel[j])), cf, 0u, false);
                    packed |= (uint32_t)vmix(b0, b1, h0, h1) << (8 * j);   // <= 255: the weights sum to <= 2049
                }
            } else {
                const uint8_t *R0 = reinterpret_cast<const uint8_t *>(prev + omv::mul_u24(y.sx0 - bp.need_lo, sndw));
                const uint8_t *R1 = reinterpret_cast<const uint8_t *>(prev + omv::mul_u24(y.sx1 - bp.need_lo, sndw));
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int dx = dx0 + j;
                    if (dx < L.w) {
                        const XTab x = xs[dx];
                        const int a0 = (short)(x.coef & 0xffff), a1 = (short)(x.coef >> 16);
                        const int h0 = R0[x.sx0] * a0 + R0[x.sx1] * a1;
                        const int h1 = R1[x.sx0] * a0 + R1[x.sx1] * a1;
                        const int v = vmix(b0, b1, h0, h1);
                        packed |= (uint32_t)min(v, 255) << (8 * j);
                    }
                }
            }
            cur[omv::mul_u24(r, cndw) + qd] = packed;   // the next level's source row (bytes past the width are never read)
            if (dy >= bc.own_lo && dy < bc.own_hi) {
                uint8_t *dst = pyr + (size_t)img * g.pyr_bytes + L.off + (size_t)dy * L.pitch;
                if (dx0 + 3 < L.w) {
                    *reinterpret_cast<uint32_t *>(dst + dx0) = packed;
                } else {
                    for (int j = 0; j < 4 && dx0 + j < L.w; ++j) dst[dx0 + j] = (uint8_t)(packed >> (8 * j));
                }
            }
        }
        __syncthreads();
        uint32_t *t = prev;
        prev = cur, cur = t;
    }
}

// K2 --------------------------------------------------------------------------------------------
// FAST-9 strength: max over the 16 circular 9-arcs of min(d) (darker) and of min(-d) (brighter),
// d = centre - ring.  A pixel is a FAST corner at threshold t iff S > t, and OpenCV's
// cornerScore<16>(t) then returns S - 1 (the threshold floor max(t, .) never binds for a corner).
typedef short pk16 __attribute__((ext_vector_type(2)));   // packed int16 pair (v_pk_* ops)

// The strength on packed f16 pairs (k, k+8): 1024 + n is the f16 bit pattern 0x6400 | n (n < 1024), so the
// differences d = v - ring are exact, and every min / max of integers in [-255, 255] is exact.  gfx950's
// v_pk_minimum3_f16 / v_pk_maximum3_f16 take three operands: the 9-arc is min3 of three 3-runs.
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 h2_swap(h2 x) { return h2{x.y, x.x}; }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 h2_biased(const uint8_t *lo, const uint8_t *hi) {   // (1024 + *lo, 1024 + *hi)
    const u16x2 v{(unsigned short)*lo, (unsigned short)*hi};   // ds_read_u8_d16 / _d16_hi
    return __builtin_bit_cast(h2, __builtin_bit_cast(uint32_t, v) | 0x64006400u);
}

template <int RS>
__device__ __forceinline__ int fast_strength_h(const uint8_t *p, int stride_rt) {
    const int stride = RS > 0 ? RS : stride_rt;
    const int o[16] = {3 * stride, 3 * stride + 1, 2 * stride + 2, stride + 3, 3, -stride + 3, -2 * stride + 2,
                       -3 * stride + 1, -3 * stride, -3 * stride - 1, -2 * stride - 2, -stride - 3, -3, stride - 3,
                       2 * stride - 2, 3 * stride - 1};
    const h2 vv = h2_biased(p, p);
    h2 d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = vv - h2_biased(p + o[k], p + o[k + 8]);
    auto Q = [&](const h2 *a, int k) { return k < 8 ? a[k] : h2_swap(a[k - 8]); };
    h2 t3n[8], t3x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        t3n[k] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(d[k], Q(d, k + 1)), Q(d, k + 2));
        t3x[k] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(d[k], Q(d, k + 1)), Q(d, k + 2));
    }
    h2 a{(_Float16)-1000, (_Float16)-1000}, b{(_Float16)1000, (_Float16)1000};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const h2 m9 = __builtin_elementwise_minimum(__builtin_elementwise_minimum(t3n[k], Q(t3n, k + 3)), Q(t3n, k + 6));
        const h2 M9 = __builtin_elementwise_maximum(__builtin_elementwise_maximum(t3x[k], Q(t3x, k + 3)), Q(t3x, k + 6));
        a = __builtin_elementwise_maximum(a, m9);
        b = __builtin_elementwise_minimum(b, M9);
    }
    const int A = (int)__builtin_elementwise_maximum(a.x, a.y), B = (int)__builtin_elementwise_minimum(b.x, b.y);
    return max(A, -B);
}

// Inclusive wave64 prefix sum by DPP (row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15 / 31);
// every lane of the wave must be active.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    return v;
}

// One wavefront (= one workgroup of 64) per cell.  The cell's region is staged into LDS with dword
// loads (row stride rs, 4-byte aligned; pixel (r, q) at pix[r * rs + q]); then
//   1. prefilter at min(iniTh, minTh): a 9-arc of the 16-ring always holds two adjacent compass points
//      (ring positions 0/4/8/12), so a pixel can be a corner only if some adjacent compass pair is
//      brighter (d < -t) or darker (d > t) together -- exact, not a heuristic; survivors are compacted
//      in row-major order (ballot prefix) into an LDS list;
//   2. the full FAST strength for the survivors only (the strength map S stays 0 elsewhere, which is
//      what the NMS of any threshold >= t sees for non-corners);
//   3. NMS (3x3, strict >) at iniTh and minTh in one pass over the survivors;
//   4. emission at iniTh, or minTh if the cell had no iniTh keypoint (ORBextractor.cc:764-782).
#ifdef OMV_FAST_PROFILE
__device__ unsigned long long g_fast_stats[8];
#endif
template <int RS>   // LDS row stride in bytes (0: per cell, rounded up to 4)
__global__ void __launch_bounds__(64) fast_cells_kernel(Geom g, const Cell *cells, const uint8_t *images,
                                                        size_t img_stride, size_t pitch0, const uint8_t *pyr,
                                                        int *cell_cnt, uint32_t *cell_kp, int rmax, int smax,
                                                        int n_blocks) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int blk = omv::xcd_block(n_blocks);
    if (blk < 0) return;
    const int img = blk / g.n_cells;
    const int ci = blk - img * g.n_cells;
    const Cell c = cells[ci];
    const int lane = threadIdx.x;
    const int rw = c.x1 - c.x0, rh = c.y1 - c.y0;
    int sp;
    const uint8_t *src = level_base(g, images, img_stride, pitch0, pyr, img, c.level, &sp);
    const uint8_t *row0 = src + (size_t)c.y0 * sp + c.x0;
    const bool dwords = ((sp & 3) == 0) && ((((uintptr_t)src) & 3) == 0);
    const int o = dwords ? (int)(((uintptr_t)row0) & 3) : 0;
    const int rs = RS > 0 ? RS : ((rw + o + 3) & ~3);
    uint8_t *pix = smem + o;
    // the strength map covers the NMS reach only: rows / columns 2 .. n-3 of the region, (r, q) at
    // S[(r - 2) * sw + q - 2] (the region's outer rows never hold a candidate or an NMS neighbour)
    uint8_t *S = smem + rmax;
    const int sw = rw - 4;
    uint16_t *cand = (uint16_t *)(smem + rmax + smax);
    if (dwords) {
        const int nd = (rw + o + 3) >> 2;   // dwords of a row read (the LDS row holds rs / 4)
        const uint32_t *g0 = (const uint32_t *)(row0 - o);
        const int sw = sp >> 2;
        uint32_t *l0 = (uint32_t *)smem;
        // lane -> (row lr of a band of rpi rows, dword w); the band steps down the region by pointer increments
        const int rpi = 64 / nd, lr = lane / nd, w = lane - lr * nd;
        if (lr < rpi) {
            const uint32_t *gs = g0 + (size_t)lr * sw + w;
            uint32_t *ld = l0 + lr * (rs >> 2) + w;
            const size_t gstep = (size_t)rpi * sw;
            const int lstep = rpi * (rs >> 2);
#pragma unroll 4
            for (int r = lr; r < rh; r += rpi, gs += gstep, ld += lstep) *ld = *gs;
        }
    } else {
        for (int i = lane; i < rw * rh; i += 64) {
            const int r = i / rw, q = i - r * rw;
            pix[r * rs + q] = row0[(size_t)r * sp + q];
        }
    }
    for (int i = lane; i < (sw * (rh - 4) + 15) >> 4; i += 64) ((uint4 *)S)[i] = make_uint4(0, 0, 0, 0);   // rmax % 16 == 0
    __syncthreads();
    const int dw = rw - 6, dh = rh - 6;   // detection window [3, rw-4] x [3, rh-4]
    const int ndet = (dw > 0 && dh > 0) ? dw * dh : 0;
    // i / dw by multiply-shift with m = floor(2^20/dw) + 1: exact while i * dw < 2^20 (cells are < 80 px wide)
    const uint32_t mdw = dw > 0 ? (1u << 20) / (uint32_t)dw + 1u : 0u;
    auto rowcol = [&](int i, int &r, int &q) {
        const int rr = omv::mul_u24(i, (int)mdw) >> 20;
        r = 3 + rr, q = 3 + i - omv::mul_u24(rr, dw);   // 24-bit multiplies: full rate
    };
    const uint64_t lt = (1ull << lane) - 1ull;
    // compass prefilter at threshold t: the row-major candidate list cand[0..n) (returns n)
    auto prefilter = [&](int t) {
        int ncand = 0;
        if (dwords && ndet > 0) {
            // 8 pixels per lane: LDS dwords j, j+1 of a row (bytes = columns 4j+k-o) with their compass
            // neighbours as whole dwords (up / down rows; left / right as byte windows of the adjacent dwords, one
            // v_perm each), the tests on packed int16 pairs.  The adjacent-pair test (a0&a4)|(a4&a8)|(a8&a12)|(a12&a0) is (a0|a8)&(a4|a12).  Survivors go to the
            // list by a DPP wave scan of the per-lane counts, each lane then writing its set bits.
            const uint32_t *w32 = reinterpret_cast<const uint32_t *>(smem);
            const int jq0 = (o + 3) >> 2, jq1 = (o + rw - 4) >> 2, nqr = jq1 - jq0 + 1, rsw = rs >> 2;
            const int npr = (nqr + 1) >> 1;   // dword pairs per row
            const int np = npr * dh;
            const uint32_t mp = (1u << 20) / (uint32_t)npr + 1u;   // tp / npr, exact while tp * npr < 2^20
            const pk16 T0{(short)t, (short)t};
            // bytes s, s+1 (lo) / s+2, s+3 (hi) of the 8-byte {a:b} as a packed int16 pair
            auto lo = [](uint32_t a, uint32_t b, uint32_t s) {
                return __builtin_bit_cast(pk16, __builtin_amdgcn_perm(a, b, 0x0c000c00u | ((s + 1) << 16) | s));
            };
            auto hi = [](uint32_t a, uint32_t b, uint32_t s) {
                return __builtin_bit_cast(pk16, __builtin_amdgcn_perm(a, b, 0x0c000c00u | ((s + 3) << 16) | (s + 2)));
            };
            auto test = [&](pk16 v, pk16 n0, pk16 n4, pk16 n8, pk16 n12) {   // bits 15 / 31: the pair passes
                // brighter pair (n0 | n8 > v + t) & (n4 | n12 > v + t) <=> min(max(n0, n8), max(n4, n12)) > v + t,
                // darker pair <=> max(min(n0, n8), min(n4, n12)) < v - t; each test is the sign of one difference
                // (v_pk_max_i16 / v_pk_min_i16: 11 packed ops per pixel pair instead of 17)
                const pk16 vp = v + T0, vm = v - T0;
                auto sg = [](pk16 x) { return __builtin_bit_cast(uint32_t, x); };
                const pk16 hi = __builtin_elementwise_min(__builtin_elementwise_max(n0, n8), __builtin_elementwise_max(n4, n12));
                const pk16 lo = __builtin_elementwise_max(__builtin_elementwise_min(n0, n8), __builtin_elementwise_min(n4, n12));
                return (sg(vp - hi) | sg(lo - vm)) & 0x80008000u;
            };
            for (int t0 = 0; t0 < np; t0 += 64) {
                const int tp = t0 + lane;
                uint32_t bits = 0;
                int r = 3, jq = jq0;
                if (tp < np) {
                    const int rr = omv::mul_u24(tp, (int)mp) >> 20;   // tp < 2^13, mp <= 2^20 + 1
                    r = 3 + rr, jq = jq0 + 2 * (tp - omv::mul_u24(rr, npr));
                    const int j = omv::mul_u24(r, rsw) + jq;
                    const uint32_t Wm = w32[j - 1], C0 = w32[j], C1 = w32[j + 1], Wp = w32[j + 2];
                    const uint32_t D0 = w32[j + 3 * rsw], D1 = w32[j + 3 * rsw + 1];
                    const uint32_t U0 = w32[j - 3 * rsw], U1 = w32[j - 3 * rsw + 1];
                    // left neighbours: {C:prev} from byte 1; right: {next:C} from byte 3
                    const uint32_t p0 = test(lo(C0, C0, 0), lo(D0, D0, 0), lo(C1, C0, 3), lo(U0, U0, 0), lo(C0, Wm, 1));
                    const uint32_t p1 = test(hi(C0, C0, 0), hi(D0, D0, 0), hi(C1, C0, 3), hi(U0, U0, 0), hi(C0, Wm, 1));
                    const uint32_t p2 = test(lo(C1, C1, 0), lo(D1, D1, 0), lo(Wp, C1, 3), lo(U1, U1, 0), lo(C1, C0, 1));
                    const uint32_t p3 = test(hi(C1, C1, 0), hi(D1, D1, 0), hi(Wp, C1, 3), hi(U1, U1, 0), hi(C1, C0, 1));
                    // bit 2k = p_k bit 15, bit 2k + 1 = p_k bit 31: the shifts land the bit-15s on 0, 2, 4, 6 and the
                    // bit-31s on 16, 18, 20, 22
                    const uint32_t xb = (p0 >> 15) | (p1 >> 13) | (p2 >> 11) | (p3 >> 9);
                    bits = (xb & 0x55u) | ((xb >> 15) & 0xaau);
                    // columns q0 + k of the pair outside [3, rw - 4] (the second dword of a row's last pair
                    // may lie wholly past it)
                    const int q0 = 4 * jq - o;
                    const int klo = min(max(3 - q0, 0), 8), khi = min(max(rw - 3 - q0, 0), 8);
                    bits &= ((1u << khi) - 1u) & ~((1u << klo) - 1u);
                }
                const int cnt = __popc(bits);
                const int incl = wave_incl_scan_dpp(cnt);
                int pos = ncand + incl - cnt;
                const int ibase = omv::mul_u24(r - 3, dw) + (4 * jq - o) - 3;
                // row-major: lanes hold consecutive pairs, bit k = column q0 + k (a few set bits per lane)
                for (uint32_t b = bits; b; b &= b - 1u) cand[pos++] = (uint16_t)(ibase + __builtin_ctz(b));
                ncand += __builtin_amdgcn_readlane(incl, 63);
            }
        } else {
            for (int i0 = 0; i0 < ndet; i0 += 64) {
                const int i = i0 + lane;
                bool pass = false;
                if (i < ndet) {
                    int r, q;
                    rowcol(i, r, q);
                    const uint8_t *p = pix + r * rs + q;
                    const int v = p[0];
                    const int d0 = v - p[3 * rs], d4 = v - p[3], d8 = v - p[-3 * rs], d12 = v - p[-3];
                    const bool a0 = d0 > t, a4 = d4 > t, a8 = d8 > t, a12 = d12 > t;
                    const bool b0 = d0 < -t, b4 = d4 < -t, b8 = d8 < -t, b12 = d12 < -t;
                    pass = (a0 && a4) || (a4 && a8) || (a8 && a12) || (a12 && a0) || (b0 && b4) || (b4 && b8) ||
                           (b8 && b12) || (b12 && b0);
                }
                const uint64_t m = __ballot(pass);
                if (pass) cand[ncand + __popcll(m & lt)] = (uint16_t)i;
                ncand += __popcll(m);
            }
        }
        __syncthreads();
        // FAST strength of the candidates (threshold-free; non-candidates keep S = 0)
        for (int k = lane; k < ncand; k += 64) {
            const int i = cand[k];
            int r, q;
            rowcol(i, r, q);
            const int sv = fast_strength_h<RS>(pix + r * rs + q, rs);
            S[omv::mul_u24(r - 2, sw) + (q - 2)] = (uint8_t)min(max(sv, 0), 255);
        }
        __syncthreads();
        return ncand;
    };
    // NMS at threshold th over the candidates: keypoint k survives iff S > th and S - 1 > every neighbour's
    // cornerScore (S - 1 if S > th, else 0) -- i.e. S > max(th, 1, every neighbour's S).  Returns the count;
    // with `out`, emits row-major.
    auto nms = [&](int ncand, int th, uint32_t *out) {
        int base = 0;
        for (int k0 = 0; k0 < ncand; k0 += 64) {
            const int k = k0 + lane;
            bool keep = false;
            uint32_t packed = 0;
            if (k < ncand) {
                const int i = cand[k];
                int r, q;
                rowcol(i, r, q);
                const uint8_t *sp8 = S + omv::mul_u24(r - 2, sw) + (q - 2);
                const int v = sp8[0];
                // v > th and v - 1 > (nv > th ? nv - 1 : 0) for all 8 neighbours <=> v > max(nv..., th, 1)
                int m = max(th, 1);
#pragma unroll
                for (int n = 0; n < 9; ++n)
                    if (n != 4) m = max(m, (int)sp8[(n / 3 - 1) * sw + (n % 3 - 1)]);
                keep = v > m;
                const int x = c.x0 + q - kMinB, y = c.y0 + r - kMinB;
                packed = (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)(v - 1) << 24);
            }
            const uint64_t m = __ballot(keep);
            const int pos = base + __popcll(m & lt);
            if (out && keep && pos < g.cell_cap) out[pos] = packed;
            base += __popcll(m);
        }
        return base;
    };
    // iniThFAST first; minThFAST only for a cell without an iniTh keypoint (ORBextractor.cc:745-782).  Every
    // pixel with S > th passes the compass prefilter at th, so the iniTh pass only needs those candidates:
    // the NMS treats non-candidates (S = 0) as the reference treats scores <= th.
    // keypoints are emitted row-major by the counting pass itself (coordinates relative to the FAST border,
    // minBorder = 16); a cell without an iniTh keypoint wrote nothing and is redone at minTh
    uint32_t *out = cell_kp + (size_t)blk * g.cell_cap;
    int th = g.ini_th;
    int ncand = prefilter(th);
#ifdef OMV_FAST_PROFILE
    const int ncand0 = ncand;
#endif
    int total = nms(ncand, th, out);
    if (total == 0) {
        th = g.min_th;
        ncand = prefilter(th);
        total = nms(ncand, th, out);
    }
    // cap = max NMS survivors of the window, so this cannot trigger (writes past it were dropped)
    if (lane == 0) cell_cnt[blk] = total > g.cell_cap ? -1 : total;
#ifdef OMV_FAST_PROFILE
    // totals over the launch: cells, detection-window pixels, prefilter candidates (both passes), minTh retries,
    // keypoints; the last cell prints them
    {
        __shared__ int dummy;
        (void)dummy;
        if (lane == 0) {
            atomicAdd(&g_fast_stats[0], 1ull);
            atomicAdd(&g_fast_stats[1], (unsigned long long)ndet);
            atomicAdd(&g_fast_stats[2], (unsigned long long)ncand0);
            atomicAdd(&g_fast_stats[3], th == g.min_th && g.min_th != g.ini_th ? 1ull : 0ull);
            atomicAdd(&g_fast_stats[4], (unsigned long long)ncand);
            atomicAdd(&g_fast_stats[5], (unsigned long long)total);
            __threadfence();
            const unsigned long long done = atomicAdd(&g_fast_stats[7], 1ull) + 1;
            if (done == (unsigned long long)n_blocks)
                printf("fast: cells %llu pixels %llu cand(iniTh) %llu retries %llu cand(last pass) %llu keypoints %llu\n",
                       g_fast_stats[0], g_fast_stats[1], g_fast_stats[2], g_fast_stats[3], g_fast_stats[4],
                       g_fast_stats[5]);
        }
    }
#endif
}

// K3 --------------------------------------------------------------------------------------------
// (every lane active: the DPP form, six VALU ops instead of six LDS-latency permutes)
__device__ __forceinline__ int wave_incl_scan(int v) { return wave_incl_scan_dpp(v); }

// In-place exclusive scan of a[0..n) in LDS by the whole (256-thread) block; returns the total.
__device__ int block_excl_scan(int *a, int n, int *tmp) {
    const int tid = threadIdx.x, T = blockDim.x;
    const int chunk = (n + T - 1) / T;
    const int b = min(n, tid * chunk), e = min(n, b + chunk);
    int s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    const int incl = wave_incl_scan(s);
    const int wave = tid >> 6, nw = T >> 6;
    __syncthreads();
    if ((tid & 63) == 63) tmp[wave] = incl;
    __syncthreads();
    int woff = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        if (w < wave) woff += tmp[w];
        tot += tmp[w];
    }
    int run = woff + incl - s;
    for (int i = b; i < e; ++i) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return tot;
}

// Two independent in-place exclusive scans (a[0..na), b[0..nb)) with one set of barriers; tmp holds 16 ints.
// Thread t scans the same chunks as block_excl_scan, so a caller that wrote exactly those entries itself needs no
// barrier before the call.
__device__ int2 block_excl_scan2(int *a, int na, int *b, int nb, int *tmp) {
    const int tid = threadIdx.x, T = blockDim.x;
    const int ca = (na + T - 1) / T, a0 = min(na, tid * ca), a1 = min(na, a0 + ca);
    const int cb = (nb + T - 1) / T, b0 = min(nb, tid * cb), b1 = min(nb, b0 + cb);
    int sa = 0, sb = 0;
    for (int i = a0; i < a1; ++i) sa += a[i];
    for (int i = b0; i < b1; ++i) sb += b[i];
    const int ia = wave_incl_scan(sa), ib = wave_incl_scan(sb);
    const int wave = tid >> 6, nw = T >> 6;
    __syncthreads();
    if ((tid & 63) == 63) tmp[wave] = ia, tmp[8 + wave] = ib;
    __syncthreads();
    int oa = 0, ta = 0, ob = 0, tb = 0;
    for (int w = 0; w < nw; ++w) {
        if (w < wave) oa += tmp[w], ob += tmp[8 + w];
        ta += tmp[w], tb += tmp[8 + w];
    }
    int run = oa + ia - sa;
    for (int i = a0; i < a1; ++i) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    run = ob + ib - sb;
    for (int i = b0; i < b1; ++i) {
        const int v = b[i];
        b[i] = run;
        run += v;
    }
    __syncthreads();
    return make_int2(ta, tb);
}

__device__ int block_sum(int v, int *tmp) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += tmp[w];
    __syncthreads();
    return t;
}

// Node rectangles as packed 16-bit pairs (x0 | x1 << 16, y0 | y1 << 16; level coordinates < 2^15): 3 ints per node
// instead of 5, so the workgroup's LDS stays under 20 KB (eight workgroups per CU)
struct NodeSoA {
    int *xx, *yy, *cnt;
    __device__ __forceinline__ int x0(int i) const { return xx[i] & 0xffff; }
    __device__ __forceinline__ int x1(int i) const { return (int)((uint32_t)xx[i] >> 16); }
    __device__ __forceinline__ int y0(int i) const { return yy[i] & 0xffff; }
    __device__ __forceinline__ int y1(int i) const { return (int)((uint32_t)yy[i] >> 16); }
    __device__ __forceinline__ void set(int i, int ax0, int ax1, int ay0, int ay1) const {
        xx[i] = ax0 | (ax1 << 16), yy[i] = ay0 | (ay1 << 16);
    }
    __device__ __forceinline__ void copy_from(int i, const NodeSoA &o, int k) const {
        xx[i] = o.xx[k], yy[i] = o.yy[k], cnt[i] = o.cnt[k];
    }
};

// Quadrant of key (x, y) in node i: 0 = n1 (UL), 1 = n2 (UR), 2 = n3 (BL), 3 = n4 (BR)  (DivideNode)
__device__ __forceinline__ int node_mid_x(const NodeSoA &A, int i) {
    return A.x0(i) + (int)ceilf((float)(A.x1(i) - A.x0(i)) / 2);
}
__device__ __forceinline__ int node_mid_y(const NodeSoA &A, int i) {
    return A.y0(i) + (int)ceilf((float)(A.y1(i) - A.y0(i)) / 2);
}
__device__ __forceinline__ void child_rect(const NodeSoA &A, int i, int t, const NodeSoA &Bo, int j) {
    const int xm = node_mid_x(A, i), ym = node_mid_y(A, i);
    Bo.set(j, (t & 1) ? xm : A.x0(i), (t & 1) ? A.x1(i) : xm, (t & 2) ? ym : A.y0(i), (t & 2) ? A.y1(i) : ym);
}

constexpr uint32_t kSplitFlag = 0x80000000u;

struct OctArgs {
    const int *cell_cnt;
    const uint32_t *cell_kp;
    uint32_t *cand;        // compact candidates scratch
    uint32_t *nid;         // per-candidate node id scratch
    uint32_t *lvl_out;     // [img][out_per_img] packed x|y|score of selected keypoints
    uint32_t *lvl_cls;     // [img][out_per_img] rank | lap << 31
    int *lvl_cnt;          // [img][L][3] total, mono, lap
    const int *lapping;    // device [img][2]
    int *err;
};

constexpr int kOctSmallImages = 16;      // extractions of up to this many images: octree_kernel<1>
#ifndef OMV_OCT_WGS
#define OMV_OCT_WGS 8   // workgroups per CU the register budget targets (LDS: 20 KB each; measured 6 / 7 / 8 with
                        // the level-major order: 0.232 / 0.221 / 0.213 ms per 128-frame launch; 8 spills a few
                        // registers but wins since the long level-0 workgroups overlap more of each other)
#endif
// WGS: workgroups per CU the register budget targets -- OMV_OCT_WGS for batches; 1 for a frame or two, where only a
// few dozen workgroups run and the level-0 ones are the critical path (no spills at the full register budget).
template <int WGS>
__global__ void __launch_bounds__(256, WGS) octree_kernel(Geom g, OctArgs a) {
    extern __shared__ __attribute__((aligned(16))) int osm[];
    // level-major block order: the finest levels (most keys, the longest workgroups) of every image are dispatched
    // first and the short coarse levels fill the launch's tail (longest-job-first)
    const int n_img = gridDim.x / g.nlevels;
    const int l = blockIdx.x / n_img;
    const int img = blockIdx.x - l * n_img;
    const LevelGeom &L = g.lv[l];
    const int tid = threadIdx.x, T = blockDim.x;
    const int NC = g.node_cap;
    // LDS carve-up
    int *tmp = osm;                  // 16
    int *shared_int = osm + 16;      // 16 scalars
    int *buf = osm + 32;
    NodeSoA A{buf, buf + NC, buf + 2 * NC};
    NodeSoA B{buf + 3 * NC, buf + 4 * NC, buf + 5 * NC};
    int *ccnt = buf + 6 * NC;        // ccnt_cap (>= 4 * NC)
    int *cellscan = ccnt;            // the level's cells (<= ccnt_cap by host check), gather phase only
    int *rest = ccnt + g.ccnt_cap;
    int *scanA = rest;               // NC
    int *scanB = rest + NC;          // NC
    int *map = rest + 2 * NC;        // NC: new index of an unsplit/unprocessed node, or -1
    int *vlist = rest + 3 * NC;      // NC
    int *vpos = rest + 4 * NC;       // NC: position in the sorted V list, or -1
    omv::SortItem *items = reinterpret_cast<omv::SortItem *>(rest + 5 * NC);   // NC items (3 ints)
    int *sstack = rest + 8 * NC;     // the sort's range queues: introsort_queue_ints(NC) (<= oct_queue(NC))

#ifdef OMV_OCT_PROFILE
    long long pf_t0 = wall_clock64(), pf_sort = 0, pf_p1 = 0, pf_p2 = 0, pf_gather = 0;
    int pf_r1 = 0, pf_r2 = 0;
#endif
    const int ncell = L.cell_end - L.cell_begin;
    uint32_t *cand = a.cand + (size_t)img * g.cand_per_img + L.cand_off;
    uint32_t *nid = a.nid + (size_t)img * g.cand_per_img + L.cand_off;
    const int N = L.quota;

    // ---- gather candidates of this level in cell order (vToDistributeKeys order) ----
    for (int i = tid; i < ncell; i += T) {
        const int cc = a.cell_cnt[(size_t)img * g.n_cells + L.cell_begin + i];
        if (cc < 0) atomicOr(a.err, OMV_ERR_CAPACITY);
        cellscan[i] = max(cc, 0);
    }
    __syncthreads();
    const int K = block_excl_scan(cellscan, ncell, tmp);
    if (K > L.cand_cap) {
        if (tid == 0) atomicOr(a.err, OMV_ERR_CAPACITY);
        return;
    }
    // one thread per cell: its keys to [start, next start), eight loads in flight before their stores (the store
    // to cand could alias the next load as far as the compiler knows, which serialised load -> store pairs)
    for (int i = tid; i < ncell; i += T) {
        const int k0 = cellscan[i], k1 = i + 1 < ncell ? cellscan[i + 1] : K;
        const uint32_t *src = a.cell_kp + ((size_t)img * g.n_cells + L.cell_begin + i) * g.cell_cap;
        for (int b = k0; b < k1; b += 8) {
            const int nb = min(8, k1 - b);
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[b - k0 + min(u, nb - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (u < nb) cand[b + u] = v[u];
        }
    }
    __syncthreads();

    int *cnt_out = a.lvl_cnt + ((size_t)img * g.nlevels + l) * 3;
    uint32_t *out = a.lvl_out + (size_t)img * g.out_per_img + L.out_off;
    uint32_t *cls = a.lvl_cls + (size_t)img * g.out_per_img + L.out_off;
    if (K == 0) {
        if (tid == 0) cnt_out[0] = cnt_out[1] = cnt_out[2] = 0;
        return;
    }

    // ---- initial vertical strips ----
    const int nIni = L.nIni;
    const float hX = L.hX;
    const int Hn = L.maxBY - kMinB;
    if (nIni > NC) {
        if (tid == 0) atomicOr(a.err, OMV_ERR_CAPACITY);
        return;
    }
    for (int i = tid; i < nIni; i += T) {
        B.set(i, (int)(hX * (float)i), (int)(hX * (float)(i + 1)), 0, Hn);
        B.cnt[i] = 0;
    }
    __syncthreads();
    // the passes over the keys below keep four global loads in flight per thread (clamped indices: unconditional
    // loads, so the compiler does not serialise them behind their guards); nid / cand live in global scratch
    constexpr int kKB = 4;
    for (int k0 = tid; k0 < K; k0 += kKB * T) {
        uint32_t cv[kKB];
#pragma unroll
        for (int i = 0; i < kKB; ++i) cv[i] = cand[min(k0 + i * T, K - 1)];
#pragma unroll
        for (int i = 0; i < kKB; ++i) {
            const int k = k0 + i * T;
            if (k < K) {
                const float x = (float)(cv[i] & 0xfff);
                const int n = (int)(x / hX);
                nid[k] = (uint32_t)n;
                atomicAdd(&B.cnt[n], 1);
            }
        }
    }
    __syncthreads();
    // drop empty strips, keep order
    for (int i = tid; i < nIni; i += T) scanA[i] = B.cnt[i] > 0 ? 1 : 0;
    __syncthreads();
    int m = block_excl_scan(scanA, nIni, tmp);
    for (int i = tid; i < nIni; i += T)
        if (B.cnt[i] > 0) {
            const int j = scanA[i];
            A.copy_from(j, B, i);
        }
    __syncthreads();
    for (int k0 = tid; k0 < K; k0 += kKB * T) {
        uint32_t nv4[kKB];
#pragma unroll
        for (int i = 0; i < kKB; ++i) nv4[i] = nid[min(k0 + i * T, K - 1)];
#pragma unroll
        for (int i = 0; i < kKB; ++i)
            if (k0 + i * T < K) nid[k0 + i * T] = (uint32_t)scanA[nv4[i]];
    }
    __syncthreads();

#ifdef OMV_OCT_PROFILE
    pf_gather = wall_clock64() - pf_t0;
#endif
    // ---- subdivision rounds ----
    // phase 1: every node with > 1 key splits (list walk :562-613)
    // phase 2: only the expandable list of the last round, largest (size, UL.x) first (:621-679)
    bool phase2 = false;
    int nv = 0;   // phase 2: |V|, V stored in vlist (indices into A, creation order)
    for (int guard = 0; guard < 4096; ++guard) {
        const int prev = m;
#ifdef OMV_OCT_PROFILE
        const long long pf_r = wall_clock64();
        const bool pf_ph2 = phase2;
#endif
        // 1. mark which nodes split this round (phase 1: every node with > 1 key), zero child counts.  No barrier
        // here: each node's entries are written by one thread, and the phase-2 sort reads only A and the V list
        // (both final since the previous round's last barrier) before its own first barrier.
        for (int i = tid; i < m; i += T) {
            map[i] = -1;
            vpos[i] = !phase2 && A.cnt[i] > 1 ? 0 : -1;
            ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
        }
        if (phase2) {
            // sort V by (size, UL.x) exactly as libstdc++'s std::sort moves the elements: the introsort
            // partitions one recursion depth at a time, a range per wavefront, the final insertion sort as a
            // stable rank over the block (B is free until step 4: its x0 / x1 / y0 rows hold the items' scratch)
            // (std::sort's exact element moves are needed: equal (size, UL.x) keys occur in every phase-2 list of
            // the bench images -- siblings share UL.x -- so a rank sort of distinct keys never applies)
            for (int j = tid; j < nv; j += T) items[j] = omv::SortItem{A.cnt[vlist[j]], A.x0(vlist[j]), vlist[j]};
            __syncthreads();
            omv::block_introsort_loop(items, nv, sstack, scanA, scanB, tid, T);
            omv::block_final_insertion_sort(items, nv, reinterpret_cast<omv::SortItem *>(B.xx), tid, T);   // B: 3 NC ints
#ifdef OMV_OCT_PROFILE
            pf_sort += wall_clock64() - pf_r;
#endif
            for (int j = tid; j < nv; j += T) vpos[items[j].payload] = j;
        }
        __syncthreads();
        // 2. quadrant counts for the candidate nodes
        for (int k0 = tid; k0 < K; k0 += kKB * T) {
            uint32_t nv4[kKB], pv4[kKB];
#pragma unroll
            for (int i = 0; i < kKB; ++i) {
                const int kc = min(k0 + i * T, K - 1);
                nv4[i] = nid[kc], pv4[i] = cand[kc];
            }
#pragma unroll
            for (int i = 0; i < kKB; ++i) {
                const int k = k0 + i * T;
                if (k >= K) continue;
                const uint32_t n = nv4[i] & ~kSplitFlag;
                if (vpos[n] >= 0) {
                    const uint32_t p = pv4[i];
                    const int x = p & 0xfff, y = (p >> 12) & 0xfff;
                    const int t = (x < node_mid_x(A, n) ? 0 : 1) + (y < node_mid_y(A, n) ? 0 : 2);
                    atomicAdd(&ccnt[4 * n + t], 1);
                    nid[k] = kSplitFlag | (n << 2) | t;
                } else {
                    nid[k] = n;
                }
            }
        }
        __syncthreads();
        // 3. which candidate nodes are actually divided, and in what order children are created
        //    processed[i]: scanA holds #non-empty children in creation order position
        int n_proc_nodes;   // number of divided nodes
        if (!phase2) {
            // creation order = list order; every candidate node is divided.  Each thread writes the chunk of
            // entries the scans below give it, so no barrier separates the two
            const int chunk = (m + T - 1) / T, i0 = min(m, tid * chunk), i1 = min(m, i0 + chunk);
            for (int i = i0; i < i1; ++i) {
                int nk = 0;
                if (vpos[i] >= 0)
                    for (int t = 0; t < 4; ++t) nk += ccnt[4 * i + t] > 0;
                scanA[i] = nk;
                scanB[i] = vpos[i] >= 0 ? 0 : 1;
            }
            n_proc_nodes = m;   // scan domain
        } else {
            // divide from the back of the sorted list until the list holds >= N nodes (:633-675)
            // the list size after dividing items[nv-1 .. j] is m + sum (children - 1) over them: a suffix
            // sum (block scan over r = nv-1-j); the walk stops at the first r reaching N, else at j = 0
            int *dv = B.cnt, *dv1 = B.yy;   // B is free until step 4
            for (int r = tid; r < nv; r += T) {
                const int n = items[nv - 1 - r].payload;
                int nk = 0;
                for (int t = 0; t < 4; ++t) nk += ccnt[4 * n + t] > 0;
                dv[r] = dv1[r] = nk - 1;
            }
            if (tid == 0) shared_int[0] = nv;
            __syncthreads();
            block_excl_scan(dv, nv, tmp);
            for (int r = tid; r < nv; r += T)
                if (m + dv[r] + dv1[r] >= N) atomicMin(&shared_int[0], r);
            __syncthreads();
            const int jstar = shared_int[0] < nv ? nv - 1 - shared_int[0] : 0;
            n_proc_nodes = nv - jstar;
            // processing position p = 0.. corresponds to items[nv-1-p]
            for (int p = tid; p < n_proc_nodes; p += T) {
                const int n = items[nv - 1 - p].payload;
                int nk = 0;
                for (int t = 0; t < 4; ++t) nk += ccnt[4 * n + t] > 0;
                scanA[p] = nk;
            }
            // vpos now marks processed nodes only: position p, else -1
            __syncthreads();
            for (int i = tid; i < m; i += T) vpos[i] = -1;
            __syncthreads();
            for (int p = tid; p < n_proc_nodes; p += T) vpos[items[nv - 1 - p].payload] = p;
            __syncthreads();
            for (int i = tid; i < m; i += T) scanB[i] = vpos[i] >= 0 ? 0 : 1;
            __syncthreads();
        }
        const int2 QU = block_excl_scan2(scanA, n_proc_nodes, scanB, m, tmp);
        const int Q = QU.x, newm = QU.x + QU.y;
        if (newm > NC) {
            if (tid == 0) atomicOr(a.err, OMV_ERR_CAPACITY);
            return;
        }
        // 4. build the new list: children (reverse creation order) then survivors (old order); xf[r]: the child
        //    created r-th has > 1 key (the next round's V list, step 6).  xf aliases the sort items, dead by now
        int *xf = reinterpret_cast<int *>(items);
        for (int i = tid; i < m; i += T) {
            const int p = phase2 ? vpos[i] : (vpos[i] >= 0 ? i : -1);
            if (p >= 0) {
                int r = scanA[p];
                for (int t = 0; t < 4; ++t) {
                    const int c = ccnt[4 * i + t];
                    if (c > 0) {
                        const int j = Q - 1 - r;
                        child_rect(A, i, t, B, j);
                        B.cnt[j] = c;
                        xf[r] = c > 1 ? 1 : 0;
                        ccnt[4 * i + t] = -(j + 1);   // remember the child's new index
                        ++r;
                    }
                }
            } else {
                const int j = Q + scanB[i];
                B.copy_from(j, A, i);
                map[i] = j;
            }
        }
        __syncthreads();
        // 5. relabel keys
        for (int k0 = tid; k0 < K; k0 += kKB * T) {
            uint32_t nv4[kKB];
#pragma unroll
            for (int i = 0; i < kKB; ++i) nv4[i] = nid[min(k0 + i * T, K - 1)];
#pragma unroll
            for (int i = 0; i < kKB; ++i) {
                const int k = k0 + i * T;
                if (k >= K) continue;
                const uint32_t v = nv4[i];
                if (v & kSplitFlag) {
                    const int n = (v & ~kSplitFlag) >> 2, t = v & 3;
                    const bool divided = phase2 ? vpos[n] >= 0 : true;
                    nid[k] = divided ? (uint32_t)(-ccnt[4 * n + t] - 1) : (uint32_t)map[n];
                } else {
                    nid[k] = (uint32_t)map[v];
                }
            }
        }
        // 6. expandable children (> 1 key) in creation order = new indices Q-1 down to 0
        const int nexp = block_excl_scan(xf, Q, tmp);
        for (int j = tid; j < Q; j += T)
            if (B.cnt[Q - 1 - j] > 1) vlist[xf[j]] = Q - 1 - j;
        // the new list becomes A (the roles of the two node arrays swap; no copy)
        {
            const NodeSoA t = A;
            A = B;
            B = t;
        }
        __syncthreads();
        m = newm;
#ifdef OMV_OCT_PROFILE
        if (pf_ph2) pf_p2 += wall_clock64() - pf_r, ++pf_r2;
        else pf_p1 += wall_clock64() - pf_r, ++pf_r1;
#endif
        if (m >= N || m == prev) break;
        if (!phase2) {
            if (m + nexp * 3 > N) phase2 = true;
        }
        nv = nexp;
        if (phase2 && nv == 0) {
            // nothing left to expand: the next round would leave the size unchanged
            break;
        }
    }

    // ---- keep the strongest key of each node (first on ties) ----
    int *best = scanA;
    for (int i = tid; i < m; i += T) best[i] = -1;
    __syncthreads();
    for (int k0 = tid; k0 < K; k0 += kKB * T) {
        uint32_t nv4[kKB], pv4[kKB];
#pragma unroll
        for (int i = 0; i < kKB; ++i) {
            const int kc = min(k0 + i * T, K - 1);
            nv4[i] = nid[kc], pv4[i] = cand[kc];
        }
#pragma unroll
        for (int i = 0; i < kKB; ++i) {
            const int k = k0 + i * T;
            if (k < K) atomicMax(&best[(int)nv4[i]], (int)((pv4[i] >> 24) << 23) | (0x7fffff - k));
        }
    }
    __syncthreads();
    const int lap0 = a.lapping[2 * img], lap1 = a.lapping[2 * img + 1];
    for (int i = tid; i < m; i += T) {
        const int k = 0x7fffff - (best[i] & 0x7fffff);
        const uint32_t p = cand[k];
        out[i] = p;
        float xs = (float)((int)(p & 0xfff) + kMinB);
        if (l != 0) xs *= L.scale;
        scanB[i] = (xs >= (float)lap0 && xs <= (float)lap1) ? 1 : 0;
    }
    __syncthreads();
    for (int i = tid; i < m; i += T) map[i] = scanB[i];
    __syncthreads();
    const int nlap = block_excl_scan(scanB, m, tmp);
    for (int i = tid; i < m; i += T) {
        const int lapf = map[i];
        const int rank = lapf ? scanB[i] : i - scanB[i];
        cls[i] = (uint32_t)rank | ((uint32_t)lapf << 31);
    }
    if (tid == 0) {
        cnt_out[0] = m;
        cnt_out[1] = m - nlap;
        cnt_out[2] = nlap;
    }
#ifdef OMV_OCT_PROFILE
    if (tid == 0 && img < 2)
        printf("oct img %d level %d K %d N %d m %d ticks(100MHz) total %lld gather %lld p1 %lld (%d rounds) p2 %lld (%d rounds, sort %lld)\n",
               img, l, K, N, m, wall_clock64() - pf_t0, pf_gather, pf_p1, pf_r1, pf_p2, pf_r2, pf_sort);
#endif
}

// K4 --------------------------------------------------------------------------------------------
// Orientation + blur + rBRIEF, one wavefront per output slot (inactive slots leave at once).  The reference
// blurs every level whole (GaussianBlur 7x7 sigma 2, ORBextractor.cc:1035-1036, OpenCV's bit-exact 8U path,
// BORDER_REFLECT_101 on the level) and then samples 512 pixels of it per keypoint; only the blurred values
// within radius 18.4 of a keypoint are ever read, so the blur is evaluated here, per keypoint, from the
// un-blurred level -- no blurred pyramid is written or re-read:
//   stage   the raw 43 x 43 patch (rows cy-21 .. cy+21, cols cx-21 .. cx+21, reflect-101 outside the level)
//           into this wave's LDS, three 16-byte loads per lane (byte loads near the level's left / right edge);
//   IC_Angle (:19-43) over the r = 15 disc of that raw patch: lane = (disc row, 16-byte half), five LDS dwords,
//           four v_dot4 items with the lane's in-disc byte masks (row sum -> m01) and weights u + 15 (m10) from a
//           per-lane table; a wave reduction; fastAtan2 (degrees, float);
//   blur    horizontal 7-tap sums (two v_dot4_u32_u8 per sum on byte-aligned dwords, exact in u16) of the
//           (row pair, column quad) items any rotation of the pattern can reach (a host table, 189 of 220),
//           stored column-major with the two rows of a pair in one dword; the vertical 7 taps only at the 512
//           sample points: two ds_read2 + three v_dot2_u32_u16 + one mad, (sum_i k_i h_i + 2^15) >> 16,
//           k = [18, 34, 48, 56, 48, 34, 18] -- OpenCV's separable fixed-point integers, so every sampled value
//           equals the reference's blurred pixel;
//   rBRIEF (computeOrbDescriptor :46-90): lane = pattern pair (4 rounds of 64), steering by (cos, sin) with
//           cvRound, bit = I(a) < I(b) collected by 4 ballots = 32 bytes.
struct DescArgs {
    const uint8_t *images;
    size_t img_stride, pitch0;
    const uint8_t *pyr;
    const uint32_t *lvl_out, *lvl_cls;
    const int *lvl_cnt;
    omv_kp *kps;
    uint8_t *desc;
    int *n_out, *mono;
    int n_images;
    const uint32_t *disc;    // [64][8] per lane: (row-sum mask, weight mask) of its four centroid dot4 items
    float *harris;           // optional [n_images][n_max]: OpenCV ORB's Harris response per output row
};

constexpr int kRawRows = 43, kRawDw = 12;   // raw patch: rows cy-21 .. cy+21, 48 bytes each (43 used + alignment)
constexpr int kHCols = 40, kHStride = 23;   // horizontal sums: 40 columns x 22 row pairs (stride 23 dwords)
// LDS dwords per wave (3,680 B): the horizontal sums overwrite the raw patch once its centroid is summed and its MFMA
// operands are in registers (a separate table was 5,744 B per wave: 24 instead of 36 waves per CU)
constexpr int kDescDw = kHCols * kHStride > kRawRows * kRawDw ? kHCols * kHStride : kRawRows * kRawDw;
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));   // 16-byte access, dword-aligned
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void wave_lds_sync() {
    // other lanes read what this wave just wrote: a wave's LDS operations complete in order; keep the compiler's too
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) describe_kernel(Geom g, DescArgs a, int n_blocks) {
    // the wave index is wave-uniform: everything derived from the slot (record, level, counts, patch origin) is
    // scalar work and scalar loads
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int blk = omv::xcd_block(n_blocks);
    if (blk < 0) return;
    const int slot = blk * 4 + wave;
    const int img = slot / g.out_per_img;
    const int s = slot - img * g.out_per_img;
    if (img >= a.n_images) return;
    int l = 0;
    while (l + 1 < g.nlevels && s >= g.lv[l + 1].out_off) ++l;
    const LevelGeom &L = g.lv[l];
    const int j = s - L.out_off;
    const int *cnts = a.lvl_cnt + (size_t)img * g.nlevels * 3;
    if (s == 0 && lane == 0) {
        int tot = 0, mono = 0;
        for (int q = 0; q < g.nlevels; ++q) tot += cnts[3 * q], mono += cnts[3 * q + 1];
        a.n_out[img] = tot;
        a.mono[img] = mono;
    }
    // the slot's record is loaded with the level count (one round trip; slots past the count are in bounds)
    const uint32_t p = a.lvl_out[(size_t)img * g.out_per_img + s];
    const uint32_t cl = a.lvl_cls[(size_t)img * g.out_per_img + s];
    if (j >= cnts[3 * l]) return;
    // the lane's constant tables (independent of the record: in flight together)
    const uint4 dm0 = reinterpret_cast<const uint4 *>(a.disc)[2 * lane], dm1 = reinterpret_cast<const uint4 *>(a.disc)[2 * lane + 1];
    float4 pat[4];
#pragma unroll
    for (int rd = 0; rd < 4; ++rd) pat[rd] = *reinterpret_cast<const float4 *>(c_patternf.v[rd * 64 + lane]);
    const int cx = (int)(p & 0xfff) + kMinB, cy = (int)((p >> 12) & 0xfff) + kMinB;
    const int score = (int)(p >> 24);
    int sp;
    const uint8_t *src = level_base(g, a.images, a.img_stride, a.pitch0, a.pyr, img, l, &sp);
    __shared__ __attribute__((aligned(16))) uint32_t lds[4][kDescDw];
    uint32_t *raw = lds[wave];
    uint32_t *H = lds[wave];   // after the raw patch: H[c * kHStride + m] = h[2m][c] | h[2m+1][c] << 16
    // Keypoints lie in [19, w-20] x [19, h-20] of their level, so the patch reaches at most 2 pixels past an
    // edge (reflected).  Fast path: the level's rows are dword aligned and the 48 bytes from the aligned start
    // stay inside [0, w): three 16-byte loads per lane; raw byte po + c is column cx - 21 + c.
    const int x0 = cx - 21;
    const bool dw_rows = ((((uintptr_t)src) | (uintptr_t)sp) & 3) == 0;
    int po = dw_rows ? (x0 & 3) : 0;
    if (dw_rows && x0 - po >= 0 && x0 - po + 4 * kRawDw <= L.w) {
        const uint8_t *base = src + (x0 - po);
        u32x4a pv[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int i = min(lane + 64 * t, kRawRows * 3 - 1);
            const int r = i / 3, w = i - 3 * r;
            const int yy = omv::reflect101(cy - 21 + r, L.h);
            pv[t] = *reinterpret_cast<const u32x4a *>(base + (size_t)yy * sp + 16 * w);
        }
#pragma unroll
        for (int t = 0; t < 3; ++t)
            if (lane + 64 * t < kRawRows * 3) reinterpret_cast<u32x4a *>(raw)[lane + 64 * t] = pv[t];
    } else {
        po = 0;   // byte loads, columns reflected (near the level's left / right edge, or rows not dword aligned)
        for (int i = lane; i < kRawRows * kRawDw; i += 64) {
            const int r = i / kRawDw, d = i - kRawDw * r;
            const uint8_t *row = src + (size_t)omv::reflect101(cy - 21 + r, L.h) * sp;
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (4 * d + b < 43) v |= (uint32_t)row[omv::reflect101(x0 + 4 * d + b, L.w)] << (8 * b);
            raw[i] = v;
        }
    }
    wave_lds_sync();
    // intensity centroid: lane = (disc row vr = lane >> 1, half h = lane & 1) = bytes cx-15+16h .. +15 of row
    // cy-15+vr (raw row 6 + vr, raw byte po + 6 + 16h) as four dot4 items over five LDS dwords; lanes 62, 63 and
    // the bytes outside the disc have zero masks
    int m01 = 0, m10 = 0;
    {
        const int vr = min(lane >> 1, 30), h = lane & 1;
        const int b = po + 6 + 16 * h;
        const uint32_t *al = raw + (6 + vr) * kRawDw + (b >> 2);
        const int sh = b & 3;
        const uint32_t qq[5] = {al[0], al[1], al[2], al[3], al[4]};
        const uint32_t mk[8] = {dm0.x, dm0.y, dm0.z, dm0.w, dm1.x, dm1.y, dm1.z, dm1.w};
        int rs = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w = __builtin_amdgcn_alignbyte(qq[k + 1], qq[k], sh);
            rs = (int)__builtin_amdgcn_udot4(w, mk[2 * k], (uint32_t)rs, false);
            m10 += (int)__builtin_amdgcn_udot4(w, mk[2 * k + 1], 0u, false);
        }
        m10 -= __mul24(15, rs);
        m01 = __mul24(vr - 15, rs);
    }
    for (int d = 32; d >= 1; d >>= 1) {
        m01 += __shfl_xor(m01, d, 64);
        m10 += __shfl_xor(m10, d, 64);
    }
    // optional Harris response (OpenCV ORB's HarrisResponses, blockSize 7, k 0.04 -- the north star's "Harris score";
    // the reference's response is FAST's): lane k < 49 = block pixel (cy - 3 + k / 7, cx - 3 + k % 7) of the raw patch
    float harris = 0.f;
    if (a.harris) {
        int ha = 0, hb = 0, hc = 0;
        if (lane < 49) {
            const int i = lane / 7, jj = lane - 7 * i;
            const uint8_t *rb = reinterpret_cast<const uint8_t *>(raw) + (18 + i) * (4 * kRawDw) + po + 18 + jj;
            const int st = 4 * kRawDw;
            const int Ix = (rb[1] - rb[-1]) * 2 + (rb[-st + 1] - rb[-st - 1]) + (rb[st + 1] - rb[st - 1]);
            const int Iy = (rb[st] - rb[-st]) * 2 + (rb[st - 1] - rb[-st - 1]) + (rb[st + 1] - rb[-st + 1]);
            ha = Ix * Ix, hb = Iy * Iy, hc = Ix * Iy;
        }
        for (int d = 32; d >= 1; d >>= 1) {
            ha += __shfl_xor(ha, d, 64);
            hb += __shfl_xor(hb, d, 64);
            hc += __shfl_xor(hc, d, 64);
        }
        const float scale = 1.f / ((1 << 2) * 7 * 255.f);
        const float scale_sq_sq = scale * scale * scale * scale;
        harris = ((float)ha * hb - (float)hc * hc - 0.04f * ((float)ha + hb) * ((float)ha + hb)) * scale_sq_sq;
    }
    // horizontal 7-tap sums H(r, c) = sum_j g[j] raw[r][po + c + j] (column c = level column cx - 18 + c) on the
    // matrix cores: per (row tile rt, column tile t) of 16 x 16 sums, the product of 16 raw rows' bytes 16t .. 16t + 31
    // (A, as i8: x - 128) and the banded Toeplitz B[k][c'] = g[k - c' - po] (zero outside the 7 taps; the same for
    // every tile, k <= 15 + 3 + 6 < 32), with the accumulator started at 128 * sum(g) = 128 * 256: integer, exact.
    // v_mfma_i32_16x16x32_i8: lane l holds A[row l & 15][k = 8 (l >> 4) + j] and B[k = 8 (l >> 4) + j][col l & 15]
    // (byte j of a 64-bit operand); D[i] = sum at (row 4 (l >> 4) + i, col l & 15).  Rows 43 .. 47 and columns 40 .. 47
    // of the last tiles read bytes past the patch / multiply zeros and are not stored.  Every operand is read before
    // the first sum is stored: the sums take the patch's place.
    {
        const int sB = 8 * (lane >> 4) - (lane & 15) - po;   // B byte j = g[j + sB]
        constexpr uint64_t kG7 = 0x0012223038302212ull;     // g[0..6] = 18, 34, 48, 56, 48, 34, 18 (byte i = g[i])
        const long Bop = (long)(sB >= 8 || sB <= -8 ? 0ull : sB >= 0 ? kG7 >> (8 * sB) : kG7 << (-8 * sB));
        const uint8_t *rawb = reinterpret_cast<const uint8_t *>(raw);
        const int m0 = 2 * (lane >> 4);   // this lane's first row pair inside a row tile
        uint64_t av[3][3];
#pragma unroll
        for (int rt = 0; rt < 3; ++rt)
#pragma unroll
            for (int t = 0; t < 3; ++t)
                av[rt][t] = *reinterpret_cast<const uint64_t *>(rawb + (16 * rt + (lane & 15)) * (4 * kRawDw) + 16 * t +
                                                                8 * (lane >> 4));
        wave_lds_sync();   // every lane's patch reads before any sum overwrites the patch
#pragma unroll
        for (int rt = 0; rt < 3; ++rt) {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const i32x4 d = __builtin_amdgcn_mfma_i32_16x16x32_i8((long)(av[rt][t] ^ 0x8080808080808080ull), Bop,
                                                                      i32x4{32768, 32768, 32768, 32768}, 0, 0, 0);
                const int c = 16 * t + (lane & 15), m = 8 * rt + m0;
                if (c < kHCols && m < 22) {   // rows <= 43 (pair 21), columns < 40
                    uint32_t *hp = H + c * kHStride + m;
                    hp[0] = (uint32_t)d[0] | ((uint32_t)d[1] << 16);
                    hp[1] = (uint32_t)d[2] | ((uint32_t)d[3] << 16);
                }
            }
        }
    }
    const float angle = omv::fast_atan2_deg((float)m01, (float)m10);
    float sn, cs;
    omv::glibc_sincosf(angle * (float)(3.14159265358979323846 / 180.f), &sn, &cs);
    const float fa = cs, fb = sn;
    wave_lds_sync();   // the horizontal sums of every lane are in LDS
    // the blurred pixel at (cx + dx, cy + dy), |dx|, |dy| <= 18: column dx + 18, sum rows R0 = dy + 18 .. R0 + 6
    // = the four pair dwords from R0 >> 1, realigned by a half when R0 is odd
    auto blurred = [&](int dx, int dy) -> uint32_t {
        const int R0 = dy + 18;   // 0 .. 36, and dx + 18 too: 24-bit multiplies (full rate)
        const uint32_t *q = H + omv::mul_u24(dx + 18, kHStride) + (R0 >> 1);
        const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
        const uint32_t sh = (uint32_t)(R0 & 1) << 4;
        const uint32_t w0 = __builtin_amdgcn_alignbit(d1, d0, sh), w1 = __builtin_amdgcn_alignbit(d2, d1, sh),
                       w2 = __builtin_amdgcn_alignbit(d3, d2, sh);
        uint32_t acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w0), u16x2{18, 34}, 32768u, false);
        acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w1), u16x2{48, 56}, acc, false);
        acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w2), u16x2{48, 34}, acc, false);
        return (acc + 18u * ((d3 >> sh) & 0xffffu)) >> 16;
    };
    uint64_t words[4];
#pragma unroll
    for (int rd = 0; rd < 4; ++rd) {
        const float ax = pat[rd].x, ay = pat[rd].y, bx = pat[rd].z, by = pat[rd].w;
        const int ady = omv::round_even(ax * fb + ay * fa);
        const int adx = omv::round_even(ax * fa - ay * fb);
        const int bdy = omv::round_even(bx * fb + by * fa);
        const int bdx = omv::round_even(bx * fa - by * fb);
        words[rd] = __ballot(blurred(adx, ady) < blurred(bdx, bdy));
    }
    // final row: monoIndex order (front) or lapping order (back, reversed)
    int mono_before = 0, lap_before = 0, total = 0;
    for (int q = 0; q < g.nlevels; ++q) {
        total += cnts[3 * q];
        if (q < l) mono_before += cnts[3 * q + 1], lap_before += cnts[3 * q + 2];
    }
    const int rank = (int)(cl & 0x7fffffffu);
    const int row = (cl >> 31) ? total - 1 - (lap_before + rank) : mono_before + rank;
    omv_kp *kp = a.kps + (size_t)img * g.n_max + row;
    uint64_t *dst = reinterpret_cast<uint64_t *>(a.desc + ((size_t)img * g.n_max + row) * 32);
    if (lane < 4) dst[lane] = words[lane];
    if (a.harris && lane == 0) a.harris[(size_t)img * g.n_max + row] = harris;
    if (lane == 0) {
        float x = (float)cx, y = (float)cy;
        if (l != 0) x *= L.scale, y *= L.scale;
        *kp = omv_kp{x, y, L.size, angle, (float)score, l};
    }
}

// ---------------------------------------------------------------------------------------------
#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

inline int host_round_even(float v) { return (int)std::nearbyint(v); }

// Test hook: the octree's device sort (wave_introsort_loop + block_final_insertion_sort) on one array.
__global__ void __launch_bounds__(256) node_sort_selftest_kernel(const int *k1, const int *k2, int n, int *perm) {
    extern __shared__ __attribute__((aligned(16))) int ssm[];
    omv::SortItem *items = reinterpret_cast<omv::SortItem *>(ssm);
    omv::SortItem *tmp = items + n;
    int *LS = reinterpret_cast<int *>(tmp + n), *RS = LS + n, *stk = RS + n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) items[i] = omv::SortItem{k1[i], k2[i], i};
    __syncthreads();
    omv::block_introsort_loop(items, n, stk, LS, RS, threadIdx.x, blockDim.x);
    omv::block_final_insertion_sort(items, n, tmp, threadIdx.x, blockDim.x);
    for (int i = threadIdx.x; i < n; i += blockDim.x) perm[i] = items[i].payload;
}

}  // namespace

struct omv_orb {
    omv_orb_params p;
    int W, H, max_images;
    int pyr_mode = -1;   // test knob OMV_PYR_MODE read at creation: -1 unset, 0 "levels", 1 "chain"
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> quota;
    int umax[16];
    Geom g;
    // device
    Cell *d_cells = nullptr;
    XTab *d_xt = nullptr, *d_yt = nullptr;
    XQuad *d_xq = nullptr;
    uint32_t *d_disc = nullptr;   // K4's per-lane centroid masks
    float *harris = nullptr;   // optional Harris output of the next batches (omv_orb_set_harris)
    uint8_t *d_pyr = nullptr;
    int *d_cell_cnt = nullptr;
    uint32_t *d_cell_kp = nullptr, *d_cand = nullptr, *d_nid = nullptr, *d_lvl_out = nullptr, *d_lvl_cls = nullptr;
    int *d_lvl_cnt = nullptr, *d_lap = nullptr, *d_err = nullptr;
    int rmax = 0;
    int smax = 0;          // K2 strength-map bytes
    int fast_rs = 0;       // K2 LDS row stride: 68 (17 dwords, odd: rows spread over the banks) when every cell row (plus misalignment) fits, else per cell
    size_t fast_lds = 0;   // K2 dynamic LDS: region + strength map (rmax each) + the candidate list (u16)
    size_t oct_lds = 0;
    size_t pyr_lds[kMaxLevels] = {};   // K1 dynamic LDS per level: x table + the widest row block
    PyrBand *d_bands = nullptr;        // K1 as one launch (pyr_chain_kernel): per (band, level) rows
    int pyr_nb = 0, pyr_buf_dw = 0;    //   bands per image, dwords per LDS ping-pong buffer (0: per-level launches)
    int pyr_tab_dw = 0, pyr_rows = 0;  //   dwords of the staged x table, the most rows a band needs at a level >= 1
    // host staging for the synchronous path
    uint8_t *d_img1 = nullptr;
    omv_kp *d_kp1 = nullptr;
    uint8_t *d_desc1 = nullptr;
    int *d_n1 = nullptr;
    std::vector<int> h_lap;   // the lapping array last uploaded to d_lap (re-uploaded only when it changes)
    hipStream_t last_stream = nullptr;
    int last_n = 0;
    int device = 0;
    // optional per-stage HIP-event timing (bench.py): events recorded on the launch stream
    bool timing = false;
    std::vector<hipEvent_t> ev;   // 5 events per batch: before K1, K2, K3, K4, after K4
    double stage_ms[kOrbStages] = {};
    long long stage_calls = 0;
};

static void flush_timing(omv_orb *o) {
    for (size_t b = 0; b + kOrbStages + 1 <= o->ev.size(); b += kOrbStages + 1) {
        for (int k = 0; k < kOrbStages; ++k) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, o->ev[b + k], o->ev[b + k + 1]);
            o->stage_ms[k] += ms;
        }
        o->stage_calls++;
    }
    for (hipEvent_t e : o->ev) (void)hipEventDestroy(e);
    o->ev.clear();
}

static void mark(omv_orb *o, hipStream_t st) {
    if (!o->timing) return;
    hipEvent_t e;
    (void)hipEventCreate(&e);
    (void)hipEventRecord(e, st);
    o->ev.push_back(e);
}

static omv_status build_geometry(omv_orb *o, std::vector<Cell> &cells, std::vector<XTab> &xt, std::vector<XTab> &yt, std::vector<XQuad> &xq) {
    const omv_orb_params &p = o->p;
    const int nl = p.nlevels;
    // ORBextractor ctor tables (:362-391): scaleFactor is a double member
    const double sf = (double)p.scale_factor;
    o->scale.assign(nl, 1.f), o->sigma2.assign(nl, 1.f), o->inv_scale.resize(nl), o->inv_sigma2.resize(nl);
    for (int i = 1; i < nl; ++i) {
        o->scale[i] = (float)(o->scale[i - 1] * sf);
        o->sigma2[i] = o->scale[i] * o->scale[i];
    }
    for (int i = 0; i < nl; ++i) o->inv_scale[i] = 1.0f / o->scale[i], o->inv_sigma2[i] = 1.0f / o->sigma2[i];
    o->quota.assign(nl, 0);
    const float f = (float)(1.0f / sf);
    float per = p.nfeatures * (1 - f) / (1 - (float)std::pow((double)f, (double)nl));
    int sum = 0;
    for (int l = 0; l < nl - 1; ++l) {
        o->quota[l] = host_round_even(per);
        sum += o->quota[l];
        per *= f;
    }
    o->quota[nl - 1] = std::max(p.nfeatures - sum, 0);
    const int vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) o->umax[v] = (int)std::nearbyint(std::sqrt(225.0 - v * v));
    for (int v = 15, v0 = 0; v >= vmin; --v) {
        while (o->umax[v0] == o->umax[v0 + 1]) ++v0;
        o->umax[v] = v0;
        ++v0;
    }

    Geom &g = o->g;
    memset(&g, 0, sizeof(g));
    for (int v = 0; v < 16; ++v) g.umax_pk |= (unsigned long long)(o->umax[v] & 15) << (4 * v);
    g.nlevels = nl, g.W = o->W, g.H = o->H, g.ini_th = std::min(std::max(p.ini_th_fast, 0), 255);
    g.min_th = std::min(std::max(p.min_th_fast, 0), 255);
    long long pyr_off = 0, cand_off = 0;
    int out_off = 0, max_rw = 0, max_rh = 0, max_cells_lvl = 0, max_nodes = 0;
    int prev_w = o->W, prev_h = o->H;
    for (int l = 0; l < nl; ++l) {
        LevelGeom &L = g.lv[l];
        L.w = host_round_even((float)o->W * o->inv_scale[l]);
        L.h = host_round_even((float)o->H * o->inv_scale[l]);
        if (L.w > 4000 || L.h > 4000) return OMV_ERR_ARG;   // 12-bit packed coordinates
        L.pitch = (L.w + 15) & ~15;
        L.off = l == 0 ? 0 : pyr_off;
        if (l > 0) pyr_off += (long long)L.pitch * L.h;
        L.maxBX = L.w - kEdge + 3;
        L.maxBY = L.h - kEdge + 3;
        L.scale = o->scale[l];
        L.size = (float)(int)(31 * o->scale[l]);
        L.quota = o->quota[l];
        // FAST cells (:718-742)
        const float width = (float)(L.maxBX - kMinB), height = (float)(L.maxBY - kMinB);
        const int nCols = (int)(width / 35.f), nRows = (int)(height / 35.f);
        if (nCols < 1 || nRows < 1) return OMV_ERR_ARG;   // level too small: the reference divides by 0
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        L.cell_begin = (int)cells.size();
        long long cap_lvl = 0;
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(kMinB + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= L.maxBY - 3) continue;
            if (maxY > L.maxBY) maxY = (float)L.maxBY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(kMinB + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= L.maxBX - 6) continue;
                if (maxX > L.maxBX) maxX = (float)L.maxBX;
                Cell c{l, (int)iniY, (int)maxY, (int)iniX, (int)maxX};
                cells.push_back(c);
                max_rw = std::max(max_rw, c.x1 - c.x0);
                max_rh = std::max(max_rh, c.y1 - c.y0);
            }
        }
        L.cell_end = (int)cells.size();
        max_cells_lvl = std::max(max_cells_lvl, L.cell_end - L.cell_begin);
        // octree initial strips (:505-507)
        const int Wn = L.maxBX - kMinB, Hn = L.maxBY - kMinB;
        L.nIni = (int)std::round((float)Wn / Hn);
        if (L.nIni < 1) return OMV_ERR_ARG;   // the reference divides by zero here
        L.hX = (float)Wn / L.nIni;
        L.out_cap = std::max(L.quota + 2, 4 * L.nIni);
        L.out_off = out_off;
        out_off += L.out_cap;
        max_nodes = std::max(max_nodes, std::max(L.quota + 3, 4 * L.nIni + 4));
        (void)cap_lvl;
        // resize tables (cv::resize INTER_LINEAR, :1083)
        if (l > 0) {
            const int sw = prev_w, sh = prev_h, dw = L.w, dh = L.h;
            L.xtab_off = (int)xt.size();
            L.ytab_off = (int)yt.size();
            const double sx_scale = 1.0 / ((double)dw / sw), sy_scale = 1.0 / ((double)dh / sh);
            int xmax = dw;
            std::vector<XTab> row(dw);
            for (int dx = 0; dx < dw; ++dx) {
                float fx = (float)((dx + 0.5) * sx_scale - 0.5);
                int sx = (int)std::floor(fx);
                fx -= sx;
                if (sx < 0) fx = 0, sx = 0;
                if (sx + 1 >= sw) {
                    xmax = std::min(xmax, dx);
                    if (sx >= sw - 1) fx = 0, sx = sw - 1;
                }
                int a0 = (short)host_round_even((1.f - fx) * 2048.f), a1 = (short)host_round_even(fx * 2048.f);
                row[dx] = XTab{sx, std::min(sx + 1, sw - 1), (a0 & 0xffff) | (a1 << 16)};
            }
            for (int dx = xmax; dx < dw; ++dx) row[dx].coef = 2048, row[dx].sx1 = row[dx].sx0;
            xt.insert(xt.end(), row.begin(), row.end());
            // quad table: each pixel pair's two source bytes within two dwords of its first pixel's sx0
            L.xq_off = (int)xq.size();
            L.use_xq = 1;
            for (int q = 0; q < (dw + 3) / 4; ++q) {
                XQuad X{};
                for (int p = 0; p < 2; ++p) X.a[p] = (row[std::min(4 * q + 2 * p, dw - 1)].sx0) >> 2;
                for (int j = 0; j < 4; ++j) {
                    const int dx = 4 * q + j;
                    if (dx >= dw) {
                        X.sel[j] = 0x0c0c0c0cu, X.cf[j] = 0;
                        continue;
                    }
                    const int base = 4 * X.a[j >> 1], o0 = row[dx].sx0 - base, o1 = row[dx].sx1 - base;
                    const int a0 = (short)(row[dx].coef & 0xffff), a1 = (short)(row[dx].coef >> 16);
                    if (o0 < 0 || o0 > 7 || o1 < 0 || o1 > 7 || a0 < 0 || a1 < 0) L.use_xq = 0;
                    X.sel[j] = (uint32_t)(o0 & 7) | 0x0c00u | ((uint32_t)(o1 & 7) << 16) | 0x0c000000u;
                    X.cf[j] = (uint32_t)(a0 & 0xffff) | ((uint32_t)(a1 & 0xffff) << 16);
                }
                xq.push_back(X);
            }
            for (int dy = 0; dy < dh; ++dy) {
                float fy = (float)((dy + 0.5) * sy_scale - 0.5);
                int sy = (int)std::floor(fy);
                fy -= sy;
                int b0 = (short)host_round_even((1.f - fy) * 2048.f), b1 = (short)host_round_even(fy * 2048.f);
                const int r0 = std::min(std::max(sy, 0), sh - 1), r1 = std::min(std::max(sy + 1, 0), sh - 1);
                yt.push_back(XTab{r0, r1, (b0 & 0xffff) | (b1 << 16)});
            }
        }
        prev_w = L.w, prev_h = L.h;
        auto divm = [](int d) { return (uint32_t)((0x100000000ull + (uint64_t)d - 1) / (uint64_t)d); };
        L.m_quads = divm((L.w + 3) / 4), L.m_groups = divm((L.w + 15) / 16), L.m_w = divm(L.w);
    }
    g.n_cells = (int)cells.size();
    if (max_rw > 80 || max_rh > 80) return OMV_ERR_ARG;   // K2's index arithmetic (cells are ~35-45 px)
    const int dw = max_rw - 6, dh = max_rh - 6;
    g.cell_cap = ((dw + 1) / 2) * ((dh + 1) / 2);
    for (int l = 0; l < nl; ++l) {
        LevelGeom &L = g.lv[l];
        L.cand_off = cand_off;
        L.cand_cap = (L.cell_end - L.cell_begin) * g.cell_cap;
        cand_off += L.cand_cap;
    }
    g.pyr_bytes = (pyr_off + 255) & ~255LL;
    g.cand_per_img = cand_off;
    g.out_per_img = out_off;
    g.n_max = out_off;
    g.node_cap = (max_nodes + 15) & ~15;   // <= quota + 3 nodes exist at once (DistributeOctTree's stop rules)
    g.ccnt_cap = (std::max(4 * g.node_cap, max_cells_lvl) + 15) & ~15;
    // K2's row stride: an odd dword count (rows spread over the LDS banks) -- 13 dwords when every cell row plus its
    // misalignment fits, else 17, else per cell; OMV_FAST_RS=68 forces the wider stride (A/B)
    o->fast_rs = max_rw + 3 <= 52 ? 52 : max_rw + 3 <= 68 ? 68 : 0;
    if (const char *e = getenv("OMV_FAST_RS"))
        if (std::atoi(e) == 68 && max_rw + 3 <= 68) o->fast_rs = 68;
    o->rmax = ((o->fast_rs ? o->fast_rs * max_rh : ((max_rw + 6) & ~3) * max_rh) + 15) & ~15;   // rows: rw + misalignment
    // the strength map over rows / columns 2 .. n-3 (the NMS reach), then the candidate list (u16, worst case every
    // detection-window pixel): the LDS per wave sets K2's occupancy
    o->smax = ((std::max(0, (max_rw - 4) * (max_rh - 4))) + 15) & ~15;
    o->fast_lds = (size_t)o->rmax + o->smax + 2 * (size_t)std::max(0, (max_rw - 6) * (max_rh - 6));
    o->oct_lds = (size_t)(32 + 14 * g.node_cap + g.ccnt_cap + 6 * (g.node_cap / 17 + 1) + 2) * sizeof(int);
    return OMV_OK;
}

// K4's per-lane constant table.  disc[lane][2k], disc[lane][2k+1]: the row-sum and the weight (u + 15) byte masks of
// the lane's centroid item k (disc row vr = min(lane >> 1, 30), bytes 16 (lane & 1) + 4k .. +3 of cx-15 ..; zero
// outside the r = 15 disc, IC_Angle's umax rows, and for lanes 62, 63).
static std::vector<uint32_t> disc_table(const int umax[16]) {
    std::vector<uint32_t> t(64 * 8, 0u);
    for (int lane = 0; lane < 62; ++lane) {
        const int vr = std::min(lane >> 1, 30), h = lane & 1;
        const int um = umax[vr < 15 ? 15 - vr : vr - 15];
        for (int k = 0; k < 4; ++k) {
            const int kd = 4 * h + k;
            const int blo = std::min(std::max(15 - um - 4 * kd, 0), 4), bhi = std::min(std::max(15 + um - 4 * kd, -1), 3);
            const uint32_t keep = (blo >= 4 ? 0u : (0xffffffffu << (8 * blo))) & (bhi < 0 ? 0u : (0xffffffffu >> (8 * (3 - bhi))));
            t[8 * lane + 2 * k] = 0x01010101u & keep;
            t[8 * lane + 2 * k + 1] = (0x03020100u + 0x04040404u * (uint32_t)kd) & keep;
        }
    }
    return t;
}

extern "C" {

omv_status omv_orb_create(const omv_orb_params *params, int width, int height, int max_images, omv_orb **out) {
    if (!params || !out || width <= 0 || height <= 0 || max_images <= 0) return OMV_ERR_ARG;
    if (params->nlevels < 1 || params->nlevels > kMaxLevels || params->nfeatures <= 0) return OMV_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return OMV_ERR_NO_DEVICE;
    omv_orb *o = new omv_orb();
    o->p = *params;
    o->W = width, o->H = height, o->max_images = max_images;
    if (const char *pm = getenv("OMV_PYR_MODE")) o->pyr_mode = std::strcmp(pm, "chain") == 0 ? 1 : 0;
    (void)hipGetDevice(&o->device);
    std::vector<Cell> cells;
    std::vector<XTab> xt, yt;
    std::vector<XQuad> xq;
    omv_status st = build_geometry(o, cells, xt, yt, xq);
    if (st != OMV_OK) {
        delete o;
        return st;
    }
    if (o->oct_lds > 160 * 1024) {
        delete o;
        return OMV_ERR_ARG;
    }
    // 1080p levels hold ~1,500 cells: the octree's node lists then exceed the default 64 KB dynamic LDS
    if (o->oct_lds > 64 * 1024 &&
        (hipFuncSetAttribute((const void *)octree_kernel<OMV_OCT_WGS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)o->oct_lds) != hipSuccess ||
         hipFuncSetAttribute((const void *)octree_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)o->oct_lds) != hipSuccess)) {
        delete o;
        return OMV_ERR_HIP;
    }
    const Geom &g = o->g;
    const size_t n = (size_t)max_images;
    HIP_OK(hipMalloc(&o->d_cells, sizeof(Cell) * cells.size()));
    HIP_OK(hipMemcpy(o->d_cells, cells.data(), sizeof(Cell) * cells.size(), hipMemcpyHostToDevice));
    for (int l = 1; l < g.nlevels; ++l) {   // K1 LDS: the level's x table + the most source rows a row block reads
        const LevelGeom &L = g.lv[l];
        int nr = 0;
        for (int dy0 = 0; dy0 < L.h; dy0 += kPyrBlock) {
            const int dy1 = std::min(dy0 + kPyrBlock, L.h);
            nr = std::max(nr, yt[L.ytab_off + dy1 - 1].sx1 - yt[L.ytab_off + dy0].sx0 + 1);
        }
        o->pyr_lds[l] = sizeof(uint32_t) * (12 * (size_t)((L.w + 3) / 4) + (size_t)nr * (((g.lv[l - 1].w + 15) / 16) * 4) + 4 +
                                            3 * kPyrBlock);
        if (o->pyr_lds[l] > 160 * 1024) {   // images wider than ~8000 px
            delete o;
            return OMV_ERR_ARG;
        }
        if (o->pyr_lds[l] > 64 * 1024)
            (void)hipFuncSetAttribute((const void *)pyr_resize_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)o->pyr_lds[l]);
    }
    {   // K1 as one launch: the fewest bands per image whose largest level band (halo rows included) fits 32 KB of
        // LDS (two workgroups per CU), else 64 KB (wide images); no plan: the per-level launches
        const int L = g.nlevels;
        auto plan = [&](int nb, std::vector<PyrBand> &bands) {
            bands.assign((size_t)nb * kMaxLevels, PyrBand{0, 0, 0, 0});
            int worst = 0;
            for (int b = 0; b < nb; ++b) {
                PyrBand *B = &bands[(size_t)b * kMaxLevels];
                for (int l = 1; l < L; ++l)
                    B[l].own_lo = (int)((long long)b * g.lv[l].h / nb), B[l].own_hi = (int)((long long)(b + 1) * g.lv[l].h / nb);
                B[L - 1].need_lo = B[L - 1].own_lo, B[L - 1].need_hi = B[L - 1].own_hi;
                for (int l = L - 1; l >= 1; --l) {
                    int lo = INT_MAX, hi = INT_MIN;   // the source rows of level l's needed rows
                    if (B[l].need_hi > B[l].need_lo)
                        lo = yt[g.lv[l].ytab_off + B[l].need_lo].sx0, hi = yt[g.lv[l].ytab_off + B[l].need_hi - 1].sx1 + 1;
                    if (l - 1 >= 1 && B[l - 1].own_hi > B[l - 1].own_lo)
                        lo = std::min(lo, B[l - 1].own_lo), hi = std::max(hi, B[l - 1].own_hi);
                    if (hi > lo) B[l - 1].need_lo = std::max(0, lo), B[l - 1].need_hi = std::min(g.lv[l - 1].h, hi);
                }
                for (int l = 0; l < L; ++l)
                    worst = std::max(worst, (B[l].need_hi - B[l].need_lo) * (((g.lv[l].w + 15) / 16) * 4));
            }
            return worst;
        };
        std::vector<PyrBand> bands;
        for (int budget : {8192, 16384}) {
            for (int nb = 8; nb <= 128 && L > 1 && !o->pyr_nb; ++nb) {
                const int worst = plan(nb, bands);
                if (worst > budget) continue;
                int tab = 0, rows = 0;
                for (int l = 1; l < L; ++l) {
                    tab = std::max(tab, g.lv[l].use_xq ? 12 * ((g.lv[l].w + 3) / 4) : 3 * g.lv[l].w);
                    for (int b = 0; b < nb; ++b) {
                        const PyrBand &pb = bands[(size_t)b * kMaxLevels + l];
                        rows = std::max(rows, pb.need_hi - pb.need_lo);
                    }
                }
                o->pyr_nb = nb, o->pyr_buf_dw = worst, o->pyr_tab_dw = (tab + 3) & ~3, o->pyr_rows = rows;
                HIP_OK(hipMalloc(&o->d_bands, sizeof(PyrBand) * bands.size()));
                HIP_OK(hipMemcpy(o->d_bands, bands.data(), sizeof(PyrBand) * bands.size(), hipMemcpyHostToDevice));
                const int lds = (int)(sizeof(uint32_t) * (2 * (size_t)worst + 4 + o->pyr_tab_dw + 3 * (size_t)rows));
                if (lds > 160 * 1024) {   // no plan: the per-level launches
                    (void)hipFree(o->d_bands);
                    o->d_bands = nullptr, o->pyr_nb = 0;
                    break;
                }
                if (lds > 64 * 1024)
                    (void)hipFuncSetAttribute((const void *)pyr_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            }
        }
    }
    HIP_OK(hipMalloc(&o->d_xt, sizeof(XTab) * std::max<size_t>(1, xt.size())));
    HIP_OK(hipMalloc(&o->d_yt, sizeof(XTab) * std::max<size_t>(1, yt.size())));
    if (!xt.empty()) HIP_OK(hipMemcpy(o->d_xt, xt.data(), sizeof(XTab) * xt.size(), hipMemcpyHostToDevice));
    if (!yt.empty()) HIP_OK(hipMemcpy(o->d_yt, yt.data(), sizeof(XTab) * yt.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMalloc(&o->d_xq, sizeof(XQuad) * std::max<size_t>(1, xq.size())));
    if (!xq.empty()) HIP_OK(hipMemcpy(o->d_xq, xq.data(), sizeof(XQuad) * xq.size(), hipMemcpyHostToDevice));
    {
        const std::vector<uint32_t> dt = disc_table(o->umax);
        HIP_OK(hipMalloc(&o->d_disc, sizeof(uint32_t) * dt.size()));
        HIP_OK(hipMemcpy(o->d_disc, dt.data(), sizeof(uint32_t) * dt.size(), hipMemcpyHostToDevice));
    }
    HIP_OK(hipMalloc(&o->d_pyr, std::max<size_t>(256, (size_t)g.pyr_bytes * n)));
    HIP_OK(hipMalloc(&o->d_cell_cnt, sizeof(int) * g.n_cells * n));
    HIP_OK(hipMalloc(&o->d_cell_kp, sizeof(uint32_t) * (size_t)g.n_cells * g.cell_cap * n));
    HIP_OK(hipMalloc(&o->d_cand, sizeof(uint32_t) * (size_t)g.cand_per_img * n));
    HIP_OK(hipMalloc(&o->d_nid, sizeof(uint32_t) * (size_t)g.cand_per_img * n));
    HIP_OK(hipMalloc(&o->d_lvl_out, sizeof(uint32_t) * (size_t)g.out_per_img * n));
    HIP_OK(hipMalloc(&o->d_lvl_cls, sizeof(uint32_t) * (size_t)g.out_per_img * n));
    HIP_OK(hipMalloc(&o->d_lvl_cnt, sizeof(int) * 3 * g.nlevels * n));
    HIP_OK(hipMalloc(&o->d_lap, sizeof(int) * 2 * n));
    HIP_OK(hipMalloc(&o->d_err, sizeof(int)));
    HIP_OK(hipMemset(o->d_err, 0, sizeof(int)));
    *out = o;
    return OMV_OK;
}

omv_status omv_orb_destroy(omv_orb *o) {
    if (!o) return OMV_ERR_ARG;
    for (hipEvent_t e : o->ev) (void)hipEventDestroy(e);
    void *ptrs[] = {o->d_bands, o->d_cells, o->d_xt, o->d_yt, o->d_xq, o->d_disc, o->d_pyr, o->d_cell_cnt, o->d_cell_kp, o->d_cand, o->d_nid,
                    o->d_lvl_out, o->d_lvl_cls, o->d_lvl_cnt, o->d_lap, o->d_err, o->d_img1, o->d_kp1,
                    o->d_desc1, o->d_n1};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete o;
    return OMV_OK;
}

int omv_orb_max_keypoints(const omv_orb *o) { return o ? o->g.n_max : 0; }

omv_status omv_orb_scale_tables(const omv_orb *o, float *scale, float *inv_scale, float *sigma2, float *inv_sigma2) {
    if (!o) return OMV_ERR_ARG;
    for (int l = 0; l < o->p.nlevels; ++l) {
        if (scale) scale[l] = o->scale[l];
        if (inv_scale) inv_scale[l] = o->inv_scale[l];
        if (sigma2) sigma2[l] = o->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = o->inv_sigma2[l];
    }
    return OMV_OK;
}

omv_status omv_orb_extract_batch(omv_orb *o, int n, const uint8_t *images, size_t image_stride, size_t pitch,
                                 const int *lapping, omv_kp *kps, uint8_t *desc, int *n_out, int *mono_index,
                                 void *stream) {
    if (!o || n <= 0 || n > o->max_images || !images || !lapping || !kps || !desc || !n_out || !mono_index)
        return OMV_ERR_ARG;
    if (pitch < (size_t)o->W || image_stride < pitch * o->H) return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    o->last_stream = st;
    o->last_n = n;
    const Geom &g = o->g;
    // the lapping areas are constant per camera: a pageable host->device copy only when they change, so a
    // steady stream of batches enqueues kernels only (no host stall between launches)
    if (o->h_lap.size() < (size_t)2 * n || std::memcmp(o->h_lap.data(), lapping, sizeof(int) * 2 * n) != 0) {
        HIP_OK(hipMemcpyAsync(o->d_lap, lapping, sizeof(int) * 2 * n, hipMemcpyHostToDevice, st));
        o->h_lap.assign(lapping, lapping + 2 * n);
    }
    mark(o, st);
    // K1: pyramid, every level in one launch (level by level when no band plan fits LDS); test knob OMV_PYR_MODE =
    // "levels" / "chain" (read at omv_orb_create) picks the path
    const bool chain = o->pyr_mode >= 0 ? o->pyr_mode == 1 : n <= kPyrChainMaxImages;
    if (o->pyr_nb > 0 && chain) {
        const size_t lds = sizeof(uint32_t) * (2 * (size_t)o->pyr_buf_dw + 4 + o->pyr_tab_dw + 3 * (size_t)o->pyr_rows);
        pyr_chain_kernel<<<dim3(o->pyr_nb, n), 256, lds, st>>>(g, images, image_stride, pitch, o->d_pyr, o->d_xt, o->d_yt,
                                                               o->d_xq, o->d_bands, o->pyr_buf_dw, o->pyr_tab_dw);
    } else {
        for (int l = 1; l < g.nlevels; ++l) {
            pyr_resize_kernel<<<dim3((g.lv[l].h + kPyrBlock - 1) / kPyrBlock, n), 256, o->pyr_lds[l], st>>>(
                g, l, images, image_stride, pitch, o->d_pyr, o->d_xt, o->d_yt, o->d_xq, n);
        }
    }
    mark(o, st);
    // K2: FAST per cell
    if (o->fast_rs == 52)
        fast_cells_kernel<52><<<omv::xcd_grid(g.n_cells * n), 64, o->fast_lds, st>>>(
            g, o->d_cells, images, image_stride, pitch, o->d_pyr, o->d_cell_cnt, o->d_cell_kp, o->rmax, o->smax,
            g.n_cells * n);
    else if (o->fast_rs == 68)
        fast_cells_kernel<68><<<omv::xcd_grid(g.n_cells * n), 64, o->fast_lds, st>>>(
            g, o->d_cells, images, image_stride, pitch, o->d_pyr, o->d_cell_cnt, o->d_cell_kp, o->rmax, o->smax,
            g.n_cells * n);
    else
        fast_cells_kernel<0><<<omv::xcd_grid(g.n_cells * n), 64, o->fast_lds, st>>>(
            g, o->d_cells, images, image_stride, pitch, o->d_pyr, o->d_cell_cnt, o->d_cell_kp, o->rmax, o->smax,
            g.n_cells * n);
    mark(o, st);
    // K3: octree per (image, level)
    OctArgs oa{o->d_cell_cnt, o->d_cell_kp, o->d_cand, o->d_nid, o->d_lvl_out, o->d_lvl_cls, o->d_lvl_cnt, o->d_lap, o->d_err};
    if (n <= kOctSmallImages) octree_kernel<1><<<g.nlevels * n, 256, o->oct_lds, st>>>(g, oa);
    else octree_kernel<OMV_OCT_WGS><<<g.nlevels * n, 256, o->oct_lds, st>>>(g, oa);
    mark(o, st);
    // K4: orientation + blur at the samples + descriptors, one wave per output slot
    DescArgs da{images, image_stride, pitch, o->d_pyr, o->d_lvl_out, o->d_lvl_cls, o->d_lvl_cnt, kps, desc, n_out, mono_index, n,
                o->d_disc, o->harris};
    const int waves = g.out_per_img * n;
    describe_kernel<<<omv::xcd_grid((waves + 3) / 4), 256, 0, st>>>(g, da, (waves + 3) / 4);
    mark(o, st);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_orb_set_harris(omv_orb *o, float *harris) {
    if (!o) return OMV_ERR_ARG;
    o->harris = harris;
    return OMV_OK;
}

omv_status omv_orb_enable_timing(omv_orb *o, int on) {
    if (!o) return OMV_ERR_ARG;
    o->timing = on != 0;
    return OMV_OK;
}

omv_status omv_orb_stage_ms(omv_orb *o, double *ms4, long long *calls, int reset) {
    if (!o || !ms4) return OMV_ERR_ARG;
    HIP_OK(hipStreamSynchronize(o->last_stream));
    flush_timing(o);
    for (int k = 0; k < kOrbStages; ++k) ms4[k] = o->stage_ms[k];
    if (calls) *calls = o->stage_calls;
    if (reset) {
        for (int k = 0; k < kOrbStages; ++k) o->stage_ms[k] = 0;
        o->stage_calls = 0;
    }
    return OMV_OK;
}

omv_status omv_orb_last_error(omv_orb *o) {
    if (!o) return OMV_ERR_ARG;
    HIP_OK(hipStreamSynchronize(o->last_stream));
    int e = 0;
    HIP_OK(hipMemcpy(&e, o->d_err, sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(o->d_err, 0, sizeof(int)));
    return e;
}

omv_status omv_orb_extract_host(omv_orb *o, const uint8_t *image, size_t pitch, int lap0, int lap1, omv_kp *kps,
                                uint8_t *desc, int *n_out, int *mono_index) {
    if (!o || !image || !kps || !desc || !n_out || !mono_index) return OMV_ERR_ARG;
    const size_t dp = (size_t)o->W;
    if (!o->d_img1) {
        HIP_OK(hipMalloc(&o->d_img1, dp * o->H));
        HIP_OK(hipMalloc(&o->d_kp1, sizeof(omv_kp) * o->g.n_max));
        HIP_OK(hipMalloc(&o->d_desc1, 32 * (size_t)o->g.n_max));
        HIP_OK(hipMalloc(&o->d_n1, 2 * sizeof(int)));
    }
    HIP_OK(hipMemcpy2D(o->d_img1, dp, image, pitch, o->W, o->H, hipMemcpyHostToDevice));
    int lap[2] = {lap0, lap1};
    omv_status s = omv_orb_extract_batch(o, 1, o->d_img1, dp * o->H, dp, lap, o->d_kp1, o->d_desc1, o->d_n1,
                                         o->d_n1 + 1, nullptr);
    if (s != OMV_OK) return s;
    s = omv_orb_last_error(o);
    if (s != OMV_OK) return s;
    int hn[2];
    HIP_OK(hipMemcpy(hn, o->d_n1, sizeof(hn), hipMemcpyDeviceToHost));
    *n_out = hn[0];
    *mono_index = hn[1];
    HIP_OK(hipMemcpy(kps, o->d_kp1, sizeof(omv_kp) * hn[0], hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(desc, o->d_desc1, 32 * (size_t)hn[0], hipMemcpyDeviceToHost));
    return OMV_OK;
}

omv_status omv_orb_last_counts(omv_orb *o, long long *n_candidates, long long *n_keypoints) {
    if (!o || !n_candidates || !n_keypoints) return OMV_ERR_ARG;
    HIP_OK(hipStreamSynchronize(o->last_stream));
    const int n = o->last_n;
    std::vector<int> cc((size_t)n * o->g.n_cells), lc((size_t)n * o->g.nlevels * 3);
    if (n > 0) {
        HIP_OK(hipMemcpy(cc.data(), o->d_cell_cnt, sizeof(int) * cc.size(), hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(lc.data(), o->d_lvl_cnt, sizeof(int) * lc.size(), hipMemcpyDeviceToHost));
    }
    long long c = 0, k = 0;
    for (int v : cc) c += v > 0 ? v : 0;
    for (size_t i = 0; i < lc.size(); i += 3) k += lc[i];
    *n_candidates = c, *n_keypoints = k;
    return OMV_OK;
}

omv_status omv_orb_debug_level(omv_orb *o, int img, int level, uint8_t *out, int *w, int *h) {
    if (!o || level < 1 || level >= o->p.nlevels || img < 0 || img >= o->max_images) return OMV_ERR_ARG;
    const LevelGeom &L = o->g.lv[level];
    *w = L.w, *h = L.h;
    if (!out) return OMV_OK;
    HIP_OK(hipStreamSynchronize(o->last_stream));
    HIP_OK(hipMemcpy2D(out, L.w, o->d_pyr + (size_t)img * o->g.pyr_bytes + L.off, L.pitch, L.w, L.h,
                       hipMemcpyDeviceToHost));
    return OMV_OK;
}

omv_status omv_selftest_node_sort(const int *k1, const int *k2, int n, int *perm, void *stream) {
    if (n < 0 || n > 2048 || (n > 0 && (!k1 || !k2 || !perm))) return OMV_ERR_ARG;
    if (n == 0) return OMV_OK;
    const size_t lds = (size_t)n * (2 * sizeof(omv::SortItem) + 2 * sizeof(int)) + (6 * (n / 17 + 1) + 2) * sizeof(int);
    if (hipFuncSetAttribute((const void *)node_sort_selftest_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        return OMV_ERR_HIP;
    node_sort_selftest_kernel<<<1, 256, lds, (hipStream_t)stream>>>(k1, k2, n, perm);
    return hipGetLastError() == hipSuccess ? OMV_OK : OMV_ERR_HIP;
}

}  // extern "C"
