// MI355X-native Hamming matchers for the multi-camera frame.
//
//   grid_kernel      Frame::AssignFeaturesToGrid / PosInGrid (src/Frame.cc:541-582, :969-978):
//                    one wavefront per (frame, camera) builds a 64x48 CSR grid with a counting sort
//                    that keeps ascending keypoint order inside each cell (the reference push_backs
//                    in index order, and GetFeaturesInArea's output order depends on it).
//   cand_kernel      ORBmatcher::SearchByProjection (src/ORBmatcher.cc:23-340), speculative part:
//                    one thread per (frame, map point, camera block) walks the GetFeaturesInArea
//                    window (src/Frame.cc:890-967) and keeps the 4 best candidates by
//                    (Hamming distance, window order) — best/second-best are exactly the first two
//                    of that order, so claims made by earlier map points only need the next ones.
//   resolve_kernel   the order-dependent part: one wavefront per frame takes map points 64 at a
//                    time, each lane evaluates its point against the claims committed so far, and
//                    the wave commits the longest prefix of lanes whose best/second candidates were
//                    not claimed by an earlier lane of the same batch; the first conflicting lane is
//                    re-evaluated.  Results are identical to the reference's sequential loop
//                    (a keypoint taken by an earlier point with Observations() > 0 is skipped).
//   knn2_kernel      cv::BFMatcher(NORM_HAMMING).knnMatch(k=2) (src/Frame.cc:1483): train tiles in
//                    LDS, one query per lane, 4 x popcount64 per pair, first index wins ties.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../include/omv.h"
#include "omv_device.h"

namespace {

constexpr int kGridCols = 64, kGridRows = 48, kCells = kGridCols * kGridRows;
constexpr int kTH_HIGH = 100;
constexpr int kTop = 16;   // candidates kept per (point, camera): rescans only when >14 are claimed
constexpr int kMaxCams = 8;
constexpr size_t kResolveLds = 150 * 1024;   // dynamic LDS of the resolve workgroup (set as its maximum)

#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

struct FrameArgs {
    int n_cams, kp_cap, nlevels;
    float min_x, max_x, min_y, max_y, invW, invH;
    float scale[16];
    int model[8];             // camera type per block (omv_frame_geom::cam_model)
    const omv_kp *kps;        // [frame][cam][kp_cap]
    const uint8_t *desc;      // [frame][cam][kp_cap][32]
    const int *n_kp;          // [frame][cam]
    const int32_t *cell_start;   // [frame][cam][kCells + 1]
    const int32_t *cell_idx;     // [frame][cam][kp_cap]
};

// ---------------------------------------------------------------------------------------------
// One 256-thread workgroup per (frame, camera): per-cell counts by LDS atomics, a block scan of the 3,072
// counts, an unordered scatter by per-cell cursors, then each cell's (short) run sorted by keypoint index —
// the reference push_backs in index order, and GetFeaturesInArea's output order depends on it.
__global__ void __launch_bounds__(256) grid_kernel(FrameArgs f, int32_t *cell_start, int32_t *cell_idx) {
    __shared__ int cnt[kCells];
    __shared__ int cur[kCells];
    __shared__ int wsum[4];
    const int fc = blockIdx.x;   // frame * n_cams + cam
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = f.n_kp[fc];
    const omv_kp *kp = f.kps + (size_t)fc * f.kp_cap;
    for (int c = tid; c < kCells; c += 256) cnt[c] = 0;
    __syncthreads();
    auto cell_of = [&](int i) {
        const int px = (int)roundf((kp[i].x - f.min_x) * f.invW);
        const int py = (int)roundf((kp[i].y - f.min_y) * f.invH);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) return -1;
        return px * kGridRows + py;   // mGrid[ix][iy]
    };
    for (int i = tid; i < n; i += 256) {
        const int c = cell_of(i);
        if (c >= 0) atomicAdd(&cnt[c], 1);
    }
    __syncthreads();
    // exclusive scan of 3,072 counts: 12 per thread, wave scan, then the 4 wave totals
    constexpr int per = kCells / 256;
    int v[per], s = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) v[k] = cnt[tid * per + k], s += v[k];
    int incl = s;
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int run = incl - s;
    for (int q = 0; q < wv; ++q) run += wsum[q];
    int32_t *cs = cell_start + (size_t)fc * (kCells + 1);
#pragma unroll
    for (int k = 0; k < per; ++k) {
        const int c = tid * per + k;
        cs[c] = run;
        cnt[c] = run;   // start of the cell's run
        cur[c] = run;   // scatter cursor
        run += v[k];
    }
    if (tid == 255) cs[kCells] = run;
    __syncthreads();
    int32_t *out = cell_idx + (size_t)fc * f.kp_cap;
    for (int i = tid; i < n; i += 256) {
        const int c = cell_of(i);
        if (c >= 0) out[atomicAdd(&cur[c], 1)] = i;
    }
    __syncthreads();
    // ascending index order inside each cell (runs are a few entries long)
    for (int c = tid; c < kCells; c += 256) {
        const int b0 = cnt[c], e0 = cur[c];
        for (int p = b0 + 1; p < e0; ++p) {
            const int x = out[p];
            int q = p - 1;
            while (q >= b0 && out[q] > x) out[q + 1] = out[q], --q;
            out[q + 1] = x;
        }
    }
}

// ---------------------------------------------------------------------------------------------
struct MpArgs {
    const uint8_t *desc;
    const float *proj_x, *proj_y, *view_cos;
    const int32_t *level;
    const uint8_t *in_view;
    const float *track_depth;
    const uint8_t *is_bad, *has_obs;
    int M;
};

// Record entry: keypoint index (bits 0-15) | Hamming distance (bits 16-24) | octave (bits 25-29).
struct Rec {
    uint32_t e[kTop];
};
// SearchByProjection(F, MPs) records carry their own validity: bit 31 marks a filled entry (entries 0 .. n-1, n =
// min(count, kTop)), bit 30 of entry 0 that the window held more than kTop unblocked candidates (no count array).
constexpr uint32_t kRecValid = 1u << 31, kRecOver = 1u << 30;
template <class TopT>
__device__ __forceinline__ void store_record(Rec *dst, const TopT &t) {
    uint4 *o4 = reinterpret_cast<uint4 *>(dst);   // 64-B record as four 16-B stores
    uint32_t w[kTop];
#pragma unroll
    for (int q = 0; q < kTop; ++q) w[q] = q < t.n ? t.rec(q) | kRecValid : 0u;
    w[0] |= t.count > kTop ? kRecOver : 0u;
#pragma unroll
    for (int v = 0; v < kTop / 4; ++v) o4[v] = make_uint4(w[4 * v], w[4 * v + 1], w[4 * v + 2], w[4 * v + 3]);
}
__device__ __forceinline__ int rec_idx(uint32_t v) { return (int)(v & 0xffff); }
__device__ __forceinline__ int rec_dist(uint32_t v) { return (int)((v >> 16) & 0x1ff); }
__device__ __forceinline__ int rec_oct(uint32_t v) { return (int)((v >> 25) & 0x1f); }

// The kTop best candidates as sorted 64-bit keys dist << 40 | window order << 20 | octave << 16 | idx,
// kept in registers: insertion is a branch-free compare-and-shift over compile-time indices (no
// dynamically indexed arrays, hence no scratch).  Keys are unique (window order), so ties in
// distance keep window order exactly like the reference's strict `<` scans.
struct Top {
    uint64_t key[kTop];
    int n, count, seq;
    __device__ __forceinline__ void reset() {
#pragma unroll
        for (int q = 0; q < kTop; ++q) key[q] = ~0ull;
        n = count = seq = 0;
    }
    __device__ __forceinline__ void insert(int idx, int dist, int oct) { insert_at(idx, dist, oct, seq++); }
    // q: the candidate's position in the window's iteration order (< 2^20)
    __device__ __forceinline__ void insert_at(int idx, int dist, int oct, int q) {
        const uint64_t k = ((uint64_t)dist << 40) | ((uint64_t)q << 20) | ((uint64_t)oct << 16) | (uint64_t)idx;
#pragma unroll
        for (int q = kTop - 1; q > 0; --q) key[q] = k < key[q - 1] ? key[q - 1] : (k < key[q] ? k : key[q]);
        key[0] = k < key[0] ? k : key[0];
        n = min(n + 1, kTop);
    }
    __device__ __forceinline__ int idx(int q) const { return (int)(key[q] & 0xffff); }
    __device__ __forceinline__ int oct(int q) const { return (int)((key[q] >> 16) & 0xf); }
    __device__ __forceinline__ int dist(int q) const { return (int)(key[q] >> 40); }
    __device__ __forceinline__ uint32_t rec(int q) const {   // Rec entry: idx | dist << 16 | oct << 25
        return (uint32_t)idx(q) | ((uint32_t)dist(q) << 16) | ((uint32_t)oct(q) << 25);
    }
};

// The two smallest keys of Top's form (a lane's share of a wave-cooperative rescan, which needs best / second only).
struct Top2 {
    uint64_t key[2];
    int count;
    __device__ __forceinline__ void reset() { key[0] = key[1] = ~0ull, count = 0; }
    __device__ __forceinline__ void insert_at(int idx, int dist, int oct, int q) {
        const uint64_t k = ((uint64_t)dist << 40) | ((uint64_t)q << 20) | ((uint64_t)oct << 16) | (uint64_t)idx;
        key[1] = k < key[0] ? key[0] : (k < key[1] ? k : key[1]);
        key[0] = k < key[0] ? k : key[0];
    }
};
__device__ __forceinline__ uint32_t key_rec(uint64_t k) {   // Top key -> Rec entry idx | dist << 16 | oct << 25
    return (uint32_t)(k & 0xffff) | ((uint32_t)(k >> 40) << 16) | ((uint32_t)((k >> 16) & 0xf) << 25);
}

// The same list for one lane inserting in window order: 32-bit keys dist << 23 | oct << 16 | idx compared by
// distance alone (k | 0x7fffff < key <=> dist(k) < dist(key)), so a new key moves past strictly larger
// distances only and equal distances keep window order -- the strict `<` scans' tie rule, at half the
// compare / select work of the 64-bit keys.
struct TopSeq {
    uint32_t key[kTop];
    int n, count;
    __device__ __forceinline__ void reset() {
#pragma unroll
        for (int q = 0; q < kTop; ++q) key[q] = ~0u;
        n = count = 0;
    }
    __device__ __forceinline__ void insert(int idx, int dist, int oct) {
        const uint32_t k = ((uint32_t)dist << 23) | ((uint32_t)oct << 16) | (uint32_t)idx;
        const uint32_t kk = k | 0x7fffffu;
#pragma unroll
        for (int q = kTop - 1; q > 0; --q) key[q] = kk < key[q - 1] ? key[q - 1] : (kk < key[q] ? k : key[q]);
        key[0] = kk < key[0] ? k : key[0];
        n = min(n + 1, kTop);
    }
    __device__ __forceinline__ int idx(int q) const { return (int)(key[q] & 0xffff); }
    __device__ __forceinline__ int oct(int q) const { return (int)((key[q] >> 16) & 0x7f); }
    __device__ __forceinline__ int dist(int q) const { return (int)(key[q] >> 23); }
    __device__ __forceinline__ uint32_t rec(int q) const {   // Rec entry: idx | dist << 16 | oct << 25
        return (uint32_t)idx(q) | ((uint32_t)dist(q) << 16) | ((uint32_t)oct(q) << 25);
    }
};

__device__ __forceinline__ void load_desc(const uint8_t *p, uint64_t d[4]) {
    const uint64_t *q = reinterpret_cast<const uint64_t *>(p);
    d[0] = q[0], d[1] = q[1], d[2] = q[2], d[3] = q[3];
}

// Window of GetFeaturesInArea(x, y, r, level-1, level, cam), in the reference's iteration order;
// keeps the kTop best unblocked candidates by (dist, order).
template <class Blocked, class TopT>
__device__ void scan_window(const FrameArgs &f, int frame, int cam, float x, float y, float r, int minL, int maxL,
                            const uint64_t dmp[4], Blocked blocked, TopT &t) {
    t.reset();
    const int nMinCellX = max(0, (int)floorf((x - f.min_x - r) * f.invW));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - f.min_x + r) * f.invW));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - f.min_y - r) * f.invH));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - f.min_y + r) * f.invH));
    if (nMaxCellY < 0) return;
    const bool checkLevels = (minL > 0) || (maxL >= 0);
    const size_t fc = (size_t)frame * f.n_cams + cam;
    const int32_t *cs = f.cell_start + fc * (kCells + 1);
    const int32_t *ci = f.cell_idx + fc * f.kp_cap;
    const omv_kp *kp = f.kps + fc * f.kp_cap;
    const uint8_t *dd = f.desc + fc * f.kp_cap * 32;
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int c0 = ix * kGridRows + nMinCellY, c1 = ix * kGridRows + nMaxCellY;
        const int e = cs[c1 + 1];
        // cells iy = min..max of column ix are contiguous.  Latency-bound gathers, so one step's loads go
        // out together: the keypoint and its descriptor (speculatively) with the next index
        int p = cs[c0];
        int inext = p < e ? ci[p] : 0;
        for (; p < e; ++p) {
            const int i = inext;
            if (p + 1 < e) inext = ci[p + 1];
            const omv_kp k = kp[i];
            uint64_t d[4];
            load_desc(dd + (size_t)i * 32, d);
            if (checkLevels) {
                if (k.octave < minL) continue;
                if (maxL >= 0 && k.octave > maxL) continue;
            }
            if (!(fabsf(k.x - x) < r && fabsf(k.y - y) < r)) continue;
            if (blocked(cam * f.kp_cap + i)) continue;
            ++t.count;
            t.insert(i, omv::hamming256(dmp, d), k.octave);
        }
    }
}

// scan_window over G cooperating lanes (g = the lane's rank in its group): the window's candidates in the
// reference's iteration order (columns ix ascending, each column's cells iy ascending = one contiguous CSR run)
// are dealt round-robin, each lane keeps its own top kTop keyed by window position, then merge_top() selects the
// group's kTop smallest keys — the same list scan_window builds on one lane.  For small batches, where one
// lane's chain of dependent gathers through a large window is the kernel's critical path.
template <int G, class Blocked, class TopT>
__device__ void scan_window_coop(const FrameArgs &f, int frame, int cam, float x, float y, float r, int minL, int maxL,
                                 const uint64_t dmp[4], Blocked blocked, TopT &t, int g) {
    t.reset();
    const int nMinCellX = max(0, (int)floorf((x - f.min_x - r) * f.invW));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - f.min_x + r) * f.invW));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - f.min_y - r) * f.invH));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - f.min_y + r) * f.invH));
    if (nMaxCellY < 0) return;
    const bool checkLevels = (minL > 0) || (maxL >= 0);
    const size_t fc = (size_t)frame * f.n_cams + cam;
    const int32_t *cs = f.cell_start + fc * (kCells + 1);
    const int32_t *ci = f.cell_idx + fc * f.kp_cap;
    const omv_kp *kp = f.kps + fc * f.kp_cap;
    const uint8_t *dd = f.desc + fc * f.kp_cap * 32;
    int pos = g, acc = 0;   // this lane's next window position; window positions before the current column
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int b = cs[ix * kGridRows + nMinCellY], e = cs[ix * kGridRows + nMaxCellY + 1];
        for (; pos < acc + (e - b); pos += G) {
            const int i = ci[b + pos - acc];
            const omv_kp k = kp[i];
            uint64_t d[4];
            load_desc(dd + (size_t)i * 32, d);
            if (checkLevels) {
                if (k.octave < minL) continue;
                if (maxL >= 0 && k.octave > maxL) continue;
            }
            if (!(fabsf(k.x - x) < r && fabsf(k.y - y) < r)) continue;
            if (blocked(cam * f.kp_cap + i)) continue;
            ++t.count;
            t.insert_at(i, omv::hamming256(dmp, d), k.octave, pos);
        }
        acc += e - b;
    }
}

// The group's kTop smallest keys (unique: window positions differ) into every lane's t, counts summed.
template <int G>
__device__ __forceinline__ void merge_top(Top &t) {
    uint64_t out[kTop];
#pragma unroll
    for (int r = 0; r < kTop; ++r) {
        const uint64_t h = t.key[0];
        uint64_t mn = h;
#pragma unroll
        for (int s = 1; s < G; s <<= 1) {
            const uint64_t o = __shfl_xor(mn, s, 64);
            mn = o < mn ? o : mn;
        }
        out[r] = mn;
        const bool own = h == mn && h != ~0ull;
#pragma unroll
        for (int q = 0; q < kTop - 1; ++q) t.key[q] = own ? t.key[q + 1] : t.key[q];
        t.key[kTop - 1] = own ? ~0ull : t.key[kTop - 1];
    }
    int cnt = t.count;
#pragma unroll
    for (int s = 1; s < G; s <<= 1) cnt += __shfl_xor(cnt, s, 64);
    t.count = cnt;
    t.n = 0;
#pragma unroll
    for (int r = 0; r < kTop; ++r) {
        t.key[r] = out[r];
        t.n += out[r] != ~0ull;
    }
}

__device__ __forceinline__ bool mp_skipped(const MpArgs &m, int frame, int i, int C, int far_points, float th_far) {
    const size_t b = (size_t)frame * m.M + i;
    bool any = false;
    for (int c = 0; c < C; ++c) any = any || m.in_view[b * C + c];
    if (!any) return true;
    if (far_points && m.track_depth[b] > th_far) return true;
    return m.is_bad[b] != 0;
}

__device__ __forceinline__ float window_radius(const FrameArgs &f, const MpArgs &m, size_t bc, int c, float th,
                                               bool bFactor) {
    float r = m.view_cos[bc] > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos (:342-347)
    if (c == 0 && bFactor) r *= th;                   // th scales the left block only (:51-52)
    return r * f.scale[m.level[bc]];
}

// Candidates per (frame, map point, camera).
// Per-point flag word for the resolve stage: bits 0..C-1 in_view per camera, bit 16 skipped
// (mp_skipped), bit 17 has observations.
constexpr int kFlagSkip = 1 << 16, kFlagObs = 1 << 17;
constexpr int kFlagActive = 8;   // bits 8 .. 8+C-1: in view with a valid predicted level (the slots that have a record)
__device__ __forceinline__ int point_flags(const MpArgs &m, const FrameArgs &f, size_t fm, int frame, int i, int C,
                                           int far_points, float th_far) {
    int fl = 0;
    for (int q = 0; q < C; ++q) {
        const bool iv = m.in_view[fm * C + q];
        const int lv = m.level[fm * C + q];
        fl |= iv ? (1 << q) : 0;
        fl |= iv && lv >= 0 && lv < f.nlevels ? (1 << (kFlagActive + q)) : 0;
    }
    if (mp_skipped(m, frame, i, C, far_points, th_far)) fl |= kFlagSkip;
    if (m.has_obs[fm]) fl |= kFlagObs;
    return fl;
}

// Work compaction: a point is in view in ~1-2 of the C cameras, so a wave over consecutive (point, camera)
// slots would idle most lanes through the window scans.  Each wave takes kCandChunk consecutive slots,
// compacts the active ones (in view, valid predicted level; the others get no record) into an LDS queue
// (ballot prefix, slot order kept) and scans them 64 at a time.
constexpr int kCandChunk = 192;

// G: lanes per window (1 for large batches; 8 when the batch is a frame or two and the windows' gather chains,
// not the slot count, set the kernel's time).
template <int G>
__global__ void __launch_bounds__(256, 4) cand_kernel(FrameArgs f, MpArgs m, int n_frames, float th,
                                                   const uint8_t *occ_init, Rec *recs, int *counts, int *flags,
                                                   int far_points, float th_far, int n_blocks) {
    constexpr int kChunk = kCandChunk / G;   // slots per wave: G lanes per active slot keep ~one pass per wave
    __shared__ int queue[4][kChunk];
    const int C = f.n_cams;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long total = (long long)n_frames * m.M * C;
    const int blk = omv::xcd_block(n_blocks);   // consecutive slots (one frame's map points) on one XCD's L2
    if (blk < 0) return;
    const long long g0 = ((long long)blk * 4 + wave) * kChunk;
    const uint64_t lt = (1ull << lane) - 1ull;
    int nq = 0;
    for (int s0 = 0; s0 < kChunk; s0 += 64) {
        const long long gid = g0 + s0 + lane;
        bool act = false;
        if (s0 + lane < kChunk && gid < total) {
            const int c = (int)(gid % C);
            const long long fm = gid / C;
            const int frame = (int)(fm / m.M), i = (int)(fm % m.M);
            const size_t bc = (size_t)gid;
            if (c == 0) {
                flags[fm] = point_flags(m, f, (size_t)fm, frame, i, C, far_points, th_far);
            }
            const int lvl = m.level[bc];
            act = m.in_view[bc] && lvl >= 0 && lvl < f.nlevels;   // no record for the others: resolve never reads it
        }
        const uint64_t am = __ballot(act);
        if (act) queue[wave][nq + __popcll(am & lt)] = s0 + lane;
        nq += __popcll(am);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int g = lane % G;
    for (int q0 = 0; q0 < nq; q0 += 64 / G) {
        if (q0 + lane / G >= nq) break;   // whole groups leave together
        const long long gid = g0 + queue[wave][q0 + lane / G];
        const int c = (int)(gid % C);
        const long long fm = gid / C;
        const int frame = (int)(fm / m.M);
        const size_t bc = (size_t)gid;
        std::conditional_t<G == 1, TopSeq, Top> t;
        t.reset();
        uint64_t dmp[4];
        load_desc(m.desc + (size_t)fm * 32, dmp);
        const float r = window_radius(f, m, bc, c, th, th != 1.0f);
        const uint8_t *occ = occ_init ? occ_init + (size_t)frame * C * f.kp_cap : nullptr;
        if constexpr (G == 1) {
            scan_window(f, frame, c, m.proj_x[bc], m.proj_y[bc], r, m.level[bc] - 1, m.level[bc], dmp,
                        [&](int slot) { return occ && occ[slot]; }, t);
        } else {
            scan_window_coop<G>(f, frame, c, m.proj_x[bc], m.proj_y[bc], r, m.level[bc] - 1, m.level[bc], dmp,
                                [&](int slot) { return occ && occ[slot]; }, t, g);
            merge_top<G>(t);
        }
        if (g == 0) store_record(&recs[bc], t);
    }
}

// ---------------------------------------------------------------------------------------------
// The same candidates with the camera's keypoints staged in LDS.  One 512-thread workgroup per (frame, camera,
// chunk of 8 * pw map points): the camera's grid-ordered keypoints (CSR position p -> x, y, octave | index |
// blocked bit, 32-B descriptor) and its cell starts are copied into LDS once, then every in-view slot of the
// chunk walks its window there.  The global-memory version pays one dependent L2/HBM gather per window entry
// (cell index -> keypoint and descriptor) per (map point, camera); here a window step is two LDS reads, the
// descriptor only for entries that pass the level / radius / blocked tests, and the cell-index hop is gone
// (entries sit in CSR order).  Same window order and tie rule as scan_window, hence the same records.
constexpr int kStageThreads = 512;
constexpr uint32_t kStageBlocked = 1u << 31;
constexpr size_t kStageLdsMax = 80 * 1024;   // two workgroups per CU
constexpr int kScanGroup = 4;                 // window entries read per LDS round trip
constexpr int kStageUnroll = 3;               // staged entries per thread per pass (1,536 per pass)
constexpr int kStageMaxIt = 4;                // map points per wave <= 256
constexpr int kStageBuckets = 32;             // window-size classes: 2 x predicted level (nlevels <= 16)

__host__ __device__ inline size_t stage_lds_bytes(int kp_cap, int pw) {
    return (size_t)kp_cap * (32 + 8 + 4) + (size_t)(kCells + 1) * 4 + (size_t)(kStageThreads / 64) * pw * 4;
}

__device__ __forceinline__ void scan_window_lds(const FrameArgs &f, float x, float y, float r, int minL, int maxL,
                                                const uint64_t dmp[4], const int *scs, const float2 *sxy,
                                                const uint32_t *smeta, const uint4 *sdesc, TopSeq &t) {
    t.reset();
    const int nMinCellX = max(0, (int)floorf((x - f.min_x - r) * f.invW));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - f.min_x + r) * f.invW));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - f.min_y - r) * f.invH));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - f.min_y + r) * f.invH));
    if (nMaxCellY < 0) return;
    const bool checkLevels = (minL > 0) || (maxL >= 0);
    // a column's run in groups of kScanGroup entries: the group's position / meta reads go out together (one LDS
    // round trip per group instead of per entry; reads past the run stay inside the staged arrays and are masked)
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix) {
        const int e = scs[ix * kGridRows + nMaxCellY + 1];
        for (int p0 = scs[ix * kGridRows + nMinCellY]; p0 < e; p0 += kScanGroup) {
            float2 k[kScanGroup];
            uint32_t meta[kScanGroup];
#pragma unroll
            for (int u = 0; u < kScanGroup; ++u) k[u] = sxy[p0 + u], meta[u] = smeta[p0 + u];
#pragma unroll
            for (int u = 0; u < kScanGroup; ++u) {
                const int oct = (int)((meta[u] >> 16) & 0x7f);
                bool ok = p0 + u < e;
                if (checkLevels) ok = ok && oct >= minL && !(maxL >= 0 && oct > maxL);
                ok = ok && fabsf(k[u].x - x) < r && fabsf(k[u].y - y) < r && !(meta[u] & kStageBlocked);
                if (!ok) continue;
                const int p = p0 + u;
                const uint4 a = sdesc[2 * p], b = sdesc[2 * p + 1];
                const uint64_t d[4] = {(uint64_t)a.x | ((uint64_t)a.y << 32), (uint64_t)a.z | ((uint64_t)a.w << 32),
                                       (uint64_t)b.x | ((uint64_t)b.y << 32), (uint64_t)b.z | ((uint64_t)b.w << 32)};
                ++t.count;
                t.insert((int)(meta[u] & 0xffff), omv::hamming256(dmp, d), oct);
            }
        }
    }
}

// blockIdx -> (frame, cam, chunk) logical block, XCD-aware: a (frame, camera)'s chunks share one XCD's L2 for
// their staging reads.  pw: map points per wave.
__global__ void __launch_bounds__(kStageThreads) cand_stage_kernel(FrameArgs f, MpArgs m, int n_frames, float th,
                                                                   const uint8_t *occ_init, Rec *recs, int *counts,
                                                                   int *flags, int far_points, float th_far,
                                                                   int n_chunks, int pw, int n_blocks) {
    extern __shared__ __align__(16) unsigned char stage_lds[];
    const int C = f.n_cams, cap = f.kp_cap, M = m.M;
    const int blk = omv::xcd_block(n_blocks);
    if (blk < 0) return;
    const int chunk = blk % n_chunks, fc = blk / n_chunks, cam = fc % C, frame = fc / C;
    uint4 *sdesc = reinterpret_cast<uint4 *>(stage_lds);
    float2 *sxy = reinterpret_cast<float2 *>(stage_lds + (size_t)cap * 32);
    uint32_t *smeta = reinterpret_cast<uint32_t *>(stage_lds + (size_t)cap * 40);
    int *scs = reinterpret_cast<int *>(stage_lds + (size_t)cap * 44);
    int *queue = scs + kCells + 1;   // [8 * pw] the chunk's active points (workgroup-local index), sorted
    __shared__ int bucket[kStageBuckets + 1];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (tid <= kStageBuckets) bucket[tid] = 0;
    __syncthreads();
    // Latency chains overlapped: the cell starts and the first staging pass's cell indices are loaded, then the
    // chunk's map-point activity, then the keypoints / descriptors behind those cell indices.
    const int32_t *cs = f.cell_start + (size_t)fc * (kCells + 1);
    const int32_t *ci = f.cell_idx + (size_t)fc * cap;
    const omv_kp *kp = f.kps + (size_t)fc * cap;
    const uint4 *dd = reinterpret_cast<const uint4 *>(f.desc + (size_t)fc * cap * 32);
    const uint8_t *occ = occ_init ? occ_init + ((size_t)frame * C + cam) * cap : nullptr;
    const int n_in = cs[kCells];
    for (int c = tid; c <= kCells; c += kStageThreads) scs[c] = cs[c];
    int idx[kStageUnroll];
#pragma unroll
    for (int u = 0; u < kStageUnroll; ++u) {
        const int p = u * kStageThreads + tid;
        idx[u] = p < n_in ? ci[p] : -1;
    }
    // The chunk's map points: the in-view ones with a valid predicted level counting-sorted by window size
    // (predicted level, RadiusByViewingCos) into one workgroup queue, so that a wavefront's 64 lanes walk windows of
    // similar length (a wave takes the time of its longest window).
    const int p0 = chunk * (kStageThreads / 64) * pw;
    int key[kStageMaxIt], lv[kStageMaxIt];
    bool iv[kStageMaxIt];
    float vc[kStageMaxIt];
#pragma unroll
    for (int it = 0; it < kStageMaxIt; ++it) {
        const int i = p0 + wave * pw + it * 64 + lane;
        const bool valid = it * 64 + lane < pw && i < M;
        const size_t bc = ((size_t)frame * M + (valid ? i : 0)) * C + cam;
        iv[it] = valid && m.in_view[bc];
        lv[it] = valid ? m.level[bc] : -1;
        vc[it] = valid ? m.view_cos[bc] : 0.0f;
    }
#pragma unroll
    for (int it = 0; it < kStageMaxIt; ++it) {
        key[it] = -1;
        const int i = p0 + wave * pw + it * 64 + lane;
        if (it * 64 + lane >= pw || i >= M) continue;
        const size_t fm = (size_t)frame * M + i, bc = fm * C + cam;
        if (cam == 0) {
            flags[fm] = point_flags(m, f, fm, frame, i, C, far_points, th_far);
        }
        if (iv[it] && lv[it] >= 0 && lv[it] < f.nlevels) {   // only these have records (resolve's visit skips the
            key[it] = 2 * lv[it] + (vc[it] > 0.998 ? 0 : 1);   // others before it reads one)
            atomicAdd(&bucket[key[it]], 1);
        }
    }
    // stage the grid-ordered keypoints: kStageUnroll entries per thread per pass, all cell-index loads first, then all
    // keypoint / descriptor loads (two dependent global round trips per pass instead of two per entry)
    for (int s0 = 0; s0 < n_in; s0 += kStageThreads * kStageUnroll) {
        if (s0 > 0) {
#pragma unroll
            for (int u = 0; u < kStageUnroll; ++u) {
                const int p = s0 + u * kStageThreads + tid;
                idx[u] = p < n_in ? ci[p] : -1;
            }
        }
        float x[kStageUnroll], y[kStageUnroll];
        int oct[kStageUnroll];
        uint4 da[kStageUnroll], db[kStageUnroll];
        bool bl[kStageUnroll];
#pragma unroll
        for (int u = 0; u < kStageUnroll; ++u) {
            const int i = max(idx[u], 0);
            x[u] = kp[i].x, y[u] = kp[i].y, oct[u] = kp[i].octave;
            da[u] = dd[2 * i], db[u] = dd[2 * i + 1];
            bl[u] = occ && occ[i];
        }
#pragma unroll
        for (int u = 0; u < kStageUnroll; ++u) {
            const int p = s0 + u * kStageThreads + tid;
            if (idx[u] < 0) continue;
            sxy[p] = make_float2(x[u], y[u]);
            smeta[p] = (uint32_t)idx[u] | ((uint32_t)(oct[u] & 0x7f) << 16) | (bl[u] ? kStageBlocked : 0u);
            sdesc[2 * p] = da[u], sdesc[2 * p + 1] = db[u];
        }
    }
    __syncthreads();   // staging and bucket counts complete
    if (tid < 64) {    // exclusive scan of the 32 bucket counts
        const int c = tid < kStageBuckets ? bucket[tid] : 0;
        int incl = c;
        for (int d = 1; d < 32; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        if (tid < kStageBuckets) bucket[tid] = incl - c;
        if (tid == kStageBuckets - 1) bucket[kStageBuckets] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kStageMaxIt; ++it)
        if (key[it] >= 0) queue[atomicAdd(&bucket[key[it]], 1)] = wave * pw + it * 64 + lane;
    __syncthreads();
    const int nq = bucket[kStageBuckets];
    for (int q = wave * 64 + lane; q - lane < nq; q += kStageThreads) {
        if (q >= nq) break;
        const int i = p0 + queue[q];
        const size_t fm = (size_t)frame * M + i, bc = fm * C + cam;
        TopSeq t;
        uint64_t dmp[4];
        load_desc(m.desc + fm * 32, dmp);
        const float r = window_radius(f, m, bc, cam, th, th != 1.0f);
        scan_window_lds(f, m.proj_x[bc], m.proj_y[bc], r, m.level[bc] - 1, m.level[bc], dmp, scs, sxy, smeta, sdesc, t);
        store_record(&recs[bc], t);
    }
}

// ---------------------------------------------------------------------------------------------
// Claim resolution (the order-dependent part of SearchByProjection).
//
// Decomposition: the keypoint slots of camera blocks >= 2 are only ever touched by searches in their own block,
// blocks 0 and 1 are coupled by the stereo-partner writes (ORBmatcher.cc:125-131, :194-200).  So the claims form
// independent domains D0 = {block 0, block 1} and Dc-1 = {block c} for c >= 2.  A point visits its cameras in
// order and a failed ratio test ends its visit (the `continue` of :116 / :185 / ...), so domain w may evaluate a
// point only once the domains of its earlier cameras have decided whether it stopped there.  One wavefront per
// domain: each walks the points in view of its domain in map-point order, 64 at a time, with the prefix-commit
// rounds below; per-point stop cameras and per-domain progress counters in LDS order the domains (a domain
// waits until every earlier domain has finished the points of its current block; the order is acyclic, so the
// workgroup always drains).
//
// Rounds (per domain wave): every lane evaluates its point against the committed claims; lanes whose best /
// second candidate was claimed by an earlier lane of the same batch (or after a full rescan, or after an earlier
// lane without observations overwrote a blocked keypoint) end the committed prefix; the prefix commits in
// parallel (the highest lane writes a shared slot last) and the rest is re-evaluated.
constexpr int kMaxRevived = 64;   // initially-occupied keypoints freed during the call, per domain (rare)
constexpr int kMaxDomains = kMaxCams - 1;
constexpr int kListCap = 128;     // per-domain ring of member point indices (the next block is built ahead)

struct ResolveArgs {
    FrameArgs f;
    MpArgs m;
    const Rec *recs;
    const int *counts;   // candidates in the window not blocked when the record was built
    const int *flags;    // per point: in_view bits | active bits (kFlagActive) | kFlagSkip | kFlagObs
    const int32_t *l2r, *r2l;
    const uint8_t *occ_init;
    int32_t *kp_to_mp;
    int *n_matches;
    int *err;
    float th, th_far, nnratio;
    int far_points;
    int lds_k2m;         // the frame's assignment is kept in LDS (else updated in global memory)
};

// Each domain wave issues only wave-private LDS traffic on its own slots between its rounds; a wavefront-scope
// fence orders the wave's own LDS operations (no barrier: the other waves run their own rounds).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bool bit_of(const uint32_t *bits, int s) { return (bits[s >> 5] >> (s & 31)) & 1u; }

// Does keypoint slot `slot` (camera c) fall in the GetFeaturesInArea window of (x, y, r, lvl)?
__device__ bool in_window(const FrameArgs &f, int frame, int c, int slot, float x, float y, float r, int lvl) {
    const omv_kp k = f.kps[((size_t)frame * f.n_cams) * f.kp_cap + slot];
    const int px = (int)roundf((k.x - f.min_x) * f.invW), py = (int)roundf((k.y - f.min_y) * f.invH);
    if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) return false;   // not in the grid
    const int x0 = max(0, (int)floorf((x - f.min_x - r) * f.invW));
    const int x1 = min(kGridCols - 1, (int)ceilf((x - f.min_x + r) * f.invW));
    const int y0 = max(0, (int)floorf((y - f.min_y - r) * f.invH));
    const int y1 = min(kGridRows - 1, (int)ceilf((y - f.min_y + r) * f.invH));
    if (px < x0 || px > x1 || py < y0 || py > y1) return false;
    if (k.octave < lvl - 1 || k.octave > lvl) return false;
    return fabsf(k.x - x) < r && fabsf(k.y - y) < r;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));   // a register vector (uint4 copies go by memcpy)

// One (point, camera) record held in registers: the kTop candidates, the unblocked count, the predicted level.
// Only the first 4 of the 16 entries are prefetched: the best / second unblocked ones are nearly always among them;
// the rest are loaded from the record when a wave needs them.
struct RegRec {
    u32x4 e0;
};

// Best / second-best unblocked candidates of one (point, camera) record.  The reference walks the window and
// skips keypoints held by a point with observations (ORBmatcher.cc:77-79); the record holds the kTop best
// candidates in (distance, window order), so the walk takes the first two unblocked entries, 4 entries (their
// blocked bits fetched together) at a time.  The only own earlier write of the
// point that can fall into a later camera's block is camera 0's stereo-partner claim in block 1 (pa0,
// ORBmatcher.cc:125-131): it reads as blocked iff the point itself has observations.
struct Pick {
    int b1, b2, d1, d2, o1, o2;
    bool rescan;   // the 16 entries ran out with more candidates in the window
};

__device__ __forceinline__ Pick pick_record(const RegRec &r, const Rec *rp, int c, int cap, const uint32_t *bits, int pa0,
                                            bool obs) {
    // groups of 4 entries (their blocked bits fetched together), until every lane of the wave holds two unblocked
    // ones or has run out: nearly always the first group (claims are few against 16 candidates per window); groups
    // past the first come from the record in memory
    int k1 = -1, k2 = -1;
    uint32_t v1 = 0, v2 = 0, e_last = 0;   // e_last: the previous group's last entry (entries are filled in order)
#pragma unroll
    for (int g = 0; g < kTop / 4; ++g) {
        uint32_t e[4];
        if (g == 0) {
            e[0] = r.e0.x, e[1] = r.e0.y, e[2] = r.e0.z, e[3] = r.e0.w;
        } else {
            if (__all(k2 >= 0 || !(e_last & kRecValid))) break;
            const u32x4 q = reinterpret_cast<const u32x4 *>(rp)[g];
            e[0] = q.x, e[1] = q.y, e[2] = q.z, e[3] = q.w;
        }
        uint32_t w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int slot = c * cap + rec_idx(e[u]);
            w[u] = bits[slot >> 5];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = 4 * g + u;
            const int slot = c * cap + rec_idx(e[u]);
            bool b = (w[u] >> (slot & 31)) & 1u;
            if (slot == pa0) b = obs;
            const bool un = (e[u] & kRecValid) && !b;
            const bool t2 = un && k1 >= 0 && k2 < 0;
            v2 = t2 ? e[u] : v2;
            k2 = t2 ? k : k2;
            const bool t1 = un && k1 < 0;
            v1 = t1 ? e[u] : v1;
            k1 = t1 ? k : k1;
        }
        e_last = e[3];
    }
    Pick p;
    p.b1 = k1 >= 0 ? rec_idx(v1) : -1, p.d1 = k1 >= 0 ? rec_dist(v1) : 256, p.o1 = k1 >= 0 ? rec_oct(v1) : -1;
    p.b2 = k2 >= 0 ? rec_idx(v2) : -1, p.d2 = k2 >= 0 ? rec_dist(v2) : 256, p.o2 = k2 >= 0 ? rec_oct(v2) : -1;
    p.rescan = k2 < 0 && (r.e0.x & kRecOver);
    return p;
}

// Full GetFeaturesInArea rescan of one window against the current claims (freed initially-occupied keypoints, or more
// than kTop - 2 candidates claimed): rare, and done by the whole wavefront for one lane's window (uniform arguments,
// every lane active) -- the window's entries dealt over the 64 lanes, then the wave's two smallest (distance, window
// order) keys: the first two of the sequential scan's order.  A single lane's dependent gather chain through a large
// window was ~25 us.
__device__ __forceinline__ uint2 rescan_window_wave(const ResolveArgs &a, int frame, size_t fm, int c, int lvl,
                                                             const uint32_t *bits, int pa0, bool obs, int lane) {
    const FrameArgs &f = a.f;
    const MpArgs &m = a.m;
    const size_t bc = fm * f.n_cams + c;
    uint64_t dmp[4];
    load_desc(m.desc + fm * 32, dmp);
    const float x = m.proj_x[bc], y = m.proj_y[bc], r = window_radius(f, m, bc, c, a.th, a.th != 1.0f);
    const int minL = lvl - 1, maxL = lvl;
    Top2 t;
    t.reset();
    const int nMinCellX = max(0, (int)floorf((x - f.min_x - r) * f.invW));
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - f.min_x + r) * f.invW));
    const int nMinCellY = max(0, (int)floorf((y - f.min_y - r) * f.invH));
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - f.min_y + r) * f.invH));
    if (nMinCellX < kGridCols && nMaxCellX >= 0 && nMinCellY < kGridRows && nMaxCellY >= 0) {
        const bool checkLevels = (minL > 0) || (maxL >= 0);
        const size_t fc = (size_t)frame * f.n_cams + c;
        const int32_t *cs = f.cell_start + fc * (kCells + 1);
        const int32_t *ci = f.cell_idx + fc * f.kp_cap;
        const omv_kp *kp = f.kps + fc * f.kp_cap;
        const uint8_t *dd = f.desc + fc * f.kp_cap * 32;
        // lane j holds column nMinCellX + j's contiguous CSR run [b, b + len) (<= 64 columns) and its offset in the
        // window's iteration order; then the window's entries are dealt 64 per pass, one gather round per pass
        const int ncol = nMaxCellX - nMinCellX + 1;
        int cb = 0, len = 0;
        if (lane < ncol) {
            const int ix = nMinCellX + lane;
            cb = cs[ix * kGridRows + nMinCellY];
            len = cs[ix * kGridRows + nMaxCellY + 1] - cb;
        }
        int incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int u = __shfl_up(incl, d, 64);
            if (lane >= d) incl += u;
        }
        const int off = incl - len, total = __shfl(incl, 63, 64);
        for (int p0 = 0; p0 < total; p0 += 64) {
            const int pos = p0 + lane;
            int p = -1;
            for (int j = 0; j < ncol; ++j) {   // the column holding window position pos
                const int oj = __shfl(off, j, 64), lj = __shfl(len, j, 64), bj = __shfl(cb, j, 64);
                if (pos >= oj && pos < oj + lj) p = bj + pos - oj;
            }
            if (p < 0) continue;
            const int i = ci[p];
            const omv_kp k = kp[i];
            uint64_t d[4];
            load_desc(dd + (size_t)i * 32, d);
            if (checkLevels) {
                if (k.octave < minL) continue;
                if (maxL >= 0 && k.octave > maxL) continue;
            }
            if (!(fabsf(k.x - x) < r && fabsf(k.y - y) < r)) continue;
            const int slot = c * f.kp_cap + i;
            if (slot == pa0 ? obs : bit_of(bits, slot)) continue;
            t.insert_at(i, omv::hamming256(dmp, d), k.octave, pos);
        }
    }
    uint64_t mn[2];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const uint64_t h = t.key[0];
        uint64_t v = h;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint64_t o = __shfl_xor(v, s, 64);
            v = o < v ? o : v;
        }
        mn[rr] = v;
        const bool own = h == v && h != ~0ull;   // keys are unique (window positions)
        t.key[0] = own ? t.key[1] : t.key[0];
        t.key[1] = own ? ~0ull : t.key[1];
    }
    // packed as record entries, 0: none (bit 31 marks an entry)
    return make_uint2(mn[0] != ~0ull ? key_rec(mn[0]) | 0x80000000u : 0u, mn[1] != ~0ull ? key_rec(mn[1]) | 0x80000000u : 0u);
}

// A rescan's best / second entries (rescan_window_wave's packing) as a Pick.
__device__ __forceinline__ Pick unpack_pick(uint2 w) {
    Pick p;
    p.rescan = false;
    p.b1 = w.x ? rec_idx(w.x) : -1, p.d1 = w.x ? rec_dist(w.x) : 256, p.o1 = w.x ? rec_oct(w.x) : -1;
    p.b2 = w.y ? rec_idx(w.y) : -1, p.d2 = w.y ? rec_dist(w.y) : 256, p.o2 = w.y ? rec_oct(w.y) : -1;
    return p;
}

// Does a freed initially-occupied keypoint of this domain fall into this (point, camera) window?  (rare)
__device__ __forceinline__ bool revived_in_window(const ResolveArgs &a, int frame, size_t fm, int c, int lvl,
                                                  const int *revived, int nrevived, int self_rev) {
    const FrameArgs &f = a.f;
    const MpArgs &m = a.m;
    if (nrevived > kMaxRevived) return true;   // list overflowed: rescan every window (exact, slow)
    const int cap = f.kp_cap;
    const size_t bc = fm * f.n_cams + c;
    const float rad = window_radius(f, m, bc, c, a.th, a.th != 1.0f);
    for (int q = 0; q < nrevived; ++q) {
        const int s = revived[q];
        if (s / cap == c && in_window(f, frame, c, s, m.proj_x[bc], m.proj_y[bc], rad, lvl)) return true;
    }
    return c == 1 && self_rev >= 0 && in_window(f, frame, c, self_rev, m.proj_x[bc], m.proj_y[bc], rad, lvl);
}

// One point's visit of the NC cameras c0 .. c0+NC-1 of a domain (ORBmatcher.cc:45-330 for one pMP), against the
// committed claims.  NC = 2 for D0 (blocks 0 and 1, stereo partners), 1 for the side domains.  Claims and the
// slots that decided the result stay in registers (compile-time indices).
template <int NC>
struct Visit {
    int claim[2 * NC];   // slots written (mvpMapPoints = pMP), -1 none
    int rel[2 * NC];     // best / second slots per camera, -1 none
    int nmatch;
    int stop;            // camera whose ratio test failed (the visit ended there), 255 none
    bool fallback;       // needed a full window rescan
    bool unblock;        // overwrote a blocked slot while having no observations
    int pending;         // camera (index in the domain) whose window needs a rescan first: the visit stopped there, -1 none
    int pend_pa0;        // the stereo-partner slot that rescan treats specially (ORBmatcher.cc:125-131)
};

template <int NC>
__device__ __forceinline__ void visit(const ResolveArgs &a, int frame, int i, int c0, int fl, const RegRec (&rr)[NC],
                                      const uint32_t *bits, const uint32_t *occ0, const int *revived, int nrevived,
                                      const int32_t *l2r, const int32_t *r2l, const uint2 (&forced)[NC], int fmask,
                                      Visit<NC> &v) {
    const FrameArgs &f = a.f;
    const int C = f.n_cams, cap = f.kp_cap;
#pragma unroll
    for (int q = 0; q < 2 * NC; ++q) v.claim[q] = v.rel[q] = -1;
    v.nmatch = 0, v.stop = 255, v.fallback = v.unblock = false, v.pending = -1, v.pend_pa0 = -1;
    const size_t fm = (size_t)frame * a.m.M + i;
    const bool obs = (fl & kFlagObs) != 0;
    auto claim = [&](int q, int slot) {
        if (!obs && bit_of(bits, slot)) v.unblock = true;   // overwrites a keypoint later points saw blocked
        v.claim[q] = slot;
    };
    // the left block's stereo partner claim (ORBmatcher.cc:125-131) by a point without observations frees an
    // initially-occupied right keypoint for this point's own right-block search (:150-160); the right-block
    // record was built without it (occupied at the call), so that window is rescanned
    int self_rev = -1, pa0 = -1;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const int c = c0 + k;
        // in view with a valid predicted level (c > 0: nPredictedLevel == -1 skips, :142) -- the slots with a record
        if (!((fl >> (kFlagActive + c)) & 1)) continue;
        bool need_rescan = (nrevived > 0 || (c == 1 && self_rev >= 0)) &&
                           revived_in_window(a, frame, fm, c, a.m.level[fm * C + c], revived, nrevived, self_rev);
        const bool forced_k = (fmask >> k) & 1;   // the wave rescanned this window for this visit (same claims)
        if (!(rr[k].e0.x & kRecValid) && !need_rescan && !forced_k) continue;   // vIndices empty or all initially blocked
        Pick p;
        if (forced_k) {
            p = unpack_pick(forced[k]);
            v.fallback = true;
        } else {
            if (!need_rescan) {
                p = pick_record(rr[k], a.recs + fm * C + c, c, cap, bits, c == 1 ? pa0 : -1, obs);
                need_rescan = p.rescan;
            }
            if (need_rescan) {   // the wave rescans the window, then this visit runs again
                v.pending = k, v.pend_pa0 = c == 1 ? pa0 : -1;
                return;
            }
        }
        v.rel[2 * k] = p.b1 >= 0 ? c * cap + p.b1 : -1;
        v.rel[2 * k + 1] = p.b2 >= 0 ? c * cap + p.b2 : -1;
        if (p.d1 <= kTH_HIGH) {
            if (p.o1 == p.o2 && (float)p.d1 > a.nnratio * p.d2) {   // `continue` to the next map point
                v.stop = c;
                return;
            }
            if (c == 0) {
                claim(0, p.b1);
                if (C > 1 && l2r[p.b1] != -1) {
                    const int ps = cap + l2r[p.b1];
                    if (!obs && bit_of(occ0, ps) && bit_of(bits, ps)) self_rev = ps;
                    claim(1, ps), v.nmatch++;
                    pa0 = ps;
                }
                v.nmatch++;
            } else if (c == 1) {
                if (r2l[p.b1] != -1) claim(2 * k, r2l[p.b1]), v.nmatch++;
                claim(2 * k + 1, cap + p.b1);
                v.nmatch++;
            } else {
                claim(2 * k, c * cap + p.b1);
                v.nmatch++;
            }
        }
    }
}

// Shared LDS state of one frame's resolve (all domains).
struct ResolveShared {
    uint32_t *bits;    // blocked: mvpMapPoints[s] has observations (atomics: a word may hold two domains' slots)
    uint32_t *occ0;    // initially occupied (not in the records)
    int *owner;        // per slot: phase-stamped claim word (see run_domain)
    int32_t *l2r, *r2l;
    int32_t *k2m;      // this frame's mvpMapPoints (LDS or global)
    uint8_t *stop;     // per point: the camera whose ratio test ended its visit (255 none)
    int *prog;         // per domain: points below this index are final in that domain
    int *list;         // per domain ring of member point indices [kMaxDomains][kListCap]
    int *listfl;       // their flag words (same ring positions)
    int *revived;      // per domain [kMaxDomains][kMaxRevived]
    int *nrevived;     // per domain
    int *total;
};

// The rounds of one domain (wave w) over its member points.
template <int NC>
__device__ __forceinline__ void run_domain(const ResolveArgs &a, const ResolveShared &sh, int frame, int w, int c0,
                                           int lane) {
    const int C = a.f.n_cams, M = a.m.M;
    const uint64_t lt = (1ull << lane) - 1ull;
    int *list = sh.list + w * kListCap, *listfl = sh.listfl + w * kListCap;
    int *revived = sh.revived + w * kMaxRevived;
    const int *flags_f = a.flags + (size_t)frame * M;
    const size_t rec_base = (size_t)frame * M;
    const uint32_t dom_mask = ((1u << NC) - 1u) << c0;
    // member list: points [0, fscan) scanned; ring entries [head, tail)
    int fscan = 0, head = 0, tail = 0;
    // flags of the next 4 chunks of 64 points, prefetched
    int fr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) fr[q] = q * 64 + lane < M ? flags_f[q * 64 + lane] : kFlagSkip;
    // append members until the ring holds a full block past `from` (or the points run out)
    auto fill = [&](int from) {
        while (tail - from < 64 && fscan < M) {
            const int fl = fr[0];
            fr[0] = fr[1], fr[1] = fr[2], fr[2] = fr[3];
            const int nxt = fscan + 4 * 64 + lane;
            fr[3] = nxt < M ? flags_f[nxt] : kFlagSkip;
            const bool mem = fscan + lane < M && !(fl & kFlagSkip) && (fl & dom_mask);
            const uint64_t bm = __ballot(mem);
            if (mem) {
                const int pos = (tail + __popcll(bm & lt)) & (kListCap - 1);
                list[pos] = fscan + lane, listfl[pos] = fl;
            }
            tail += __popcll(bm);
            fscan += 64;
        }
        wave_sync();
    };
    // register prefetch of a block's records (lane l: member point l of the block)
    RegRec cur[NC], nxt[NC];
    int cur_flag = 0, nxt_flag = 0;
    auto load_block = [&](int h, RegRec (&rr)[NC], int &flag) {
        const int nb = min(64, tail - h);
        const int pos = (h + min(lane, max(nb - 1, 0))) & (kListCap - 1);
        const int pt = list[pos];
        flag = listfl[pos];
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            const size_t bc = (rec_base + pt) * C + c0 + k;
            rr[k].e0 = *reinterpret_cast<const u32x4 *>(a.recs + bc);
        }
    };
    fill(0);
    if (tail > head) load_block(head, nxt, nxt_flag);
    int total = 0;
    int phase = 0x3fffff;   // owner stamp of the current conflict phase (commit phase = phase - 1)
#ifdef OMV_RESOLVE_PROFILE
    long long tp[5] = {0, 0, 0, 0, 0}, tl = wall_clock64();
    int nblocks = 0, nrounds = 0, nfall = 0;
    long long tp4 = 0;   // visit ticks of each block's first round
#define OMV_TP(k) (tp[k] += wall_clock64() - tl, tl = wall_clock64())
#else
#define OMV_TP(k) ((void)0)
#endif
    while (tail > head) {
        const int nb = min(64, tail - head);
        const int pt = list[(head + min(lane, nb - 1)) & (kListCap - 1)];
        const int pmax = list[(head + nb - 1) & (kListCap - 1)];
#pragma unroll
        for (int k = 0; k < NC; ++k) cur[k] = nxt[k];
        cur_flag = nxt_flag;
        // build and prefetch the next block while this one resolves
        const int head2 = head + nb;
        fill(head2);
        if (tail > head2) load_block(head2, nxt, nxt_flag);
        // the earlier domains must have decided every point of this block
        for (int q = 0; q < w; ++q)
            while (__hip_atomic_load(&sh.prog[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= pmax)
                __builtin_amdgcn_s_sleep(1);
        OMV_TP(0);
        const bool alive = lane < nb && (w == 0 || sh.stop[pt] > c0);
        int start = 0;
        while (start < nb) {
            const bool active = alive && lane >= start;
            Visit<NC> v;
            const int nrev = min(sh.nrevived[w], kMaxRevived + 1);
            OMV_TP(1);
            uint2 forced[NC];
            int fmask = 0;
            if (active) {
                visit<NC>(a, frame, pt, c0, cur_flag, cur, sh.bits, sh.occ0, revived, nrev, sh.l2r, sh.r2l, forced, fmask, v);
            } else {
#pragma unroll
                for (int q = 0; q < 2 * NC; ++q) v.claim[q] = v.rel[q] = -1;
                v.nmatch = 0, v.stop = 255, v.fallback = v.unblock = false, v.pending = -1;
            }
            // windows that ran out of candidates: rescanned one at a time by the whole wave, then those lanes' visits
            // run again with the result (at most NC times: a camera is rescanned once per visit)
            uint64_t pm = __ballot(active && v.pending >= 0);
            if (__builtin_expect(pm != 0, 0)) {
                do {
                    while (pm) {
                        const int L = __ffsll((long long)pm) - 1;
                        pm &= pm - 1;
                        const int k = __shfl(v.pending, L, 64), pa0L = __shfl(v.pend_pa0, L, 64), ptL = __shfl(pt, L, 64);
                        const bool obsL = (__shfl(cur_flag, L, 64) & kFlagObs) != 0;
                        const size_t fmL = (size_t)frame * M + ptL;
                        const int c = c0 + k;
                        const uint2 p = rescan_window_wave(a, frame, fmL, c, a.m.level[fmL * C + c], sh.bits, pa0L, obsL,
                                                           lane);
                        if (lane == L) {
                            if (k == 0) forced[0] = p;
                            else forced[NC - 1] = p;
                            fmask |= 1 << k;
                        }
                    }
                    if (active && v.pending >= 0)
                        visit<NC>(a, frame, pt, c0, cur_flag, cur, sh.bits, sh.occ0, revived, nrev, sh.l2r, sh.r2l, forced,
                                  fmask, v);
                    pm = __ballot(active && v.pending >= 0);
                } while (pm);
            }
#ifdef OMV_RESOLVE_PROFILE
            if (start == 0) tp4 += wall_clock64() - tl;
#endif
            OMV_TP(2);
            const bool obs = active && (cur_flag & kFlagObs);
            const int keyA = (phase << 7) | lane, keyB = ((phase - 1) << 7) | (63 - lane);
            if (obs) {
#pragma unroll
                for (int q = 0; q < 2 * NC; ++q)
                    if (v.claim[q] >= 0) atomicMin(&sh.owner[v.claim[q]], keyA);
            }
            wave_sync();
            bool conflict = false;
            if (active && lane > start) {
                conflict = v.fallback;   // a full rescan saw the whole window: only safe at the batch head
#pragma unroll
                for (int q = 0; q < 2 * NC; ++q)
                    if (v.rel[q] >= 0) {
                        const int o = sh.owner[v.rel[q]];
                        conflict = conflict || ((o >> 7) == phase && (o & 127) < lane);
                    }
            }
            uint64_t cm = __ballot(conflict);
            const uint64_t um = __ballot(active && v.unblock);
            if (um) {
                // a point without observations overwrote a blocked keypoint: later lanes saw it blocked
                const int u = __ffsll((long long)um) - 1;
                cm |= (u >= 63) ? 0ull : (~0ull << (u + 1));
            }
            const int j0 = cm ? min(nb, __ffsll((long long)cm) - 1) : nb;
            // commit lanes [start, j0): the highest committing lane writes a shared slot last
            const bool committed = active && lane < j0;
            if (committed) {
#pragma unroll
                for (int q = 0; q < 2 * NC; ++q)
                    if (v.claim[q] >= 0) atomicMin(&sh.owner[v.claim[q]], keyB);
            }
            wave_sync();
            if (committed) {
#pragma unroll
                for (int q = 0; q < 2 * NC; ++q) {
                    const int s = v.claim[q];
                    if (s < 0 || sh.owner[s] != keyB) continue;
                    sh.k2m[s] = pt;
                    if (obs) {
                        atomicOr(&sh.bits[s >> 5], 1u << (s & 31));
                    } else {
                        if (bit_of(sh.occ0, s) && bit_of(sh.bits, s)) {   // an initially occupied keypoint is freed
                            const int r = atomicAdd(&sh.nrevived[w], 1);
                            if (r < kMaxRevived) revived[r] = s;
                        }
                        atomicAnd(&sh.bits[s >> 5], ~(1u << (s & 31)));
                    }
                }
                if (v.stop != 255) sh.stop[pt] = (uint8_t)v.stop;
                total += v.nmatch;
            }
            phase -= 2;
            start = j0;
            wave_sync();
            OMV_TP(3);
#ifdef OMV_RESOLVE_PROFILE
            ++nrounds;
            nfall += __popcll(__ballot(active && v.fallback));
#endif
        }
#ifdef OMV_RESOLVE_PROFILE
        ++nblocks;
#endif
        head = head2;
        // every point below the next block's first member is final in this domain
        if (lane == 0)
            __hip_atomic_store(&sh.prog[w], tail > head ? list[head & (kListCap - 1)] : M, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (lane == 0) __hip_atomic_store(&sh.prog[w], M, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef OMV_RESOLVE_PROFILE
    if (lane == 0 && frame < 2)
        printf("resolve frame %d domain %d blocks %d rounds %d revived %d rescans %d ticks(100MHz): block-start+deps %lld rounds-pre %lld visit %lld commit %lld\n",
               frame, w, nblocks, nrounds, sh.nrevived[w], nfall, tp[0], tp[1], tp[2], tp[3]);
    if (lane == 0 && frame < 2) printf("resolve frame %d domain %d first-round visit ticks %lld\n", frame, w, tp4);
#endif
#undef OMV_TP
    for (int d = 32; d >= 1; d >>= 1) total += __shfl_xor(total, d, 64);
    if (lane == 0) atomicAdd(sh.total, total);
}

// One workgroup per frame, one wavefront per claim domain (1 + max(0, n_cams - 2) waves).
template <bool kLdsK2m>
__global__ void __launch_bounds__(64 * kMaxDomains) resolve_kernel(ResolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rsm[];
    __shared__ int list[kMaxDomains * kListCap], listfl[kMaxDomains * kListCap];
    __shared__ int revived[kMaxDomains * kMaxRevived];
    __shared__ int nrevived[kMaxDomains], prog[kMaxDomains], total;
    const int frame = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const int C = a.f.n_cams, cap = a.f.kp_cap, S = C * cap, M = a.m.M;
    const int nwords = (S + 31) >> 5;
    ResolveShared sh;
    sh.bits = rsm;
    sh.occ0 = rsm + nwords;
    sh.owner = reinterpret_cast<int *>(rsm + 2 * nwords);
    sh.l2r = sh.owner + S;
    sh.r2l = sh.l2r + cap;
    int32_t *const k2m_g = a.kp_to_mp + (size_t)frame * S;
    sh.k2m = kLdsK2m ? sh.r2l + cap : k2m_g;
    sh.stop = reinterpret_cast<uint8_t *>(sh.r2l + cap + (kLdsK2m ? S : 0));
    sh.prog = prog, sh.list = list, sh.listfl = listfl, sh.revived = revived, sh.nrevived = nrevived, sh.total = &total;
    const uint8_t *occ = a.occ_init ? a.occ_init + (size_t)frame * S : nullptr;
    for (int w = tid; w < nwords; w += nt) {
        uint32_t v = 0;
        if (occ) {
            uint8_t o[32];   // all 32 byte loads in flight together
#pragma unroll
            for (int b = 0; b < 32; ++b) o[b] = occ[min(w * 32 + b, S - 1)];
#pragma unroll
            for (int b = 0; b < 32; ++b) v |= (w * 32 + b < S && o[b]) ? 1u << b : 0u;
        }
        sh.bits[w] = v;
        sh.occ0[w] = v;
    }
    for (int s = tid; s < S; s += nt) sh.owner[s] = INT_MAX;
    if (kLdsK2m)
        for (int s = tid; s < S; s += nt) sh.k2m[s] = k2m_g[s];
    for (int s = tid; s < cap; s += nt) {
        sh.l2r[s] = a.l2r[(size_t)frame * cap + s];
        sh.r2l[s] = a.r2l[(size_t)frame * cap + s];
    }
    for (int p = tid; p < M; p += nt) sh.stop[p] = 255;
    if (tid < kMaxDomains) nrevived[tid] = 0, prog[tid] = 0;
    if (tid == 0) total = 0;
    __syncthreads();
    const int w = tid >> 6, lane = tid & 63;
    if (w == 0) {
        if (C >= 2) run_domain<2>(a, sh, frame, 0, 0, lane);
        else run_domain<1>(a, sh, frame, 0, 0, lane);
    } else {
        run_domain<1>(a, sh, frame, w, w + 1, lane);
    }
    __syncthreads();
    if (kLdsK2m)
        for (int s = tid; s < S; s += nt) k2m_g[s] = sh.k2m[s];
    if (tid == 0) a.n_matches[frame] = total;
}

// ---------------------------------------------------------------------------------------------
// knnMatch(k=2): block = 256 queries of one (query set, train set) pair.
struct KnnArgs {
    const uint8_t *q, *t;
    long long q_stride, t_stride;   // bytes between pairs
    const int *nq, *nt;             // per pair
    const int *q_off, *t_off;       // per pair row offset (may be null)
    int pair_stride_off;            // stride of q_off/t_off arrays
    int32_t *idx2, *dist2;          // [pair][out_cap][2]
    int out_cap;
};

// G lanes per query: lane g of a query's group scores train rows g, g+G, ... of every LDS tile (its own top-2 by
// (distance, index), strict updates in index order), then the group merges its G top-2 lists with shuffles.  The
// result is the two smallest (distance, index) pairs — exactly knnMatch's "first index wins ties".  G > 1 cuts
// the per-query chain and multiplies the waves (see launch_knn2).
template <int G>
__global__ void __launch_bounds__(256) knn2_kernel(KnnArgs a, int n_pairs) {
    __shared__ __attribute__((aligned(16))) uint64_t tile[256][4];
    constexpr int QB = 256 / G;   // queries per block
    const int pair = blockIdx.y;
    const int qo = a.q_off ? a.q_off[pair * a.pair_stride_off] : 0;
    const int to = a.t_off ? a.t_off[pair * a.pair_stride_off] : 0;
    const int nq = a.nq[pair * a.pair_stride_off] - qo;
    const int nt = a.nt[pair * a.pair_stride_off] - to;
    const int g = threadIdx.x % G;
    const int qi = blockIdx.x * QB + threadIdx.x / G;
    if (blockIdx.x * QB >= max(nq, 0)) return;   // block-uniform
    uint64_t dq[4] = {0, 0, 0, 0};
    if (qi < nq) load_desc(a.q + pair * a.q_stride + (size_t)(qo + qi) * 32, dq);
    // keys (distance << 32 | index): "none" = (INT_MAX, -1) sorts last
    uint64_t k0 = ~0ull >> 1, k1 = ~0ull >> 1;
    int d0 = INT_MAX, d1 = INT_MAX, i0 = -1, i1 = -1;
    for (int b = 0; b < nt; b += 256) {
        __syncthreads();
        const int j = b + threadIdx.x;
        if (j < nt) load_desc(a.t + pair * a.t_stride + (size_t)(to + j) * 32, tile[threadIdx.x]);
        __syncthreads();
        const int e = min(256, nt - b);
        for (int k = g; k < e; k += G) {
            const int d = omv::hamming256(dq, tile[k]);
            if (d < d1) {
                if (d0 > d) d1 = d0, i1 = i0, d0 = d, i0 = b + k;
                else d1 = d, i1 = b + k;
            }
        }
    }
    k0 = ((uint64_t)(uint32_t)d0 << 32) | (uint32_t)i0;
    k1 = ((uint64_t)(uint32_t)d1 << 32) | (uint32_t)i1;
#pragma unroll
    for (int m = 1; m < G; m <<= 1) {   // merge with the partner group-lane's top-2
        const uint64_t o0 = __shfl_xor(k0, m, 64), o1 = __shfl_xor(k1, m, 64);
        const uint64_t r0 = k0 < o0 ? k0 : o0;
        const uint64_t r1 = k0 < o0 ? (k1 < o0 ? k1 : o0) : (k0 < o1 ? k0 : o1);
        k0 = r0, k1 = r1;
    }
    if (qi < nq && g == 0) {
        int32_t *oi = a.idx2 + ((size_t)pair * a.out_cap + qi) * 2;
        int32_t *od = a.dist2 + ((size_t)pair * a.out_cap + qi) * 2;
        oi[0] = (int32_t)(uint32_t)k0, oi[1] = (int32_t)(uint32_t)k1;
        od[0] = (int32_t)(k0 >> 32), od[1] = (int32_t)(k1 >> 32);
    }
}

// 8 lanes per query at every batch size: one frame (1,200 queries) needs the spread to fill the chip, and at 128
// frames the shorter per-lane chains and 8x the waves still win over one lane per query (0.150 vs 0.189 ms per
// 128-frame launch; G = 2 / 4: 0.169 / 0.154).
static void launch_knn2(const KnnArgs &a, int n_pairs, int q_cap, hipStream_t st) {
    if ((long long)n_pairs * q_cap <= 4096)   // a frame or three: 32 lanes per query, shorter chains
        knn2_kernel<32><<<dim3((q_cap + 7) / 8, n_pairs), 256, 0, st>>>(a, n_pairs);
    else
        knn2_kernel<8><<<dim3((q_cap + 31) / 32, n_pairs), 256, 0, st>>>(a, n_pairs);
}

// Lowe ratio on the lapping-area knn of camera blocks 0 and 1 (Frame.cc:1488-1491); candidate
// stereo pairs before the TriangulateMatches depth check.
__global__ void stereo_pairs_kernel(const int32_t *idx2, const int32_t *dist2, int out_cap, const int *n_kp,
                                    const int *mono, int n_cams, int kp_cap, double ratio, int32_t *l2r,
                                    int32_t *r2l, int n_frames) {
    // one thread per left slot q of the frame's [0, kp_cap): every l2r entry is written here (-1 unless q is a
    // lapping left keypoint passing the ratio test), so only r2l needs a reset before the launch
    const int frame = blockIdx.y;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= kp_cap) return;
    const int m0 = mono[frame * n_cams], m1 = mono[frame * n_cams + 1];
    const int nq = n_kp[frame * n_cams] - m0, qi = q - m0;
    int32_t v = -1;
    if (qi >= 0 && qi < nq) {
        const int32_t *oi = idx2 + ((size_t)frame * out_cap + qi) * 2;
        const int32_t *od = dist2 + ((size_t)frame * out_cap + qi) * 2;
        // fewer than 2 matches: none; `distance * 0.8` is a double product (:1491)
        if (oi[1] >= 0 && (double)od[0] < (double)od[1] * ratio) {
            v = m1 + oi[0];
            atomicMax(&r2l[(size_t)frame * kp_cap + m1 + oi[0]], q);   // later left index wins
        }
    }
    l2r[(size_t)frame * kp_cap + q] = v;
}

// ---------------------------------------------------------------------------------------------
// Frame::isInFrustum, multi-camera branch: one thread per (frame, map point), the camera-block
// transforms of the frame composed once per workgroup in LDS (same float operation order as the
// reference's per-point Eigen expressions: 3x3 products summed left to right, no contraction).
// KannalaBrandt8.cpp / MapPoint.cc call the C double cos / sin / log on float arguments.
__device__ __forceinline__ void mat3f(const float *a, const float *b, float *r) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
__device__ __forceinline__ void matvec3f(const float *a, const float *x, float *r) {
    for (int i = 0; i < 3; ++i) r[i] = a[3 * i] * x[0] + a[3 * i + 1] * x[1] + a[3 * i + 2] * x[2];
}

__global__ void __launch_bounds__(256) frustum_kernel(const omv_frame_pose *poses, omv_rig rig, omv_mp_world mp, int M,
                                                      float cos_limit, omv_mp_track out, int32_t *n_in_view) {
    __shared__ float Rc[kMaxCams][9], tc[kMaxCams][3], twc[kMaxCams][3];
    const int frame = blockIdx.y, C = rig.n_cams;
    const omv_frame_pose &pose = poses[frame];
    if (threadIdx.x < C) {
        const int c = threadIdx.x;
        if (c == 0) {
            for (int q = 0; q < 9; ++q) Rc[0][q] = pose.Rcw[q];
            for (int q = 0; q < 3; ++q) tc[0][q] = pose.tcw[q], twc[0][q] = pose.Ow[q];
        } else {
            float R[9], t[3];
            mat3f(rig.R_cl[c], pose.Rcw, R);
            for (int q = 0; q < 9; ++q) Rc[c][q] = R[q];
            matvec3f(rig.R_cl[c], pose.tcw, t);
            for (int q = 0; q < 3; ++q) tc[c][q] = t[q] + rig.t_cl[c][q];
            matvec3f(pose.Rwc, rig.t_lc[c], t);
            for (int q = 0; q < 3; ++q) twc[c][q] = t[q] + pose.Ow[q];
        }
    }
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const size_t fm = (size_t)frame * M + i;
    const float P[3] = {mp.pos[3 * fm], mp.pos[3 * fm + 1], mp.pos[3 * fm + 2]};
    const float Pn[3] = {mp.normal[3 * fm], mp.normal[3 * fm + 1], mp.normal[3 * fm + 2]};
    const float mind = mp.min_dist[fm], maxd = mp.max_dist[fm];
    bool any = false;
    for (int c = 0; c < C; ++c) {
        const size_t o = fm * C + c;
        float px = -1.f, py = -1.f;
        int lvl = -1;
        bool vis = false;
        float Pc[3];
        matvec3f(Rc[c], P, Pc);
        for (int q = 0; q < 3; ++q) Pc[q] = Pc[q] + tc[c][q];
        const float Pc_dist = omv::sqrtf_cr(Pc[0] * Pc[0] + Pc[1] * Pc[1] + Pc[2] * Pc[2]);
        if (Pc[2] >= 0.0f) {
            const float *k = rig.cam[c];
            float u, v;
            if (rig.model[c] == OMV_CAM_PINHOLE) {   // Pinhole::project(Vector3f) (Pinhole.cpp:26-32)
                u = k[0] * Pc[0] / Pc[2] + k[2];
                v = k[1] * Pc[1] / Pc[2] + k[3];
            } else {                                 // KannalaBrandt8::project(Vector3f)
                const float x2y2 = Pc[0] * Pc[0] + Pc[1] * Pc[1];
                const float theta = omv::glibc_atan2f(omv::sqrtf_cr(x2y2), Pc[2]);
                const float psi = omv::glibc_atan2f(Pc[1], Pc[0]);
                const float t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
                const float r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9;
                u = (float)((double)(k[0] * r) * cos((double)psi) + (double)k[2]);
                v = (float)((double)(k[1] * r) * sin((double)psi) + (double)k[3]);
            }
            if (!(u < rig.min_x || u > rig.max_x || v < rig.min_y || v > rig.max_y)) {
                const float maxD = 1.2f * maxd, minD = 0.8f * mind;
                const float PO[3] = {P[0] - twc[c][0], P[1] - twc[c][1], P[2] - twc[c][2]};
                const float dist = omv::sqrtf_cr(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
                if (!(dist < minD || dist > maxD)) {
                    const float vc = (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) / dist;
                    if (!(vc < cos_limit)) {
                        const float ratio = maxd / dist;
                        int ns = (int)ceil(log((double)ratio) / (double)rig.log_scale_factor);
                        ns = ns < 0 ? 0 : (ns >= rig.n_levels ? rig.n_levels - 1 : ns);
                        px = u, py = v, lvl = ns, vis = true;
                        out.view_cos[o] = vc;
                        if (c == 0) out.track_depth[fm] = Pc_dist;
                    }
                }
            }
        }
        out.proj_x[o] = px, out.proj_y[o] = py, out.level[o] = lvl, out.in_view[o] = vis ? 1 : 0;
        any = any || vis;
    }
    if (n_in_view) {
        const uint64_t m = __ballot(any);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(n_in_view + frame, __popcll(m));
    }
}

// ---------------------------------------------------------------------------------------------
// SearchByProjection(Frame&, const Frame& LastFrame, th, bMono): a candidate pass per (frame, last
// slot, block) — projection (Sophus quaternion rotation, float KB8) and the 16 best window candidates
// by (distance, window order) — then one wave per frame resolving slots in order against the claims
// (a claimed keypoint with observations blocks later points), then the rotation-histogram filter.
struct LastArgs {
    const float *pos;
    const uint8_t *desc, *valid, *has_obs;
    const omv_kp *kps;
    int S;
};
struct LfGeo {
    float cam0[8];
    omv_se3f Trl;
    float th, mb;
    int bMono;
};

__device__ __forceinline__ void cross3f(const float *a, const float *b, float *r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}
// Eigen Quaternion::_transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv
__device__ __forceinline__ void quat_rotate(const float *q, const float *v, float *r) {
    float uv[3], c[3];
    cross3f(q, v, uv);
    for (int i = 0; i < 3; ++i) uv[i] = uv[i] + uv[i];
    cross3f(q, uv, c);
    for (int i = 0; i < 3; ++i) r[i] = v[i] + q[3] * uv[i] + c[i];
}
__device__ __forceinline__ void se3_apply(const omv_se3f &T, const float *p, float *r) {
    quat_rotate(T.q, p, r);
    for (int i = 0; i < 3; ++i) r[i] = r[i] + T.t[i];
}
// KannalaBrandt8::project(const Eigen::Vector3f&) (KannalaBrandt8.cpp:48-67)
__device__ __forceinline__ void kb8_project_f(const float *k, const float *X, float &u, float &v) {
    const float x2y2 = X[0] * X[0] + X[1] * X[1];
    const float theta = omv::glibc_atan2f(omv::sqrtf_cr(x2y2), X[2]);
    const float psi = omv::glibc_atan2f(X[1], X[0]);
    const float t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
    const float r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9;
    u = (float)((double)(k[0] * r) * cos((double)psi) + (double)k[2]);
    v = (float)((double)(k[1] * r) * sin((double)psi) + (double)k[3]);
}
// GeometricCamera::project(const Eigen::Vector3f&) by the block's camera type: KannalaBrandt8, or
// Pinhole::project (Pinhole.cpp:26-32: fx * x / z + cx in float, left to right)
__device__ __forceinline__ void cam_project_f(int model, const float *k, const float *X, float &u, float &v) {
    if (model == OMV_CAM_PINHOLE) {
        u = k[0] * X[0] / X[2] + k[2];
        v = k[1] * X[1] / X[2] + k[3];
    } else {
        kb8_project_f(k, X, u, v);
    }
}

// Window of last slot s in block c of frame `frame`: false if the point is skipped entirely.
__device__ bool lf_window(const FrameArgs &f, const LastArgs &L, const LfGeo &G, const omv_se3f &Tcw,
                          const omv_se3f &Tlw, int frame, int s, int c, float &x, float &y, float &r, int &minL,
                          int &maxL) {
    const size_t fs = (size_t)frame * L.S + s;
    if (!L.valid[fs]) return false;
    float x3[3];
    se3_apply(Tcw, L.pos + 3 * fs, x3);
    const float invzc = (float)(1.0 / (double)x3[2]);
    if (invzc < 0) return false;
    float u, v;
    cam_project_f(f.model[0], G.cam0, x3, u, v);   // CurrentFrame.mpCamera->project (ORBmatcher.cc:2022)
    if (u < f.min_x || u > f.max_x || v < f.min_y || v > f.max_y) return false;
    x = u, y = v;
    if (c == 1) {
        float xr[3];
        se3_apply(G.Trl, x3, xr);
        cam_project_f(f.model[0], G.cam0, xr, x, y);   // the same camera on Trl * x3Dc (:2134)
    }
    // bForward / bBackward from tlc = Tlw * twc, twc = -(q^-1 t)
    const omv_se3f inv{{-Tcw.q[0], -Tcw.q[1], -Tcw.q[2], Tcw.q[3]}, {0, 0, 0}};
    float twc[3], tlc[3];
    quat_rotate(inv.q, Tcw.t, twc);
    for (int i = 0; i < 3; ++i) twc[i] = -twc[i];
    se3_apply(Tlw, twc, tlc);
    const bool fwd = tlc[2] > G.mb && !G.bMono, bwd = -tlc[2] > G.mb && !G.bMono;
    const int oct = L.kps[fs].octave;
    r = G.th * f.scale[oct];
    if (fwd) minL = oct, maxL = -1;
    else if (bwd) minL = 0, maxL = oct;
    else minL = oct - 1, maxL = oct + 1;
    return true;
}

__global__ void __launch_bounds__(256) lf_cand_kernel(FrameArgs f, LastArgs L, LfGeo G, const omv_se3f *Tcw,
                                                      const omv_se3f *Tlw, int n_frames, const uint8_t *occ_init,
                                                      Rec *recs, int *counts) {
    const int C = f.n_cams;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long long)n_frames * L.S * C) return;
    const int c = (int)(gid % C);
    const long long fs = gid / C;
    const int frame = (int)(fs / L.S), s = (int)(fs % L.S);
    TopSeq t;
    t.reset();
    float x, y, r;
    int minL, maxL;
    if (lf_window(f, L, G, Tcw[frame], Tlw[frame], frame, s, c, x, y, r, minL, maxL)) {
        uint64_t dmp[4];
        load_desc(L.desc + (size_t)fs * 32, dmp);
        const uint8_t *occ = occ_init ? occ_init + (size_t)frame * C * f.kp_cap : nullptr;
        scan_window(f, frame, c, x, y, r, minL, maxL, dmp, [&](int slot) { return occ && occ[slot]; }, t);
    }
    Rec &out = recs[(size_t)fs * C + c];
    uint4 *o4 = reinterpret_cast<uint4 *>(&out);
#pragma unroll
    for (int v = 0; v < kTop / 4; ++v)
        o4[v] = make_uint4(4 * v < t.n ? t.rec(4 * v) : 0u, 4 * v + 1 < t.n ? t.rec(4 * v + 1) : 0u,
                           4 * v + 2 < t.n ? t.rec(4 * v + 2) : 0u, 4 * v + 3 < t.n ? t.rec(4 * v + 3) : 0u);
    counts[(size_t)fs * C + c] = t.count;
}

struct LfResolveArgs {
    FrameArgs f;
    LastArgs L;
    LfGeo G;
    const omv_se3f *Tcw, *Tlw;
    const Rec *recs;
    const int *counts;
    const uint8_t *occ_init;
    int32_t *kp_to_mp;
    int *n_matches;
    int2 *pushes;   // [frame][S * C] (slot, bin) in claim order
    int *n_push;
    int check_ori;
};

// One wavefront per frame; lanes evaluate 64 consecutive last-frame slots, the longest prefix whose
// chosen keypoints were not claimed (with observations) by an earlier lane of the batch commits.
__global__ void __launch_bounds__(64) lf_resolve_kernel(LfResolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lsm[];
    const int frame = blockIdx.x, lane = threadIdx.x;
    const FrameArgs &f = a.f;
    const int C = f.n_cams, cap = f.kp_cap, S = C * cap;
    const int nwords = (S + 31) >> 5;
    uint32_t *bits = lsm;                                        // blocked slots
    // first claiming lane (with obs) in the conflict phase, 63 - the last committing writer in the commit phase
    int *owner = reinterpret_cast<int *>(lsm + nwords);
    const uint8_t *occ = a.occ_init ? a.occ_init + (size_t)frame * S : nullptr;
    for (int w = lane; w < nwords; w += 64) {
        uint32_t v = 0;
        for (int b = 0; b < 32; ++b) {
            const int s = w * 32 + b;
            if (s < S && occ && occ[s]) v |= 1u << b;
        }
        bits[w] = v;
    }
    for (int s = lane; s < S; s += 64) owner[s] = INT_MAX;
    wave_sync();
    int32_t *k2m = a.kp_to_mp + (size_t)frame * S;
    int2 *push = a.pushes + (size_t)frame * a.L.S * C;
    int total = 0, npush = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int base = 0; base < a.L.S; base += 64) {
        const int nb = min(64, a.L.S - base);
        const int s = base + lane;
        int start = 0;
        while (start < nb) {
            const bool active = lane >= start && lane < nb;
            int claim[kMaxCams], bin[kMaxCams];
            int nclaim = 0;
            bool fallback = false, unblock = false;
            const size_t fs = (size_t)frame * a.L.S + s;
            const bool obs = active && a.L.has_obs[fs];
            if (active && a.L.valid[fs]) {
                for (int c = 0; c < C; ++c) {
                    const size_t rc = fs * C + c;
                    const int cnt = a.counts[rc];
                    int best = -1, bd = 256;
                    if (cnt > 0) {
                        const Rec &r = a.recs[rc];
                        const int avail = min(cnt, kTop);
                        for (int k = 0; k < avail; ++k) {
                            const uint32_t v = r.e[k];
                            if (bit_of(bits, c * cap + rec_idx(v))) continue;
                            best = rec_idx(v), bd = rec_dist(v);
                            break;
                        }
                        if (best < 0 && cnt > kTop) {   // every kept candidate is claimed: rescan the window
                            fallback = true;
                            float x, y, rr;
                            int minL, maxL;
                            lf_window(f, a.L, a.G, a.Tcw[frame], a.Tlw[frame], frame, s, c, x, y, rr, minL, maxL);
                            uint64_t dmp[4];
                            load_desc(a.L.desc + fs * 32, dmp);
                            TopSeq t;
                            scan_window(f, frame, c, x, y, rr, minL, maxL, dmp,
                                        [&](int slot) { return bit_of(bits, slot); }, t);
                            if (t.n > 0) best = t.idx(0), bd = t.dist(0);
                        }
                    }
                    if (best >= 0 && bd <= kTH_HIGH) {
                        const int slot = c * cap + best;
                        if (!obs && bit_of(bits, slot)) unblock = true;
                        claim[nclaim] = slot;
                        float rot = a.L.kps[fs].angle - f.kps[(size_t)frame * S + slot].angle;
                        if (rot < 0.0f) rot += 360.0f;
                        int b = (int)roundf(rot * (1.0f / 30));
                        if (b == 30) b = 0;
                        bin[nclaim++] = b;
                    }
                }
            }
            if (obs)
                for (int q = 0; q < nclaim; ++q) atomicMin(&owner[claim[q]], lane);
            wave_sync();
            bool conflict = false;
            if (active && lane > start) {
                conflict = fallback;   // a rescan saw the whole window: only safe at the batch head
                for (int q = 0; q < nclaim && !conflict; ++q) conflict = owner[claim[q]] < lane;
            }
            wave_sync();
            if (obs)
                for (int q = 0; q < nclaim; ++q) owner[claim[q]] = 64;
            wave_sync();
            uint64_t cm = __ballot(conflict);
            const uint64_t um = __ballot(active && unblock);
            if (um) {
                const int u = __ffsll((long long)um) - 1;
                cm |= (u >= 63) ? 0ull : (~0ull << (u + 1));
            }
            const int j0 = cm ? min(nb, __ffsll((long long)cm) - 1) : nb;
            const bool committed = lane >= start && lane < j0;
            // pushes of committed lanes in lane order
            int np = committed ? nclaim : 0, incl = np;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int t = __shfl_up(incl, d, 64);
                if (lane >= d) incl += t;
            }
            const int ptot = __shfl(incl, 63, 64);
            if (committed) {
                for (int q = 0; q < nclaim; ++q) {
                    atomicMin(&owner[claim[q]], 63 - lane);
                    if (a.check_ori) push[npush + incl - np + q] = make_int2(claim[q], bin[q]);
                }
            }
            npush += ptot;
            total += ptot;
            wave_sync();
            if (committed)
                for (int q = 0; q < nclaim; ++q) {
                    const int slot = claim[q];
                    if (owner[slot] != 63 - lane) continue;
                    k2m[slot] = s;
                    if (obs) atomicOr(&bits[slot >> 5], 1u << (slot & 31));
                    else atomicAnd(&bits[slot >> 5], ~(1u << (slot & 31)));
                }
            wave_sync();
            if (committed)
                for (int q = 0; q < nclaim; ++q) owner[claim[q]] = 64;
            start = j0;
            wave_sync();
            (void)lt;
        }
    }
    if (lane == 0) {
        a.n_matches[frame] = total;
        a.n_push[frame] = npush;
    }
}

// Rotation consistency (ORBmatcher.cc:2396-2410 + ComputeThreeMaxima): keep the three largest bins
// (second / third only when >= 10% of the first), undo every claim pushed into another bin.
__global__ void __launch_bounds__(256) lf_histo_kernel(const int2 *pushes, const int *n_push, int per_frame,
                                                       int S, int32_t *kp_to_mp, int *n_matches) {
    __shared__ int hist[30];
    __shared__ int keep[3];
    __shared__ int removed;
    const int frame = blockIdx.x;
    const int n = n_push[frame];
    const int2 *p = pushes + (size_t)frame * per_frame;
    if (threadIdx.x < 30) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) removed = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[p[i].y], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < 30; i++) {
            const int sz = hist[i];
            if (sz > max1) {
                max3 = max2, max2 = max1, max1 = sz, ind3 = ind2, ind2 = ind1, ind1 = i;
            } else if (sz > max2) {
                max3 = max2, max2 = sz, ind3 = ind2, ind2 = i;
            } else if (sz > max3) {
                max3 = sz, ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) ind2 = -1, ind3 = -1;
        else if (max3 < 0.1f * (float)max1) ind3 = -1;
        keep[0] = ind1, keep[1] = ind2, keep[2] = ind3;
    }
    __syncthreads();
    int32_t *k2m = kp_to_mp + (size_t)frame * S;
    int rm = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int b = p[i].y;
        if (b != keep[0] && b != keep[1] && b != keep[2]) {
            k2m[p[i].x] = -1;
            ++rm;
        }
    }
    atomicAdd(&removed, rm);
    __syncthreads();
    if (threadIdx.x == 0) n_matches[frame] -= removed;
}

// ---------------------------------------------------------------------------------------------
// Keyframe-side projection searches (omv_matcher_search_kf): ORBmatcher::Fuse (both overloads,
// ORBmatcher.cc:1458-1769), SearchByProjection(KF, Sim3, ...) (:668-893) and
// SearchByProjection(Frame&, KF, ...) (:2415-2535).
//   kf_cand_kernel     one thread per (job, map point): SE3f transform, float KB8 projection, the mode's
//                      depth / bounds / distance / viewing tests, PredictScale, and the 16 best window
//                      candidates by (distance, window order) passing the level filter, Fuse's
//                      reprojection gate and the claims present at the call.  The Fuse modes read no
//                      state the loop changes, so their answer is final here.
//   kf_resolve_kernel  claim modes: one wavefront per keyframe walks its jobs and points in order; a
//                      point takes the first of its candidates not claimed so far (ballot over the 16),
//                      rescanning the window when all are taken and it held more; then
//                      OMV_KF_SBP_FRAME's rotation histogram un-claims matches outside the top 3 bins.
// Slots claimed at the call are never freed during it (the histogram only removes this call's claims),
// so filtering them in the candidate pass is exact.
struct KfArgs {
    FrameArgs f;
    const omv_kf_search_job *jobs;
    int n_jobs, n_kf;
    const int32_t *mp_list;
    int n_entries;
    omv_kf_mps mps;
    int mode, check_ori;
    float th, max_dist, bf;
    const float *uright;
    float invs2[16], log_scale;
    int n_levels;
    float cams[kMaxCams][8];
    const float *mp_angle;
    int32_t *kp_match, *best_idx, *best_dist, *n_matches;
    Rec *recs;
    int *counts;
    float4 *geo;   // per entry: window centre x, y, radius, predicted level (bits) for rescans
};

__device__ __forceinline__ bool kf_claim_mode(int mode) { return mode == OMV_KF_SBP_SIM3 || mode == OMV_KF_SBP_FRAME; }

// The job whose run of mp_list holds entry e (jobs tile mp_list in order; the last of equal starts).
__device__ __forceinline__ int kf_job_of(const KfArgs &a, int e) {
    int lo = 0, hi = a.n_jobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.jobs[mid].mp_start <= e) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Level window: the KeyFrame modes filter [pred-1, pred] in their loop, OMV_KF_SBP_FRAME's
// Frame::GetFeaturesInArea takes [pred-1, pred+1].
__device__ __forceinline__ void kf_levels(int mode, int pred, int &minL, int &maxL) {
    minL = pred - 1;
    maxL = mode == OMV_KF_SBP_FRAME ? pred + 1 : pred;
}

__device__ __forceinline__ int kf_block_offset(const FrameArgs &f, int kf, int cam) {   // N-index of the block's kp 0
    int off = 0;
    for (int c = 0; c < cam; ++c) off += f.n_kp[(size_t)kf * f.n_cams + c];
    return off;
}

__global__ void __launch_bounds__(256) kf_cand_kernel(KfArgs a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n_entries) return;
    const int j = kf_job_of(a, e);
    const omv_kf_search_job &J = a.jobs[j];
    const int kf = J.kf, cam = J.cam, mode = a.mode, C = a.f.n_cams, cap = a.f.kp_cap;
    const bool claim = kf_claim_mode(mode);
    const int mp = a.mp_list[e];
    TopSeq t;
    t.reset();
    float4 g = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
    do {
        const float P[3] = {a.mps.pos[3 * (size_t)mp], a.mps.pos[3 * (size_t)mp + 1], a.mps.pos[3 * (size_t)mp + 2]};
        float Pc[3];
        se3_apply(J.Tcw, P, Pc);
        if (mode != OMV_KF_SBP_FRAME && Pc[2] < 0.0f) break;   // depth must be positive
        float u, v;
        cam_project_f(a.f.model[cam], a.cams[cam], Pc, u, v);   // pCamera / GetCamera(camId) (:1536, :1710, :2443)
        if (mode == OMV_KF_SBP_FRAME) {   // CurrentFrame.mnMinX .. mnMaxX, inclusive
            if (u < a.f.min_x || u > a.f.max_x || v < a.f.min_y || v > a.f.max_y) break;
        } else if (!(u >= a.f.min_x && u < a.f.max_x && v >= a.f.min_y && v < a.f.max_y)) {   // KeyFrame::IsInImage
            break;
        }
        const float invz = 1 / Pc[2];
        const float ur = u - a.bf * invz;
        const float maxd = a.mps.max_dist[mp];
        const float maxDistance = 1.2f * maxd, minDistance = 0.8f * a.mps.min_dist[mp];
        const float PO[3] = {P[0] - J.Ow[0], P[1] - J.Ow[1], P[2] - J.Ow[2]};
        const float dist3D = omv::sqrtf_cr(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
        if (mode != OMV_KF_FUSE_SIM3 && (dist3D < minDistance || dist3D > maxDistance)) break;
        if (mode == OMV_KF_FUSE || mode == OMV_KF_SBP_SIM3) {   // viewing angle < 60 deg
            const float *Pn = a.mps.normal + 3 * (size_t)mp;
            if ((double)(PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) < 0.5 * (double)dist3D) break;
        }
        int pred = (int)ceil(log((double)(maxd / dist3D)) / (double)a.log_scale);   // MapPoint::PredictScale
        pred = pred < 0 ? 0 : (pred >= a.n_levels ? a.n_levels - 1 : pred);
        const float radius = a.th * a.f.scale[pred];
        int minL, maxL;
        kf_levels(mode, pred, minL, maxL);
        uint64_t dmp[4];
        load_desc(a.mps.desc + (size_t)mp * 32, dmp);
        const int32_t *cl = claim ? a.kp_match + (size_t)kf * C * cap : nullptr;
        const omv_kp *kk = a.f.kps + (size_t)kf * C * cap;
        const float *urow = a.uright ? a.uright + (size_t)kf * cap : nullptr;
        scan_window(a.f, kf, cam, u, v, radius, minL, maxL, dmp,
                    [&](int slot) {
                        if (claim) return cl[slot] >= 0;
                        if (mode != OMV_KF_FUSE) return false;
                        const omv_kp k = kk[slot];   // reprojection gate (ORBmatcher.cc:1594-1615)
                        const float ex = u - k.x, ey = v - k.y;
                        const int i = slot - cam * cap;
                        if (cam == 0 && urow[i] >= 0) {
                            const float er = ur - urow[i];
                            const float e2 = ex * ex + ey * ey + er * er;
                            return (double)(e2 * a.invs2[k.octave]) > 7.8;
                        }
                        const float e2 = ex * ex + ey * ey;
                        return (double)(e2 * a.invs2[k.octave]) > 5.99;
                    },
                    t);
        g = make_float4(u, v, radius, __int_as_float(pred));
    } while (false);
    if (!claim) {
        int bi = -1, bd = -1;
        if (t.n > 0) bi = kf_block_offset(a.f, kf, cam) + t.idx(0), bd = t.dist(0);
        a.best_idx[e] = bi, a.best_dist[e] = bd;
        if (bi >= 0 && (float)bd <= a.max_dist) atomicAdd(a.n_matches + j, 1);
        return;
    }
    uint4 *o4 = reinterpret_cast<uint4 *>(&a.recs[e]);
#pragma unroll
    for (int q = 0; q < kTop / 4; ++q)
        o4[q] = make_uint4(4 * q < t.n ? t.rec(4 * q) : 0u, 4 * q + 1 < t.n ? t.rec(4 * q + 1) : 0u,
                           4 * q + 2 < t.n ? t.rec(4 * q + 2) : 0u, 4 * q + 3 < t.n ? t.rec(4 * q + 3) : 0u);
    a.counts[e] = t.count;
    a.geo[e] = g;
}

// Rotation bin of a SearchByProjection(Frame&, KF, ...) match (:2502-2510).
__device__ __forceinline__ int kf_rot_bin(float kf_angle, float frame_angle) {
    float rot = kf_angle - frame_angle;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / 30));
    return bin == 30 ? 0 : bin;
}

__global__ void __launch_bounds__(64) kf_resolve_kernel(KfArgs a) {
    extern __shared__ uint32_t claimed[];
    __shared__ int hist[30];
    const int kf = blockIdx.x, lane = threadIdx.x;
    const int C = a.f.n_cams, cap = a.f.kp_cap, S = C * cap, W = (S + 31) / 32;
    int32_t *cl = a.kp_match + (size_t)kf * S;
    for (int w = lane; w < W; w += 64) {
        uint32_t bits = 0;
        for (int b = 0; b < 32; ++b) {
            const int s = w * 32 + b;
            if (s < S && cl[s] >= 0) bits |= 1u << b;
        }
        claimed[w] = bits;
    }
    wave_sync();
    const bool ori = a.mode == OMV_KF_SBP_FRAME && a.check_ori;
    for (int j = 0; j < a.n_jobs; ++j) {
        const omv_kf_search_job &J = a.jobs[j];
        if (J.kf != kf) continue;
        const int cam = J.cam, off = kf_block_offset(a.f, kf, cam);
        const omv_kp *kk = a.f.kps + (size_t)kf * S;
        int nm = 0;
        if (lane < 30) hist[lane] = 0;
        wave_sync();
        for (int e = J.mp_start; e < J.mp_start + J.mp_count; ++e) {
            const int cnt = a.counts[e];
            int idx = -1, dist = 0;
            if (cnt > 0) {
                const int nrec = min(cnt, kTop);
                const uint32_t r = lane < nrec ? a.recs[e].e[lane] : 0u;
                const bool free = lane < nrec && !bit_of(claimed, cam * cap + rec_idx(r));
                const uint64_t m = __ballot(free);
                if (m) {
                    const uint32_t rf = __shfl(r, __ffsll((long long)m) - 1, 64);
                    idx = rec_idx(rf), dist = rec_dist(rf);
                } else if (cnt > kTop) {   // all 16 taken and the window held more: rescan (rare)
                    if (lane == 0) {
                        const float4 g = a.geo[e];
                        int minL, maxL;
                        kf_levels(a.mode, __float_as_int(g.w), minL, maxL);
                        uint64_t dmp[4];
                        load_desc(a.mps.desc + (size_t)a.mp_list[e] * 32, dmp);
                        TopSeq t;
                        scan_window(a.f, kf, cam, g.x, g.y, g.z, minL, maxL, dmp,
                                    [&](int slot) { return bit_of(claimed, slot); }, t);
                        if (t.n > 0) idx = t.idx(0), dist = t.dist(0);
                    }
                    idx = __shfl(idx, 0, 64), dist = __shfl(dist, 0, 64);
                }
            }
            const bool ok = idx >= 0 && (float)dist <= a.max_dist;
            if (lane == 0) {
                if (ok) {
                    const int slot = cam * cap + idx;
                    claimed[slot >> 5] |= 1u << (slot & 31);
                    cl[slot] = a.mp_list[e];
                    a.best_idx[e] = off + idx, a.best_dist[e] = dist;
                    if (ori) ++hist[kf_rot_bin(a.mp_angle[e], kk[slot].angle)];
                } else {
                    a.best_idx[e] = -1, a.best_dist[e] = -1;
                }
            }
            nm += ok ? 1 : 0;
            wave_sync();
        }
        if (ori) {   // ComputeThreeMaxima (:2537-2573), then un-claim the matches outside the top bins
            if (lane == 0) {
                int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
                for (int i = 0; i < 30; i++) {
                    const int sz = hist[i];
                    if (sz > max1) max3 = max2, max2 = max1, max1 = sz, ind3 = ind2, ind2 = ind1, ind1 = i;
                    else if (sz > max2) max3 = max2, max2 = sz, ind3 = ind2, ind2 = i;
                    else if (sz > max3) max3 = sz, ind3 = i;
                }
                if (max2 < 0.1f * (float)max1) ind2 = -1, ind3 = -1;
                else if (max3 < 0.1f * (float)max1) ind3 = -1;
                for (int e = J.mp_start; e < J.mp_start + J.mp_count; ++e) {
                    const int bi = a.best_idx[e];
                    if (bi < 0) continue;
                    const int slot = cam * cap + (bi - off);
                    const int bin = kf_rot_bin(a.mp_angle[e], kk[slot].angle);
                    if (bin == ind1 || bin == ind2 || bin == ind3) continue;
                    claimed[slot >> 5] &= ~(1u << (slot & 31));
                    cl[slot] = -1;
                    a.best_idx[e] = -1, a.best_dist[e] = -1;
                    --nm;
                }
            }
            nm = __shfl(nm, 0, 64);
            wave_sync();
        }
        if (lane == 0) a.n_matches[j] = nm;
    }
}

// ---- ORBmatcher::SearchBySim3 (ORBmatcher.cc:1771-1983) ------------------------------------------------
//   sbs3_cand_kernel   one thread per entry of either side: side 1 (:1812-1885) T1w then S21 into pKF2,
//                      side 2 (:1888-1961) T2w then S12 into pKF1; pinhole with pKF1's intrinsics in both
//                      directions, IsInImage, distance invariance on |p3Dc|, PredictScale, the window's best
//                      at levels [pred-1, pred] (strict <, so the first of equal distances), kept at <= TH_HIGH.
//                      vnMatch1 per side-1 entry; vnMatch2 scattered into a dense [job][N] table.
//   sbs3_agree_kernel  the agreement check (:1964-1979) per side-1 entry.
// No state changes between the points of a pass, so every entry is independent.
struct Sim3Args {
    FrameArgs f;
    const omv_sim3_job *jobs;
    int n_jobs, n1, n2, N;             // N = n_cams * kp_cap: the keyframe N-index bound
    const int32_t *kp1, *mp1, *kp2, *mp2;
    omv_kf_mps mps;
    float th, log_scale;
    int n_levels;
    int32_t *vn1;                      // [n1] vnMatch1 per side-1 entry
    int32_t *vn2;                      // [n_jobs][N] vnMatch2 (-1 initially)
    int32_t *match12, *n_found;
};

// Sophus RxSO3 * p + t (rxso3.hpp:265-272, sim3.hpp:226-229): s p + (w 2(v x p) + v x 2(v x p)) + t
__device__ __forceinline__ void sim3_apply(const omv_sim3f &S, const float *p, float *r) {
    float two[3], c[3];
    cross3f(S.q, p, two);
    for (int i = 0; i < 3; ++i) two[i] = two[i] + two[i];
    cross3f(S.q, two, c);
    for (int i = 0; i < 3; ++i) r[i] = (S.scale * p[i] + (S.q[3] * two[i] + c[i])) + S.t[i];
}

// The job whose run of the side's list holds entry k (runs tile the list in order; the last of equal starts).
__device__ __forceinline__ int sbs3_job_of(const Sim3Args &a, bool one, int k) {
    int lo = 0, hi = a.n_jobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((one ? a.jobs[mid].start1 : a.jobs[mid].start2) <= k) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ void __launch_bounds__(256) sbs3_cand_kernel(Sim3Args a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n1 + a.n2) return;
    const bool one = e < a.n1;
    const int k = one ? e : e - a.n1;
    const int j = sbs3_job_of(a, one, k);
    const omv_sim3_job &J = a.jobs[j];
    const int mp = one ? a.mp1[k] : a.mp2[k];
    const int tgt = one ? J.kf2 : J.kf1;
    int best = -1;
    do {
        const float P[3] = {a.mps.pos[3 * (size_t)mp], a.mps.pos[3 * (size_t)mp + 1], a.mps.pos[3 * (size_t)mp + 2]};
        float Pc[3], Pt[3];
        se3_apply(one ? J.T1w : J.T2w, P, Pc);
        sim3_apply(one ? J.S21 : J.S12, Pc, Pt);
        if (Pt[2] < 0.0f) break;   // depth must be positive
        // invz = 1.0 / z in double, stored as float: equal to the float quotient (53 >= 2 * 24 + 2)
        const float invz = 1.0f / Pt[2];
        const float x = Pt[0] * invz, y = Pt[1] * invz;
        const float u = J.fx * x + J.cx, v = J.fy * y + J.cy;
        if (!(u >= a.f.min_x && u < a.f.max_x && v >= a.f.min_y && v < a.f.max_y)) break;   // IsInImage
        const float maxd = a.mps.max_dist[mp];
        const float maxDistance = 1.2f * maxd, minDistance = 0.8f * a.mps.min_dist[mp];
        const float dist3D = omv::sqrtf_cr(Pt[0] * Pt[0] + Pt[1] * Pt[1] + Pt[2] * Pt[2]);
        if (dist3D < minDistance || dist3D > maxDistance) break;
        int pred = (int)ceil(log((double)(maxd / dist3D)) / (double)a.log_scale);   // MapPoint::PredictScale
        pred = pred < 0 ? 0 : (pred >= a.n_levels ? a.n_levels - 1 : pred);
        const float radius = a.th * a.f.scale[pred];
        uint64_t dmp[4];
        load_desc(a.mps.desc + (size_t)mp * 32, dmp);
        TopSeq t;
        scan_window(a.f, tgt, 0, u, v, radius, pred - 1, pred, dmp, [](int) { return false; }, t);
        if (t.n > 0 && t.dist(0) <= kTH_HIGH) best = t.idx(0);   // block 0: the N-index is the block index
    } while (false);
    if (one) {
        a.vn1[k] = best;
    } else if (best >= 0) {
        const int i2 = a.kp2[k];
        if ((unsigned)i2 < (unsigned)a.N) a.vn2[(size_t)j * a.N + i2] = best;
    }
}

__global__ void __launch_bounds__(256) sbs3_agree_kernel(Sim3Args a) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.n1) return;
    const int j = sbs3_job_of(a, true, k);
    const int i2 = a.vn1[k];
    const bool ok = i2 >= 0 && a.vn2[(size_t)j * a.N + i2] == a.kp1[k];
    a.match12[k] = ok ? i2 : -1;
    if (ok) atomicAdd(a.n_found + j, 1);
}

// ---- ORBmatcher::SearchForInitialization (ORBmatcher.cc:895-1004) ---------------------------------------
// The claims are sequential (vMatchedDistance / vnMatches21 of F2 change with every accepted match), but a claim
// only ever EXCLUDES window candidates: the scan skips F2 keypoints whose claimed distance is <= the new one
// (`vMatchedDistance[i2] <= dist`, :937), and a claimed distance only decreases.  So the launch is two kernels:
//  1. init_spec_kernel, one wavefront per F1 keypoint of every pair (the whole chip): the window scan with NO
//     claim filter, keeping the eight smallest (distance, window position) keys and their F2 indices;
//  2. init_kernel, one wavefront per pair walking F1 in order: exclusion only removes candidates, so the
//     filtered best and second are the first two of those keys the current claims leave -- known whenever two
//     of them survive (or the window held fewer than eight).  Otherwise the wavefront rescans the window with
//     the filter, as the reference's loop does.
// For one window scan the lanes take the candidates of each grid column (GetFeaturesInArea order: columns ix,
// the column's cells iy contiguous in the CSR, keypoints ascending), each keeping its K smallest keys; K wave
// reductions give the reference's best (first minimal distance) and second.  The F2 claim state, F1's
// matches and rotation bins live in LDS.
struct InitArgs {
    FrameArgs f;
    const int32_t *pairs;   // [n][2] (F1, F2) frame indices
    float *prev;            // [n][kp_cap][2] vbPrevMatched in/out
    int window;
    float nnratio;
    int check_ori;
    int32_t *m12;           // [n][kp_cap]
    int32_t *n_matches;     // [n]
    uint4 *spec;            // [n][kp_cap][4] {8 smallest keys}, {their F2 indices}, without the claim filter
};

constexpr int kInitChunk = 256;   // F1 keypoints whose speculative keys are staged in LDS at a time
__host__ __device__ inline size_t init_lds_bytes(int cap) { return kInitChunk * 64 + (size_t)cap * 17 + 4 * 36 + 16; }

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

constexpr uint32_t kNoKey = 0xffffffffu;
constexpr int kInitSpec = 8;   // speculative keys kept per F1 keypoint (two uint4 of keys, two of F2 indices)

// Frame::GetFeaturesInArea(x, y, windowSize, 0, 0) window (Frame.cc:890-967) scanned by one wavefront.  Returns
// the wave-uniform K smallest keys ((dist << 16) | window position, ascending) and their F2 indices (kNoKey / -1
// past the candidates); mdist == nullptr scans without the claim filter.
template <int K>
__device__ __forceinline__ void init_window_scan(const FrameArgs &f, const int32_t *cs, const int32_t *ci,
                                                 const omv_kp *kp2, const uint8_t *ds2, const uint64_t d1[4],
                                                 float x, float y, float r, const int *mdist, int lane,
                                                 uint32_t (&ok)[K], int (&oi)[K]) {
    uint32_t kk[K];
    int ii[K];
#pragma unroll
    for (int t = 0; t < K; ++t) ok[t] = kk[t] = kNoKey, oi[t] = ii[t] = -1;
    const int nMinCellX = max(0, (int)floorf((x - f.min_x - r) * f.invW));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - f.min_x + r) * f.invW));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - f.min_y - r) * f.invH));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - f.min_y + r) * f.invH));
    if (nMaxCellY < 0) return;
    // the window's columns are contiguous CSR runs; lane j < ncol holds column j's run, an inclusive scan
    // flattens them in GetFeaturesInArea order, and the lanes walk the flattened list 64 at a time (one
    // gather chain per 64 candidates instead of one per column)
    const int ncol = nMaxCellX - nMinCellX + 1;
    int cp0 = 0, clen = 0;
    if (lane < ncol) {
        const int ix = nMinCellX + lane;
        cp0 = cs[ix * kGridRows + nMinCellY];
        clen = cs[ix * kGridRows + nMaxCellY + 1] - cp0;
    }
    int incl = clen;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
    }
    const int excl = incl - clen, total = __shfl(incl, 63, 64);
    for (int base = 0; base < total; base += 64) {
        const int pos = base + lane;   // the shuffles run on the whole wavefront (uniform loop)
        int j = 0;
        for (int t = 1; t < ncol; ++t) j = __shfl(excl, t, 64) <= pos ? t : j;
        const int p = __shfl(cp0, j, 64) + pos - __shfl(excl, j, 64);
        if (pos >= total) continue;
        const int i2 = ci[p];
        const omv_kp k = kp2[i2];
        if (k.octave != 0) continue;   // levels [0, 0]
        if (!(fabsf(k.x - x) < r && fabsf(k.y - y) < r)) continue;
        uint64_t d2[4];
        load_desc(ds2 + (size_t)i2 * 32, d2);
        const int dist = omv::hamming256(d1, d2);
        if (mdist && mdist[i2] <= dist) continue;
        const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)pos;   // unique: distinct window positions
#pragma unroll
        for (int t = K - 1; t >= 0; --t)   // sorted insert (reads kk[t - 1] before step t - 1 writes it)
            if (kk[t] > key) {
                if (t > 0 && kk[t - 1] > key) kk[t] = kk[t - 1], ii[t] = ii[t - 1];
                else kk[t] = key, ii[t] = i2;
            }
    }
#pragma unroll
    for (int t = 0; t < K; ++t) {   // K rounds of wave minimum over the lanes' heads, the winner pops its head
        const uint32_t m = wave_min_u32(kk[0]);
        if (m == kNoKey) return;
        const int src = __ffsll((long long)__ballot(kk[0] == m)) - 1;
        ok[t] = m, oi[t] = __shfl(ii[0], src, 64);
        if (lane == src) {
#pragma unroll
            for (int u = 0; u + 1 < K; ++u) kk[u] = kk[u + 1], ii[u] = ii[u + 1];
            kk[K - 1] = kNoKey;
        }
    }
}

__global__ void __launch_bounds__(256) init_spec_kernel(InitArgs a) {
    const FrameArgs &f = a.f;
    const int cap = f.kp_cap, lane = threadIdx.x & 63, pr = blockIdx.y;
    const int i1 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t fc1 = (size_t)a.pairs[2 * pr] * f.n_cams, fc2 = (size_t)a.pairs[2 * pr + 1] * f.n_cams;   // block 0
    const int n1 = f.n_kp[fc1];
    if (i1 >= n1) return;   // wave-uniform
    uint32_t k[kInitSpec];
    int id[kInitSpec];
#pragma unroll
    for (int t = 0; t < kInitSpec; ++t) k[t] = kNoKey, id[t] = -1;
    const omv_kp k1 = f.kps[fc1 * cap + i1];
    if (k1.octave == 0) {
        const float *prev = a.prev + ((size_t)pr * cap + i1) * 2;
        uint64_t d1[4];
        load_desc(f.desc + (fc1 * cap + i1) * 32, d1);
        init_window_scan<kInitSpec>(f, f.cell_start + fc2 * (kCells + 1), f.cell_idx + fc2 * cap, f.kps + fc2 * cap,
                                    f.desc + fc2 * cap * 32, d1, prev[0], prev[1], (float)a.window, nullptr, lane, k, id);
    }
    if (lane == 0) {
        uint4 *o = a.spec + ((size_t)pr * cap + i1) * 4;
        o[0] = uint4{k[0], k[1], k[2], k[3]};
        o[1] = uint4{k[4], k[5], k[6], k[7]};
        o[2] = uint4{(uint32_t)id[0], (uint32_t)id[1], (uint32_t)id[2], (uint32_t)id[3]};
        o[3] = uint4{(uint32_t)id[4], (uint32_t)id[5], (uint32_t)id[6], (uint32_t)id[7]};
    }
}

__global__ void __launch_bounds__(64) init_kernel(InitArgs a) {
    extern __shared__ __attribute__((aligned(16))) int ism_raw[];
    const FrameArgs &f = a.f;
    const int cap = f.kp_cap, lane = threadIdx.x, pr = blockIdx.x;
    uint4 *sbuf = reinterpret_cast<uint4 *>(ism_raw);   // [kInitChunk][4] speculative keys of the current chunk
    int *ism = ism_raw + kInitChunk * 16;
    int *mdist = ism, *m21 = ism + cap, *m12 = ism + 2 * cap;
    int *acc2 = ism + 3 * cap;   // [n1] the F2 keypoint F1 keypoint i1 was accepted with (rotHist push), or -1
    int *cnt = ism + 4 * cap, *ind = cnt + 30;
    uint8_t *bins = reinterpret_cast<uint8_t *>(ind + 4);
    const size_t fc1 = (size_t)a.pairs[2 * pr] * f.n_cams, fc2 = (size_t)a.pairs[2 * pr + 1] * f.n_cams;   // block 0
    const int n1 = f.n_kp[fc1], n2 = f.n_kp[fc2];
    const omv_kp *kp1 = f.kps + fc1 * cap, *kp2 = f.kps + fc2 * cap;
    const uint8_t *ds1 = f.desc + fc1 * cap * 32, *ds2 = f.desc + fc2 * cap * 32;
    const int32_t *cs = f.cell_start + fc2 * (kCells + 1), *ci = f.cell_idx + fc2 * cap;
    float *prev = a.prev + (size_t)pr * cap * 2;
    const uint4 *spec = a.spec + (size_t)pr * cap * 4;
    for (int i = lane; i < n1; i += 64) m12[i] = -1, acc2[i] = -1, bins[i] = 0xff;
    for (int i = lane; i < n2; i += 64) mdist[i] = INT_MAX, m21[i] = -1;
    if (lane < 30) cnt[lane] = 0;
    __syncthreads();
    const float r = (float)a.window;
    int nm = 0;
    // the speculative keys are staged in LDS kInitChunk keypoints at a time (one global round trip per chunk,
    // not one per step of the walk's chain); the next keypoint's entry is read one step ahead
    auto stage = [&](int i0) {
        const int m = min(kInitChunk, n1 - i0) * 4;
        for (int q = lane; q < m; q += 64) sbuf[q] = spec[4 * i0 + q];
        wave_sync();
    };
    // lane t < kInitSpec holds key t and its F2 index; the checks against the claims are one LDS load per lane
    const uint32_t *sb = reinterpret_cast<const uint32_t *>(sbuf);
    const bool kl = lane < kInitSpec;
    uint32_t nkey = kNoKey;
    int nidx = -1;
    if (n1 > 0) {
        stage(0);
        if (kl) nkey = sb[lane], nidx = (int)sb[kInitSpec + lane];
    }
    for (int i1 = 0; i1 < n1; ++i1) {
        const uint32_t mykey = nkey;
        const int myidx = nidx;
        if (i1 + 1 < n1) {
            const int c = (i1 + 1) & (kInitChunk - 1);
            if (c == 0) stage(i1 + 1);
            if (kl) nkey = sb[16 * c + lane], nidx = (int)sb[16 * c + kInitSpec + lane];
        }
        // no candidate without the filter: none with it (or not level 0 / off-grid)
        if ((uint32_t)__builtin_amdgcn_readfirstlane(mykey) == kNoKey) continue;
        // the filtered best and second are the two smallest keys the claims leave; known unless fewer than two of
        // the kept keys survive while more candidates may lie beyond them
        int md = 0, mo = -1;
        if (kl && mykey != kNoKey) md = mdist[myidx], mo = m21[myidx];
        const uint64_t ok = __ballot(kl && mykey != kNoKey && md > (int)(mykey >> 16));
        uint32_t g[2] = {kNoKey, kNoKey};
        int bi[2] = {-1, -1}, old = -1;
        if (ok) {
            const int t0 = __ffsll((long long)ok) - 1;
            g[0] = (uint32_t)__builtin_amdgcn_readlane((int)mykey, t0);
            bi[0] = __builtin_amdgcn_readlane(myidx, t0), old = __builtin_amdgcn_readlane(mo, t0);
            const uint64_t rest = ok & (ok - 1);
            if (rest) g[1] = (uint32_t)__builtin_amdgcn_readlane((int)mykey, __ffsll((long long)rest) - 1);
        }
        const int found = __popcll(ok);
        if (found < 2 && (uint32_t)__builtin_amdgcn_readlane((int)mykey, kInitSpec - 1) != kNoKey) {   // filtered scan
            uint64_t d1[4];
            load_desc(ds1 + (size_t)i1 * 32, d1);
            init_window_scan<2>(f, cs, ci, kp2, ds2, d1, prev[2 * i1], prev[2 * i1 + 1], r, mdist, lane, g, bi);
            if (g[0] != kNoKey) old = m21[bi[0]];
        }
        if (g[0] == kNoKey) continue;
        const int bestIdx2 = bi[0], bestDist = (int)(g[0] >> 16), bestDist2 = g[1] == kNoKey ? INT_MAX : (int)(g[1] >> 16);
        if (bestDist <= 50 && (float)bestDist < (float)bestDist2 * a.nnratio) {
            if (old >= 0) --nm;
            ++nm;
            if (lane == 0) {
                if (old >= 0) m12[old] = -1;
                m12[i1] = bestIdx2, m21[bestIdx2] = i1, mdist[bestIdx2] = bestDist, acc2[i1] = bestIdx2;
            }
        }
        wave_sync();   // the claim state before the next F1 keypoint (one wavefront, LDS only)
    }
    if (a.check_ori) {   // ComputeThreeMaxima, then every push outside the top bins that is still matched
        // the rotation histogram of every accept (each F1 keypoint is accepted at most once, so its bin is a
        // function of (i1, acc2[i1]); the counts do not depend on the push order): off the walk's chain
        for (int i = lane; i < n1; i += 64) {
            const int j = acc2[i];
            if (j < 0) continue;
            float rot = kp1[i].angle - kp2[j].angle;   // rot = angle1 - angle2, +360 if negative
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * (1.0f / 30));   // bin = round(rot / 30), 30 -> 0
            if (bin == 30) bin = 0;
            bins[i] = (uint8_t)bin;
            atomicAdd(cnt + bin, 1);
        }
        __syncthreads();
        if (lane == 0) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < 30; i++) {
                const int s = cnt[i];
                if (s > max1) {
                    max3 = max2, max2 = max1, max1 = s;
                    ind3 = ind2, ind2 = ind1, ind1 = i;
                } else if (s > max2) {
                    max3 = max2, max2 = s;
                    ind3 = ind2, ind2 = i;
                } else if (s > max3) {
                    max3 = s;
                    ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                ind2 = -1, ind3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                ind3 = -1;
            }
            ind[0] = ind1, ind[1] = ind2, ind[2] = ind3;
        }
        __syncthreads();
        int removed = 0;
        for (int i = lane; i < n1; i += 64) {
            const int bn = bins[i];
            if (bn != 0xff && bn != ind[0] && bn != ind[1] && bn != ind[2] && m12[i] >= 0) m12[i] = -1, ++removed;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) removed += __shfl_xor(removed, d, 64);
        nm -= removed;
        __syncthreads();
    }
    int32_t *out = a.m12 + (size_t)pr * cap;
    for (int i = lane; i < n1; i += 64) {
        const int m = m12[i];
        out[i] = m;
        if (m >= 0) prev[2 * i] = kp2[m].x, prev[2 * i + 1] = kp2[m].y;   // vbPrevMatched update
    }
    if (lane == 0) a.n_matches[pr] = nm;
}

}  // namespace

// =============================================================================================
struct omv_matcher {
    int max_frames, n_cams, kp_cap, max_mps;
    int32_t *d_cell_start = nullptr, *d_cell_idx = nullptr;
    Rec *d_recs = nullptr;
    int *d_counts = nullptr;
    int *d_flags = nullptr;   // per (frame, point): in_view bits | skip | has_obs (cand -> resolve)
    int2 *d_push = nullptr;   // SearchByProjection(last frame): (slot, rotation bin) per claim, in order
    float4 *d_geo = nullptr;  // keyframe searches: per entry window geometry (claim-mode rescans)
    size_t geo_cap = 0;
    omv_kf_search_job *d_jobs = nullptr;
    size_t jobs_cap = 0;
    int *d_npush = nullptr;
    size_t push_cap = 0;
    int32_t *d_knn_i = nullptr, *d_knn_d = nullptr;
    int *d_err = nullptr;
    FrameArgs f{};
    hipStream_t last = nullptr;
    // optional per-stage HIP-event timing: 0 grid, 1 stereo knn, 2 candidates, 3 resolve
    bool timing = false;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev;
    double stage_ms[4] = {0, 0, 0, 0};
    omv::MatcherKnobs knobs;   // test knobs, read from the environment once at creation
};

omv::MatcherKnobs omv::matcher_knobs(const omv_matcher *m) { return m ? m->knobs : omv::MatcherKnobs{}; }
size_t omv::matcher_kf_entry_cap(const omv_matcher *m) {
    return m ? (size_t)m->max_frames * m->n_cams * std::max(1, m->max_mps) : 0;
}

static hipEvent_t mk_event(hipStream_t st) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    (void)hipEventRecord(e, st);
    return e;
}

// Camera types of the first n entries: KB8 or Pinhole only (tri / lba / pose reject anything else the same way).
static bool cam_models_ok(const int *models, int n) {
    for (int c = 0; c < n; ++c)
        if (models[c] != OMV_CAM_KB8 && models[c] != OMV_CAM_PINHOLE) return false;
    return true;
}

static void fill_frame(omv_matcher *h, const omv_frame_geom *g, const omv_kp *kps, const uint8_t *desc, const int *n_kp,
                       FrameArgs &f) {
    f.n_cams = h->n_cams;
    f.kp_cap = h->kp_cap;
    f.nlevels = g->nlevels;
    f.min_x = g->min_x, f.max_x = g->max_x, f.min_y = g->min_y, f.max_y = g->max_y;
    f.invW = (float)kGridCols / (g->max_x - g->min_x);   // Frame.cc:1878-1879
    f.invH = (float)kGridRows / (g->max_y - g->min_y);
    for (int l = 0; l < 16; ++l) f.scale[l] = g->scale_factors[l];
    for (int c = 0; c < 8; ++c) f.model[c] = g->cam_model[c];
    f.kps = kps, f.desc = desc, f.n_kp = n_kp;
    f.cell_start = h->d_cell_start, f.cell_idx = h->d_cell_idx;
}

// resolve workspace (dynamic LDS): blocked / initially-occupied bitmaps, the per-slot owner word, l2r / r2l, the
// per-point stop camera and, when it fits, the frame's assignment (*lds_k2m = 1)
constexpr size_t kResolveStaticLds = 4 * ((size_t)kMaxDomains * (2 * kListCap + kMaxRevived + 2) + 1);
static size_t resolve_lds_bytes(int C, int cap, int M, int *lds_k2m = nullptr) {
    const size_t S = (size_t)C * cap;
    const size_t b = sizeof(uint32_t) * 2 * ((S + 31) / 32) + sizeof(int) * S + 2 * sizeof(int32_t) * cap + ((size_t)M + 3) / 4 * 4;
    const size_t with_k2m = b + sizeof(int32_t) * S;
    const bool fits = with_k2m + kResolveStaticLds <= kResolveLds;
    if (lds_k2m) *lds_k2m = fits;
    return fits ? with_k2m : b;
}
static size_t lf_resolve_lds_bytes(int C, int cap) {
    const size_t S = (size_t)C * cap;
    return sizeof(uint32_t) * ((S + 31) / 32) + sizeof(int) * S;
}

extern "C" {

omv_status omv_frustum(int n_frames, const omv_frame_pose *poses, const omv_rig *rig, const omv_mp_world *mp, int M,
                       float viewing_cos_limit, const omv_mp_track *out, int32_t *n_in_view, void *stream) {
    if (n_frames <= 0 || !poses || !rig || !mp || !out || M < 0 || rig->n_cams <= 0 || rig->n_cams > kMaxCams ||
        rig->n_levels <= 0 || !cam_models_ok(rig->model, rig->n_cams))
        return OMV_ERR_ARG;
    if (M == 0) return OMV_OK;
    hipStream_t st = (hipStream_t)stream;
    frustum_kernel<<<dim3((M + 255) / 256, n_frames), 256, 0, st>>>(poses, *rig, *mp, M, viewing_cos_limit, *out,
                                                                    n_in_view);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_matcher_create(int max_frames, int n_cams, int kp_cap, int max_mps, omv_matcher **out) {
    if (!out || max_frames <= 0 || n_cams <= 0 || n_cams > kMaxCams || kp_cap <= 0 || kp_cap > 65535 || max_mps < 0)
        return OMV_ERR_ARG;
    if (resolve_lds_bytes(n_cams, kp_cap, max_mps) > kResolveLds - kResolveStaticLds || lf_resolve_lds_bytes(n_cams, kp_cap) > kResolveLds)
        return OMV_ERR_ARG;   // resolve workspaces must fit LDS
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return OMV_ERR_NO_DEVICE;
    const int resolve_dyn = (int)(kResolveLds - kResolveStaticLds);
    HIP_OK(hipFuncSetAttribute((const void *)resolve_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, resolve_dyn));
    HIP_OK(hipFuncSetAttribute((const void *)resolve_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, resolve_dyn));
    HIP_OK(hipFuncSetAttribute((const void *)lf_resolve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResolveLds));
    HIP_OK(hipFuncSetAttribute((const void *)cand_stage_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStageLdsMax));
    omv_matcher *h = new omv_matcher();
    h->max_frames = max_frames, h->n_cams = n_cams, h->kp_cap = kp_cap, h->max_mps = max_mps;
    if (const char *e = getenv("OMV_BOW_TOP")) h->knobs.bow_top = atoi(e);
    if (const char *e = getenv("OMV_TRI_SLICES")) h->knobs.tri_slices = atoi(e);
    if (const char *e = getenv("OMV_TRI_ECAP")) h->knobs.tri_ecap = atoi(e);
    if (const char *e = getenv("OMV_TRI_WALK")) h->knobs.tri_walk_seq = strcmp(e, "seq") == 0 ? 1 : 0;
    if (const char *e = getenv("OMV_CAND")) h->knobs.cand_mode = strcmp(e, "global") == 0 ? 1 : strcmp(e, "lds") == 0 ? 2 : 0;
    if (const char *e = getenv("OMV_CAND_PW")) h->knobs.cand_pw = atoi(e);
    const size_t fc = (size_t)max_frames * n_cams;
    HIP_OK(hipMalloc(&h->d_cell_start, sizeof(int32_t) * fc * (kCells + 1)));
    HIP_OK(hipMalloc(&h->d_cell_idx, sizeof(int32_t) * fc * kp_cap));
    HIP_OK(hipMalloc(&h->d_recs, sizeof(Rec) * std::max<size_t>(1, fc * max_mps)));
    HIP_OK(hipMalloc(&h->d_counts, sizeof(int) * std::max<size_t>(1, fc * max_mps)));
    HIP_OK(hipMalloc(&h->d_flags, sizeof(int) * std::max<size_t>(1, (size_t)max_frames * max_mps)));
    HIP_OK(hipMalloc(&h->d_knn_i, sizeof(int32_t) * 2 * max_frames * kp_cap));
    HIP_OK(hipMalloc(&h->d_knn_d, sizeof(int32_t) * 2 * max_frames * kp_cap));
    HIP_OK(hipMalloc(&h->d_err, sizeof(int)));
    HIP_OK(hipMemset(h->d_err, 0, sizeof(int)));
    *out = h;
    return OMV_OK;
}

omv_status omv_matcher_enable_timing(omv_matcher *h, int on) {
    if (!h) return OMV_ERR_ARG;
    h->timing = on != 0;
    return OMV_OK;
}

omv_status omv_matcher_stage_ms(omv_matcher *h, double *ms4, int reset) {
    if (!h || !ms4) return OMV_ERR_ARG;
    HIP_OK(hipStreamSynchronize(h->last));
    for (auto &p : h->ev) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, p.second.first, p.second.second);
        h->stage_ms[p.first] += ms;
        (void)hipEventDestroy(p.second.first);
        (void)hipEventDestroy(p.second.second);
    }
    h->ev.clear();
    for (int k = 0; k < 4; ++k) ms4[k] = h->stage_ms[k];
    if (reset)
        for (int k = 0; k < 4; ++k) h->stage_ms[k] = 0;
    return OMV_OK;
}

omv_status omv_matcher_last_error(omv_matcher *h) {
    if (!h) return OMV_ERR_ARG;
    HIP_OK(hipStreamSynchronize(h->last));
    int e = 0;
    HIP_OK(hipMemcpy(&e, h->d_err, sizeof(int), hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(h->d_err, 0, sizeof(int)));
    return e;
}

omv_status omv_matcher_destroy(omv_matcher *h) {
    if (!h) return OMV_ERR_ARG;
    void *p[] = {h->d_cell_start, h->d_cell_idx, h->d_recs, h->d_counts, h->d_flags, h->d_knn_i, h->d_knn_d, h->d_err,
                 h->d_push, h->d_npush, h->d_geo, h->d_jobs};
    for (void *q : p)
        if (q) (void)hipFree(q);
    delete h;
    return OMV_OK;
}

omv_status omv_matcher_assign_grid(omv_matcher *h, int n_frames, const omv_frame_geom *g, const omv_kp *kps,
                                   const int *n_kp, void *stream) {
    if (!h || !g || !kps || !n_kp || n_frames <= 0 || n_frames > h->max_frames || g->n_cams != h->n_cams)
        return OMV_ERR_ARG;
    FrameArgs f;
    if (!cam_models_ok(g->cam_model, h->n_cams)) return OMV_ERR_ARG;
    fill_frame(h, g, kps, nullptr, n_kp, f);
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    hipEvent_t e0 = h->timing ? mk_event(st) : nullptr;
    grid_kernel<<<n_frames * h->n_cams, 256, 0, st>>>(f, h->d_cell_start, h->d_cell_idx);
    if (h->timing) h->ev.push_back({0, {e0, mk_event(st)}});
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_matcher_grid_debug(omv_matcher *h, int frame, int cam, int32_t *cell_start, int32_t *idx) {
    if (!h || frame < 0 || frame >= h->max_frames || cam < 0 || cam >= h->n_cams) return OMV_ERR_ARG;
    HIP_OK(hipStreamSynchronize(h->last));
    const size_t fc = (size_t)frame * h->n_cams + cam;
    HIP_OK(hipMemcpy(cell_start, h->d_cell_start + fc * (kCells + 1), sizeof(int32_t) * (kCells + 1),
                     hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(idx, h->d_cell_idx + fc * h->kp_cap, sizeof(int32_t) * h->kp_cap, hipMemcpyDeviceToHost));
    return OMV_OK;
}

omv_status omv_matcher_search_projection(omv_matcher *h, int n_frames, const omv_frame_geom *g, const omv_kp *kps,
                                         const uint8_t *desc, const int *n_kp, const omv_mp_view *mps, int M, float th,
                                         int far_points, float th_far, float nnratio, const int32_t *l2r,
                                         const int32_t *r2l, const uint8_t *kp_occ_init, int32_t *kp_to_mp,
                                         int *n_matches, void *stream) {
    if (!h || !g || !kps || !desc || !n_kp || !mps || !kp_to_mp || !n_matches || n_frames <= 0 ||
        n_frames > h->max_frames || M < 0 || M > h->max_mps || g->n_cams != h->n_cams)
        return OMV_ERR_ARG;
    if (h->n_cams > 1 && (!l2r || !r2l)) return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    FrameArgs f;
    if (!cam_models_ok(g->cam_model, h->n_cams)) return OMV_ERR_ARG;
    fill_frame(h, g, kps, desc, n_kp, f);
    MpArgs m{mps->desc, mps->proj_x, mps->proj_y, mps->view_cos, mps->level, mps->in_view, mps->track_depth,
             mps->is_bad, mps->has_obs, M};
    hipEvent_t e0 = h->timing ? mk_event(st) : nullptr;
    if (M > 0) {
        const long long tot = (long long)n_frames * M * h->n_cams;
        // LDS-staged candidates: map points per wave as large as keeps >= ~1,024 workgroups (at least 16)
        int pw = 128;
        while (pw > 16 && (long long)n_frames * h->n_cams * ((M + 8 * pw - 1) / (8 * pw)) < 1024) pw >>= 1;
        if (h->knobs.cand_pw > 0) pw = min(h->knobs.cand_pw, 64 * kStageMaxIt);
        // staged for batches (throughput); a frame or a few keep cand_kernel<8>, whose 8 lanes per window cut the
        // longest window's chain, which sets a small launch's time (measured: B=1 51 us vs 70 us staged)
        const bool staged = h->knobs.cand_mode == 2 || (h->knobs.cand_mode == 0 && tot > 262144);
        if (staged && stage_lds_bytes(h->kp_cap, pw) <= kStageLdsMax) {
            const int n_chunks = (M + 8 * pw - 1) / (8 * pw);
            const int nb = n_frames * h->n_cams * n_chunks;
            cand_stage_kernel<<<omv::xcd_grid(nb), kStageThreads, stage_lds_bytes(h->kp_cap, pw), st>>>(
                f, m, n_frames, th, kp_occ_init, h->d_recs, h->d_counts, h->d_flags, far_points, th_far, n_chunks, pw, nb);
        } else if (tot <= 65536) {   // a frame or two: 16 lanes per window (the longest window sets the time)
            const int nb = (int)((tot + 4 * (kCandChunk / 16) - 1) / (4 * (kCandChunk / 16)));
            cand_kernel<16><<<omv::xcd_grid(nb), 256, 0, st>>>(f, m, n_frames, th, kp_occ_init, h->d_recs, h->d_counts,
                                                               h->d_flags, far_points, th_far, nb);
        } else if (tot <= 262144) {   // up to ~10 frames: spread each window over 8 lanes so the launch fills the chip
            const int nb = (int)((tot + 4 * (kCandChunk / 8) - 1) / (4 * (kCandChunk / 8)));
            cand_kernel<8><<<omv::xcd_grid(nb), 256, 0, st>>>(f, m, n_frames, th, kp_occ_init, h->d_recs, h->d_counts,
                                                              h->d_flags, far_points, th_far, nb);
        } else {
            const int nb = (int)((tot + 4 * kCandChunk - 1) / (4 * kCandChunk));
            cand_kernel<1><<<omv::xcd_grid(nb), 256, 0, st>>>(f, m, n_frames, th, kp_occ_init, h->d_recs, h->d_counts,
                                                              h->d_flags, far_points, th_far, nb);
        }
    }
    hipEvent_t e1 = h->timing ? mk_event(st) : nullptr;
    hipEvent_t e2 = h->timing ? mk_event(st) : nullptr;   // own start event: every event is destroyed once
    int staged = 1;   // the assignment fits in LDS
    const size_t lds = resolve_lds_bytes(h->n_cams, h->kp_cap, M, &staged);
    ResolveArgs ra{f, m, h->d_recs, h->d_counts, h->d_flags, l2r, r2l, kp_occ_init, kp_to_mp, n_matches, h->d_err, th, th_far, nnratio,
                   far_points, staged};
    const int n_dom = 1 + max(0, h->n_cams - 2);   // one wavefront per claim domain
    if (staged)
        resolve_kernel<true><<<n_frames, 64 * n_dom, lds, st>>>(ra);
    else
        resolve_kernel<false><<<n_frames, 64 * n_dom, lds, st>>>(ra);
    if (h->timing) {
        h->ev.push_back({2, {e0, e1}});
        h->ev.push_back({3, {e2, mk_event(st)}});
    }
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_matcher_search_last_frame(omv_matcher *h, int n_frames, const omv_frame_geom *g, const omv_kp *kps,
                                         const uint8_t *desc, const int *n_kp, const float *cams, const omv_se3f *Tcw,
                                         const omv_se3f *Tlw, const omv_se3f *Trl, const omv_last_frame *last, float th,
                                         int bMono, float mb, int check_ori, const uint8_t *kp_occ_init,
                                         int32_t *kp_to_mp, int32_t *n_matches, void *stream) {
    if (!h || !g || !kps || !desc || !n_kp || !cams || !Tcw || !Tlw || !last || !kp_to_mp || !n_matches ||
        n_frames <= 0 || n_frames > h->max_frames || g->n_cams != h->n_cams || last->S < 0 || last->S > h->max_mps ||
        (h->n_cams > 1 && !Trl))
        return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    FrameArgs f;
    if (!cam_models_ok(g->cam_model, h->n_cams)) return OMV_ERR_ARG;
    fill_frame(h, g, kps, desc, n_kp, f);
    LastArgs L{last->pos, last->desc, last->valid, last->has_obs, last->kps, last->S};
    LfGeo G{};
    for (int q = 0; q < 8; ++q) G.cam0[q] = cams[q];
    if (Trl) G.Trl = *Trl;
    G.th = th, G.mb = mb, G.bMono = bMono;
    const int C = h->n_cams;
    const size_t per_frame = (size_t)std::max(1, last->S) * C;
    if (h->push_cap < per_frame * n_frames) {
        if (h->d_push) (void)hipFree(h->d_push);
        if (h->d_npush) (void)hipFree(h->d_npush);
        HIP_OK(hipMalloc(&h->d_push, sizeof(int2) * per_frame * n_frames));
        HIP_OK(hipMalloc(&h->d_npush, sizeof(int) * h->max_frames));
        h->push_cap = per_frame * n_frames;
    }
    if (last->S > 0) {
        const long long tot = (long long)n_frames * last->S * C;
        lf_cand_kernel<<<(int)((tot + 255) / 256), 256, 0, st>>>(f, L, G, Tcw, Tlw, n_frames, kp_occ_init, h->d_recs,
                                                                 h->d_counts);
    }
    LfResolveArgs ra{f, L, G, Tcw, Tlw, h->d_recs, h->d_counts, kp_occ_init, kp_to_mp, n_matches, h->d_push, h->d_npush,
                     check_ori};
    const int S = C * h->kp_cap;
    lf_resolve_kernel<<<n_frames, 64, lf_resolve_lds_bytes(C, h->kp_cap), st>>>(ra);
    if (check_ori) lf_histo_kernel<<<n_frames, 256, 0, st>>>(h->d_push, h->d_npush, (int)per_frame, S, kp_to_mp, n_matches);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_matcher_search_kf(omv_matcher *h, int n_kf, const omv_frame_geom *g, const omv_kp *kps,
                                 const uint8_t *desc, const int *n_kp, int n_jobs, const omv_kf_search_job *jobs,
                                 int n_entries, const int32_t *mp_list, const omv_kf_mps *mps,
                                 const omv_kf_search_params *p, int32_t *kp_match, int32_t *best_idx,
                                 int32_t *best_dist, int32_t *n_matches, void *stream) {
    if (!h || !g || !kps || !desc || !n_kp || !mps || !p || n_kf <= 0 || n_kf > h->max_frames ||
        g->n_cams != h->n_cams || n_jobs < 0 || n_entries < 0 || (n_jobs > 0 && (!jobs || !n_matches)) ||
        (n_entries > 0 && (!mp_list || !best_idx || !best_dist || !mps->pos || !mps->desc || !mps->min_dist ||
                           !mps->max_dist || !mps->normal)))
        return OMV_ERR_ARG;
    if (p->mode < OMV_KF_FUSE || p->mode > OMV_KF_SBP_FRAME || p->n_levels <= 0 || p->n_levels > 16) return OMV_ERR_ARG;
    const bool claim = p->mode == OMV_KF_SBP_SIM3 || p->mode == OMV_KF_SBP_FRAME;
    if ((claim && !kp_match) || (p->mode == OMV_KF_FUSE && !p->uright) ||
        (p->mode == OMV_KF_SBP_FRAME && p->check_ori && n_entries > 0 && !p->mp_angle))
        return OMV_ERR_ARG;
    int next = 0;   // jobs must tile mp_list in order, name a keyframe of the batch and one of its blocks
    for (int j = 0; j < n_jobs; ++j) {
        const omv_kf_search_job &J = jobs[j];
        if (J.kf < 0 || J.kf >= n_kf || J.cam < 0 || J.cam >= h->n_cams || J.mp_start != next || J.mp_count < 0)
            return OMV_ERR_ARG;
        if (p->mode == OMV_KF_SBP_FRAME && J.cam != 0) return OMV_ERR_ARG;   // CurrentFrame.mpCamera, left grid
        next += J.mp_count;
    }
    if (next != n_entries || !cam_models_ok(g->cam_model, h->n_cams)) return OMV_ERR_ARG;
    if ((size_t)n_entries > (size_t)h->max_frames * h->n_cams * std::max(1, h->max_mps)) return OMV_ERR_CAPACITY;
    if (n_jobs == 0) return OMV_OK;
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    if (h->jobs_cap < (size_t)n_jobs) {
        if (h->d_jobs) (void)hipFree(h->d_jobs);
        h->d_jobs = nullptr, h->jobs_cap = 0;
        HIP_OK(hipMalloc(&h->d_jobs, sizeof(omv_kf_search_job) * n_jobs));
        h->jobs_cap = n_jobs;
    }
    if (claim && h->geo_cap < (size_t)std::max(1, n_entries)) {
        if (h->d_geo) (void)hipFree(h->d_geo);
        h->d_geo = nullptr, h->geo_cap = 0;
        HIP_OK(hipMalloc(&h->d_geo, sizeof(float4) * std::max(1, n_entries)));
        h->geo_cap = std::max(1, n_entries);
    }
    HIP_OK(hipMemcpyAsync(h->d_jobs, jobs, sizeof(omv_kf_search_job) * n_jobs, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(n_matches, 0, sizeof(int32_t) * n_jobs, st));
    KfArgs a{};
    fill_frame(h, g, kps, desc, n_kp, a.f);
    a.jobs = h->d_jobs, a.n_jobs = n_jobs, a.n_kf = n_kf;
    a.mp_list = mp_list, a.n_entries = n_entries, a.mps = *mps;
    a.mode = p->mode, a.check_ori = p->check_ori;
    a.th = p->th, a.max_dist = p->max_dist, a.bf = p->bf, a.uright = p->uright;
    for (int l = 0; l < 16; ++l) a.invs2[l] = p->inv_level_sigma2[l];
    a.log_scale = p->log_scale_factor, a.n_levels = p->n_levels;
    for (int c = 0; c < h->n_cams; ++c)
        for (int q = 0; q < 8; ++q) a.cams[c][q] = p->cams[c][q];
    a.mp_angle = p->mp_angle;
    a.kp_match = kp_match, a.best_idx = best_idx, a.best_dist = best_dist, a.n_matches = n_matches;
    a.recs = h->d_recs, a.counts = h->d_counts, a.geo = h->d_geo;
    if (n_entries > 0) kf_cand_kernel<<<(n_entries + 255) / 256, 256, 0, st>>>(a);
    if (claim) {
        const size_t lds = sizeof(uint32_t) * (((size_t)h->n_cams * h->kp_cap + 31) / 32);
        kf_resolve_kernel<<<n_kf, 64, lds, st>>>(a);
    }
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_matcher_search_by_sim3(omv_matcher *h, int n_kf, const omv_frame_geom *g, const omv_kp *kps,
                                      const uint8_t *desc, const int *n_kp, int n_jobs, const omv_sim3_job *jobs,
                                      int n1, const int32_t *kp1, const int32_t *mp1, int n2, const int32_t *kp2,
                                      const int32_t *mp2, const omv_kf_mps *mps, float th, float log_scale_factor,
                                      int n_levels, int32_t *match12, int32_t *n_found, void *stream) {
    if (!h || !g || !kps || !desc || !n_kp || !mps || n_kf <= 0 || n_kf > h->max_frames || g->n_cams != h->n_cams ||
        n_jobs < 0 || n1 < 0 || n2 < 0 || (n_jobs > 0 && (!jobs || !n_found)) || (n1 > 0 && (!kp1 || !mp1 || !match12)) ||
        (n2 > 0 && (!kp2 || !mp2)) || ((n1 + n2) > 0 && (!mps->pos || !mps->desc || !mps->min_dist || !mps->max_dist)) ||
        n_levels <= 0 || n_levels > 16)
        return OMV_ERR_ARG;
    int next1 = 0, next2 = 0;   // runs tile both lists in order; keyframes of the batch
    for (int j = 0; j < n_jobs; ++j) {
        const omv_sim3_job &J = jobs[j];
        if (J.kf1 < 0 || J.kf1 >= n_kf || J.kf2 < 0 || J.kf2 >= n_kf || J.start1 != next1 || J.count1 < 0 ||
            J.start2 != next2 || J.count2 < 0)
            return OMV_ERR_ARG;
        next1 += J.count1, next2 += J.count2;
    }
    if (next1 != n1 || next2 != n2) return OMV_ERR_ARG;
    if (!cam_models_ok(g->cam_model, h->n_cams)) return OMV_ERR_ARG;
    if (n_jobs == 0) return OMV_OK;
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    const int N = h->n_cams * h->kp_cap;
    const size_t job_b = ((sizeof(omv_sim3_job) * n_jobs + 255) / 256) * 256;
    const size_t vn1_b = ((sizeof(int32_t) * std::max(1, n1) + 255) / 256) * 256;
    const size_t vn2_b = sizeof(int32_t) * (size_t)n_jobs * N;
    uint8_t *buf = nullptr;
    HIP_OK(hipMallocAsync((void **)&buf, job_b + vn1_b + vn2_b, st));
    Sim3Args a{};
    fill_frame(h, g, kps, desc, n_kp, a.f);
    a.jobs = reinterpret_cast<const omv_sim3_job *>(buf);
    a.n_jobs = n_jobs, a.n1 = n1, a.n2 = n2, a.N = N;
    a.kp1 = kp1, a.mp1 = mp1, a.kp2 = kp2, a.mp2 = mp2, a.mps = *mps;
    a.th = th, a.log_scale = log_scale_factor, a.n_levels = n_levels;
    a.vn1 = reinterpret_cast<int32_t *>(buf + job_b);
    a.vn2 = reinterpret_cast<int32_t *>(buf + job_b + vn1_b);
    a.match12 = match12, a.n_found = n_found;
    HIP_OK(hipMemcpyAsync(buf, jobs, sizeof(omv_sim3_job) * n_jobs, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(a.vn2, 0xff, vn2_b, st));
    HIP_OK(hipMemsetAsync(n_found, 0, sizeof(int32_t) * n_jobs, st));
    if (n1 + n2 > 0) sbs3_cand_kernel<<<(n1 + n2 + 255) / 256, 256, 0, st>>>(a);
    if (n1 > 0) sbs3_agree_kernel<<<(n1 + 255) / 256, 256, 0, st>>>(a);
    HIP_OK(hipGetLastError());
    HIP_OK(hipFreeAsync(buf, st));
    return OMV_OK;
}

omv_status omv_bf_knn2(int n_pairs, const uint8_t *query, int q_cap, const int *nq, const uint8_t *train, int t_cap,
                       const int *nt, int32_t *idx2, int32_t *dist2, void *stream) {
    if (n_pairs <= 0 || !query || !train || !nq || !nt || !idx2 || !dist2 || q_cap <= 0 || t_cap <= 0)
        return OMV_ERR_ARG;
    KnnArgs a{query, train, (long long)q_cap * 32, (long long)t_cap * 32, nq, nt, nullptr, nullptr, 1, idx2, dist2, q_cap};
    launch_knn2(a, n_pairs, q_cap, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_matcher_stereo_lapping(omv_matcher *h, int n_frames, const uint8_t *desc, const int *n_kp,
                                      const int *mono, double ratio, int32_t *l2r, int32_t *r2l, void *stream) {
    if (!h || h->n_cams < 2 || !desc || !n_kp || !mono || !l2r || !r2l || n_frames <= 0 || n_frames > h->max_frames)
        return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    const int cap = h->kp_cap, C = h->n_cams;
    hipEvent_t e0 = h->timing ? mk_event(st) : nullptr;
    HIP_OK(hipMemsetAsync(r2l, 0xff, sizeof(int32_t) * n_frames * cap, st));   // l2r: written whole by stereo_pairs
    // query = camera 0 rows [mono0, n0), train = camera 1 rows [mono1, n1)
    KnnArgs a{desc, desc + (size_t)cap * 32, (long long)C * cap * 32, (long long)C * cap * 32, n_kp, n_kp + 1,
              mono, mono + 1, C, h->d_knn_i, h->d_knn_d, cap};
    launch_knn2(a, n_frames, cap, st);
    dim3 g2((cap + 255) / 256, n_frames);
    stereo_pairs_kernel<<<g2, 256, 0, st>>>(h->d_knn_i, h->d_knn_d, cap, n_kp, mono, C, cap, ratio, l2r, r2l, n_frames);
    if (h->timing) h->ev.push_back({1, {e0, mk_event(st)}});
    HIP_OK(hipGetLastError());
    return OMV_OK;
}


omv_status omv_matcher_search_for_initialization(omv_matcher *h, int n_pairs, const int32_t *pairs,
                                                 const omv_frame_geom *g, const omv_kp *kps, const uint8_t *desc,
                                                 const int *n_kp, float *prev_matched, int window, float nnratio,
                                                 int check_ori, int32_t *matches12, int32_t *n_matches, void *stream) {
    if (!h || n_pairs < 0 || (n_pairs > 0 && (!pairs || !g || !kps || !desc || !n_kp || !prev_matched || !matches12 ||
                                              !n_matches)) ||
        g->n_cams != h->n_cams || window < 0)
        return OMV_ERR_ARG;
    if (n_pairs == 0) return OMV_OK;
    for (int i = 0; i < 2 * n_pairs; ++i)
        if (pairs[i] < 0 || pairs[i] >= h->max_frames) return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    h->last = st;
    FrameArgs f;
    if (!cam_models_ok(g->cam_model, h->n_cams)) return OMV_ERR_ARG;
    fill_frame(h, g, kps, desc, n_kp, f);
    const size_t lds = init_lds_bytes(h->kp_cap);
    if (lds > 160 * 1024) return OMV_ERR_CAPACITY;
    HIP_OK(hipFuncSetAttribute((const void *)init_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int32_t *d_pairs = nullptr;
    HIP_OK(hipMallocAsync((void **)&d_pairs, sizeof(int32_t) * 2 * n_pairs, st));
    HIP_OK(hipMemcpyAsync(d_pairs, pairs, sizeof(int32_t) * 2 * n_pairs, hipMemcpyHostToDevice, st));
    uint4 *d_spec = nullptr;
    HIP_OK(hipMallocAsync((void **)&d_spec, sizeof(uint4) * 4 * (size_t)n_pairs * h->kp_cap, st));
    InitArgs ia{f, d_pairs, prev_matched, window, nnratio, check_ori, matches12, n_matches, d_spec};
    init_spec_kernel<<<dim3((h->kp_cap + 3) / 4, n_pairs), 256, 0, st>>>(ia);
    init_kernel<<<n_pairs, 64, lds, st>>>(ia);
    HIP_OK(hipGetLastError());
    HIP_OK(hipFreeAsync(d_spec, st));
    HIP_OK(hipFreeAsync(d_pairs, st));
    return OMV_OK;
}

}  // extern "C"
