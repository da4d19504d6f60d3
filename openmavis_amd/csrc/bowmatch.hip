// MI355X-native ORBmatcher::SearchByBoW (src/ORBmatcher.cc:349-666 for (KeyFrame, Frame), :1006-1129 for
// (KeyFrame, KeyFrame)): Hamming matching of the keypoints that share a DBoW2 FeatureVector node, in the
// reference's sequential order (common node ids ascending, keyframe keypoints in node order), with the
// claims of earlier keyframe keypoints, the per-camera-block best / second and the rotation-consistency
// filter (ComputeThreeMaxima, :2537-2573).
//
// Two launches.  bow_cand_kernel, one thread per keyframe keypoint (position in its FeatureVector CSR): the
// node's candidates in the other view under the static filters (block ranges, map points, idx < N), their
// distances, and per camera block the kTop best by (distance, node position) -- the order the reference's
// strict `<` update ranks them.  bow_resolve_kernel, one wavefront per job: the reference's sequential walk
// (common nodes ascending = the keyframe CSR order), where only the claims of earlier keyframe keypoints can
// change a pick: the first two unclaimed entries of each block are its best and second, and a block whose
// short list runs out while it holds more candidates is rescanned on the wave.  The walk runs in batches of
// 64 / NB keypoints picked in parallel against the batch-start claims; the prefix before the first keypoint
// whose examined entries an earlier batch keypoint claims commits at once (that keypoint is then walked alone):
// 1.5x (KF, F) / 2.4x (KF, KF) over the keypoint-at-a-time walk.  Claims live in an LDS bitmap, the matches'
// rotation bins in LDS bytes; the top-3 filter runs over them at the end.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <vector>

#include "../../include/omv.h"
#include "omv_device.h"

namespace {

#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

constexpr int TH_LOW = 50, kHisto = 30;
constexpr int kMaxKp = 16384;      // keypoints per view (LDS claim bitmap + rotation bins)
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kFree = 0x7fffffff;
std::atomic<int64_t> g_bow_rescans{0};   // walk rescans over all SearchByBoW calls (diagnostic)

// rot = angle1 - angle2 (float), +360 if negative, bin = round(rot / 30) with 30 -> 0 (ORBmatcher.cc:475-481)
__device__ __forceinline__ int rot_bin(float a1, float a2) {
    const float factor = 1.0f / kHisto;
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == kHisto) bin = 0;
    return bin;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// ComputeThreeMaxima (ORBmatcher.cc:2537-2573)
__device__ void three_maxima(const int *cnt, int *ind) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHisto; i++) {
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

// camera block of a frame keypoint (ORBmatcher.cc:398-465): L [0, Nleft), R [Nleft, +Nright), SL, SR when the
// frame has side cameras; a single-camera frame (Nleft == -1) has one block
__device__ __forceinline__ int frame_block(const omv_kf_view &F, int idx) {
    if (F.n_left == -1) return 0;
    if (idx < F.n_left) return 0;
    if (idx < F.n_left + F.n_right) return 1;
    if (F.n_sideleft >= 0) {
        if (idx < F.n_left + F.n_right + F.n_sideleft) return 2;
        if (idx < F.n) return 3;
    }
    return -1;
}

// Candidate records, one per position q of the keyframe's FeatureVector CSR (the resolve's walk order):
// [0] o0 (-1: no search) [1] o1 [2] idx1 [3] counts of blocks 0|1 (u16 each) [4] counts 2|3 [5..7] pad,
// [8 + kTop c + k] the k-th best static candidate of block c as (distance << 23 | rotation bin << 16 | keypoint
// index), ascending by (distance, node position); 0xffffffff past the end.  Claims are the only dynamic filter, so the first two
// unclaimed entries are the reference's best and second whenever the block holds <= kTop candidates or two
// of them are unclaimed; otherwise the resolve rescans the node.
// Per mode: (KeyFrame, Frame) keeps 16 entries per camera block -- its four blocks' short lists ran out (a node rescan
// on one wavefront) for ~4 % of the keypoints at 8 -- and (KeyFrame, KeyFrame) 8.  kChunk * kRecWords: a multiple of 64.
template <int MODE>
struct BowCfg {
    static constexpr int top = MODE == OMV_BOW_KF_FRAME ? 16 : 8;
    static constexpr int rec = 8 + 4 * top;
    static constexpr int chunk = MODE == OMV_BOW_KF_FRAME ? 16 : 32;
};
constexpr int kBowWaves = 4;   // wavefronts per resolve workgroup (kChunk * kBowWaves records staged per chunk)

// Static filters + camera block of candidate idx2 (-1: not a candidate whatever the claims)
template <int MODE>
__device__ __forceinline__ int cand_block(const omv_kf_view &O, int idx2) {
    if (MODE == OMV_BOW_KF_FRAME) return frame_block(O, idx2);
    if (O.n_left != -1 && idx2 >= O.n) return -1;
    return O.has_mp[idx2] ? 0 : -1;
}

template <int MODE>
__global__ void __launch_bounds__(256) bow_cand_kernel(const omv_bow_job *jobs, const int *rec_off, uint32_t *recs) {
    constexpr int NB = MODE == OMV_BOW_KF_FRAME ? 4 : 1;
    constexpr int kTop = BowCfg<MODE>::top, kRecWords = BowCfg<MODE>::rec;
    const omv_bow_job &J = jobs[blockIdx.y];
    const omv_kf_view &K = J.kf, &O = J.other;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= K.n) return;
    uint32_t *R = recs + ((size_t)rec_off[blockIdx.y] + q) * kRecWords;
    // the FeatureVector lists only the keypoints of non-stopped words (TemplatedVocabulary.h:1157 `if (w > 0)`):
    // positions past its end carry no search
    const int n_list = K.n_nodes > 0 ? K.node_start[K.n_nodes] : 0;
    const int idx1 = q < n_list ? K.node_idx[q] : 0;
    int o0 = -1, o1 = -1;
    if (q < n_list && K.has_mp[idx1] && !(MODE == OMV_BOW_KF_KF && K.n_left != -1 && idx1 >= K.n)) {
        int lo = 0, hi = K.n_nodes - 1;   // the node holding position q: the last a with node_start[a] <= q
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (K.node_start[mid] <= q) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t id = K.node_id[lo];
        int l = 0, h = O.n_nodes;   // the same node id in the other view
        while (l < h) {
            const int mid = (l + h) >> 1;
            if (O.node_id[mid] < id) l = mid + 1;
            else h = mid;
        }
        if (l < O.n_nodes && O.node_id[l] == id) o0 = O.node_start[l], o1 = O.node_start[l + 1];
    }
    uint32_t key[NB][kTop], ent[NB][kTop];
    int cnt[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        cnt[c] = 0;
#pragma unroll
        for (int k = 0; k < kTop; ++k) key[c][k] = kNone, ent[c][k] = kNone;
    }
    if (o0 >= 0) {
        const uint64_t *dq = reinterpret_cast<const uint64_t *>(K.desc + 32 * (size_t)idx1);
        const uint64_t d1[4] = {dq[0], dq[1], dq[2], dq[3]};
        for (int p = o0; p < o1; ++p) {
            const int idx2 = O.node_idx[p];
            const int blk = cand_block<MODE>(O, idx2);
            if (blk < 0) continue;
            const uint64_t *q2 = reinterpret_cast<const uint64_t *>(O.desc + 32 * (size_t)idx2);
            const uint64_t d2[4] = {q2[0], q2[1], q2[2], q2[3]};
            const int dist = omv::hamming256(d1, d2);
            const int bin = rot_bin(K.kps[idx1].angle, O.kps[idx2].angle);   // static: both angles are fixed
            uint32_t kk = ((uint32_t)dist << 16) | (uint32_t)(p - o0),
                     ee = ((uint32_t)dist << 23) | ((uint32_t)bin << 16) | (uint32_t)idx2;
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                if (c != blk) continue;
                ++cnt[c];
#pragma unroll
                for (int k = 0; k < kTop; ++k) {   // insertion into the sorted top list
                    if (kk < key[c][k]) {
                        const uint32_t tk = key[c][k], te = ent[c][k];
                        key[c][k] = kk, ent[c][k] = ee;
                        kk = tk, ee = te;
                    }
                }
            }
        }
    }
    R[0] = (uint32_t)o0, R[1] = (uint32_t)o1, R[2] = (uint32_t)idx1;
    R[3] = (uint32_t)min(cnt[0], 0xffff) | (NB > 1 ? (uint32_t)min(cnt[NB > 1 ? 1 : 0], 0xffff) << 16 : 0u);
    R[4] = NB > 2 ? ((uint32_t)min(cnt[NB > 2 ? 2 : 0], 0xffff) | (uint32_t)min(cnt[NB > 3 ? 3 : 0], 0xffff) << 16) : 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int k = 0; k < kTop; ++k) R[8 + kTop * c + k] = c < NB ? ent[c < NB ? c : 0][k] : kNone;
}

// The full scan of one keyframe keypoint's node with the current claims (the rare fallback): per block the
// best (distance, node position) key and second distance over the wave.
template <int MODE, int NB>
__device__ void scan_node(const omv_kf_view &O, const uint32_t *claimed, const uint64_t d1[4], int o0, int o1,
                          int lane, int *bd, int *bi, int *bs) {
    uint32_t bk[NB];
    int sec[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) bk[c] = kNone, sec[c] = 256;
    for (int p = o0 + lane; p < o1; p += 64) {
        const int idx2 = O.node_idx[p];
        const int blk = cand_block<MODE>(O, idx2);
        if (blk < 0 || ((claimed[idx2 >> 5] >> (idx2 & 31)) & 1u)) continue;
        const uint64_t *q = reinterpret_cast<const uint64_t *>(O.desc + 32 * (size_t)idx2);
        const uint64_t d2[4] = {q[0], q[1], q[2], q[3]};
        const int dist = omv::hamming256(d1, d2);
        const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)(p - o0);
#pragma unroll
        for (int c = 0; c < NB; ++c) {
            if (c != blk) continue;
            if (key < bk[c]) {   // this lane's candidates arrive in node order
                if (bk[c] != kNone) sec[c] = min(sec[c], (int)(bk[c] >> 16));
                bk[c] = key;
            } else {
                sec[c] = min(sec[c], dist);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        const uint32_t g = wave_min_u32(bk[c]);
        const uint32_t other = bk[c] == g ? (uint32_t)sec[c] : (bk[c] == kNone ? 256u : bk[c] >> 16);
        bs[c] = (int)wave_min_u32(other);
        bd[c] = g == kNone ? 256 : (int)(g >> 16);
        bi[c] = g == kNone ? -1 : O.node_idx[o0 + (int)(g & 0xffffu)];
    }
}

// One workgroup of W wavefronts per job: the reference's sequential walk over the records (common nodes ascending,
// keyframe keypoints in node order), claims in an LDS bitmap, then the rotation filter.  The walk's batches span the
// whole workgroup (64 W / NB keypoints), so a conflict-free stretch of the walk commits in 1/W of the batches a
// single wavefront needs; a conflicting keypoint is walked alone by wavefront 0.
template <int MODE, int W>
__global__ void __launch_bounds__(64 * W) bow_resolve_kernel(const omv_bow_job *jobs, const int *rec_off,
                                                             const uint32_t *recs, float nnratio, int check_ori,
                                                             int32_t *n_matches, int *err, int lim) {
    // err[0]: status; err[1]: rescans of the walk (diagnostic, omv_matcher_bow_rescans)
    constexpr int kTop = BowCfg<MODE>::top, kRecWords = BowCfg<MODE>::rec, kChunk = BowCfg<MODE>::chunk;
    __shared__ uint32_t claimed[kMaxKp / 32];
    __shared__ uint8_t bins[kMaxKp];
    __shared__ int16_t match[kMaxKp];   // the output, written to memory once at the end (no stores in the walk)
    constexpr int T = 64 * W, kChunkW = kChunk * W;
    __shared__ uint32_t recbuf[2][kChunkW * kRecWords];
    __shared__ int owner[kMaxKp];   // batch claims: the first batch keypoint claiming an other-view keypoint, or kFree
    __shared__ int cnt[kHisto];
    __shared__ int ind[3];
    __shared__ int s_first, s_nm;
    constexpr int NB = MODE == OMV_BOW_KF_FRAME ? 4 : 1, S = T / NB;
    const omv_bow_job &J = jobs[blockIdx.x];
    const omv_kf_view &K = J.kf, &O = J.other;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_out = MODE == OMV_BOW_KF_FRAME ? O.n : K.n;
    if (O.n > kMaxKp || K.n > kMaxKp) {
        if (tid == 0) *err = OMV_ERR_CAPACITY;
        return;
    }
    for (int i = tid; i < n_out; i += T) match[i] = -1, bins[i] = 0xff;
    for (int i = tid; i < (O.n + 31) / 32; i += T) claimed[i] = 0;
    for (int i = tid; i < O.n; i += T) owner[i] = kFree;
    if (tid < kHisto) cnt[tid] = 0;
    if (tid == 0) s_first = INT_MAX, s_nm = 0;
    __syncthreads();
    // records staged through LDS a chunk at a time (one coalesced load per chunk, the next chunk in flight while
    // the current one is walked): the walk itself then only waits on LDS
    const uint32_t *R = recs + (size_t)rec_off[blockIdx.x] * kRecWords;
    const int n_words = K.n * kRecWords;
    constexpr int kPer = kChunkW * kRecWords / T;
    uint32_t nxt[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) nxt[k] = T * k + tid < n_words ? R[T * k + tid] : 0u;
    int nm = 0, buf = 0;
#ifdef OMV_BOW_PROFILE
    long long tb[4] = {0, 0, 0, 0}, tl = wall_clock64();
    int n_batch = 0, n_lone = 0, n_searched = 0, n_iter = 0;
#define OMV_TB(k) (tb[k] += wall_clock64() - tl, tl = wall_clock64())
#else
#define OMV_TB(k) ((void)0)
#endif
    for (int base = 0; base < K.n; base += kChunkW) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) recbuf[buf][T * k + tid] = nxt[k];
        const int nb = base + kChunkW;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int w = nb * kRecWords + T * k + tid;
            nxt[k] = w < n_words ? R[w] : 0u;
        }
        __syncthreads();
        OMV_TB(0);
        // one keyframe keypoint with the live claims (the batch's conflict / rescan case)
        auto walk_one = [&](const uint32_t *cr) {
        const int o0 = (int)cr[0];
        if (o0 < 0) return;
        const int o1 = (int)cr[1], idx1 = (int)cr[2];
        const uint32_t c01 = cr[3], c23 = cr[4];
        // lane c < NB: the block's first two unclaimed entries
        const int c = lane < NB ? lane : 0;
        uint32_t e[kTop];
#pragma unroll
        for (int k = 0; k < kTop; ++k) e[k] = cr[8 + kTop * c + k];
        const int total = (int)(((c < 2 ? c01 : c23) >> (16 * (c & 1))) & 0xffffu);
        // all claim words first (independent LDS reads, one latency), then a branch-free pick
        uint32_t cw[kTop];
#pragma unroll
        for (int k = 0; k < kTop; ++k) cw[k] = claimed[(e[k] == kNone ? 0u : e[k] & 0xffffu) >> 5];
        uint32_t best = kNone;
        int d2 = 256, found = 0;
#pragma unroll
        for (int k = 0; k < kTop; ++k) {
            const uint32_t x = e[k];
            const bool ok = k < lim && x != kNone && !((cw[k] >> (x & 31u)) & 1u);
            best = ok && found == 0 ? x : best;
            d2 = ok && found == 1 ? (int)(x >> 23) : d2;
            found += ok && found < 2 ? 1 : 0;
        }
        const bool rescan = lane < NB && found < 2 && total > lim;
        int bd[NB], bi[NB], bs[NB], bb[NB];
        if (__ballot(rescan)) {
            if (lane == 0) atomicAdd(err + 1, 1);
            const uint64_t *dq = reinterpret_cast<const uint64_t *>(K.desc + 32 * (size_t)idx1);
            const uint64_t d1[4] = {dq[0], dq[1], dq[2], dq[3]};
            scan_node<MODE, NB>(O, claimed, d1, o0, o1, lane, bd, bi, bs);
#pragma unroll
            for (int cc = 0; cc < NB; ++cc)
                bb[cc] = check_ori && bd[cc] <= TH_LOW ? rot_bin(K.kps[idx1].angle, O.kps[bi[cc]].angle) : 0;
        } else {
#pragma unroll
            for (int cc = 0; cc < NB; ++cc) {   // lane cc's pick, read into scalar registers
                const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)best, cc);
                bd[cc] = b == kNone ? 256 : (int)(b >> 23);
                bi[cc] = b == kNone ? -1 : (int)(b & 0xffffu);
                bb[cc] = (int)((b >> 16) & 31u);
                bs[cc] = __builtin_amdgcn_readlane(d2, cc);
            }
        }
        if (MODE == OMV_BOW_KF_FRAME) {
            if (bd[0] <= TH_LOW) {
#pragma unroll
                for (int cc = 0; cc < NB; ++cc) {
                    if (bd[cc] > TH_LOW) continue;
                    // left: the nnratio test; right / side: `... || true` (ORBmatcher.cc:520-521, ...)
                    if (cc == 0 && !((float)bd[0] < nnratio * (float)bs[0])) continue;
                    const int idxF = bi[cc];
                    if (lane == 0) {
                        match[idxF] = (int16_t)idx1;
                        claimed[idxF >> 5] |= 1u << (idxF & 31);
                        if (check_ori) {
                            bins[idxF] = (uint8_t)bb[cc];
                            ++cnt[bb[cc]];
                        }
                    }
                    ++nm;
                }
            }
        } else if (bd[0] < TH_LOW && (float)bd[0] < nnratio * (float)bs[0]) {
            const int idx2 = bi[0];
            if (lane == 0) {
                match[idx1] = (int16_t)idx2;
                claimed[idx2 >> 5] |= 1u << (idx2 & 31);   // vbMatched2
                if (check_ori) {
                    bins[idx1] = (uint8_t)bb[0];
                    ++cnt[bb[0]];
                }
            }
            ++nm;
        }
        // the claims before the next keyframe keypoint's pick: one wavefront, LDS only -- a wave-scope fence
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        // Batches of S = 64 W / NB consecutive keyframe keypoints, lane (s, c) = keypoint q + s, camera block c.  The
        // picks are iterated to the reference's: each round every lane picks against the claims committed before the
        // batch plus the claims of the earlier batch keypoints' current picks (`owner`: the first claimer), and the
        // rounds stop when no pick changes.  The fixed point is unique and is the sequential walk's (keypoint 0's
        // pick is final after one round, keypoint s's once those before it are), and conflicting keypoints only
        // cost another round (a one-entry claim chain a round) instead of a walk alone.  A keypoint whose short
        // list runs out (a node rescan) ends the batch: the keypoints before it commit, it is walked alone.
        const int qend = min(nb, K.n);
        for (int q = base; q < qend;) {
            const int nbatch = min(S, qend - q);
            const int s = tid / NB, c = tid % NB;
            const bool act = s < nbatch;
            const uint32_t *cr = recbuf[buf] + (act ? q + s - base : 0) * kRecWords;
            const int o0 = act ? (int)cr[0] : -1, idx1 = (int)cr[2];
            const uint32_t c01 = cr[3], c23 = cr[4];
            uint32_t e[kTop];
#pragma unroll
            for (int k = 0; k < kTop; ++k) e[k] = cr[8 + kTop * c + k];
            const int total = (int)(((c < 2 ? c01 : c23) >> (16 * (c & 1))) & 0xffffu);
            uint32_t cw[kTop];
#pragma unroll
            for (int k = 0; k < kTop; ++k) cw[k] = claimed[(e[k] == kNone ? 0u : e[k] & 0xffffu) >> 5];
            const bool search = o0 >= 0;
            uint32_t best = kNone;
            int d2 = 256, myclaim = -1;
            bool rescan = false;
            for (int it = 0;; ++it) {
                uint32_t nbest = kNone;
                int nd2 = 256, found = 0;
#pragma unroll
                for (int k = 0; k < kTop; ++k) {
                    const uint32_t x = e[k];
                    const bool ok = k < lim && x != kNone && !((cw[k] >> (x & 31u)) & 1u) &&
                                    owner[x == kNone ? 0u : x & 0xffffu] >= s;
                    nbest = ok && found == 0 ? x : nbest;
                    nd2 = ok && found == 1 ? (int)(x >> 23) : nd2;
                    found += ok && found < 2 ? 1 : 0;
                }
                const bool nresc = search && found < 2 && total > lim;
                const int bd = nbest == kNone ? 256 : (int)(nbest >> 23), bi = (int)(nbest & 0xffffu);
                const int bd0 = __shfl(bd, lane - c, 64), bs0 = __shfl(nd2, lane - c, 64);   // keypoint s's block 0
                bool claim;
                if (MODE == OMV_BOW_KF_FRAME)
                    claim = search && bd0 <= TH_LOW && bd <= TH_LOW && (c != 0 || (float)bd0 < nnratio * (float)bs0);
                else
                    claim = search && bd < TH_LOW && (float)bd < nnratio * (float)nd2;
                const bool changed = act && (nbest != best || nd2 != d2 || nresc != rescan);
                best = nbest, d2 = nd2, rescan = nresc;
                if (!__syncthreads_or(changed ? 1 : 0) && it > 0) break;   // owner already holds these picks' claims
                if (it > 2 * S + 4) {   // cannot happen (S + 1 rounds suffice); kept so the loop always ends:
                    rescan = act;       // the batch then commits nothing and its first keypoint is walked alone
                    break;
                }
                if (myclaim >= 0) owner[myclaim] = kFree;
                __syncthreads();
                myclaim = claim ? bi : -1;
                if (myclaim >= 0) atomicMin(&owner[myclaim], s);
                __syncthreads();
#ifdef OMV_BOW_PROFILE
                if (tid == 0) ++n_iter;
#endif
            }
            const uint64_t rm = __ballot(act && rescan);
            if (rm && lane == 0) atomicMin(&s_first, wave * (64 / NB) + (int)(__builtin_ctzll(rm) / NB));
            __syncthreads();
            const int sstar = min(s_first, nbatch);   // first keypoint to walk alone
            const bool commit = myclaim >= 0 && s < sstar;
            if (commit) {
                atomicOr(&claimed[myclaim >> 5], 1u << (myclaim & 31));
                const int at = MODE == OMV_BOW_KF_FRAME ? myclaim : idx1;
                match[at] = (int16_t)(MODE == OMV_BOW_KF_FRAME ? idx1 : myclaim);
                if (check_ori) {
                    const int bb = (int)((best >> 16) & 31u);
                    bins[at] = (uint8_t)bb;
                    atomicAdd(&cnt[bb], 1);
                }
            }
            nm += __popcll(__ballot(commit));   // this wavefront's commits
            if (myclaim >= 0) owner[myclaim] = kFree;
            __syncthreads();
            if (tid == 0) s_first = INT_MAX;   // read by every thread above; the next batch sets it after a barrier
            OMV_TB(1);
#ifdef OMV_BOW_PROFILE
            ++n_batch;
            n_searched += __popcll(__ballot(act && search && c == 0));
#endif
            if (sstar < nbatch) {
                if (wave == 0) walk_one(recbuf[buf] + (q + sstar - base) * kRecWords);
                __syncthreads();
                q += sstar + 1;
#ifdef OMV_BOW_PROFILE
                ++n_lone;
#endif
                OMV_TB(2);
            } else {
                q += nbatch;
            }
        }
        buf ^= 1;
    }
    __syncthreads();
#ifdef OMV_BOW_PROFILE
    OMV_TB(3);
    if (tid == 0 && blockIdx.x < 3)
        printf("bow job %d mode %d n %d: chunk staging %lld batches %lld lone walks %lld tail %lld ticks; batches %d lone %d searched(wave0) %d rounds %d\n",
               blockIdx.x, MODE, K.n, tb[0], tb[1], tb[2], tb[3], n_batch, n_lone, n_searched, n_iter);
#endif
#undef OMV_TB
    if (check_ori) {
        if (tid == 0) three_maxima(cnt, ind);
        __syncthreads();
    }
    int removed = 0;
    for (int i = tid; i < n_out; i += T) {
        const int bn = bins[i];
        const bool drop = check_ori && bn != 0xff && bn != ind[0] && bn != ind[1] && bn != ind[2];
        removed += drop ? 1 : 0;
        J.match[i] = drop ? -1 : (int32_t)match[i];
    }
    nm -= wave_sum_i32(removed);   // per wavefront: its commits (wave 0: also the lone walks) less its drops
    if (lane == 0) atomicAdd(&s_nm, nm);
    __syncthreads();
    if (tid == 0) n_matches[blockIdx.x] = s_nm;
}

}  // namespace

extern "C" {

omv_status omv_matcher_search_by_bow(omv_matcher *m, int n_jobs, const omv_bow_job *jobs, int mode, float nnratio,
                                     int check_ori, int32_t *n_matches, void *stream) {
    if (!m || n_jobs < 0 || (n_jobs > 0 && (!jobs || !n_matches)) || (mode != OMV_BOW_KF_FRAME && mode != OMV_BOW_KF_KF))
        return OMV_ERR_ARG;
    if (n_jobs == 0) return OMV_OK;
    for (int i = 0; i < n_jobs; ++i) {
        const omv_bow_job &j = jobs[i];
        if (!j.match || j.kf.n < 0 || j.other.n < 0 || j.kf.n_nodes < 0 || j.other.n_nodes < 0 ||
            (j.kf.n_nodes > 0 && (!j.kf.node_id || !j.kf.node_start || !j.kf.node_idx)) ||
            (j.other.n_nodes > 0 && (!j.other.node_id || !j.other.node_start || !j.other.node_idx)))
            return OMV_ERR_ARG;
        if (j.kf.n > kMaxKp || j.other.n > kMaxKp) return OMV_ERR_CAPACITY;
    }
    hipStream_t st = (hipStream_t)stream;
    std::vector<int> off(n_jobs + 1, 0);
    int max_n = 1;
    for (int i = 0; i < n_jobs; ++i) off[i + 1] = off[i] + jobs[i].kf.n, max_n = std::max(max_n, jobs[i].kf.n);
    const size_t job_bytes = (sizeof(omv_bow_job) * n_jobs + 15) & ~(size_t)15;
    const size_t off_bytes = (sizeof(int) * (n_jobs + 1) + 15) & ~(size_t)15;
    char *d_buf = nullptr;
    const int rec_words = mode == OMV_BOW_KF_FRAME ? BowCfg<OMV_BOW_KF_FRAME>::rec : BowCfg<OMV_BOW_KF_KF>::rec;
    const int top = mode == OMV_BOW_KF_FRAME ? BowCfg<OMV_BOW_KF_FRAME>::top : BowCfg<OMV_BOW_KF_KF>::top;
    HIP_OK(hipMallocAsync((void **)&d_buf, job_bytes + off_bytes + 16 + (size_t)off[n_jobs] * rec_words * 4, st));
    omv_bow_job *d_jobs = (omv_bow_job *)d_buf;
    int *d_off = (int *)(d_buf + job_bytes);
    int *d_err = (int *)(d_buf + job_bytes + off_bytes);
    uint32_t *d_recs = (uint32_t *)(d_buf + job_bytes + off_bytes + 16);
    HIP_OK(hipMemcpyAsync(d_jobs, jobs, sizeof(omv_bow_job) * n_jobs, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(d_off, off.data(), sizeof(int) * (n_jobs + 1), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(d_err, 0, 2 * sizeof(int), st));
    const dim3 cg((max_n + 255) / 256, n_jobs);
    // short-list entries the walk uses (test knob OMV_BOW_TOP: fewer make the node rescans run on small inputs)
    int lim = top;
    const omv::MatcherKnobs kn = omv::matcher_knobs(m);
    if (kn.bow_top >= 0) lim = std::max(2, std::min(top, kn.bow_top));
    if (mode == OMV_BOW_KF_FRAME) {
        bow_cand_kernel<OMV_BOW_KF_FRAME><<<cg, 256, 0, st>>>(d_jobs, d_off, d_recs);
        bow_resolve_kernel<OMV_BOW_KF_FRAME, kBowWaves><<<n_jobs, 64 * kBowWaves, 0, st>>>(d_jobs, d_off, d_recs, nnratio,
                                                                                         check_ori, n_matches, d_err, lim);
    } else {
        bow_cand_kernel<OMV_BOW_KF_KF><<<cg, 256, 0, st>>>(d_jobs, d_off, d_recs);
        bow_resolve_kernel<OMV_BOW_KF_KF, kBowWaves><<<n_jobs, 64 * kBowWaves, 0, st>>>(d_jobs, d_off, d_recs, nnratio,
                                                                                      check_ori, n_matches, d_err, lim);
    }
    HIP_OK(hipGetLastError());
    int h_err[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(h_err, d_err, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_OK(hipFreeAsync(d_buf, st));
    HIP_OK(hipStreamSynchronize(st));
    g_bow_rescans += h_err[1];
    return h_err[0] ? (omv_status)h_err[0] : OMV_OK;
}

omv_status omv_matcher_bow_rescans(int64_t *total, int reset) {
    if (!total) return OMV_ERR_ARG;
    *total = g_bow_rescans.load();
    if (reset) g_bow_rescans = 0;
    return OMV_OK;
}

}  // extern "C"
