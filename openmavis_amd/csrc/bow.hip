// MI355X-native DBoW2 vocabulary transform: TemplatedVocabulary<FORB>::transform(features, BowVector&,
// FeatureVector&, levelsup) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1194, :1217-1259) for a batch of
// descriptor sets (Frame::ComputeBoW / KeyFrame::ComputeBoW, src/KeyFrame.cc:207-214).
//   bow_descend_kernel  one thread per descriptor: the tree descent (k Hamming distances per level over the
//                       node's children in file order, first child wins ties), the word, its weight and the
//                       FeatureVector node at level L - levelsup.
//   bow_build_kernel    one 1024-thread workgroup per set: the std::map semantics of BowVector::addWeight /
//                       addIfNotExist and FeatureVector::addFeature as a bitonic sort of (word | feature)
//                       and (node | feature) keys in LDS (<= 16384 keys = 128 KB), runs summed in feature
//                       order (the reference's += order), then BowVector::normalize with the norm summed in
//                       ascending word order by one thread (the reference's map iteration), so the doubles
//                       are bit-identical to the restatement in oracle/bow_oracle.cpp.
#include <hip/hip_runtime.h>

#include <cstdio>

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

constexpr int kMaxSet = 16384;   // keys carry the feature index in 14 bits
constexpr int kBuildThreads = 1024;

__device__ __forceinline__ void load_desc(const uint8_t *p, uint64_t d[4]) {
    const uint64_t *q = reinterpret_cast<const uint64_t *>(p);
    d[0] = q[0], d[1] = q[1], d[2] = q[2], d[3] = q[3];
}

__global__ void __launch_bounds__(256) bow_descend_kernel(omv_vocab v, const uint8_t *desc, int cap, const int *n_desc,
                                                          int n_sets, int levelsup, int32_t *word, double *wval,
                                                          int32_t *node) {
    const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long long)n_sets * cap) return;
    const int set = (int)(g / cap), i = (int)(g % cap);
    if (i >= n_desc[set]) return;
    if (v.n_words == 0) {   // empty(): nothing is transformed
        word[g] = -1, wval[g] = 0.0, node[g] = -1;
        return;
    }
    uint64_t f[4];
    load_desc(desc + (size_t)g * 32, f);
    const int nid_level = v.L - levelsup;
    int nid = nid_level <= 0 ? 0 : -1;
    int final_id = 0, level = 0;
    do {   // TemplatedVocabulary::transform (:1232-1254)
        ++level;
        const int c0 = v.child_start[final_id], c1 = v.child_start[final_id + 1];
        final_id = v.child_ids[c0];
        uint64_t d[4];
        load_desc(v.desc + 32 * (size_t)final_id, d);
        int best_d = omv::hamming256(f, d);
        for (int c = c0 + 1; c < c1; ++c) {
            const int id = v.child_ids[c];
            load_desc(v.desc + 32 * (size_t)id, d);
            const int dd = omv::hamming256(f, d);
            if (dd < best_d) best_d = dd, final_id = id;
        }
        if (level == nid_level) nid = final_id;
    } while (v.child_start[final_id] != v.child_start[final_id + 1]);
    word[g] = v.word_id[final_id];
    wval[g] = v.weight[final_id];
    node[g] = nid;
}

// Ascending bitonic sort of P (power of two) keys in LDS.
__device__ void bitonic_sort(uint64_t *k, int P) {
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < P; t += blockDim.x) {
                const int p = t ^ stride;
                if (p > t) {
                    const uint64_t a = k[t], b = k[p];
                    const bool up = (t & size) == 0;
                    if ((a > b) == up) k[t] = b, k[p] = a;
                }
            }
            __syncthreads();
        }
}

// Exclusive prefix count of run starts over P sorted keys (field = key >> 14), kBuildThreads threads with
// P / kBuildThreads consecutive keys each; returns the run index of key t via `run`, the total in *n_runs.
__device__ void run_index(const uint64_t *k, int m, int *scan, int *n_runs) {
    const int per = (m + kBuildThreads - 1) / kBuildThreads;
    const int t0 = threadIdx.x * per;
    int c = 0;
    for (int t = t0; t < min(m, t0 + per); ++t) c += (t == 0 || (k[t] >> 14) != (k[t - 1] >> 14)) ? 1 : 0;
    scan[threadIdx.x] = c;
    __syncthreads();
    if (threadIdx.x == 0) {   // 1024 counts: serial exclusive scan
        int s = 0;
        for (int q = 0; q < kBuildThreads; ++q) {
            const int x = scan[q];
            scan[q] = s;
            s += x;
        }
        *n_runs = s;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(kBuildThreads) bow_build_kernel(omv_vocab v, int cap, const int *n_desc, const int32_t *word,
                                                                  const double *wval, const int32_t *node, int32_t *bow_word,
                                                                  double *bow_value, int32_t *bow_n, int32_t *fv_node,
                                                                  int32_t *fv_start, int32_t *fv_idx, int32_t *fv_n) {
    extern __shared__ uint64_t keys[];
    __shared__ int scan[kBuildThreads];
    __shared__ int s_m, s_runs, s_nb;
    __shared__ double s_norm;
    const int set = blockIdx.x, n = n_desc[set];
    const size_t base = (size_t)set * cap;
    int P = 1;
    while (P < n) P <<= 1;
    const int sc = v.scoring;
    const bool must = sc != 5, l2 = sc == 1, tf = v.weighting == 0 || v.weighting == 1;
    int32_t *bw = bow_word + base;
    double *bv = bow_value + base;
    for (int pass = 0; pass < 2; ++pass) {   // 0: BowVector (word keys), 1: FeatureVector (node keys)
        if (threadIdx.x == 0) s_m = 0;
        __syncthreads();
        int cnt = 0;
        for (int t = threadIdx.x; t < P; t += blockDim.x) {
            uint64_t key = ~0ull;
            if (t < n && v.n_words > 0 && wval[base + t] > 0) {   // not stopped
                const uint32_t f = pass == 0 ? (uint32_t)word[base + t] : (uint32_t)node[base + t];
                key = ((uint64_t)f << 14) | (uint64_t)t;
                ++cnt;
            }
            keys[t] = key;
        }
        atomicAdd(&s_m, cnt);
        __syncthreads();
        const int m = s_m;
        bitonic_sort(keys, P);
        run_index(keys, m, scan, &s_runs);
        const int per = (m + kBuildThreads - 1) / kBuildThreads;
        const int t0 = threadIdx.x * per;
        int r = scan[threadIdx.x];
        for (int t = t0; t < min(m, t0 + per); ++t) {
            const bool start = t == 0 || (keys[t] >> 14) != (keys[t - 1] >> 14);
            if (!start) continue;
            const uint32_t f = (uint32_t)(keys[t] >> 14);
            if (pass == 0) {   // addWeight: += in feature order; addIfNotExist: the first
                double val = wval[base + (keys[t] & 0x3fff)];
                if (tf)
                    for (int u = t + 1; u < m && (keys[u] >> 14) == f; ++u) val += wval[base + (keys[u] & 0x3fff)];
                bw[r] = (int32_t)f, bv[r] = val;
            } else {
                fv_node[base + r] = (int32_t)f;
                fv_start[(size_t)set * (cap + 1) + r] = t;
            }
            ++r;
        }
        if (pass == 1) {
            for (int t = threadIdx.x; t < m; t += blockDim.x) fv_idx[base + t] = (int32_t)(keys[t] & 0x3fff);
            if (threadIdx.x == 0) fv_start[(size_t)set * (cap + 1) + s_runs] = m, fv_n[set] = s_runs;
        } else if (threadIdx.x == 0) {
            bow_n[set] = s_runs, s_nb = s_runs;
        }
        __threadfence_block();
        __syncthreads();
    }
    const int nb = s_nb;
    if (tf && nb > 0 && !must) {
        const double nd = nb;
        for (int q = threadIdx.x; q < nb; q += blockDim.x) bv[q] /= nd;
    }
    if (must) {   // BowVector::normalize: the norm over the map in ascending word order
        if (threadIdx.x == 0) {
            double norm = 0.0;
            if (!l2) {
                for (int q = 0; q < nb; ++q) norm += fabs(bv[q]);
            } else {
                for (int q = 0; q < nb; ++q) norm += bv[q] * bv[q];
                norm = sqrt(norm);
            }
            s_norm = norm;
        }
        __syncthreads();
        const double norm = s_norm;
        if (norm > 0.0)
            for (int q = threadIdx.x; q < nb; q += blockDim.x) bv[q] /= norm;
    }
}

}  // namespace

extern "C" {

omv_status omv_bow_transform(const omv_vocab *voc, int n_sets, const uint8_t *desc, int cap, const int *n_desc,
                             int levelsup, int32_t *word, double *wval, int32_t *node, int32_t *bow_word,
                             double *bow_value, int32_t *bow_n, int32_t *fv_node, int32_t *fv_start, int32_t *fv_idx,
                             int32_t *fv_n, void *stream) {
    if (!voc || n_sets < 0 || cap <= 0 || cap > kMaxSet) return OMV_ERR_ARG;
    if (n_sets == 0) return OMV_OK;
    if (!desc || !n_desc || !word || !wval || !node || !bow_word || !bow_value || !bow_n || !fv_node || !fv_start ||
        !fv_idx || !fv_n || voc->n_nodes <= 0 || !voc->child_start || !voc->child_ids || !voc->desc || !voc->word_id ||
        !voc->weight || voc->L < 1 || voc->scoring < 0 || voc->scoring > 5 || voc->weighting < 0 || voc->weighting > 3)
        return OMV_ERR_ARG;
    static bool attr = false;
    if (!attr) {
        HIP_OK(hipFuncSetAttribute((const void *)bow_build_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)(sizeof(uint64_t) * kMaxSet)));
        attr = true;
    }
    hipStream_t st = (hipStream_t)stream;
    const long long tot = (long long)n_sets * cap;
    bow_descend_kernel<<<(int)((tot + 255) / 256), 256, 0, st>>>(*voc, desc, cap, n_desc, n_sets, levelsup, word, wval,
                                                                 node);
    int P = 1;
    while (P < cap) P <<= 1;
    bow_build_kernel<<<n_sets, kBuildThreads, sizeof(uint64_t) * P, st>>>(*voc, cap, n_desc, word, wval, node, bow_word,
                                                                          bow_value, bow_n, fv_node, fv_start, fv_idx,
                                                                          fv_n);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

}  // extern "C"
