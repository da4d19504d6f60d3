// MI355X-native ORBmatcher::SearchByBoW (src/ORBmatcher.cc:349-666 for (KeyFrame, Frame), :1006-1129 for
// (KeyFrame, KeyFrame)): Hamming matching of the keypoints that share a DBoW2 FeatureVector node, in the
// reference's sequential order (common node ids ascending, keyframe keypoints in node order), with the
// claims of earlier keyframe keypoints, the per-camera-block best / second and the rotation-consistency
// filter (ComputeThreeMaxima, :2537-2573).
//
// One wavefront per job.  The node merge and the walk over keyframe keypoints are wave-uniform; for one
// keyframe keypoint the lanes take the other view's keypoints of the node (64 at a time), each keeping its
// own best (distance, node position) key and second distance per camera block, and one min-reduction per
// block combines them: the best is the first minimal distance in node order (the reference's strict `<`
// update), the second the smallest distance of the others.  Claims live in an LDS bitmap, the matches'
// rotation bins in LDS bytes; the top-3 filter runs over them at the end.
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

constexpr int TH_LOW = 50, kHisto = 30;
constexpr int kMaxKp = 16384;      // keypoints per view (LDS claim bitmap + rotation bins)
constexpr uint32_t kNone = 0xffffffffu;

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

template <int MODE>
__global__ void __launch_bounds__(64) bow_kernel(const omv_bow_job *jobs, float nnratio, int check_ori,
                                                 int32_t *n_matches, int *err) {
    __shared__ uint32_t claimed[kMaxKp / 32];
    __shared__ uint8_t bins[kMaxKp];
    __shared__ int cnt[kHisto];
    __shared__ int ind[3];
    constexpr int NB = MODE == OMV_BOW_KF_FRAME ? 4 : 1;
    const omv_bow_job &J = jobs[blockIdx.x];
    const omv_kf_view &K = J.kf, &O = J.other;
    const int lane = threadIdx.x;
    const int n_out = MODE == OMV_BOW_KF_FRAME ? O.n : K.n;
    if (O.n > kMaxKp || K.n > kMaxKp) {
        if (lane == 0) *err = OMV_ERR_CAPACITY;
        return;
    }
    for (int i = lane; i < n_out; i += 64) J.match[i] = -1, bins[i] = 0xff;
    for (int i = lane; i < (O.n + 31) / 32; i += 64) claimed[i] = 0;
    if (lane < kHisto) cnt[lane] = 0;
    __syncthreads();
    int nm = 0;
    int a = 0, b = 0;
    while (a < K.n_nodes && b < O.n_nodes) {
        const uint32_t na = K.node_id[a], nb = O.node_id[b];
        if (na < nb) {   // lower_bound on the smaller side
            ++a;
            continue;
        }
        if (nb < na) {
            ++b;
            continue;
        }
        const int o0 = O.node_start[b], o1 = O.node_start[b + 1];
        for (int i1 = K.node_start[a]; i1 < K.node_start[a + 1]; ++i1) {
            const int idx1 = K.node_idx[i1];
            if (MODE == OMV_BOW_KF_KF && K.n_left != -1 && idx1 >= K.n) continue;
            if (!K.has_mp[idx1]) continue;
            uint64_t d1[4];
            {
                const uint64_t *q = reinterpret_cast<const uint64_t *>(K.desc + 32 * (size_t)idx1);
                d1[0] = q[0], d1[1] = q[1], d1[2] = q[2], d1[3] = q[3];
            }
            uint32_t bk[NB];
            int sec[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) bk[c] = kNone, sec[c] = 256;
            for (int p = o0 + lane; p < o1; p += 64) {
                const int idx2 = O.node_idx[p];
                int blk = 0;
                bool ok = !((claimed[idx2 >> 5] >> (idx2 & 31)) & 1u);
                if (MODE == OMV_BOW_KF_FRAME) {
                    blk = frame_block(O, idx2);
                    ok = ok && blk >= 0;
                } else {
                    ok = ok && !(O.n_left != -1 && idx2 >= O.n) && O.has_mp[idx2];
                }
                if (!ok) continue;
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
            int bd[NB], bi[NB], bs[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const uint32_t g = wave_min_u32(bk[c]);
                const uint32_t other = bk[c] == g ? (uint32_t)sec[c] : (bk[c] == kNone ? 256u : bk[c] >> 16);
                bs[c] = (int)wave_min_u32(other);
                bd[c] = g == kNone ? 256 : (int)(g >> 16);
                bi[c] = g == kNone ? -1 : O.node_idx[o0 + (int)(g & 0xffffu)];
            }
            if (MODE == OMV_BOW_KF_FRAME) {
                if (bd[0] <= TH_LOW) {
#pragma unroll
                    for (int c = 0; c < NB; ++c) {
                        if (bd[c] > TH_LOW) continue;
                        // left: the nnratio test; right / side: `... || true` (ORBmatcher.cc:520-521, ...)
                        if (c == 0 && !((float)bd[0] < nnratio * (float)bs[0])) continue;
                        const int idxF = bi[c];
                        if (lane == 0) {
                            J.match[idxF] = idx1;
                            claimed[idxF >> 5] |= 1u << (idxF & 31);
                            if (check_ori) {
                                const int bin = rot_bin(K.kps[idx1].angle, O.kps[idxF].angle);
                                bins[idxF] = (uint8_t)bin;
                                ++cnt[bin];
                            }
                        }
                        ++nm;
                    }
                }
            } else if (bd[0] < TH_LOW && (float)bd[0] < nnratio * (float)bs[0]) {
                const int idx2 = bi[0];
                if (lane == 0) {
                    J.match[idx1] = idx2;
                    claimed[idx2 >> 5] |= 1u << (idx2 & 31);   // vbMatched2
                    if (check_ori) {
                        const int bin = rot_bin(K.kps[idx1].angle, O.kps[idx2].angle);
                        bins[idx1] = (uint8_t)bin;
                        ++cnt[bin];
                    }
                }
                ++nm;
            }
            __syncthreads();   // the claims before the next keyframe keypoint's scan
        }
        ++a, ++b;
    }
    if (check_ori) {
        if (lane == 0) three_maxima(cnt, ind);
        __syncthreads();
        int removed = 0;
        for (int i = lane; i < n_out; i += 64) {
            const int bn = bins[i];
            if (bn != 0xff && bn != ind[0] && bn != ind[1] && bn != ind[2]) J.match[i] = -1, ++removed;
        }
        nm -= wave_sum_i32(removed);
    }
    if (lane == 0) n_matches[blockIdx.x] = nm;
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
        if (!j.match || j.kf.n < 0 || j.other.n < 0 || (j.kf.n_nodes > 0 && (!j.kf.node_id || !j.kf.node_start)) ||
            (j.other.n_nodes > 0 && (!j.other.node_id || !j.other.node_start)))
            return OMV_ERR_ARG;
        if (j.kf.n > kMaxKp || j.other.n > kMaxKp) return OMV_ERR_CAPACITY;
    }
    hipStream_t st = (hipStream_t)stream;
    omv_bow_job *d_jobs = nullptr;
    HIP_OK(hipMallocAsync((void **)&d_jobs, sizeof(omv_bow_job) * n_jobs + sizeof(int), st));
    int *d_err = (int *)(d_jobs + n_jobs);
    HIP_OK(hipMemcpyAsync(d_jobs, jobs, sizeof(omv_bow_job) * n_jobs, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(d_err, 0, sizeof(int), st));
    if (mode == OMV_BOW_KF_FRAME)
        bow_kernel<OMV_BOW_KF_FRAME><<<n_jobs, 64, 0, st>>>(d_jobs, nnratio, check_ori, n_matches, d_err);
    else
        bow_kernel<OMV_BOW_KF_KF><<<n_jobs, 64, 0, st>>>(d_jobs, nnratio, check_ori, n_matches, d_err);
    HIP_OK(hipGetLastError());
    int h_err = 0;
    HIP_OK(hipMemcpyAsync(&h_err, d_err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_OK(hipFreeAsync(d_jobs, st));
    HIP_OK(hipStreamSynchronize(st));
    return h_err ? (omv_status)h_err : OMV_OK;
}

}  // extern "C"
