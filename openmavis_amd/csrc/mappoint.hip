// MI355X-native map-point refresh, the pair LocalMapping calls for every new / fused map point
// (src/LocalMapping.cc:338-339, :776-778, :897-898; src/MapPoint.cc:377):
//
//   distinctive_kernel   MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:405-490): one wavefront per map
//                        point.  Its observations' descriptors (in the caller's std::map order, L / R / SL / SR per
//                        keyframe, bad keyframes left out) are staged in LDS; lane i owns descriptor i's row of the
//                        N x N Hamming distances (ORBmatcher::DescriptorDistance = popcount of the XOR) and finds the
//                        row's median vDists[0.5 (N - 1)] after std::sort as the smallest v with
//                        #{j : d_ij <= v} > (N - 1) / 2 (a 9-step bisection over 0..256, the rows never sorted);
//                        the wave's argmin of (median, i) is the reference's first strict minimum.
//   normal_depth_kernel  MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:503-588): one thread per map point, the
//                        float arithmetic in the reference's order (normal += (Pos - Owi) / |Pos - Owi| per
//                        observation entry, then / n; dist = |Pos - O_ref|, max = dist * scale[level],
//                        min = max / scale[nLevels - 1]).
// Bit-exact against oracle/mappoint_oracle.cpp (integer selection; float paths unfused, -ffp-contract=off).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>

#include "../../include/omv.h"
#include "omv_device.h"

namespace {

constexpr int kStage = 256;   // descriptors staged in LDS per map point (more: read from global memory)

__device__ __forceinline__ int hamming(const uint4 &a0, const uint4 &a1, const uint4 &b0, const uint4 &b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) + __popc(a1.x ^ b1.x) +
           __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// One wavefront per map point.  desc_start [P+1]: the point's run of descriptor rows desc_row (the observations'
// L / R / SL / SR rows in the caller's std::map order, bad keyframes already left out).
__global__ void __launch_bounds__(64) distinctive_kernel(int n_points, const int32_t *desc_start, const int32_t *desc_row,
                                                         const uint8_t *desc, int32_t *best_out, uint8_t *desc_out) {
    __shared__ uint4 sd[2 * kStage];
    const int p = blockIdx.x, lane = threadIdx.x;
    if (p >= n_points) return;
    const int e0 = desc_start[p], n = desc_start[p + 1] - e0;
    if (n <= 0) {   // no descriptor: the reference returns without touching mDescriptor
        if (lane == 0) best_out[p] = -1;
        return;
    }
    for (int j = lane; j < min(n, kStage); j += 64) {
        const uint4 *src = reinterpret_cast<const uint4 *>(desc + (size_t)desc_row[e0 + j] * 32);
        sd[2 * j] = src[0], sd[2 * j + 1] = src[1];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    auto row_of = [&](int j, uint4 &r0, uint4 &r1) {   // rows past the LDS stage from global memory (rare)
        if (j < kStage) {
            r0 = sd[2 * j], r1 = sd[2 * j + 1];
        } else {
            const uint4 *src = reinterpret_cast<const uint4 *>(desc + (size_t)desc_row[e0 + j] * 32);
            r0 = src[0], r1 = src[1];
        }
    };
    const int k = (n - 1) / 2;   // vDists[0.5 * (N - 1)]: the (k + 1)-th smallest of the row (self distance 0 included)
    int best_med = INT_MAX, best_i = INT_MAX;
    for (int i = lane; i < n; i += 64) {
        uint4 a0, a1;
        row_of(i, a0, a1);
        int lo = 0, hi = 256;   // the smallest v with #{d_ij <= v} >= k + 1
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int j = 0; j < n; ++j) {
                uint4 b0, b1;
                row_of(j, b0, b1);
                cnt += hamming(a0, a1, b0, b1) <= mid ? 1 : 0;
            }
            if (cnt >= k + 1) hi = mid;
            else lo = mid + 1;
        }
        if (lo < best_med) best_med = lo, best_i = i;   // i ascending per lane: the first of equal medians
    }
    // the first i with the strictly smallest median over the wave
    for (int d = 32; d >= 1; d >>= 1) {
        const int om = __shfl_xor(best_med, d, 64), oi = __shfl_xor(best_i, d, 64);
        if (om < best_med || (om == best_med && oi < best_i)) best_med = om, best_i = oi;
    }
    const int row = desc_row[e0 + best_i];
    if (lane == 0) best_out[p] = row;
    if (desc_out && lane < 8) {   // mDescriptor = vDescriptors[BestIdx].clone()
        const uint32_t *src = reinterpret_cast<const uint32_t *>(desc + (size_t)row * 32);
        reinterpret_cast<uint32_t *>(desc_out + (size_t)p * 32)[lane] = src[lane];
    }
}

// Eigen::Vector3f::norm() = sqrt of the left-to-right squared sum (float, correctly rounded like std::sqrt)
__device__ __forceinline__ float norm3f(float x, float y, float z) { return omv::sqrtf_cr(x * x + y * y + z * z); }

// One thread per map point.  obs_center per entry: the camera centre of that observation (GetCameraCenter /
// GetRightCameraCenter / GetSideLeftCameraCenter / GetSideRightCameraCenter of its keyframe, every entry: the
// reference does not skip bad keyframes here).
__global__ void __launch_bounds__(256) normal_depth_kernel(int n_points, const int32_t *obs_start, const float *obs_center,
                                                           const float *pos, const float *ref_center,
                                                           const float *ref_level_scale, const float *ref_max_scale,
                                                           float *normal_out, float *min_dist, float *max_dist) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_points) return;
    const int e0 = obs_start[p], e1 = obs_start[p + 1];
    if (e1 == e0) return;   // observations.empty(): untouched
    const float X = pos[3 * p], Y = pos[3 * p + 1], Z = pos[3 * p + 2];
    float nx = 0.f, ny = 0.f, nz = 0.f;
    int n = 0;
    for (int e = e0; e < e1; ++e) {
        const float dx = X - obs_center[3 * e], dy = Y - obs_center[3 * e + 1], dz = Z - obs_center[3 * e + 2];
        const float r = norm3f(dx, dy, dz);
        nx = nx + dx / r, ny = ny + dy / r, nz = nz + dz / r;
        ++n;
    }
    const float px = X - ref_center[3 * p], py = Y - ref_center[3 * p + 1], pz = Z - ref_center[3 * p + 2];
    const float dist = norm3f(px, py, pz);
    const float mx = dist * ref_level_scale[p];
    max_dist[p] = mx;
    min_dist[p] = mx / ref_max_scale[p];
    const float fn = (float)n;
    normal_out[3 * p] = nx / fn, normal_out[3 * p + 1] = ny / fn, normal_out[3 * p + 2] = nz / fn;
}

}  // namespace

extern "C" {

omv_status omv_mappoint_distinctive_descriptors(int n_points, const int32_t *desc_start, const int32_t *desc_row,
                                                const uint8_t *desc, int32_t *best_row, uint8_t *desc_out,
                                                void *stream) {
    if (n_points < 0 || (n_points > 0 && (!desc_start || !desc_row || !desc || !best_row))) return OMV_ERR_ARG;
    if (n_points == 0) return OMV_OK;
    distinctive_kernel<<<n_points, 64, 0, (hipStream_t)stream>>>(n_points, desc_start, desc_row, desc, best_row,
                                                                 desc_out);
    return hipGetLastError() == hipSuccess ? OMV_OK : OMV_ERR_HIP;
}

omv_status omv_mappoint_normal_depth(int n_points, const int32_t *obs_start, const float *obs_center, const float *pos,
                                     const float *ref_center, const float *ref_level_scale, const float *ref_max_scale,
                                     float *normal, float *min_dist, float *max_dist, void *stream) {
    if (n_points < 0 || (n_points > 0 && (!obs_start || !obs_center || !pos || !ref_center || !ref_level_scale ||
                                          !ref_max_scale || !normal || !min_dist || !max_dist)))
        return OMV_ERR_ARG;
    if (n_points == 0) return OMV_OK;
    normal_depth_kernel<<<(n_points + 255) / 256, 256, 0, (hipStream_t)stream>>>(
        n_points, obs_start, obs_center, pos, ref_center, ref_level_scale, ref_max_scale, normal, min_dist, max_dist);
    return hipGetLastError() == hipSuccess ? OMV_OK : OMV_ERR_HIP;
}

}  // extern "C"
