// MI355X-native tail of the multi-camera Frame constructor (src/Frame.cc:1913-1939):
//   * GetDepthFromUndistortedPoints (src/Frame.cc:1659-1765) -> mvuRight, one thread per keypoint:
//     cv::fisheye::undistortPoints in double, the nearest-pixel lookup into the block's undistorted
//     depth image, u_R = x - bf / d.  Work per keypoint: 24 B keypoint + one 4 B depth gather + 4 B out.
//   * the cv::vconcat of the per-camera keypoints / descriptors / mvuRight into the frame's dense rows.
// Double arithmetic without contraction (-ffp-contract=off); the one transcendental, tan(theta), is the
// device libm's (glibc's may differ by an ulp: it moves the float-rounded undistorted point only when
// the double lands within an ulp of a float rounding boundary; tests/test_frame_gpu.py says so).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../include/omv.h"

namespace {

#define HIP_OK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "omv: %s failed: %s\n", #x, hipGetErrorString(e_));      \
            return OMV_ERR_HIP;                                                      \
        }                                                                            \
    } while (0)

constexpr int kMaxBlocks = 8;

struct UrightArgs {
    const omv_kp *kps;
    const int *n_kp;
    const float *depth;
    int n_cams, n_blocks, kp_cap, w, h;
    float bf;
    omv_fisheye_undist U[kMaxBlocks];
    float *u_right, *xy;
};

// cv::fisheye::undistortPoints for one float point (R = noArray(), P = newK; criteria
// MAX_ITER + EPS, 10, 1e-8): OpenCV modules/calib3d/src/fisheye.cpp, restated.
__device__ void fisheye_undistort(const omv_fisheye_undist &U, float px, float py, float &ox, float &oy) {
    const double fx = (double)U.K[0], fy = (double)U.K[1], cx = (double)U.K[2], cy = (double)U.K[3];
    const double pwx = ((double)px - cx) / fx, pwy = ((double)py - cy) / fy;
    double scale = 1.0;
    double theta_d = sqrt(pwx * pwx + pwy * pwy);
    theta_d = fmin(fmax(-M_PI / 2., theta_d), M_PI / 2.);
    bool converged = false;
    double theta = theta_d;
    if (theta_d > 1e-8) {
        for (int j = 0; j < 10; j++) {
            const double theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2,
                         theta8 = theta6 * theta2;
            const double k0_theta2 = U.D[0] * theta2, k1_theta4 = U.D[1] * theta4, k2_theta6 = U.D[2] * theta6,
                         k3_theta8 = U.D[3] * theta8;
            const double theta_fix = (theta * (1 + k0_theta2 + k1_theta4 + k2_theta6 + k3_theta8) - theta_d) /
                                     (1 + 3 * k0_theta2 + 5 * k1_theta4 + 7 * k2_theta6 + 9 * k3_theta8);
            theta = theta - theta_fix;
            if (fabs(theta_fix) < 1e-8) {
                converged = true;
                break;
            }
        }
        scale = tan(theta) / theta_d;
    } else {
        converged = true;
    }
    const bool flipped = (theta_d < 0 && theta > 0) || (theta_d > 0 && theta < 0);
    if (converged && !flipped) {
        const double pux = pwx * scale, puy = pwy * scale;
        // RR = newK (P * I); pr = RR * (pu, 1): row sums in order, pr[2] = 0 pu + 0 pu + 1
        const double P00 = (double)U.newK[0], P02 = (double)U.newK[2], P11 = (double)U.newK[1],
                     P12 = (double)U.newK[3];
        const double pr0 = P00 * pux + 0.0 * puy + P02, pr1 = 0.0 * pux + P11 * puy + P12;
        const double pr2 = 0.0 * pux + 0.0 * puy + 1.0;
        ox = (float)(pr0 / pr2), oy = (float)(pr1 / pr2);
    } else {
        ox = -1000000.0f, oy = -1000000.0f;
    }
}

__global__ void __launch_bounds__(256) uright_kernel(UrightArgs A) {
    const int cam = blockIdx.y, frame = blockIdx.z;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int fc = frame * A.n_cams + cam, fb = frame * A.n_blocks + cam;
    if (i >= A.n_kp[fc]) return;
    const omv_kp &kp = A.kps[(size_t)fc * A.kp_cap + i];
    const size_t slot = (size_t)fb * A.kp_cap + i;
    float ux, uy;
    fisheye_undistort(A.U[cam], kp.x, kp.y, ux, uy);
    if (A.xy) A.xy[2 * slot] = ux, A.xy[2 * slot + 1] = uy;
    const int x = (int)roundf(ux), y = (int)roundf(uy);
    float d = 0.0f;
    if (!(x < 0 || x >= A.w || y < 0 || y >= A.h)) d = A.depth[((size_t)fb * A.h + y) * A.w + x];
    A.u_right[slot] = (d > 0 && d <= 20) ? kp.x - A.bf / d : -1.0f;
}

// exclusive prefix of the frames' keypoint totals (one workgroup; frames in 256-wide tiles)
__global__ void __launch_bounds__(256) pack_offsets_kernel(const int *n_kp, int n_frames, int n_cams, int n_blocks,
                                                           int *offset) {
    __shared__ int s[256];
    int carry = 0;
    for (int f0 = 0; f0 < n_frames; f0 += 256) {
        const int f = f0 + threadIdx.x;
        int v = 0;
        if (f < n_frames)
            for (int c = 0; c < n_blocks; ++c) v += n_kp[f * n_cams + c];
        s[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {
            const int o = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
            __syncthreads();
            s[threadIdx.x] += o;
            __syncthreads();
        }
        if (f < n_frames) offset[f] = carry + s[threadIdx.x] - v;
        carry += s[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) offset[n_frames] = carry;
}

struct PackArgs {
    const omv_kp *kps;
    const uint8_t *desc;
    const float *ur_in;
    const int *n_kp, *offset;
    int n_cams, n_blocks, kp_cap;
    omv_kp *kps_out;
    uint8_t *desc_out;
    float *ur_out;
};

__global__ void __launch_bounds__(256) pack_kernel(PackArgs A) {
    const int cam = blockIdx.y, frame = blockIdx.z;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int fc = frame * A.n_cams + cam;
    if (i >= A.n_kp[fc]) return;
    int row = A.offset[frame] + i;
    for (int c = 0; c < cam; ++c) row += A.n_kp[frame * A.n_cams + c];
    const size_t slot = (size_t)fc * A.kp_cap + i;
    A.kps_out[row] = A.kps[slot];
    const uint4 *src = (const uint4 *)(A.desc + 32 * slot);
    uint4 *dst = (uint4 *)(A.desc_out + 32 * (size_t)row);
    dst[0] = src[0], dst[1] = src[1];
    if (A.ur_out) A.ur_out[row] = A.ur_in[((size_t)frame * A.n_blocks + cam) * A.kp_cap + i];
}

}  // namespace

extern "C" {

omv_status omv_frame_uright(int n_frames, int n_cams, int n_blocks, int kp_cap, const omv_kp *kps, const int *n_kp,
                            const float *depth, int depth_w, int depth_h, const omv_fisheye_undist *undist, float bf,
                            float *u_right, float *undist_xy, void *stream) {
    if (n_frames < 0 || n_cams <= 0 || n_blocks <= 0 || n_blocks > n_cams || n_blocks > kMaxBlocks || kp_cap <= 0 ||
        depth_w <= 0 || depth_h <= 0)
        return OMV_ERR_ARG;
    if (n_frames == 0) return OMV_OK;
    if (!kps || !n_kp || !depth || !undist || !u_right) return OMV_ERR_ARG;
    UrightArgs A{kps, n_kp, depth, n_cams, n_blocks, kp_cap, depth_w, depth_h, bf, {}, u_right, undist_xy};
    for (int c = 0; c < n_blocks; ++c) A.U[c] = undist[c];
    const dim3 g((kp_cap + 255) / 256, n_blocks, n_frames);
    uright_kernel<<<g, 256, 0, (hipStream_t)stream>>>(A);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

omv_status omv_frame_pack(int n_frames, int n_cams, int n_blocks, int kp_cap, const omv_kp *kps, const uint8_t *desc,
                          const float *uright_in, const int *n_kp, int *offset, omv_kp *kps_out, uint8_t *desc_out,
                          float *uright_out, void *stream) {
    if (n_frames < 0 || n_cams <= 0 || n_blocks <= 0 || n_blocks > n_cams || kp_cap <= 0 || (uright_out && !uright_in))
        return OMV_ERR_ARG;
    if (!offset) return OMV_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (n_frames == 0) {
        HIP_OK(hipMemsetAsync(offset, 0, sizeof(int), st));
        return OMV_OK;
    }
    if (!kps || !desc || !n_kp || !kps_out || !desc_out) return OMV_ERR_ARG;
    pack_offsets_kernel<<<1, 256, 0, st>>>(n_kp, n_frames, n_cams, n_blocks, offset);
    PackArgs A{kps, desc, uright_in, n_kp, offset, n_cams, n_blocks, kp_cap, kps_out, desc_out, uright_out};
    const dim3 g((kp_cap + 255) / 256, n_blocks, n_frames);
    pack_kernel<<<g, 256, 0, st>>>(A);
    HIP_OK(hipGetLastError());
    return OMV_OK;
}

}  // extern "C"
