// TEST INFRASTRUCTURE ONLY — CPU restatement of the multi-camera Frame constructor's tail
// (src/Frame.cc:1913-1939) for parity tests of openmavis_amd/csrc/frame.hip.  Never shipped.
//
// GetDepthFromUndistortedPoints (src/Frame.cc:1659-1765): the keypoints of one camera block are
// undistorted with cv::fisheye::undistortPoints(points, out, origK, dist_coeff, noArray(), newK) and the
// undistorted depth image is read at the rounded pixel; mvuRight = x - bf / d for 0 < d <= 20, else -1.
// cv::fisheye::undistortPoints lives in OpenCV (modules/calib3d/src/fisheye.cpp), a third-party
// dependency absent from /root/reference (the reference does not pin its version); this restates the
// OpenCV >= 4.5 algorithm (criteria MAX_ITER + EPS, 10, 1e-8; theta clipped to +-pi/2; the theta-flip
// guard; (-1e6, -1e6) for unconverged points).  Parity against OpenCV itself is unpinned.
#include <cmath>
#include <cstdint>

#include "../include/omv.h"

namespace {

void undistort(const omv_fisheye_undist &U, float px, float py, float &ox, float &oy) {
    const double f0 = U.K[0], f1 = U.K[1], c0 = U.K[2], c1 = U.K[3];   // Vec2d f, c from the float K
    const double pw0 = ((double)px - c0) / f0, pw1 = ((double)py - c1) / f1;
    double scale = 1.0;
    double theta_d = std::sqrt(pw0 * pw0 + pw1 * pw1);
    theta_d = std::min(std::max(-M_PI / 2., theta_d), M_PI / 2.);
    bool converged = false;
    double theta = theta_d;
    if (theta_d > 1e-8) {
        for (int j = 0; j < 10; j++) {   // Newton on theta (1 + k0 t^2 + ... + k3 t^8) = theta_d
            double t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t6 * t2;
            double a = U.D[0] * t2, b = U.D[1] * t4, c = U.D[2] * t6, d = U.D[3] * t8;
            double fix = (theta * (1 + a + b + c + d) - theta_d) / (1 + 3 * a + 5 * b + 7 * c + 9 * d);
            theta = theta - fix;
            if (std::fabs(fix) < 1e-8) {
                converged = true;
                break;
            }
        }
        scale = std::tan(theta) / theta_d;
    } else {
        converged = true;
    }
    const bool flipped = (theta_d < 0 && theta > 0) || (theta_d > 0 && theta < 0);
    if (!converged || flipped) {
        ox = oy = -1000000.0f;
        return;
    }
    const double pu0 = pw0 * scale, pu1 = pw1 * scale;
    // Matx33d RR = newK * I times Vec3d(pu, 1), each row summed from 0 in column order
    const double P[9] = {U.newK[0], 0, U.newK[2], 0, U.newK[1], U.newK[3], 0, 0, 1};
    double pr[3];
    for (int i = 0; i < 3; ++i) {
        double s = 0;
        s += P[3 * i] * pu0;
        s += P[3 * i + 1] * pu1;
        s += P[3 * i + 2] * 1.0;
        pr[i] = s;
    }
    ox = (float)(pr[0] / pr[2]);
    oy = (float)(pr[1] / pr[2]);
}

}  // namespace

extern "C" {

// One camera block: keys [n] -> u_right [n] (and the undistorted points xy [n][2] when not NULL).
void oracle_depth_from_undistorted(const omv_kp *keys, int n, const float *depth, int w, int h,
                                   const omv_fisheye_undist *U, float bf, float *u_right, float *xy) {
    for (int i = 0; i < n; ++i) {
        float px, py;
        undistort(*U, keys[i].x, keys[i].y, px, py);
        if (xy) xy[2 * i] = px, xy[2 * i + 1] = py;
        const int x = (int)std::round(px), y = (int)std::round(py);
        const float d = (x < 0 || x >= w || y < 0 || y >= h) ? 0.0f : depth[(size_t)y * w + x];
        u_right[i] = (d > 0 && d <= 20) ? keys[i].x - bf / d : -1.0f;
    }
}

}  // extern "C"
