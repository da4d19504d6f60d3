// omv_adapters.hpp — the C++ adapters a maintainer drops into the reference, over the C ABI
// of omv.h only.  OpenCV / Eigen / the map database stay in the reference; these classes take the plain data
// the reference's adapters would hand over (image pointers, keypoint / descriptor vectors, flattened window
// state) so they compile and run here without them (tests/cpp/omv_consumer.cpp exercises every one).
//
//   ORBextractor            ORBextractor::ORBextractor / operator() (include/ORBextractor.h:33-38,
//                           src/ORBextractor.cc:351-414, :987-1071): one image, host memory in and out
//   MultiCameraFrame        the multi-camera Frame ctor's feature part (src/Frame.cc:1767-1949): all cameras
//                           extracted in one batched launch, AssignFeaturesToGrid, the lapping knn + Lowe test
//                           of ComputeMultiFishEyeMatches (:1461-1491), device-resident for the matchers
//   SearchByProjection      ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th, bFar, thFar)
//                           (src/ORBmatcher.cc:23-340) on a MultiCameraFrame
//   LocalInertialBAWindow   Optimizer::LocalInertialBA's graph flattening (src/Optimizer.cc:2740-3267): key
//                           frames (optimisable first, as the reference creates its vertices), points, EdgeMono
//                           and inertial edges in creation order -> omv_lba_problem -> optimize -> write-back
//   SearchByProjectionLastFrame  ORBmatcher::SearchByProjection(Frame&, const Frame& LastFrame, th, bMono)
//                           (src/ORBmatcher.cc:1985-2413) on a MultiCameraFrame
//   SearchForTriangulation  ORBmatcher::SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse)
//                           (src/ORBmatcher.cc:1131-1456, called at LocalMapping.cc:468)
//   PoseInertialOptimizer   Optimizer::PoseInertialOptimizationLastKeyFrame / LastFrame (src/Optimizer.cc:5021,
//                           :5580) on ONE frame (Tracking's call): state, mvbOutlier, return value, the Hessian
//                           of the ConstraintPoseImu
//   Fuse                    ORBmatcher::Fuse(pKF, vpMapPoints, th, cameraID) (src/ORBmatcher.cc:1458-1647,
//                           called 4x per camera at LocalMapping.cc:845-888): the chosen keypoint per point
//   PoseOptimization        Optimizer::PoseOptimization(Frame*) (src/Optimizer.cc:855-1278) on ONE frame
//   CreateNewMapPoints      LocalMapping::CreateNewMapPoints' neighbour loop (src/LocalMapping.cc:395-783):
//                           SearchForTriangulation interleaved with the geometry, the new points in creation order
//   MapPointRefresh         MapPoint::ComputeDistinctiveDescriptors / UpdateNormalAndDepth over a batch of points
//   SearchInNeighborsFuse   LocalMapping::SearchInNeighbors' fuse sequence (src/LocalMapping.cc:837-889): the final
//                           graph and the edit log (AddObservation / Replace) to replay on the reference's objects
//
// Errors: every omv_status != OMV_OK throws omv_adapt::Error (the adapters' callers are C++).
#ifndef OMV_ADAPTERS_HPP
#define OMV_ADAPTERS_HPP

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "omv.h"

namespace omv_adapt {

struct Error : std::runtime_error {
    explicit Error(const std::string &what) : std::runtime_error(what) {}
};

inline void check(omv_status s, const char *what) {
    if (s != OMV_OK) throw Error(std::string(what) + " failed (omv_status " + std::to_string(s) + ")");
}
inline void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e));
}

// Device buffer owned by an adapter.
template <class T>
struct DeviceArray {
    T *p = nullptr;
    size_t n = 0;
    DeviceArray() = default;
    explicit DeviceArray(size_t count) { resize(count); }
    DeviceArray(const DeviceArray &) = delete;
    DeviceArray &operator=(const DeviceArray &) = delete;
    ~DeviceArray() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr, n = 0;
    }
    void resize(size_t count) {
        if (count == n) return;
        release();
        if (count) hip_check(hipMalloc((void **)&p, count * sizeof(T)), "hipMalloc");
        n = count;
    }
    void upload(const T *src, size_t count, hipStream_t st) {
        resize(count);
        if (count) hip_check(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, st), "upload");
    }
    void download(T *dst, size_t count, hipStream_t st) const {
        if (count) hip_check(hipMemcpyAsync(dst, p, count * sizeof(T), hipMemcpyDeviceToHost, st), "download");
    }
};

// ---- ORBextractor ------------------------------------------------------------------------------------------
class ORBextractor {
  public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : p_{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST} {}
    ~ORBextractor() {
        if (h_) (void)omv_orb_destroy(h_);
    }
    ORBextractor(const ORBextractor &) = delete;
    ORBextractor &operator=(const ORBextractor &) = delete;

    // operator()(image, mask, keypoints, descriptors, vLappingArea): returns monoIndex; keypoints in the
    // reference's order (non-lapping from the front, lapping from the back), descriptors 32 bytes per row.
    int operator()(const uint8_t *image, int width, int height, size_t step, std::vector<omv_kp> &keypoints,
                   std::vector<uint8_t> &descriptors, const int lapping[2]) {
        if (!image || width <= 0 || height <= 0) return -1;
        if (!h_ || width != w_ || height != h0_) {
            if (h_) check(omv_orb_destroy(h_), "omv_orb_destroy");
            h_ = nullptr;
            check(omv_orb_create(&p_, width, height, 1, &h_), "omv_orb_create");
            w_ = width, h0_ = height;
        }
        const int cap = omv_orb_max_keypoints(h_);
        keypoints.resize(cap);
        descriptors.resize((size_t)cap * 32);
        int n = 0, mono = 0;
        check(omv_orb_extract_host(h_, image, step, lapping[0], lapping[1], keypoints.data(), descriptors.data(), &n,
                                   &mono),
              "omv_orb_extract_host");
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
        return mono;
    }
    // GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares / GetInverseScaleSigmaSquares
    void scale_tables(std::vector<float> &scale, std::vector<float> &inv_scale, std::vector<float> &sigma2,
                      std::vector<float> &inv_sigma2) const {
        if (!h_) throw Error("ORBextractor: no image extracted yet");
        scale.resize(p_.nlevels), inv_scale.resize(p_.nlevels), sigma2.resize(p_.nlevels), inv_sigma2.resize(p_.nlevels);
        check(omv_orb_scale_tables(h_, scale.data(), inv_scale.data(), sigma2.data(), inv_sigma2.data()),
              "omv_orb_scale_tables");
    }

  private:
    omv_orb_params p_;
    omv_orb *h_ = nullptr;
    int w_ = 0, h0_ = 0;
};

// ---- multi-camera Frame ------------------------------------------------------------------------------------
class MultiCameraFrame {
  public:
    // One rig of n_cams equal-size cameras; lapping: [n_cams][2] (vLappingArea per camera).
    MultiCameraFrame(int n_cams, int width, int height, const omv_orb_params &p, const std::vector<std::array<int, 2>> &lapping,
                     int max_map_points)
        : C_(n_cams), W_(width), H_(height), lap_(2 * n_cams) {
        for (int c = 0; c < C_; ++c) lap_[2 * c] = lapping[c][0], lap_[2 * c + 1] = lapping[c][1];
        hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
        check(omv_orb_create(&p, width, height, n_cams, &orb_), "omv_orb_create");
        cap_ = omv_orb_max_keypoints(orb_);
        check(omv_matcher_create(1, n_cams, cap_, max_map_points, &m_), "omv_matcher_create");
        scale_.resize(p.nlevels);
        std::vector<float> a(p.nlevels), b(p.nlevels), c(p.nlevels);
        check(omv_orb_scale_tables(orb_, scale_.data(), a.data(), b.data(), c.data()), "omv_orb_scale_tables");
        geom_.n_cams = n_cams;
        geom_.min_x = 0.f, geom_.max_x = (float)width, geom_.min_y = 0.f, geom_.max_y = (float)height;   // KB8 / no undistortion
        geom_.nlevels = p.nlevels;
        for (int l = 0; l < p.nlevels && l < 16; ++l) geom_.scale_factors[l] = scale_[l];
        img_.resize((size_t)n_cams * width * height);
        kps_.resize((size_t)n_cams * cap_), desc_.resize((size_t)n_cams * cap_ * 32);
        n_.resize(n_cams), mono_.resize(n_cams), l2r_.resize(cap_), r2l_.resize(cap_);
    }
    ~MultiCameraFrame() {
        if (m_) (void)omv_matcher_destroy(m_);
        if (orb_) (void)omv_orb_destroy(orb_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    MultiCameraFrame(const MultiCameraFrame &) = delete;
    MultiCameraFrame &operator=(const MultiCameraFrame &) = delete;

    // Frame::Frame(...) feature part: images [n_cams] pointers to width x height u8 (row step = width).
    void build(const std::vector<const uint8_t *> &images, double lowe_ratio = 0.8) {
        for (int c = 0; c < C_; ++c)
            hip_check(hipMemcpyAsync(img_.p + (size_t)c * W_ * H_, images[c], (size_t)W_ * H_, hipMemcpyHostToDevice, st_),
                      "upload image");
        check(omv_orb_extract_batch(orb_, C_, img_.p, (size_t)W_ * H_, W_, lap_.data(), kps_.p, desc_.p, n_.p, mono_.p, st_),
              "omv_orb_extract_batch");
        check(omv_matcher_assign_grid(m_, 1, &geom_, kps_.p, n_.p, st_), "omv_matcher_assign_grid");
        if (C_ > 1)
            check(omv_matcher_stereo_lapping(m_, 1, desc_.p, n_.p, mono_.p, lowe_ratio, l2r_.p, r2l_.p, st_),
                  "omv_matcher_stereo_lapping");
        else {
            hip_check(hipMemsetAsync(l2r_.p, 0xff, sizeof(int32_t) * cap_, st_), "l2r");
            hip_check(hipMemsetAsync(r2l_.p, 0xff, sizeof(int32_t) * cap_, st_), "r2l");
        }
        hip_check(hipStreamSynchronize(st_), "frame");
        check(omv_orb_last_error(orb_), "extraction capacity");
        check(omv_matcher_last_error(m_), "matcher capacity");
    }
    // mvKeys / mvKeysRight / ... and mDescriptors of camera block c (host copies)
    void keypoints(int c, std::vector<omv_kp> &k, std::vector<uint8_t> &d) const {
        int n = 0;
        hip_check(hipMemcpy(&n, n_.p + c, sizeof(int), hipMemcpyDeviceToHost), "n");
        k.resize(n), d.resize((size_t)n * 32);
        hip_check(hipMemcpy(k.data(), kps_.p + (size_t)c * cap_, n * sizeof(omv_kp), hipMemcpyDeviceToHost), "kps");
        hip_check(hipMemcpy(d.data(), desc_.p + (size_t)c * cap_ * 32, (size_t)n * 32, hipMemcpyDeviceToHost), "desc");
    }
    void stereo(std::vector<int32_t> &l2r, std::vector<int32_t> &r2l) const {
        l2r.resize(cap_), r2l.resize(cap_);
        hip_check(hipMemcpy(l2r.data(), l2r_.p, sizeof(int32_t) * cap_, hipMemcpyDeviceToHost), "l2r");
        hip_check(hipMemcpy(r2l.data(), r2l_.p, sizeof(int32_t) * cap_, hipMemcpyDeviceToHost), "r2l");
    }
    int n_cams() const { return C_; }
    int kp_cap() const { return cap_; }

    // GeometricCamera type per camera block (OMV_CAM_KB8 default / OMV_CAM_PINHOLE)
    void set_camera_models(const std::vector<int32_t> &models) {
        for (int c = 0; c < C_ && c < 8; ++c) geom_.cam_model[c] = c < (int)models.size() ? models[c] : OMV_CAM_KB8;
    }

  private:
    friend class SearchByProjection;
    friend class SearchByProjectionLastFrame;
    int C_, W_, H_, cap_ = 0;
    std::vector<int> lap_;
    std::vector<float> scale_;
    hipStream_t st_ = nullptr;
    omv_orb *orb_ = nullptr;
    omv_matcher *m_ = nullptr;
    omv_frame_geom geom_{};
    DeviceArray<uint8_t> img_, desc_;
    DeviceArray<omv_kp> kps_;
    DeviceArray<int> n_, mono_;
    DeviceArray<int32_t> l2r_, r2l_;
};

// ---- ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, ...) ---------------------------------
// The MapPoint fields the reference reads after Frame::isInFrustum, one entry per point of the local map (the
// adapter flattens vpMapPoints in order; per-camera arrays are [M][n_cams]).
struct LocalMapView {
    std::vector<uint8_t> desc;                       // [M][32] GetDescriptor()
    std::vector<float> proj_x, proj_y, view_cos;     // [M][C] mTrackProjX / XR / ..., mTrackViewCos*
    std::vector<int32_t> level;                      // [M][C] mnTrackScaleLevel* (-1 none)
    std::vector<uint8_t> in_view;                    // [M][C] mbTrackInView*
    std::vector<float> track_depth;                  // [M] mTrackDepth
    std::vector<uint8_t> is_bad, has_obs;            // [M] isBad(), Observations() > 0
};

class SearchByProjection {
  public:
    explicit SearchByProjection(float nnratio) : nnratio_(nnratio) {}
    // Returns nmatches; kp_to_mp [n_cams * kp_cap] in/out (F.mvpMapPoints as point indices, -1 = NULL, slot =
    // cam * kp_cap + i), occupied_init marks keypoints already holding a point with observations.
    int operator()(MultiCameraFrame &F, const LocalMapView &mp, float th, bool bFarPoints, float thFarPoints,
                   std::vector<int32_t> &kp_to_mp, const std::vector<uint8_t> *occupied_init = nullptr) {
        const int M = (int)mp.track_depth.size();
        hipStream_t st = F.st_;
        desc_.upload(mp.desc.data(), mp.desc.size(), st), px_.upload(mp.proj_x.data(), mp.proj_x.size(), st);
        py_.upload(mp.proj_y.data(), mp.proj_y.size(), st), vc_.upload(mp.view_cos.data(), mp.view_cos.size(), st);
        lv_.upload(mp.level.data(), mp.level.size(), st), iv_.upload(mp.in_view.data(), mp.in_view.size(), st);
        td_.upload(mp.track_depth.data(), mp.track_depth.size(), st), bad_.upload(mp.is_bad.data(), mp.is_bad.size(), st);
        obs_.upload(mp.has_obs.data(), mp.has_obs.size(), st);
        k2m_.upload(kp_to_mp.data(), kp_to_mp.size(), st);
        if (occupied_init) occ_.upload(occupied_init->data(), occupied_init->size(), st);
        nm_.resize(1);
        const omv_mp_view v{desc_.p, px_.p, py_.p, vc_.p, lv_.p, iv_.p, td_.p, bad_.p, obs_.p};
        check(omv_matcher_search_projection(F.m_, 1, &F.geom_, F.kps_.p, F.desc_.p, F.n_.p, &v, M, th, bFarPoints ? 1 : 0,
                                            thFarPoints, nnratio_, F.l2r_.p, F.r2l_.p, occupied_init ? occ_.p : nullptr,
                                            k2m_.p, nm_.p, st),
              "omv_matcher_search_projection");
        int n = 0;
        k2m_.download(kp_to_mp.data(), kp_to_mp.size(), st);
        nm_.download(&n, 1, st);
        hip_check(hipStreamSynchronize(st), "SearchByProjection");
        check(omv_matcher_last_error(F.m_), "matcher capacity");
        return n;
    }

  private:
    float nnratio_;
    DeviceArray<uint8_t> desc_, iv_, bad_, obs_, occ_;
    DeviceArray<float> px_, py_, vc_, td_;
    DeviceArray<int32_t> lv_, k2m_;
    DeviceArray<int> nm_;
};

// ---- Optimizer::LocalInertialBA -----------------------------------------------------------------------------
// ---- ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, th, bMono) --------------------
// The LastFrame fields the reference reads, one slot per LastFrame keypoint s = cam * last_cap + i.
struct LastFrameView {
    int last_cap = 0;                                // keypoint slots per camera block
    std::vector<float> pos;                          // [S][3] mvpMapPoints[s]->GetWorldPos()
    std::vector<uint8_t> desc;                       // [S][32] GetDescriptor()
    std::vector<uint8_t> valid;                      // [S] mvpMapPoints[s] && !mvbOutlier[s]
    std::vector<uint8_t> has_obs;                    // [S] Observations() > 0
    std::vector<omv_kp> keys;                        // [S] LastFrame keypoint s (octave, angle)
    omv_se3f Tcw{};                                  // LastFrame.GetPose() (block 0)
};

class SearchByProjectionLastFrame {
  public:
    SearchByProjectionLastFrame(float nnratio, bool checkOri) : nnratio_(nnratio), check_ori_(checkOri) {}
    // Returns nmatches; kp_to_mp [n_cams * kp_cap] in/out (CurrentFrame.mvpMapPoints as LastFrame slots, -1 NULL).
    // cams [n_cams][8] (block 0's model = CurrentFrame.mpCamera), Tcw the current pose, Trl block 1 from block 0,
    // mb = CurrentFrame.mb; occupied_init: keypoints already holding a point with observations.
    int operator()(MultiCameraFrame &F, const LastFrameView &last, const omv_se3f &Tcw, const omv_se3f &Trl,
                   const std::vector<float> &cams, float th, bool bMono, float mb, std::vector<int32_t> &kp_to_mp,
                   const std::vector<uint8_t> *occupied_init = nullptr) {
        hipStream_t st = F.st_;
        const int S = (int)last.valid.size();
        if ((int)last.pos.size() != 3 * S || (int)last.desc.size() != 32 * S || (int)last.keys.size() != S ||
            (int)last.has_obs.size() != S)
            throw Error("SearchByProjectionLastFrame: inconsistent LastFrameView");
        pos_.upload(last.pos.data(), last.pos.size(), st), desc_.upload(last.desc.data(), last.desc.size(), st);
        val_.upload(last.valid.data(), last.valid.size(), st), obs_.upload(last.has_obs.data(), last.has_obs.size(), st);
        kps_.upload(last.keys.data(), last.keys.size(), st);
        tcw_.upload(&Tcw, 1, st), tlw_.upload(&last.Tcw, 1, st);
        k2m_.upload(kp_to_mp.data(), kp_to_mp.size(), st);
        if (occupied_init) occ_.upload(occupied_init->data(), occupied_init->size(), st);
        nm_.resize(1);
        const omv_last_frame lf{pos_.p, desc_.p, val_.p, obs_.p, kps_.p, S};
        check(omv_matcher_search_last_frame(F.m_, 1, &F.geom_, F.kps_.p, F.desc_.p, F.n_.p, cams.data(), tcw_.p, tlw_.p, &Trl,
                                            &lf, th, bMono ? 1 : 0, mb, check_ori_ ? 1 : 0,
                                            occupied_init ? occ_.p : nullptr, k2m_.p, nm_.p, st),
              "omv_matcher_search_last_frame");
        int n = 0;
        k2m_.download(kp_to_mp.data(), kp_to_mp.size(), st);
        nm_.download(&n, 1, st);
        hip_check(hipStreamSynchronize(st), "SearchByProjectionLastFrame");
        check(omv_matcher_last_error(F.m_), "matcher capacity");
        return n;
    }

  private:
    float nnratio_;
    bool check_ori_;
    DeviceArray<float> pos_;
    DeviceArray<uint8_t> desc_, val_, obs_, occ_;
    DeviceArray<omv_kp> kps_;
    DeviceArray<omv_se3f> tcw_, tlw_;
    DeviceArray<int32_t> k2m_;
    DeviceArray<int> nm_;
};

// ---- ORBmatcher::SearchForTriangulation ------------------------------------------------------------------------
// The KeyFrame fields SearchForTriangulation reads, keypoints in the reference's [L | R | SL | SR] index order.
struct KeyFrameView {
    int N = 0, NLeft = -1, NRight = 0, NSideLeft = 0;
    std::vector<omv_kp> keys;                        // [N] mvKeys / mvKeysRight / mvKeysSideLeft / mvKeysSideRight
    std::vector<uint8_t> descriptors;                // [N][32] mDescriptors
    std::vector<uint8_t> has_map_point;              // [N] GetMapPoint(idx) != NULL
    std::vector<uint32_t> feat_node;                 // mFeatVec: node ids ascending ...
    std::vector<int32_t> feat_start, feat_idx;       // ... with their keypoint indices (CSR, [nodes + 1] / [..])
    std::array<float, 16> level_sigma2{};            // mvLevelSigma2
};

class SearchForTriangulation {
  public:
    SearchForTriangulation(float nnratio, bool checkOri) : check_ori_(checkOri) {
        (void)nnratio;   // the reference's ratio test is not applied in SearchForTriangulation
        hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
        check(omv_matcher_create(1, 1, 1, 1, &m_), "omv_matcher_create");
    }
    ~SearchForTriangulation() {
        if (m_) (void)omv_matcher_destroy(m_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    SearchForTriangulation(const SearchForTriangulation &) = delete;
    SearchForTriangulation &operator=(const SearchForTriangulation &) = delete;

    // Returns nmatches and vMatchedPairs (idx1, idx2) in idx1 order.  T: the 10 camera-pair transforms (R12 | t12)
    // in OMV_TRI_PAIRS order; cams [4][8] and cam_model [4] (OMV_CAM_KB8 / OMV_CAM_PINHOLE) of the L, R, SL, SR cameras.
    int operator()(const KeyFrameView &kf1, const KeyFrameView &kf2, const std::array<std::array<float, 12>, OMV_TRI_PAIRS> &T,
                   const std::vector<float> &cams, const std::vector<int32_t> &cam_model,
                   std::vector<std::pair<size_t, size_t>> &vMatchedPairs, bool bOnlyStereo, bool bCoarse = false) {
        omv_tri_pair p{};
        view(kf1, a_, p.kf1);
        view(kf2, b_, p.kf2);
        for (int q = 0; q < OMV_TRI_PAIRS; ++q) std::copy(T[q].begin(), T[q].end(), p.T[q]);
        m12_.resize(std::max(1, kf1.N));
        p.match12 = m12_.p;
        nm_.resize(1);
        check(omv_matcher_search_for_triangulation(m_, 1, &p, cams.data(), cam_model.empty() ? nullptr : cam_model.data(),
                                                   bOnlyStereo ? 1 : 0, bCoarse ? 1 : 0, check_ori_ ? 1 : 0, nm_.p, st_),
              "omv_matcher_search_for_triangulation");
        std::vector<int32_t> m12(kf1.N);
        int n = 0;
        m12_.download(m12.data(), kf1.N, st_);
        nm_.download(&n, 1, st_);
        hip_check(hipStreamSynchronize(st_), "SearchForTriangulation");
        vMatchedPairs.clear();
        for (int i = 0; i < kf1.N; ++i)
            if (m12[i] >= 0) vMatchedPairs.emplace_back((size_t)i, (size_t)m12[i]);
        return n;
    }

  private:
    struct Buf {
        DeviceArray<omv_kp> kps;
        DeviceArray<uint8_t> desc, has_mp;
        DeviceArray<uint32_t> node;
        DeviceArray<int32_t> start, idx;
    };
    void view(const KeyFrameView &k, Buf &b, omv_kf_view &v) {
        if ((int)k.keys.size() != k.N || (int)k.descriptors.size() != 32 * k.N || (int)k.has_map_point.size() != k.N ||
            k.feat_start.size() != k.feat_node.size() + 1)
            throw Error("SearchForTriangulation: inconsistent KeyFrameView");
        b.kps.upload(k.keys.data(), k.keys.size(), st_), b.desc.upload(k.descriptors.data(), k.descriptors.size(), st_);
        b.has_mp.upload(k.has_map_point.data(), k.has_map_point.size(), st_);
        b.node.upload(k.feat_node.data(), k.feat_node.size(), st_);
        b.start.upload(k.feat_start.data(), k.feat_start.size(), st_), b.idx.upload(k.feat_idx.data(), k.feat_idx.size(), st_);
        v.n = k.N, v.n_left = k.NLeft, v.n_right = k.NRight, v.n_sideleft = k.NSideLeft;
        v.kps = b.kps.p, v.desc = b.desc.p, v.has_mp = b.has_mp.p;
        v.n_nodes = (int)k.feat_node.size(), v.node_id = b.node.p, v.node_start = b.start.p, v.node_idx = b.idx.p;
        std::copy(k.level_sigma2.begin(), k.level_sigma2.end(), v.level_sigma2);
    }
    bool check_ori_;
    hipStream_t st_ = nullptr;
    omv_matcher *m_ = nullptr;
    Buf a_, b_;
    DeviceArray<int32_t> m12_;
    DeviceArray<int32_t> nm_;
};

// ---- Optimizer::PoseInertialOptimizationLastKeyFrame / LastFrame -----------------------------------------------
class PoseInertialOptimizer {
  public:
    struct State {   // a frame's (or keyframe's) VertexPose / VertexVelocity / VertexGyroBias / VertexAccBias
        std::array<double, 9> Rwb{};
        std::array<double, 3> twb{}, vel{}, bg{}, ba{};
        std::vector<std::array<double, 9>> Rcw;   // [n_cams] ImuCamPose::Rcw
        std::vector<std::array<double, 3>> tcw;   // [n_cams]
    };
    struct Mono {     // EdgeMonoOnlyPose: keypoint idx of camera `cam`, obs (u, v), invSigma2 / unc2, GetWorldPos
        int cam, kp;
        double u, v;
        float inv_sigma2;
        std::array<float, 3> Xw;
        bool close;   // mTrackDepth < 10 (bClose)
    };
    struct Stereo {   // EdgeStereoOnlyPose: obs (u, v, u_R)
        int cam, kp;
        double u, v, ur;
        float inv_sigma2;
        std::array<float, 3> Xw;
    };
    struct Prior {    // Frame::mpcpi of the previous frame (ConstraintPoseImu: Rwb twb vwb bg ba and H)
        std::array<double, 9> Rwb{};
        std::array<double, 3> twb{}, vel{}, bg{}, ba{};
        std::array<double, 225> H{};
    };

    PoseInertialOptimizer(int n_cams, std::vector<float> cams, std::vector<double> Rcb, std::vector<double> tcb,
                          std::vector<double> Rbc, std::vector<double> tbc, float bf = 0.f, std::vector<int32_t> cam_model = {})
        : C_(n_cams), cam_(std::move(cams)), Rcb_(std::move(Rcb)), tcb_(std::move(tcb)), Rbc_(std::move(Rbc)),
          tbc_(std::move(tbc)), bf_(bf), model_(std::move(cam_model)) {
        hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~PoseInertialOptimizer() {
        if (h_) (void)omv_pose_destroy(h_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    PoseInertialOptimizer(const PoseInertialOptimizer &) = delete;
    PoseInertialOptimizer &operator=(const PoseInertialOptimizer &) = delete;

    // PoseInertialOptimizationLastKeyFrame(pFrame, bRecInit): returns nInitialCorrespondences - nBad, updates `frame`
    // and mvbOutlier (the keypoints carrying an edge; [kp_cap]), H (may be null) receives the 15x15 Hessian the
    // reference hands to ConstraintPoseImu (:5529-5571).  preint: Frame::mpImuPreintegrated (OMV_PREINT_FLOATS).
    int LastKeyFrame(State &frame, const State &kf, const std::vector<float> &preint, const std::vector<Mono> &mono,
                     const std::vector<Stereo> &stereo, std::vector<uint8_t> &mvbOutlier, std::array<double, 225> *H,
                     bool bRecInit) {
        return run(frame, kf, preint, nullptr, nullptr, mono, stereo, mvbOutlier, H, bRecInit);
    }
    // PoseInertialOptimizationLastFrame(pFrame, bRecInit): `prev` = Frame::mpPrevFrame's state (free, not written
    // back), preint_frame = mpImuPreintegratedFrame, preint_kf = mpImuPreintegrated (random-walk information), prior
    // = pFp->mpcpi.  H receives Marginalize(H, 0, 14)'s frame block (:6158); ConstraintPoseImu(H) makes the next prior.
    int LastFrame(State &frame, const State &prev, const std::vector<float> &preint_frame, const std::vector<float> &preint_kf,
                  const Prior &prior, const std::vector<Mono> &mono, const std::vector<Stereo> &stereo,
                  std::vector<uint8_t> &mvbOutlier, std::array<double, 225> *H, bool bRecInit) {
        return run(frame, prev, preint_frame, &preint_kf, &prior, mono, stereo, mvbOutlier, H, bRecInit);
    }
    // The ConstraintPoseImu ctor's projection of H (include/G2oTypes.h:639-659).
    std::array<double, 225> ConstraintPoseImu(const std::array<double, 225> &H) {
        h_in_.upload(H.data(), 225, st_);
        h_out_.resize(225);
        check(omv_pose_constraint(1, h_in_.p, h_out_.p, st_), "omv_pose_constraint");
        std::array<double, 225> out{};
        h_out_.download(out.data(), 225, st_);
        hip_check(hipStreamSynchronize(st_), "ConstraintPoseImu");
        return out;
    }

  private:
    int run(State &frame, const State &other, const std::vector<float> &preint, const std::vector<float> *preint_kf,
            const Prior *prior, const std::vector<Mono> &mono, const std::vector<Stereo> &stereo,
            std::vector<uint8_t> &kpo, std::array<double, 225> *H, bool rec_init) {
        const int nm = (int)mono.size(), ns = (int)stereo.size();
        if ((int)frame.Rcw.size() != C_ || (int)frame.tcw.size() != C_ || (int)preint.size() != OMV_PREINT_FLOATS ||
            (preint_kf && (int)preint_kf->size() != OMV_PREINT_FLOATS) || kpo.empty())
            throw Error("PoseInertialOptimizer: inconsistent inputs");
        const int need = std::max(nm, ns);
        if (!h_ || need > cap_) {
            if (h_) (void)omv_pose_destroy(h_), h_ = nullptr;
            cap_ = std::max(need, std::max(1, cap_));
            check(omv_pose_create(1, cap_, &h_), "omv_pose_create");
        }
        auto st3 = [](const State &s, std::vector<double> &R, std::vector<double> &t, std::vector<double> &v,
                      std::vector<double> &g, std::vector<double> &a) {
            R.assign(s.Rwb.begin(), s.Rwb.end()), t.assign(s.twb.begin(), s.twb.end()), v.assign(s.vel.begin(), s.vel.end());
            g.assign(s.bg.begin(), s.bg.end()), a.assign(s.ba.begin(), s.ba.end());
        };
        std::vector<double> R, t, v, g, a, kR, kt, kv, kg, ka, Rc, tc;
        st3(frame, R, t, v, g, a);
        st3(other, kR, kt, kv, kg, ka);
        for (int c = 0; c < C_; ++c) {
            Rc.insert(Rc.end(), frame.Rcw[c].begin(), frame.Rcw[c].end());
            tc.insert(tc.end(), frame.tcw[c].begin(), frame.tcw[c].end());
        }
        Rwb_.upload(R.data(), 9, st_), twb_.upload(t.data(), 3, st_), vel_.upload(v.data(), 3, st_);
        bg_.upload(g.data(), 3, st_), ba_.upload(a.data(), 3, st_), Rcw_.upload(Rc.data(), Rc.size(), st_);
        tcw_.upload(tc.data(), tc.size(), st_);
        kR_.upload(kR.data(), 9, st_), kt_.upload(kt.data(), 3, st_), kv_.upload(kv.data(), 3, st_);
        kg_.upload(kg.data(), 3, st_), ka_.upload(ka.data(), 3, st_);
        pre_.upload(preint.data(), preint.size(), st_);
        std::vector<int32_t> mstart{0, nm}, sstart{0, ns}, mcam(nm), mkp(nm), scam(ns), skp(ns);
        std::vector<double> mobs(2 * (size_t)nm), sobs(3 * (size_t)ns);
        std::vector<float> mw(nm), mx(3 * (size_t)nm), sw(ns), sx(3 * (size_t)ns);
        std::vector<uint8_t> mclose(nm);
        for (int e = 0; e < nm; ++e) {
            const Mono &m = mono[e];
            mcam[e] = m.cam, mkp[e] = m.kp, mobs[2 * e] = m.u, mobs[2 * e + 1] = m.v, mw[e] = m.inv_sigma2;
            std::copy(m.Xw.begin(), m.Xw.end(), &mx[3 * e]);
            mclose[e] = m.close ? 1 : 0;
        }
        for (int e = 0; e < ns; ++e) {
            const Stereo &m = stereo[e];
            scam[e] = m.cam, skp[e] = m.kp, sobs[3 * e] = m.u, sobs[3 * e + 1] = m.v, sobs[3 * e + 2] = m.ur;
            sw[e] = m.inv_sigma2;
            std::copy(m.Xw.begin(), m.Xw.end(), &sx[3 * e]);
        }
        ms_.upload(mstart.data(), 2, st_), ss_.upload(sstart.data(), 2, st_);
        mcam_.upload(mcam.data(), nm, st_), mkp_.upload(mkp.data(), nm, st_), mobs_.upload(mobs.data(), mobs.size(), st_);
        mw_.upload(mw.data(), nm, st_), mx_.upload(mx.data(), mx.size(), st_), mclose_.upload(mclose.data(), nm, st_);
        scam_.upload(scam.data(), ns, st_), skp_.upload(skp.data(), ns, st_), sobs_.upload(sobs.data(), sobs.size(), st_);
        sw_.upload(sw.data(), ns, st_), sx_.upload(sx.data(), sx.size(), st_);
        kpo_.upload(kpo.data(), kpo.size(), st_);
        ng_.resize(1), H_.resize(225);
        omv_pose_batch b{};
        b.n_frames = 1, b.n_cams = C_, b.cam = cam_.data(), b.Rcb = Rcb_.data(), b.tcb = tcb_.data(), b.Rbc = Rbc_.data();
        b.tbc = tbc_.data(), b.bf = bf_;
        b.Rwb = Rwb_.p, b.twb = twb_.p, b.Rcw = Rcw_.p, b.tcw = tcw_.p, b.vel = vel_.p, b.bg = bg_.p, b.ba = ba_.p;
        b.kf_Rwb = kR_.p, b.kf_twb = kt_.p, b.kf_vel = kv_.p, b.kf_bg = kg_.p, b.kf_ba = ka_.p, b.preint = pre_.p;
        b.mono_start = ms_.p, b.mono_cam = mcam_.p, b.mono_kp = mkp_.p, b.mono_obs = mobs_.p, b.mono_inv_sigma2 = mw_.p;
        b.mono_xw = mx_.p, b.mono_close = mclose_.p;
        b.stereo_start = ss_.p, b.stereo_cam = scam_.p, b.stereo_kp = skp_.p, b.stereo_obs = sobs_.p;
        b.stereo_inv_sigma2 = sw_.p, b.stereo_xw = sx_.p;
        b.kp_cap = (int)kpo.size(), b.n_mono = nm, b.n_stereo = ns;
        b.cam_model = model_.empty() ? nullptr : model_.data();
        if (prior) {
            pR_.upload(prior->Rwb.data(), 9, st_), pt_.upload(prior->twb.data(), 3, st_), pv_.upload(prior->vel.data(), 3, st_);
            pg_.upload(prior->bg.data(), 3, st_), pa_.upload(prior->ba.data(), 3, st_), pH_.upload(prior->H.data(), 225, st_);
            pkf_.upload(preint_kf->data(), preint_kf->size(), st_);
            const omv_pose_prior pp{pR_.p, pt_.p, pv_.p, pg_.p, pa_.p, pH_.p, pkf_.p};
            check(omv_pose_inertial_last_frame(h_, &b, &pp, rec_init ? 1 : 0, kpo_.p, ng_.p, H ? H_.p : nullptr, st_),
                  "omv_pose_inertial_last_frame");
        } else {
            check(omv_pose_inertial_last_kf(h_, &b, rec_init ? 1 : 0, kpo_.p, ng_.p, H ? H_.p : nullptr, st_),
                  "omv_pose_inertial_last_kf");
        }
        int n_good = 0;
        ng_.download(&n_good, 1, st_);
        kpo_.download(kpo.data(), kpo.size(), st_);
        if (H) H_.download(H->data(), 225, st_);
        Rwb_.download(R.data(), 9, st_), twb_.download(t.data(), 3, st_), vel_.download(v.data(), 3, st_);
        bg_.download(g.data(), 3, st_), ba_.download(a.data(), 3, st_);
        Rcw_.download(Rc.data(), Rc.size(), st_), tcw_.download(tc.data(), tc.size(), st_);
        hip_check(hipStreamSynchronize(st_), "PoseInertialOptimizer");
        int32_t err = 0;
        check(omv_pose_last_error(h_, &err, st_), "omv_pose_last_error");
        if (err != 0) throw Error("PoseInertialOptimizer: device error " + std::to_string(err));
        std::copy_n(R.begin(), 9, frame.Rwb.begin()), std::copy_n(t.begin(), 3, frame.twb.begin());
        std::copy_n(v.begin(), 3, frame.vel.begin()), std::copy_n(g.begin(), 3, frame.bg.begin());
        std::copy_n(a.begin(), 3, frame.ba.begin());
        for (int c = 0; c < C_; ++c) {
            std::copy_n(&Rc[9 * (size_t)c], 9, frame.Rcw[c].begin());
            std::copy_n(&tc[3 * (size_t)c], 3, frame.tcw[c].begin());
        }
        return n_good;
    }

    int C_;
    std::vector<float> cam_;
    std::vector<double> Rcb_, tcb_, Rbc_, tbc_;
    float bf_;
    std::vector<int32_t> model_;
    hipStream_t st_ = nullptr;
    omv_pose *h_ = nullptr;
    int cap_ = 0;
    DeviceArray<double> Rwb_, twb_, vel_, bg_, ba_, Rcw_, tcw_, kR_, kt_, kv_, kg_, ka_, mobs_, sobs_, H_, pR_, pt_, pv_,
        pg_, pa_, pH_, h_in_, h_out_;
    DeviceArray<float> pre_, pkf_, mw_, mx_, sw_, sx_;
    DeviceArray<int32_t> ms_, ss_, mcam_, mkp_, scam_, skp_, ng_;
    DeviceArray<uint8_t> mclose_, kpo_;
};

// ---- ORBmatcher::Fuse(pKF, vpMapPoints, th, cameraID) ----------------------------------------------------------
// One keyframe whose keypoints are indexed into the grid once (KeyFrame::GetFeaturesInArea); Fuse runs per camera
// block and returns, per map point of the list, the keyframe keypoint chosen (N-index, -1 none) and its distance:
// the caller applies pMPinKF->Replace / AddObservation for best_dist <= TH_LOW in list order (:1620-1640), as the
// map-graph mutation stays with the reference.
struct FuseMapPoints {
    std::vector<float> pos, normal;                  // [M][3] GetWorldPos(), GetNormal()
    std::vector<float> min_dist, max_dist;           // [M] mfMinDistance, mfMaxDistance
    std::vector<uint8_t> desc;                       // [M][32] GetDescriptor()
};

class Fuse {
  public:
    // The keyframe: keypoints per camera block ([n_cams][kp_cap], n_kp per block), descriptors, mvuRight of block 0,
    // image bounds and scale factors; cams [n_cams][8] with their models.
    Fuse(int n_cams, int kp_cap, int width, int height, const std::vector<float> &scale_factors, const std::vector<float> &cams,
         const std::vector<int32_t> &cam_model, float bf, int max_points)
        : C_(n_cams), cap_(kp_cap), cams_(cams), bf_(bf), sf_(scale_factors) {
        hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
        check(omv_matcher_create(1, n_cams, kp_cap, std::max(1, max_points), &m_), "omv_matcher_create");
        geom_.n_cams = n_cams, geom_.min_x = 0.f, geom_.max_x = (float)width, geom_.min_y = 0.f, geom_.max_y = (float)height;
        geom_.nlevels = (int)scale_factors.size();
        for (int l = 0; l < geom_.nlevels && l < 16; ++l) geom_.scale_factors[l] = scale_factors[l];
        for (int c = 0; c < n_cams && c < 8; ++c) geom_.cam_model[c] = cam_model.empty() ? OMV_CAM_KB8 : cam_model[c];
    }
    ~Fuse() {
        if (m_) (void)omv_matcher_destroy(m_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    Fuse(const Fuse &) = delete;
    Fuse &operator=(const Fuse &) = delete;

    // The keyframe's keypoints (block-major [n_cams][kp_cap], n_kp per block), descriptors and block-0 mvuRight.
    void set_keyframe(const std::vector<omv_kp> &kps, const std::vector<uint8_t> &desc, const std::vector<int> &n_kp,
                      const std::vector<float> &uright) {
        kps_.upload(kps.data(), kps.size(), st_), desc_.upload(desc.data(), desc.size(), st_);
        n_.upload(n_kp.data(), n_kp.size(), st_), ur_.upload(uright.data(), uright.size(), st_);
        check(omv_matcher_assign_grid(m_, 1, &geom_, kps_.p, n_.p, st_), "omv_matcher_assign_grid");
    }
    // Fuse(pKF, vpMapPoints, th, cameraID): Tcw / Ow of camera block `cam` (GetPose / GetRightPose ...,
    // GetCameraCenter ...); inv_level_sigma2 = mvInvLevelSigma2.  The points the reference skips before projecting
    // (NULL, isBad(), IsInKeyFrame(pKF)) are left out of `mps` by the caller.  Returns nFused.
    int operator()(const FuseMapPoints &mps, int cam, const omv_se3f &Tcw, const std::array<float, 3> &Ow, float th,
                   const std::vector<float> &inv_level_sigma2, std::vector<int32_t> &best_idx, std::vector<int32_t> &best_dist) {
        const int M = (int)mps.min_dist.size();
        pos_.upload(mps.pos.data(), mps.pos.size(), st_), nrm_.upload(mps.normal.data(), mps.normal.size(), st_);
        mind_.upload(mps.min_dist.data(), M, st_), maxd_.upload(mps.max_dist.data(), M, st_);
        mdesc_.upload(mps.desc.data(), mps.desc.size(), st_);
        std::vector<int32_t> list(M);
        for (int i = 0; i < M; ++i) list[i] = i;
        list_.upload(list.data(), M, st_);
        bi_.resize(std::max(1, M)), bd_.resize(std::max(1, M)), nm_.resize(1);
        omv_kf_search_job job{};
        job.kf = 0, job.cam = cam, job.Tcw = Tcw, job.mp_start = 0, job.mp_count = M;
        std::copy(Ow.begin(), Ow.end(), job.Ow);
        omv_kf_search_params p{};
        p.mode = OMV_KF_FUSE, p.th = th, p.max_dist = 50.f, p.bf = bf_, p.uright = ur_.p;
        for (int l = 0; l < (int)inv_level_sigma2.size() && l < 16; ++l) p.inv_level_sigma2[l] = inv_level_sigma2[l];
        p.log_scale_factor = (float)std::log((double)sf_[1]);
        p.n_levels = geom_.nlevels;
        for (int c = 0; c < C_ && c < 8; ++c)
            for (int q = 0; q < 8; ++q) p.cams[c][q] = cams_[8 * c + q];
        const omv_kf_mps kfm{pos_.p, nrm_.p, mind_.p, maxd_.p, mdesc_.p};
        check(omv_matcher_search_kf(m_, 1, &geom_, kps_.p, desc_.p, n_.p, 1, &job, M, list_.p, &kfm, &p, nullptr, bi_.p,
                                    bd_.p, nm_.p, st_),
              "omv_matcher_search_kf");
        best_idx.resize(M), best_dist.resize(M);
        int n = 0;
        bi_.download(best_idx.data(), M, st_), bd_.download(best_dist.data(), M, st_), nm_.download(&n, 1, st_);
        hip_check(hipStreamSynchronize(st_), "Fuse");
        check(omv_matcher_last_error(m_), "matcher capacity");
        return n;
    }

  private:
    int C_, cap_;
    std::vector<float> cams_;
    float bf_;
    std::vector<float> sf_;
    hipStream_t st_ = nullptr;
    omv_matcher *m_ = nullptr;
    omv_frame_geom geom_{};
    DeviceArray<omv_kp> kps_;
    DeviceArray<uint8_t> desc_, mdesc_;
    DeviceArray<int> n_;
    DeviceArray<float> ur_, pos_, nrm_, mind_, maxd_;
    DeviceArray<int32_t> list_, bi_, bd_, nm_;
};

// ---- Optimizer::PoseOptimization(Frame*) ------------------------------------------------------------------------
// The visual-only pose optimisation of Tracking (Optimizer.cc:855-1278) on ONE frame.  The frame's edges as the
// reference creates them (:907-1121): one per matched keypoint -- a mono edge on the keypoint's camera block c (through
// T_c0 = mTrl / mTsll / mTsrl) or, on a conventional (single-camera) frame, a stereo edge instead when mvuRight >= 0.
class PoseOptimization {
  public:
    struct Mono {     // EdgeSE3ProjectXYZOnlyPose / ...ToBody / ...SLPoseToBody / ...SRPoseToBody
        int cam, kp;  // camera block, keypoint index i (mvbOutlier[i])
        double u, v;
        float inv_sigma2;
        std::array<float, 3> Xw;
    };
    struct Stereo {   // EdgeStereoSE3ProjectXYZOnlyPose (camera 0)
        int kp;
        double u, v, ur;
        float inv_sigma2;
        std::array<float, 3> Xw;
    };
    // cams [n_cams][8] with their models; rig_q / rig_t: T_c0 per camera block as the SE3Quat the reference builds from
    // GetRelativePoseTrl() / Tsll / Tsrl (entry 0 unused); bf = Frame::mbf.
    PoseOptimization(int n_cams, std::vector<float> cams, std::vector<int32_t> cam_model, float bf,
                     std::vector<std::array<double, 4>> rig_q, std::vector<std::array<double, 3>> rig_t)
        : C_(n_cams), cam_(std::move(cams)), model_(std::move(cam_model)), bf_(bf) {
        if ((int)rig_q.size() != n_cams || (int)rig_t.size() != n_cams) throw Error("PoseOptimization: rig size");
        for (auto &q : rig_q) rq_.insert(rq_.end(), q.begin(), q.end());
        for (auto &t : rig_t) rt_.insert(rt_.end(), t.begin(), t.end());
        hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~PoseOptimization() {
        if (h_) (void)omv_pose_destroy(h_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    PoseOptimization(const PoseOptimization &) = delete;
    PoseOptimization &operator=(const PoseOptimization &) = delete;

    // int Optimizer::PoseOptimization(Frame *pFrame): q / t = pFrame->GetPose() as the SE3Quat of :871-873 (in), the
    // optimised estimate (out, pFrame->SetPose); mvbOutlier [kp_cap] of the edges' keypoints; returns nGood.
    int operator()(std::array<double, 4> &q, std::array<double, 3> &t, const std::vector<Mono> &mono,
                   const std::vector<Stereo> &stereo, std::vector<uint8_t> &mvbOutlier) {
        const int nm = (int)mono.size(), ns = (int)stereo.size();
        if (mvbOutlier.empty()) throw Error("PoseOptimization: empty mvbOutlier");
        const int need = std::max(1, std::max(nm, ns));
        if (!h_ || need > cap_) {
            if (h_) (void)omv_pose_destroy(h_), h_ = nullptr;
            cap_ = need;
            check(omv_pose_create(1, cap_, &h_), "omv_pose_create");
        }
        std::vector<int32_t> mstart{0, nm}, sstart{0, ns}, mcam(nm), mkp(nm), scam(ns, 0), skp(ns);
        std::vector<double> mobs(2 * (size_t)nm), sobs(3 * (size_t)ns);
        std::vector<float> mw(nm), mx(3 * (size_t)nm), sw(ns), sx(3 * (size_t)ns);
        for (int e = 0; e < nm; ++e) {
            const Mono &m = mono[e];
            mcam[e] = m.cam, mkp[e] = m.kp, mobs[2 * e] = m.u, mobs[2 * e + 1] = m.v, mw[e] = m.inv_sigma2;
            std::copy(m.Xw.begin(), m.Xw.end(), &mx[3 * e]);
        }
        for (int e = 0; e < ns; ++e) {
            const Stereo &m = stereo[e];
            skp[e] = m.kp, sobs[3 * e] = m.u, sobs[3 * e + 1] = m.v, sobs[3 * e + 2] = m.ur, sw[e] = m.inv_sigma2;
            std::copy(m.Xw.begin(), m.Xw.end(), &sx[3 * e]);
        }
        ms_.upload(mstart.data(), 2, st_), ss_.upload(sstart.data(), 2, st_);
        mcam_.upload(mcam.data(), nm, st_), mkp_.upload(mkp.data(), nm, st_), mobs_.upload(mobs.data(), mobs.size(), st_);
        mw_.upload(mw.data(), nm, st_), mx_.upload(mx.data(), mx.size(), st_);
        scam_.upload(scam.data(), ns, st_), skp_.upload(skp.data(), ns, st_), sobs_.upload(sobs.data(), sobs.size(), st_);
        sw_.upload(sw.data(), ns, st_), sx_.upload(sx.data(), sx.size(), st_);
        kpo_.upload(mvbOutlier.data(), mvbOutlier.size(), st_);
        q_.upload(q.data(), 4, st_), t_.upload(t.data(), 3, st_);
        ng_.resize(1);
        omv_pose_batch b{};
        b.n_frames = 1, b.n_cams = C_, b.cam = cam_.data(), b.bf = bf_;
        b.cam_model = model_.empty() ? nullptr : model_.data();
        b.mono_start = ms_.p, b.mono_cam = mcam_.p, b.mono_kp = mkp_.p, b.mono_obs = mobs_.p, b.mono_inv_sigma2 = mw_.p;
        b.mono_xw = mx_.p;
        b.stereo_start = ss_.p, b.stereo_cam = scam_.p, b.stereo_kp = skp_.p, b.stereo_obs = sobs_.p;
        b.stereo_inv_sigma2 = sw_.p, b.stereo_xw = sx_.p;
        b.kp_cap = (int)mvbOutlier.size(), b.n_mono = nm, b.n_stereo = ns;
        check(omv_pose_optimization(h_, &b, rq_.data(), rt_.data(), q_.p, t_.p, kpo_.p, ng_.p, st_),
              "omv_pose_optimization");
        int n_good = 0;
        ng_.download(&n_good, 1, st_);
        kpo_.download(mvbOutlier.data(), mvbOutlier.size(), st_);
        q_.download(q.data(), 4, st_), t_.download(t.data(), 3, st_);
        hip_check(hipStreamSynchronize(st_), "PoseOptimization");
        return n_good;
    }

  private:
    int C_;
    std::vector<float> cam_;
    std::vector<int32_t> model_;
    float bf_;
    std::vector<double> rq_, rt_;
    hipStream_t st_ = nullptr;
    omv_pose *h_ = nullptr;
    int cap_ = 0;
    DeviceArray<double> mobs_, sobs_, q_, t_;
    DeviceArray<float> mw_, mx_, sw_, sx_;
    DeviceArray<int32_t> ms_, ss_, mcam_, mkp_, scam_, skp_, ng_;
    DeviceArray<uint8_t> kpo_;
};

// ---- LocalMapping::CreateNewMapPoints (LocalMapping.cc:395-783) -------------------------------------------------
// The keyframe fields the loop reads: the SearchForTriangulation view plus the geometry of the per-match checks.
struct CnmpKeyFrame {
    KeyFrameView view;                                 // kps [L|R|SL|SR], mDescriptors, GetMapPoint != NULL, mFeatVec
    std::array<std::array<float, 12>, 4> Tcw{};        // GetPose / GetRightPose / GetSideLeftPose / GetSideRightPose
    std::array<std::array<float, 3>, 4> Ow{};          // the matching camera centres
    std::array<float, 9> Rwc{};                        // mRwc (UnprojectStereo)
    std::array<float, 3> twc{};                        // mTwc.translation()
    float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mb = 0, mbf = 0;
    std::vector<float> uright, depth;                  // [N] mvuRight / mvDepth, or empty
    std::array<float, 16> scale_factors{};             // mvScaleFactors
};
// One MapPoint the loop creates, in the reference's creation order (neighbour, then idx1 ascending): new MapPoint(x3D,
// mpCurrentKeyFrame), AddObservation(pKF1, idx1) / (pKF2, idx2), AddMapPoint on both (:766-781).
struct NewMapPoint {
    int neighbour;
    size_t idx1, idx2;
    std::array<float, 3> x3D;
    bool stereo;   // bPointStereo (UnprojectStereo)
};

class CreateNewMapPoints {
  public:
    // cams [4][8] / cam_model [4] of the rig (L, R, SL, SR); n_cams 2 or 4 (the multi-camera rigs the device search
    // covers); mbInertial, mbMonocular (no baseline gate; its median-depth test arrives as `skip`), mbFarPoints /
    // mThFarPoints.
    CreateNewMapPoints(std::vector<float> cams, std::vector<int32_t> cam_model, int n_cams, bool inertial, bool monocular,
                       bool far_points, float th_far)
        : cams_(std::move(cams)), model_(std::move(cam_model)), C_(n_cams), inertial_(inertial), mono_(monocular),
          far_(far_points), th_far_(th_far) {
        hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
        check(omv_matcher_create(1, 1, 1, 1, &m_), "omv_matcher_create");
        side1_.resize(1);
    }
    ~CreateNewMapPoints() {
        if (m_) (void)omv_matcher_destroy(m_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    CreateNewMapPoints(const CreateNewMapPoints &) = delete;
    CreateNewMapPoints &operator=(const CreateNewMapPoints &) = delete;

    // The loop over vpNeighKFs [lo, hi): has_mp1 [N1] in/out (the current keyframe's GetMapPoint != NULL; the created
    // points' slots set on return); T[i]: neighbour i's ten camera-pair transforms (section 6); skip[i]: the caller's
    // `continue` (mbMonocular's median-depth test); n_matches (optional): SearchForTriangulation's counts.  `restart`
    // = the top of CreateNewMapPoints (side 1 back on the left camera); false continues from the previous call's
    // state, so a caller that checks CheckNewKeyFrames() between neighbours (:440) gets the one-call result.
    std::vector<NewMapPoint> operator()(const CnmpKeyFrame &kf1, std::vector<uint8_t> &has_mp1,
                                        const std::vector<CnmpKeyFrame> &nbs,
                                        const std::vector<std::array<std::array<float, 12>, OMV_TRI_PAIRS>> &T,
                                        const std::vector<int> &skip, bool bCoarse, float scale_factor, size_t lo,
                                        size_t hi, bool restart, std::vector<int> *n_matches = nullptr) {
        const int N1 = kf1.view.N;
        if ((int)has_mp1.size() != N1 || T.size() != nbs.size() || skip.size() != nbs.size() || hi > nbs.size() || lo > hi)
            throw Error("CreateNewMapPoints: inconsistent inputs");
        const int n = (int)(hi - lo);
        while (bufs_.size() < nbs.size() + 1) bufs_.emplace_back(new Buf());
        omv_cnmp_kf k1 = kf_struct(kf1, *bufs_[0]);
        hm_.upload(has_mp1.data(), has_mp1.size(), st_);
        if (restart) hip_check(hipMemsetAsync(side1_.p, 0, sizeof(int32_t), st_), "side1");
        std::vector<omv_cnmp_neighbour> nb(n);
        m12_.resize((size_t)std::max(1, n) * std::max(1, N1)), status_.resize((size_t)std::max(1, n) * std::max(1, N1));
        x3d_.resize((size_t)std::max(1, n) * std::max(1, N1) * 3), nm_.resize(std::max(1, n));
        for (int j = 0; j < n; ++j) {
            nb[j].kf2 = kf_struct(nbs[lo + j], *bufs_[1 + lo + j]);
            for (int q = 0; q < OMV_TRI_PAIRS; ++q) std::copy(T[lo + j][q].begin(), T[lo + j][q].end(), nb[j].T[q]);
            nb[j].skip = skip[lo + j];
            nb[j].match12 = m12_.p + (size_t)j * N1, nb[j].status = status_.p + (size_t)j * N1;
            nb[j].x3D = x3d_.p + (size_t)j * N1 * 3;
        }
        check(omv_local_mapping_create_new_map_points(m_, &k1, hm_.p, n, nb.data(), cams_.data(),
                                                      model_.empty() ? nullptr : model_.data(), C_, inertial_, !mono_,
                                                      bCoarse, far_, th_far_, scale_factor, nm_.p, side1_.p, st_),
              "omv_local_mapping_create_new_map_points");
        std::vector<int32_t> m12((size_t)n * N1), st((size_t)n * N1), nm(n);
        std::vector<float> x((size_t)n * N1 * 3);
        m12_.download(m12.data(), m12.size(), st_), status_.download(st.data(), st.size(), st_);
        x3d_.download(x.data(), x.size(), st_), nm_.download(nm.data(), n, st_);
        hm_.download(has_mp1.data(), has_mp1.size(), st_);
        hip_check(hipStreamSynchronize(st_), "CreateNewMapPoints");
        if (n_matches) n_matches->assign(nm.begin(), nm.end());
        std::vector<NewMapPoint> out;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < N1; ++i) {
                const size_t o = (size_t)j * N1 + i;
                if (st[o] > 0)
                    out.push_back(NewMapPoint{(int)(lo + j), (size_t)i, (size_t)m12[o], {x[3 * o], x[3 * o + 1], x[3 * o + 2]},
                                              st[o] == 2});
            }
        return out;
    }

  private:
    struct Buf {
        DeviceArray<omv_kp> kps;
        DeviceArray<uint8_t> desc, has_mp;
        DeviceArray<uint32_t> node;
        DeviceArray<int32_t> start, idx;
        DeviceArray<float> ur, depth;
    };
    omv_cnmp_kf kf_struct(const CnmpKeyFrame &k, Buf &b) {
        const KeyFrameView &v = k.view;
        if ((int)v.keys.size() != v.N || (int)v.descriptors.size() != 32 * v.N || (int)v.has_map_point.size() != v.N ||
            v.feat_start.size() != v.feat_node.size() + 1 || (!k.uright.empty() && (int)k.uright.size() != v.N) ||
            (!k.depth.empty() && (int)k.depth.size() != v.N))
            throw Error("CreateNewMapPoints: inconsistent CnmpKeyFrame");
        b.kps.upload(v.keys.data(), v.keys.size(), st_), b.desc.upload(v.descriptors.data(), v.descriptors.size(), st_);
        b.has_mp.upload(v.has_map_point.data(), v.has_map_point.size(), st_);
        b.node.upload(v.feat_node.data(), v.feat_node.size(), st_);
        b.start.upload(v.feat_start.data(), v.feat_start.size(), st_), b.idx.upload(v.feat_idx.data(), v.feat_idx.size(), st_);
        b.ur.upload(k.uright.data(), k.uright.size(), st_), b.depth.upload(k.depth.data(), k.depth.size(), st_);
        omv_cnmp_kf s{};
        s.kf.n = v.N, s.kf.n_left = v.NLeft, s.kf.n_right = v.NRight, s.kf.n_sideleft = v.NSideLeft;
        s.kf.kps = b.kps.p, s.kf.desc = b.desc.p, s.kf.has_mp = b.has_mp.p;
        s.kf.n_nodes = (int)v.feat_node.size(), s.kf.node_id = b.node.p, s.kf.node_start = b.start.p, s.kf.node_idx = b.idx.p;
        std::copy(v.level_sigma2.begin(), v.level_sigma2.end(), s.kf.level_sigma2);
        s.kps_raw = nullptr;
        for (int c = 0; c < 4; ++c) {
            std::copy(k.Tcw[c].begin(), k.Tcw[c].end(), s.Tcw[c]);
            std::copy(k.Ow[c].begin(), k.Ow[c].end(), s.Ow[c]);
        }
        std::copy(k.Rwc.begin(), k.Rwc.end(), s.Rwc), std::copy(k.twc.begin(), k.twc.end(), s.twc);
        s.fx = k.fx, s.fy = k.fy, s.cx = k.cx, s.cy = k.cy, s.invfx = k.invfx, s.invfy = k.invfy, s.mb = k.mb, s.mbf = k.mbf;
        s.uright = k.uright.empty() ? nullptr : b.ur.p, s.depth = k.depth.empty() ? nullptr : b.depth.p;
        std::copy(k.scale_factors.begin(), k.scale_factors.end(), s.scale_factors);
        return s;
    }
    std::vector<float> cams_;
    std::vector<int32_t> model_;
    int C_;
    bool inertial_, mono_, far_;
    float th_far_;
    hipStream_t st_ = nullptr;
    omv_matcher *m_ = nullptr;
    std::vector<std::unique_ptr<Buf>> bufs_;
    DeviceArray<uint8_t> hm_;
    DeviceArray<int32_t> m12_, status_, nm_, side1_;
    DeviceArray<float> x3d_;
};

// ---- MapPoint::ComputeDistinctiveDescriptors / UpdateNormalAndDepth over a batch of points ----------------------
class MapPointRefresh {
  public:
    MapPointRefresh() { hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate"); }
    ~MapPointRefresh() {
        if (st_) (void)hipStreamDestroy(st_);
    }
    MapPointRefresh(const MapPointRefresh &) = delete;
    MapPointRefresh &operator=(const MapPointRefresh &) = delete;

    // ComputeDistinctiveDescriptors (MapPoint.cc:405-483): point p's observation descriptors are rows
    // desc_row[desc_start[p] .. desc_start[p+1]) of `desc` [rows][32] in mObservations order (L / R / SL / SR of each
    // keyframe); returns the chosen row per point (-1: none, mDescriptor untouched) and, in desc_out [P][32], the
    // descriptors.
    std::vector<int32_t> distinctive(const std::vector<int32_t> &desc_start, const std::vector<int32_t> &desc_row,
                                     const std::vector<uint8_t> &desc, std::vector<uint8_t> &desc_out) {
        const int P = (int)desc_start.size() - 1;
        if (P < 0) throw Error("MapPointRefresh: desc_start");
        ds_.upload(desc_start.data(), desc_start.size(), st_), dr_.upload(desc_row.data(), desc_row.size(), st_);
        d_.upload(desc.data(), desc.size(), st_);
        best_.resize(std::max(1, P)), dout_.resize(32 * (size_t)std::max(1, P));
        check(omv_mappoint_distinctive_descriptors(P, ds_.p, dr_.p, d_.p, best_.p, dout_.p, st_),
              "omv_mappoint_distinctive_descriptors");
        std::vector<int32_t> best(P);
        desc_out.resize(32 * (size_t)P);
        best_.download(best.data(), P, st_), dout_.download(desc_out.data(), desc_out.size(), st_);
        hip_check(hipStreamSynchronize(st_), "distinctive");
        return best;
    }
    // UpdateNormalAndDepth (MapPoint.cc:503-588): per point its observation camera centres obs_center [E][3] (rows
    // obs_start[p] ..), mWorldPos, the reference keyframe's camera centre, mvScaleFactors[level] of its keypoint there
    // and mvScaleFactors[nLevels - 1]; out: mNormalVector, mfMinDistance, mfMaxDistance (points without entries: as
    // given).
    void normal_depth(const std::vector<int32_t> &obs_start, const std::vector<float> &obs_center,
                      const std::vector<float> &pos, const std::vector<float> &ref_center,
                      const std::vector<float> &ref_level_scale, const std::vector<float> &ref_max_scale,
                      std::vector<float> &normal, std::vector<float> &min_dist, std::vector<float> &max_dist) {
        const int P = (int)obs_start.size() - 1;
        if (P < 0 || (int)normal.size() != 3 * P || (int)min_dist.size() != P || (int)max_dist.size() != P)
            throw Error("MapPointRefresh: normal_depth sizes");
        os_.upload(obs_start.data(), obs_start.size(), st_), oc_.upload(obs_center.data(), obs_center.size(), st_);
        pos_.upload(pos.data(), pos.size(), st_), rc_.upload(ref_center.data(), ref_center.size(), st_);
        rl_.upload(ref_level_scale.data(), ref_level_scale.size(), st_);
        rm_.upload(ref_max_scale.data(), ref_max_scale.size(), st_);
        nrm_.upload(normal.data(), normal.size(), st_), mn_.upload(min_dist.data(), P, st_), mx_.upload(max_dist.data(), P, st_);
        check(omv_mappoint_normal_depth(P, os_.p, oc_.p, pos_.p, rc_.p, rl_.p, rm_.p, nrm_.p, mn_.p, mx_.p, st_),
              "omv_mappoint_normal_depth");
        nrm_.download(normal.data(), normal.size(), st_), mn_.download(min_dist.data(), P, st_);
        mx_.download(max_dist.data(), P, st_);
        hip_check(hipStreamSynchronize(st_), "normal_depth");
    }

  private:
    hipStream_t st_ = nullptr;
    DeviceArray<int32_t> ds_, dr_, best_, os_;
    DeviceArray<uint8_t> d_, dout_;
    DeviceArray<float> oc_, pos_, rc_, rl_, rm_, nrm_, mn_, mx_;
};

// ---- LocalMapping::SearchInNeighbors' fuse sequence (LocalMapping.cc:837-889) ----------------------------------
// The flattened map the sequence reads (keyframes numbered in std::map<KeyFrame*> key order, the current keyframe
// and the targets among them, block-major keypoints [n_kf][n_cams][kp_cap]) and what it returns: the final graph and
// the ordered edit log to replay with the reference's own methods ({0, mp, kf, idx}: pMP->AddObservation(pKF, idx) +
// pKF->AddMapPoint(pMP, idx); {1, a, b, -1}: a->Replace(b)).
struct FuseGraphView {
    int n_kf = 0, n_cams = 0, kp_cap = 0, width = 0, height = 0;
    std::vector<float> scale_factors, cams;            // mvScaleFactors; [n_cams][8]
    std::vector<int32_t> cam_model;                    // [n_cams] or empty (KB8)
    float bf = 0.f, th = 3.f;
    std::vector<omv_kp> kps;                           // [n_kf][n_cams][kp_cap]
    std::vector<uint8_t> desc;                         // [n_kf][n_cams][kp_cap][32]
    std::vector<int32_t> n_kp;                         // [n_kf][n_cams]
    std::vector<float> uright;                         // [n_kf][kp_cap] block-0 mvuRight
    std::vector<int32_t> n_blocks;                     // [n_kf] 1 / 2 / 4
    std::vector<omv_se3f> Tcw;                         // [n_kf][n_cams]
    std::vector<float> Ow;                             // [n_kf][n_cams][3]
    std::vector<int32_t> kf_mps;                       // [n_kf][n_cams * kp_cap] in/out, N-indexed
    std::vector<float> pos, normal, min_dist, max_dist;   // [M][3] / [M]
    std::vector<uint8_t> mp_desc;                      // [M][32] in/out
    std::vector<int32_t> bad, n_obs;                   // [M] in/out
    std::vector<int32_t> obs_start, obs_kf, obs_idx;   // in: CSR [M + 1] / [rows] / [rows][4]; out: the final ones
    std::vector<int32_t> replaced;                     // out [M]
    std::vector<int32_t> log;                          // out [n_log][4]
};

class SearchInNeighborsFuse {
  public:
    SearchInNeighborsFuse() { hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate"); }
    ~SearchInNeighborsFuse() {
        if (m_) (void)omv_matcher_destroy(m_);
        if (st_) (void)hipStreamDestroy(st_);
    }
    SearchInNeighborsFuse(const SearchInNeighborsFuse &) = delete;
    SearchInNeighborsFuse &operator=(const SearchInNeighborsFuse &) = delete;

    // Phase A + phase B for `current` and `targets` (vpTargetKFs order); returns nFused per Fuse call (phase A target-
    // major, block-minor, then phase B); g's in/out members are updated to the reference's final state.
    std::vector<int32_t> operator()(FuseGraphView &g, int current, const std::vector<int32_t> &targets,
                                    const std::vector<float> &inv_level_sigma2) {
        const int K = g.n_kf, C = g.n_cams, cap = g.kp_cap, M = (int)g.bad.size();
        if ((int)g.kps.size() != K * C * cap || (int)g.desc.size() != 32 * K * C * cap || (int)g.n_kp.size() != K * C ||
            (int)g.kf_mps.size() != K * C * cap || (int)g.obs_start.size() != M + 1)
            throw Error("SearchInNeighborsFuse: inconsistent graph");
        const int n_cur = [&] { int s = 0; for (int c = 0; c < C; ++c) s += g.n_kp[(size_t)current * C + c]; return s; }();
        const int need = std::max(1, (int)((size_t)targets.size() * C * std::max(1, n_cur) / std::max(1, K * C) + 1));
        if (!m_ || need > mps_cap_) {
            if (m_) (void)omv_matcher_destroy(m_), m_ = nullptr;
            mps_cap_ = need;
            check(omv_matcher_create(K, C, cap, mps_cap_, &m_), "omv_matcher_create");
        }
        omv_frame_geom geom{};
        geom.n_cams = C, geom.min_x = 0.f, geom.max_x = (float)g.width, geom.min_y = 0.f, geom.max_y = (float)g.height;
        geom.nlevels = (int)g.scale_factors.size();
        for (int l = 0; l < geom.nlevels && l < 16; ++l) geom.scale_factors[l] = g.scale_factors[l];
        for (int c = 0; c < C && c < 8; ++c) geom.cam_model[c] = g.cam_model.empty() ? OMV_CAM_KB8 : g.cam_model[c];
        kps_.upload(g.kps.data(), g.kps.size(), st_), desc_.upload(g.desc.data(), g.desc.size(), st_);
        nkp_.upload(g.n_kp.data(), g.n_kp.size(), st_), ur_.upload(g.uright.data(), g.uright.size(), st_);
        pos_.upload(g.pos.data(), g.pos.size(), st_), nrm_.upload(g.normal.data(), g.normal.size(), st_);
        mn_.upload(g.min_dist.data(), g.min_dist.size(), st_), mx_.upload(g.max_dist.data(), g.max_dist.size(), st_);
        md_.upload(g.mp_desc.data(), g.mp_desc.size(), st_);
        check(omv_matcher_assign_grid(m_, K, &geom, kps_.p, nkp_.p, st_), "omv_matcher_assign_grid");
        const size_t obs_cap = 4 * g.obs_kf.size() + 1024, log_cap = 4 * (size_t)M + 1024;
        std::vector<int32_t> out_start(M + 1), out_kf(obs_cap), out_idx(4 * obs_cap);
        g.replaced.assign(M, -1);
        g.log.assign(4 * log_cap, 0);
        omv_fuse_graph G{};
        G.n_kf = K, G.n_blocks = g.n_blocks.data(), G.Tcw = g.Tcw.data(), G.Ow = g.Ow.data();
        G.uright = g.uright.empty() ? nullptr : g.uright.data(), G.kf_mps = g.kf_mps.data();
        G.n_mps = M, G.bad = g.bad.data(), G.n_obs = g.n_obs.data(), G.replaced = g.replaced.data();
        G.obs_start = g.obs_start.data(), G.obs_kf = g.obs_kf.data(), G.obs_idx = g.obs_idx.data();
        G.out_obs_start = out_start.data(), G.out_obs_kf = out_kf.data(), G.out_obs_idx = out_idx.data();
        G.obs_cap = (int)obs_cap, G.log = g.log.data(), G.log_cap = (int)log_cap;
        omv_kf_search_params p{};
        p.mode = OMV_KF_FUSE, p.th = g.th, p.max_dist = 50.f, p.bf = g.bf, p.uright = ur_.p;
        for (int l = 0; l < (int)inv_level_sigma2.size() && l < 16; ++l) p.inv_level_sigma2[l] = inv_level_sigma2[l];
        p.log_scale_factor = (float)std::log((double)g.scale_factors[1]);
        p.n_levels = geom.nlevels;
        for (int c = 0; c < C && c < 8; ++c)
            for (int q = 0; q < 8; ++q) p.cams[c][q] = g.cams[8 * c + q];
        const omv_kf_mps kfm{pos_.p, nrm_.p, mn_.p, mx_.p, md_.p};
        std::vector<int32_t> n_fused(targets.size() * C + C);
        check(omv_search_in_neighbors_fuse(m_, &geom, kps_.p, desc_.p, nkp_.p, cap, &G, current, (int)targets.size(),
                                           targets.data(), &kfm, &p, n_fused.data(), st_),
              "omv_search_in_neighbors_fuse");
        md_.download(g.mp_desc.data(), g.mp_desc.size(), st_);
        hip_check(hipStreamSynchronize(st_), "SearchInNeighborsFuse");
        const int rows = out_start[M];
        g.obs_start = out_start;
        g.obs_kf.assign(out_kf.begin(), out_kf.begin() + rows);
        g.obs_idx.assign(out_idx.begin(), out_idx.begin() + 4 * (size_t)rows);
        g.log.resize(4 * (size_t)G.n_log);
        return n_fused;
    }

  private:
    hipStream_t st_ = nullptr;
    omv_matcher *m_ = nullptr;
    int mps_cap_ = 0;
    DeviceArray<omv_kp> kps_;
    DeviceArray<uint8_t> desc_, md_;
    DeviceArray<int32_t> nkp_;
    DeviceArray<float> ur_, pos_, nrm_, mn_, mx_;
};

// The window as the reference builds its graph: keyframes (each with its body pose, per-camera poses, velocity,
// biases, bImu, and whether it is fixed), map points, EdgeMono / EdgeStereo observations and inertial edges in
// creation order.  flatten() renumbers keyframes optimisable-first (the vertex order of Optimizer.cc:2800-2860) and
// produces the omv_lba_problem; optimize() runs it and writes keyframes AND points back into the window only when
// the result is not OMV_LBA_FAIL (the reference returns before any SetWorldPos / SetPose, Optimizer.cc:3317-3321).
class LocalInertialBAWindow {
  public:
    struct KeyFrame {
        std::array<double, 9> Rwb;
        std::array<double, 3> twb, vel, bg, ba;
        std::vector<std::array<double, 9>> Rcw;   // [n_cams]
        std::vector<std::array<double, 3>> tcw;   // [n_cams]
        bool imu = true, fixed = false;
    };
    struct Inertial {
        int kf1, kf2;
        std::vector<float> preint;   // OMV_PREINT_FLOATS
        bool robust;
        float info_scale;
        // The reference's rule for the i-th of N inertial edges (Optimizer.cc:2972-2981): Huber sqrt(16.92) on
        // the last edge (the one reaching the first fixed keyframe) or on every edge when bRecInit; the last
        // edge's information scaled by 1e-2.
        static Inertial make(int kf1, int kf2, std::vector<float> preint, bool is_last, bool bRecInit) {
            return Inertial{kf1, kf2, std::move(preint), is_last || bRecInit, is_last ? 1e-2f : 1.0f};
        }
    };

    LocalInertialBAWindow(int n_cams, std::vector<float> cams, std::vector<double> Rcb, std::vector<double> tcb,
                          std::vector<double> Rbc, std::vector<double> tbc, float bf = 0.f,
                          std::vector<int32_t> cam_model = {})
        : C_(n_cams), cam_(std::move(cams)), Rcb_(std::move(Rcb)), tcb_(std::move(tcb)), Rbc_(std::move(Rbc)),
          tbc_(std::move(tbc)), bf_(bf), model_(std::move(cam_model)) {}
    ~LocalInertialBAWindow() {
        if (h_) (void)omv_lba_destroy(h_);
    }
    LocalInertialBAWindow(const LocalInertialBAWindow &) = delete;
    LocalInertialBAWindow &operator=(const LocalInertialBAWindow &) = delete;

    int add_keyframe(const KeyFrame &kf) {
        kfs_.push_back(kf);
        return (int)kfs_.size() - 1;
    }
    int add_point(const std::array<double, 3> &X, float track_depth) {
        pts_.insert(pts_.end(), X.begin(), X.end());
        depth_.push_back(track_depth);
        return (int)depth_.size() - 1;
    }
    // EdgeMono (Optimizer.cc:3080-3106): camera `cam` of keyframe `kf` observes point `pt` at (u, v)
    void add_mono(int pt, int kf, int cam, double u, double v, float inv_sigma2) {
        mono_.push_back({pt, kf, cam, u, v, inv_sigma2});
    }
    // EdgeStereo (Optimizer.cc:3108-3143): a left-camera observation with mvuRight >= 0, obs (kpUn.x, kpUn.y, u_R),
    // information I3 * invSigma2 (already divided by uncertainty2), Huber sqrt(7.815)
    void add_stereo(int pt, int kf, double u, double v, double u_right, float inv_sigma2) {
        stereo_.push_back({pt, kf, u, v, u_right, inv_sigma2});
    }
    void add_inertial(const Inertial &e) { imu_.push_back(e); }
    // Landmark sharding: this window's `rank` of `world` and the caller's in-place SUM
    // collective (e.g. ncclAllReduce on the handle's stream).  Every rank adds the same full window; each optimises
    // its share of the landmarks.  Kept across handle re-creation; a communicator of one rank runs the same collective
    // call sequence.
    void set_comm(int rank, int world, omv_allreduce_fn fn, void *ctx) {
        rank_ = rank, world_ = world, ar_ = fn, ar_ctx_ = ctx;
        if (h_) check(omv_lba_set_comm(h_, rank_, world_, ar_, ar_ctx_), "omv_lba_set_comm");
    }
    // Host waits of the last optimize()'s LM loop and its trials (omv_lba_host_syncs).
    std::pair<int, int> host_syncs() const {
        int n = 0, t = 0;
        if (h_) check(omv_lba_host_syncs(h_, &n, &t), "omv_lba_host_syncs");
        return {n, t};
    }
    // Drop every keyframe, point and edge (the handle and its capacity are kept for the next window).
    void clear() { kfs_.clear(), pts_.clear(), depth_.clear(), mono_.clear(), stereo_.clear(), imu_.clear(); }

    // optimizer.optimize(opt_it) of the window (bLarge settings when `large`); returns the result.  The window
    // state is updated only when status == OMV_LBA_OK (the reference's FAIL guard, :3317-3321); the per-edge
    // chi2 / outlier flags (:3282-3311) are reported either way.
    omv_lba_result optimize(bool large, std::vector<double> *mono_chi2 = nullptr, std::vector<uint8_t> *outlier = nullptr,
                            std::vector<double> *stereo_chi2 = nullptr, std::vector<uint8_t> *stereo_outlier = nullptr) {
        flatten();
        ensure_capacity();
        check(omv_lba_set_problem(h_, &p_), "omv_lba_set_problem");
        const omv_lba_opts o{large ? 4 : 10, large ? 1e-2 : 1e0, 10, large ? 1 : 0};
        chi2_.assign(mono_.size(), 0.0), outl_.assign(mono_.size(), 0);
        schi2_.assign(stereo_.size(), 0.0), soutl_.assign(stereo_.size(), 0);
        omv_lba_result r{};
        r.mono_chi2 = chi2_.data(), r.mono_outlier = outl_.data();
        r.stereo_chi2 = schi2_.data(), r.stereo_outlier = soutl_.data();
        check(omv_lba_optimize(h_, &o, &p_, &r), "omv_lba_optimize");
        if (mono_chi2) *mono_chi2 = chi2_;
        if (outlier) *outlier = outl_;
        if (stereo_chi2) *stereo_chi2 = schi2_;
        if (stereo_outlier) *stereo_outlier = soutl_;
        if (r.status == OMV_LBA_OK) write_back();
        return r;
    }
    const std::vector<KeyFrame> &keyframes() const { return kfs_; }
    const std::vector<double> &points() const { return pts_; }

  private:
    struct Mono {
        int pt, kf, cam;
        double u, v;
        float w;
    };
    struct Stereo {
        int pt, kf;
        double u, v, ur;
        float w;
    };
    // (Re)create the handle when this window exceeds the capacity it was created with (sliding windows vary)
    void ensure_capacity() {
        const int need[5] = {(int)kfs_.size(), C_, (int)depth_.size(), (int)(mono_.size() + stereo_.size()),
                             std::max<int>(1, (int)imu_.size())};
        bool fits = h_ != nullptr;
        for (int i = 0; i < 5 && fits; ++i) fits = need[i] <= cap_[i];
        if (fits) return;
        if (h_) (void)omv_lba_destroy(h_), h_ = nullptr;
        for (int i = 0; i < 5; ++i) cap_[i] = std::max(cap_[i], need[i]);
        check(omv_lba_create(cap_[0], cap_[1], cap_[2], cap_[3], cap_[4], &h_), "omv_lba_create");
        if (ar_ || world_ > 1) check(omv_lba_set_comm(h_, rank_, world_, ar_, ar_ctx_), "omv_lba_set_comm");
    }
    void flatten() {
        const int K = (int)kfs_.size();
        order_.clear();
        for (int k = 0; k < K; ++k)
            if (!kfs_[k].fixed) order_.push_back(k);
        n_opt_ = (int)order_.size();
        for (int k = 0; k < K; ++k)
            if (kfs_[k].fixed) order_.push_back(k);
        std::vector<int> vid(K);
        for (int i = 0; i < K; ++i) vid[order_[i]] = i;
        Rwb_.clear(), twb_.clear(), Rcw_.clear(), tcw_.clear(), vel_.clear(), bg_.clear(), ba_.clear(), kimu_.clear();
        for (int k : order_) {
            const KeyFrame &f = kfs_[k];
            Rwb_.insert(Rwb_.end(), f.Rwb.begin(), f.Rwb.end()), twb_.insert(twb_.end(), f.twb.begin(), f.twb.end());
            for (int c = 0; c < C_; ++c) {
                Rcw_.insert(Rcw_.end(), f.Rcw[c].begin(), f.Rcw[c].end());
                tcw_.insert(tcw_.end(), f.tcw[c].begin(), f.tcw[c].end());
            }
            vel_.insert(vel_.end(), f.vel.begin(), f.vel.end()), bg_.insert(bg_.end(), f.bg.begin(), f.bg.end());
            ba_.insert(ba_.end(), f.ba.begin(), f.ba.end());
            kimu_.push_back(f.imu ? 1 : 0);
        }
        ptsw_ = pts_;   // the solver's copy: pts_ changes only on write_back
        mpt_.clear(), mkf_.clear(), mcam_.clear(), mobs_.clear(), mw_.clear();
        for (const Mono &m : mono_) {
            mpt_.push_back(m.pt), mkf_.push_back(vid[m.kf]), mcam_.push_back(m.cam);
            mobs_.push_back(m.u), mobs_.push_back(m.v), mw_.push_back(m.w);
        }
        spt_.clear(), skf_.clear(), sobs_.clear(), sw_.clear();
        for (const Stereo &e : stereo_) {
            spt_.push_back(e.pt), skf_.push_back(vid[e.kf]);
            sobs_.push_back(e.u), sobs_.push_back(e.v), sobs_.push_back(e.ur), sw_.push_back(e.w);
        }
        ik1_.clear(), ik2_.clear(), pre_.clear(), irob_.clear(), isc_.clear();
        for (const Inertial &e : imu_) {
            ik1_.push_back(vid[e.kf1]), ik2_.push_back(vid[e.kf2]);
            pre_.insert(pre_.end(), e.preint.begin(), e.preint.end());
            irob_.push_back(e.robust ? 1 : 0), isc_.push_back(e.info_scale);
        }
        p_ = omv_lba_problem{};
        p_.n_cams = C_, p_.cam = cam_.data(), p_.Rcb = Rcb_.data(), p_.tcb = tcb_.data(), p_.Rbc = Rbc_.data(), p_.tbc = tbc_.data();
        p_.n_kf = K, p_.n_opt = n_opt_, p_.kf_imu = kimu_.data();
        p_.Rwb = Rwb_.data(), p_.twb = twb_.data(), p_.Rcw = Rcw_.data(), p_.tcw = tcw_.data();
        p_.vel = vel_.data(), p_.bg = bg_.data(), p_.ba = ba_.data();
        p_.n_pts = (int)depth_.size(), p_.pts = ptsw_.data(), p_.pt_track_depth = depth_.data();
        p_.n_mono = (int)mono_.size(), p_.mono_pt = mpt_.data(), p_.mono_kf = mkf_.data(), p_.mono_cam = mcam_.data();
        p_.mono_obs = mobs_.data(), p_.mono_inv_sigma2 = mw_.data();
        p_.n_imu = (int)imu_.size(), p_.imu_kf1 = ik1_.data(), p_.imu_kf2 = ik2_.data(), p_.preint = pre_.data();
        p_.imu_robust = irob_.data(), p_.imu_info_scale = isc_.data();
        p_.n_stereo = (int)stereo_.size(), p_.stereo_pt = spt_.data(), p_.stereo_kf = skf_.data();
        p_.stereo_obs = sobs_.data(), p_.stereo_inv_sigma2 = sw_.data(), p_.bf = bf_;
        p_.cam_model = model_.empty() ? nullptr : model_.data();
    }
    void write_back() {   // vertex estimates back to the keyframes and points
        for (int i = 0; i < (int)order_.size(); ++i) {
            KeyFrame &f = kfs_[order_[i]];
            std::memcpy(f.Rwb.data(), &Rwb_[9 * i], 9 * sizeof(double));
            std::memcpy(f.twb.data(), &twb_[3 * i], 3 * sizeof(double));
            for (int c = 0; c < C_; ++c) {
                std::memcpy(f.Rcw[c].data(), &Rcw_[((size_t)i * C_ + c) * 9], 9 * sizeof(double));
                std::memcpy(f.tcw[c].data(), &tcw_[((size_t)i * C_ + c) * 3], 3 * sizeof(double));
            }
            std::memcpy(f.vel.data(), &vel_[3 * i], 3 * sizeof(double));
            std::memcpy(f.bg.data(), &bg_[3 * i], 3 * sizeof(double));
            std::memcpy(f.ba.data(), &ba_[3 * i], 3 * sizeof(double));
        }
        pts_ = ptsw_;
    }

    int C_;
    std::vector<float> cam_;
    std::vector<double> Rcb_, tcb_, Rbc_, tbc_;
    float bf_;
    std::vector<int32_t> model_;
    std::vector<KeyFrame> kfs_;
    std::vector<double> pts_;
    std::vector<float> depth_;
    std::vector<Mono> mono_;
    std::vector<Stereo> stereo_;
    std::vector<Inertial> imu_;
    // flattened arrays (alive for the problem's lifetime)
    std::vector<int> order_;
    int n_opt_ = 0;
    std::vector<double> Rwb_, twb_, Rcw_, tcw_, vel_, bg_, ba_, ptsw_, mobs_, sobs_, chi2_, schi2_;
    std::vector<uint8_t> kimu_, irob_, outl_, soutl_;
    std::vector<int32_t> mpt_, mkf_, mcam_, spt_, skf_, ik1_, ik2_;
    std::vector<float> mw_, sw_, pre_, isc_;
    omv_lba_problem p_{};
    omv_lba *h_ = nullptr;
    int cap_[5] = {0, 0, 0, 0, 0};   // max_kf, max_cams, max_pts, max visual edges, max_imu of h_
    int rank_ = 0, world_ = 1;
    omv_allreduce_fn ar_ = nullptr;
    void *ar_ctx_ = nullptr;
};

}  // namespace omv_adapt

#endif  // OMV_ADAPTERS_HPP
