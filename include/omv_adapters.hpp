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
//
// Errors: every omv_status != OMV_OK throws omv_adapt::Error (the adapters' callers are C++).
#ifndef OMV_ADAPTERS_HPP
#define OMV_ADAPTERS_HPP

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
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

  private:
    friend class SearchByProjection;
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
