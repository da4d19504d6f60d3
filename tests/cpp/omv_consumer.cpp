// A C++ consumer of include/omv.h through the adapters of include/omv_adapters.hpp — what the reference's
// C++ would link.  Built with g++ against the header and libomv_hip.so only (no torch, no
// Python); driven by tests/test_cpp_consumer_gpu.py, which writes the inputs as raw arrays into a directory
// and checks the outputs against the CPU oracle (ORB / SearchByProjection bit-exact) and the Python path
// (LocalInertialBA, parity bar).
//
//   omv_consumer orb   DIR   per image: ORBextractor::operator() (one image per call, host memory)
//   omv_consumer frame DIR   MultiCameraFrame (batched extraction + grid + lapping knn) + SearchByProjection
//   omv_consumer lastframe DIR  MultiCameraFrame + SearchByProjectionLastFrame (motion-model matching)
//   omv_consumer tri   DIR   SearchForTriangulation of one keyframe pair -> vMatchedPairs
//   omv_consumer pose  DIR   PoseInertialOptimizer: LastKeyFrame (meta lf 0) or LastFrame + ConstraintPoseImu (lf 1)
//   omv_consumer fuse  DIR   Fuse per camera block of one keyframe -> chosen keypoint / distance per point
//   omv_consumer posopt DIR  PoseOptimization(Frame*) on one frame -> pose, mvbOutlier, nGood
//   omv_consumer cnmp  DIR   CreateNewMapPoints' neighbour loop in two calls (a CheckNewKeyFrames boundary) -> the
//                            new points in creation order, the current keyframe's has-map-point flags
//   omv_consumer mprefresh DIR  ComputeDistinctiveDescriptors / UpdateNormalAndDepth over a batch of points
//   omv_consumer fuseseq DIR SearchInNeighbors' fuse sequence -> final graph, edit log, descriptors
//   omv_consumer lba   DIR   LocalInertialBAWindow: keyframes added in a mixed fixed / optimisable order,
//                            EdgeMono + EdgeStereo observations, inertial edges under the reference's robust
//                            rule (last edge / bRecInit), flattened optimisable-first, optimised, written back
//                            (not on FAIL); optionally a smaller window first on the same adapter; with meta
//                            rccl 1 on a one-rank RCCL communicator (omv_lba_set_comm + ncclAllReduce, §4b)
//
// DIR/meta.txt holds "key value" lines; arrays are DIR/<name>.bin in the dtype the test wrote.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "omv_adapters.hpp"

namespace {

// INTEGRATION.md §4b's collective: RCCL's in-place all-reduce on the handle's stream (counted)
int g_allreduce_calls = 0;
int nccl_sum(void *comm, double *buf, size_t n, void *stream) {
    ++g_allreduce_calls;
    return ncclAllReduce(buf, buf, n, ncclFloat64, ncclSum, (ncclComm_t)comm, (hipStream_t)stream) == ncclSuccess ? 0 : 1;
}

std::map<std::string, double> read_meta(const std::string &dir) {
    std::map<std::string, double> m;
    std::ifstream f(dir + "/meta.txt");
    std::string k;
    double v;
    while (f >> k >> v) m[k] = v;
    if (m.empty()) throw omv_adapt::Error("no " + dir + "/meta.txt");
    return m;
}

template <class T>
std::vector<T> read_bin(const std::string &dir, const std::string &name) {
    std::ifstream f(dir + "/" + name + ".bin", std::ios::binary | std::ios::ate);
    if (!f) throw omv_adapt::Error("missing " + name + ".bin");
    const size_t bytes = (size_t)f.tellg();
    std::vector<T> v(bytes / sizeof(T));
    f.seekg(0);
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)bytes);
    return v;
}

template <class T>
void write_bin(const std::string &dir, const std::string &name, const T *p, size_t n) {
    std::ofstream f(dir + "/" + name + ".bin", std::ios::binary);
    f.write(reinterpret_cast<const char *>(p), (std::streamsize)(n * sizeof(T)));
}
template <class T>
void write_bin(const std::string &dir, const std::string &name, const std::vector<T> &v) {
    write_bin(dir, name, v.data(), v.size());
}

int run_orb(const std::string &dir) {
    auto m = read_meta(dir);
    const int n = (int)m["n"], W = (int)m["W"], H = (int)m["H"];
    const auto img = read_bin<uint8_t>(dir, "images");
    const auto lap = read_bin<int32_t>(dir, "lapping");
    omv_adapt::ORBextractor ex((int)m["nfeatures"], 1.2f, 8, (int)m["ini"], (int)m["min"]);
    std::vector<int32_t> mono(n);
    for (int i = 0; i < n; ++i) {
        std::vector<omv_kp> k;
        std::vector<uint8_t> d;
        const int l[2] = {lap[2 * i], lap[2 * i + 1]};
        mono[i] = ex(img.data() + (size_t)i * W * H, W, H, W, k, d, l);
        write_bin(dir, "kps_" + std::to_string(i), k);
        write_bin(dir, "desc_" + std::to_string(i), d);
    }
    write_bin(dir, "mono", mono);
    return 0;
}

int run_frame(const std::string &dir) {
    auto m = read_meta(dir);
    const int C = (int)m["C"], W = (int)m["W"], H = (int)m["H"], M = (int)m["M"];
    const auto img = read_bin<uint8_t>(dir, "images");
    const auto lap = read_bin<int32_t>(dir, "lapping");
    std::vector<std::array<int, 2>> lapping(C);
    for (int c = 0; c < C; ++c) lapping[c] = {lap[2 * c], lap[2 * c + 1]};
    const omv_orb_params p{(int)m["nfeatures"], 1.2f, 8, (int)m["ini"], (int)m["min"]};
    omv_adapt::MultiCameraFrame F(C, W, H, p, lapping, M);
    std::vector<const uint8_t *> ims(C);
    for (int c = 0; c < C; ++c) ims[c] = img.data() + (size_t)c * W * H;
    F.build(ims);
    for (int c = 0; c < C; ++c) {
        std::vector<omv_kp> k;
        std::vector<uint8_t> d;
        F.keypoints(c, k, d);
        write_bin(dir, "kps_" + std::to_string(c), k);
        write_bin(dir, "desc_" + std::to_string(c), d);
    }
    std::vector<int32_t> l2r, r2l;
    F.stereo(l2r, r2l);
    write_bin(dir, "l2r", l2r);
    write_bin(dir, "r2l", r2l);
    if (M == 0) return 0;
    omv_adapt::LocalMapView v;
    v.desc = read_bin<uint8_t>(dir, "mp_desc"), v.proj_x = read_bin<float>(dir, "mp_proj_x");
    v.proj_y = read_bin<float>(dir, "mp_proj_y"), v.view_cos = read_bin<float>(dir, "mp_view_cos");
    v.level = read_bin<int32_t>(dir, "mp_level"), v.in_view = read_bin<uint8_t>(dir, "mp_in_view");
    v.track_depth = read_bin<float>(dir, "mp_track_depth"), v.is_bad = read_bin<uint8_t>(dir, "mp_is_bad");
    v.has_obs = read_bin<uint8_t>(dir, "mp_has_obs");
    std::vector<int32_t> k2m((size_t)C * F.kp_cap(), -1);
    omv_adapt::SearchByProjection sbp((float)m["nnratio"]);
    const int nm = sbp(F, v, (float)m["th"], m["far"] != 0, (float)m["th_far"], k2m);
    write_bin(dir, "kp_to_mp", k2m);
    write_bin(dir, "n_matches", &nm, 1);
    std::ofstream(dir + "/kp_cap.txt") << F.kp_cap() << "\n";
    return 0;
}

// optional arrays (absent file: empty)
template <class T>
std::vector<T> read_opt(const std::string &dir, const std::string &name) {
    std::ifstream f(dir + "/" + name + ".bin");
    return f ? read_bin<T>(dir, name) : std::vector<T>();
}

int run_lba(const std::string &dir) {
    auto m = read_meta(dir);
    const int C = (int)m["n_cams"], K = (int)m["n_kf"], n_opt = (int)m["n_opt"], P = (int)m["n_pts"];
    const bool rec_init = m["rec_init"] != 0;
    const auto order = read_bin<int32_t>(dir, "kf_order");   // window insertion order of the original keyframes
    const auto Rwb = read_bin<double>(dir, "Rwb"), twb = read_bin<double>(dir, "twb"), Rcw = read_bin<double>(dir, "Rcw");
    const auto tcw = read_bin<double>(dir, "tcw"), vel = read_bin<double>(dir, "vel"), bg = read_bin<double>(dir, "bg");
    const auto ba = read_bin<double>(dir, "ba");
    const auto kf_imu = read_bin<uint8_t>(dir, "kf_imu");
    const auto pts = read_bin<double>(dir, "pts");
    const auto depth = read_bin<float>(dir, "pt_track_depth");
    const auto mpt = read_bin<int32_t>(dir, "mono_pt"), mkf = read_bin<int32_t>(dir, "mono_kf"), mcam = read_bin<int32_t>(dir, "mono_cam");
    const auto mobs = read_bin<double>(dir, "mono_obs");
    const auto mw = read_bin<float>(dir, "mono_inv_sigma2");
    const auto spt = read_opt<int32_t>(dir, "stereo_pt"), skf = read_opt<int32_t>(dir, "stereo_kf");
    const auto sobs = read_opt<double>(dir, "stereo_obs");
    const auto sw = read_opt<float>(dir, "stereo_inv_sigma2");
    const auto ik1 = read_bin<int32_t>(dir, "imu_kf1"), ik2 = read_bin<int32_t>(dir, "imu_kf2");
    const auto pre = read_bin<float>(dir, "preint");
    const auto model = read_opt<int32_t>(dir, "cam_model");
    omv_adapt::LocalInertialBAWindow win(C, read_bin<float>(dir, "cam"), read_bin<double>(dir, "Rcb"), read_bin<double>(dir, "tcb"),
                                         read_bin<double>(dir, "Rbc"), read_bin<double>(dir, "tbc"), (float)m["bf"], model);
    ncclComm_t comm = nullptr;
    if (m["rccl"] != 0) {   // a one-rank RCCL communicator: the landmark-sharded call sequence on this GPU
        ncclUniqueId id;
        if (ncclGetUniqueId(&id) != ncclSuccess || ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess)
            throw omv_adapt::Error("RCCL communicator");
        win.set_comm(0, 1, nccl_sum, comm);
    }
    std::vector<int> slot(K);   // original keyframe -> window index
    // the window with its first n_pts_use points and their edges (a smaller window first exercises the handle's
    // re-creation when the next window is larger)
    auto build = [&](int n_pts_use) {
        win.clear();
        for (int w = 0; w < K; ++w) {
            const int k = order[w];
            omv_adapt::LocalInertialBAWindow::KeyFrame f;
            std::copy_n(&Rwb[9 * k], 9, f.Rwb.begin()), std::copy_n(&twb[3 * k], 3, f.twb.begin());
            std::copy_n(&vel[3 * k], 3, f.vel.begin()), std::copy_n(&bg[3 * k], 3, f.bg.begin()), std::copy_n(&ba[3 * k], 3, f.ba.begin());
            f.Rcw.resize(C), f.tcw.resize(C);
            for (int c = 0; c < C; ++c) {
                std::copy_n(&Rcw[((size_t)k * C + c) * 9], 9, f.Rcw[c].begin());
                std::copy_n(&tcw[((size_t)k * C + c) * 3], 3, f.tcw[c].begin());
            }
            f.imu = kf_imu[k] != 0, f.fixed = k >= n_opt;
            slot[k] = win.add_keyframe(f);
        }
        for (int i = 0; i < n_pts_use; ++i) win.add_point({pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}, depth[i]);
        for (size_t e = 0; e < mpt.size(); ++e)
            if (mpt[e] < n_pts_use) win.add_mono(mpt[e], slot[mkf[e]], mcam[e], mobs[2 * e], mobs[2 * e + 1], mw[e]);
        for (size_t e = 0; e < spt.size(); ++e)
            if (spt[e] < n_pts_use) win.add_stereo(spt[e], slot[skf[e]], sobs[3 * e], sobs[3 * e + 1], sobs[3 * e + 2], sw[e]);
        const int N = (int)ik1.size();
        for (int i = 0; i < N; ++i)   // the reference's robust / information rule (Optimizer.cc:2972-2981)
            win.add_inertial(omv_adapt::LocalInertialBAWindow::Inertial::make(
                slot[ik1[i]], slot[ik2[i]],
                std::vector<float>(pre.begin() + (size_t)i * OMV_PREINT_FLOATS, pre.begin() + (size_t)(i + 1) * OMV_PREINT_FLOATS),
                i == N - 1, rec_init));
    };
    if (m["warm_small"] != 0) {
        build(P / 4);
        (void)win.optimize(m["large"] != 0);
    }
    build(P);
    std::vector<double> chi2, schi2;
    std::vector<uint8_t> outl, soutl;
    const omv_lba_result r = win.optimize(m["large"] != 0, &chi2, &outl, &schi2, &soutl);
    // state back in the original keyframe order
    std::vector<double> oRwb(9 * K), otwb(3 * K), oRcw((size_t)9 * K * C), otcw((size_t)3 * K * C), ovel(3 * K), obg(3 * K), oba(3 * K);
    for (int k = 0; k < K; ++k) {
        const auto &f = win.keyframes()[slot[k]];
        std::copy(f.Rwb.begin(), f.Rwb.end(), &oRwb[9 * k]), std::copy(f.twb.begin(), f.twb.end(), &otwb[3 * k]);
        std::copy(f.vel.begin(), f.vel.end(), &ovel[3 * k]), std::copy(f.bg.begin(), f.bg.end(), &obg[3 * k]);
        std::copy(f.ba.begin(), f.ba.end(), &oba[3 * k]);
        for (int c = 0; c < C; ++c) {
            std::copy(f.Rcw[c].begin(), f.Rcw[c].end(), &oRcw[((size_t)k * C + c) * 9]);
            std::copy(f.tcw[c].begin(), f.tcw[c].end(), &otcw[((size_t)k * C + c) * 3]);
        }
    }
    write_bin(dir, "out_Rwb", oRwb), write_bin(dir, "out_twb", otwb), write_bin(dir, "out_Rcw", oRcw);
    write_bin(dir, "out_tcw", otcw), write_bin(dir, "out_vel", ovel), write_bin(dir, "out_bg", obg), write_bin(dir, "out_ba", oba);
    write_bin(dir, "out_pts", win.points());
    write_bin(dir, "out_chi2", chi2), write_bin(dir, "out_outlier", outl);
    write_bin(dir, "out_stereo_chi2", schi2), write_bin(dir, "out_stereo_outlier", soutl);
    std::ofstream o(dir + "/result.txt");
    o.precision(17);
    const auto hs = win.host_syncs();
    o << "err " << r.err << "\nerr_end " << r.err_end << "\nstatus " << r.status << "\niterations " << r.iterations
      << "\ntrials " << r.trials << "\nlambda " << r.lambda << "\nallreduce_calls " << g_allreduce_calls
      << "\nhost_syncs " << hs.first << "\n";
    if (comm) ncclCommDestroy(comm);
    return 0;
}

omv_se3f se3_of(const std::vector<float> &t7) {   // qx qy qz qw tx ty tz
    omv_se3f T{};
    for (int q = 0; q < 4; ++q) T.q[q] = t7[q];
    for (int q = 0; q < 3; ++q) T.t[q] = t7[4 + q];
    return T;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) on a MultiCameraFrame built from the images
int run_lastframe(const std::string &dir) {
    auto m = read_meta(dir);
    const int C = (int)m["C"], W = (int)m["W"], H = (int)m["H"];
    const auto img = read_bin<uint8_t>(dir, "images");
    const auto lap = read_bin<int32_t>(dir, "lapping");
    std::vector<std::array<int, 2>> lapping(C);
    for (int c = 0; c < C; ++c) lapping[c] = {lap[2 * c], lap[2 * c + 1]};
    const omv_orb_params p{(int)m["nfeatures"], 1.2f, 8, (int)m["ini"], (int)m["min"]};
    const int last_cap = (int)m["last_cap"];
    omv_adapt::MultiCameraFrame F(C, W, H, p, lapping, C * last_cap);
    F.set_camera_models(read_opt<int32_t>(dir, "cam_model"));
    std::vector<const uint8_t *> ims(C);
    for (int c = 0; c < C; ++c) ims[c] = img.data() + (size_t)c * W * H;
    F.build(ims);
    omv_adapt::LastFrameView last;
    last.last_cap = last_cap;
    last.pos = read_bin<float>(dir, "last_pos"), last.desc = read_bin<uint8_t>(dir, "last_desc");
    last.valid = read_bin<uint8_t>(dir, "last_valid"), last.has_obs = read_bin<uint8_t>(dir, "last_obs");
    last.keys = read_bin<omv_kp>(dir, "last_kps");
    last.Tcw = se3_of(read_bin<float>(dir, "Tlw"));
    const auto occ = read_bin<uint8_t>(dir, "occ");
    std::vector<int32_t> k2m((size_t)C * F.kp_cap(), -1);
    omv_adapt::SearchByProjectionLastFrame sbp((float)m["nnratio"], m["check_ori"] != 0);
    const int n = sbp(F, last, se3_of(read_bin<float>(dir, "Tcw")), se3_of(read_bin<float>(dir, "Trl")),
                      read_bin<float>(dir, "cams"), (float)m["th"], m["bmono"] != 0, (float)m["mb"], k2m, &occ);
    write_bin(dir, "kp_to_mp", k2m);
    write_bin(dir, "n_matches", &n, 1);
    return 0;
}

omv_adapt::KeyFrameView read_kf(const std::string &dir, const std::string &k, const std::map<std::string, double> &m) {
    omv_adapt::KeyFrameView v;
    v.N = (int)m.at(k + "_n"), v.NLeft = (int)m.at(k + "_n_left"), v.NRight = (int)m.at(k + "_n_right");
    v.NSideLeft = (int)m.at(k + "_n_sideleft");
    v.keys = read_bin<omv_kp>(dir, k + "_kps"), v.descriptors = read_bin<uint8_t>(dir, k + "_desc");
    v.has_map_point = read_bin<uint8_t>(dir, k + "_has_mp"), v.feat_node = read_bin<uint32_t>(dir, k + "_node_id");
    v.feat_start = read_bin<int32_t>(dir, k + "_node_start"), v.feat_idx = read_bin<int32_t>(dir, k + "_node_idx");
    const auto s2 = read_bin<float>(dir, "level_sigma2");
    std::copy_n(s2.begin(), std::min<size_t>(16, s2.size()), v.level_sigma2.begin());
    return v;
}

// SearchForTriangulation(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse)
int run_tri(const std::string &dir) {
    auto m = read_meta(dir);
    const auto kf1 = read_kf(dir, "kf1", m), kf2 = read_kf(dir, "kf2", m);
    const auto Tf = read_bin<float>(dir, "T");
    std::array<std::array<float, 12>, OMV_TRI_PAIRS> T{};
    for (int q = 0; q < OMV_TRI_PAIRS; ++q) std::copy_n(&Tf[12 * q], 12, T[q].begin());
    omv_adapt::SearchForTriangulation sft(0.6f, m["check_ori"] != 0);
    std::vector<std::pair<size_t, size_t>> pairs;
    const int n = sft(kf1, kf2, T, read_bin<float>(dir, "cams"), read_opt<int32_t>(dir, "cam_model"), pairs,
                      m["only_stereo"] != 0, m["coarse"] != 0);
    std::vector<int64_t> flat;
    for (const auto &pr : pairs) flat.push_back((int64_t)pr.first), flat.push_back((int64_t)pr.second);
    write_bin(dir, "pairs", flat);
    write_bin(dir, "n_matches", &n, 1);
    return 0;
}

omv_adapt::PoseInertialOptimizer::State read_state(const std::string &dir, const std::string &pre, int C) {
    omv_adapt::PoseInertialOptimizer::State s;
    const auto R = read_bin<double>(dir, pre + "Rwb"), t = read_bin<double>(dir, pre + "twb");
    const auto v = read_bin<double>(dir, pre + "vel"), g = read_bin<double>(dir, pre + "bg"), a = read_bin<double>(dir, pre + "ba");
    std::copy_n(R.begin(), 9, s.Rwb.begin()), std::copy_n(t.begin(), 3, s.twb.begin()), std::copy_n(v.begin(), 3, s.vel.begin());
    std::copy_n(g.begin(), 3, s.bg.begin()), std::copy_n(a.begin(), 3, s.ba.begin());
    s.Rcw.resize(C), s.tcw.resize(C);
    if (pre.empty()) {
        const auto Rc = read_bin<double>(dir, "Rcw"), tc = read_bin<double>(dir, "tcw");
        for (int c = 0; c < C; ++c) std::copy_n(&Rc[9 * c], 9, s.Rcw[c].begin()), std::copy_n(&tc[3 * c], 3, s.tcw[c].begin());
    }
    return s;
}

// PoseInertialOptimizationLastKeyFrame / LastFrame on one frame (meta lf 0 / 1)
int run_pose(const std::string &dir) {
    auto m = read_meta(dir);
    const int C = (int)m["n_cams"], cap = (int)m["kp_cap"];
    omv_adapt::PoseInertialOptimizer opt(C, read_bin<float>(dir, "cam"), read_bin<double>(dir, "Rcb"), read_bin<double>(dir, "tcb"),
                                         read_bin<double>(dir, "Rbc"), read_bin<double>(dir, "tbc"), (float)m["bf"],
                                         read_opt<int32_t>(dir, "cam_model"));
    auto frame = read_state(dir, "", C);
    const auto other = read_state(dir, "kf_", C);
    const auto mcam = read_bin<int32_t>(dir, "mono_cam"), mkp = read_bin<int32_t>(dir, "mono_kp");
    const auto mobs = read_bin<double>(dir, "mono_obs");
    const auto mw = read_bin<float>(dir, "mono_inv_sigma2"), mx = read_bin<float>(dir, "mono_xw");
    const auto mclose = read_bin<uint8_t>(dir, "mono_close");
    const auto scam = read_opt<int32_t>(dir, "stereo_cam"), skp = read_opt<int32_t>(dir, "stereo_kp");
    const auto sobs = read_opt<double>(dir, "stereo_obs");
    const auto sw = read_opt<float>(dir, "stereo_inv_sigma2"), sx = read_opt<float>(dir, "stereo_xw");
    std::vector<omv_adapt::PoseInertialOptimizer::Mono> mono;
    for (size_t e = 0; e < mcam.size(); ++e)
        mono.push_back({mcam[e], mkp[e], mobs[2 * e], mobs[2 * e + 1], mw[e], {mx[3 * e], mx[3 * e + 1], mx[3 * e + 2]},
                        mclose[e] != 0});
    std::vector<omv_adapt::PoseInertialOptimizer::Stereo> stereo;
    for (size_t e = 0; e < scam.size(); ++e)
        stereo.push_back({scam[e], skp[e], sobs[3 * e], sobs[3 * e + 1], sobs[3 * e + 2], sw[e],
                          {sx[3 * e], sx[3 * e + 1], sx[3 * e + 2]}});
    std::vector<uint8_t> outl(cap, 255);
    std::array<double, 225> H{};
    int n_good;
    if (m["lf"] != 0) {
        omv_adapt::PoseInertialOptimizer::Prior pr;
        const auto R = read_bin<double>(dir, "prior_Rwb"), t = read_bin<double>(dir, "prior_twb");
        const auto v = read_bin<double>(dir, "prior_vel"), g = read_bin<double>(dir, "prior_bg");
        const auto a = read_bin<double>(dir, "prior_ba"), Hp = read_bin<double>(dir, "prior_H");
        std::copy_n(R.begin(), 9, pr.Rwb.begin()), std::copy_n(t.begin(), 3, pr.twb.begin()), std::copy_n(v.begin(), 3, pr.vel.begin());
        std::copy_n(g.begin(), 3, pr.bg.begin()), std::copy_n(a.begin(), 3, pr.ba.begin()), std::copy_n(Hp.begin(), 225, pr.H.begin());
        n_good = opt.LastFrame(frame, other, read_bin<float>(dir, "preint"), read_bin<float>(dir, "preint_kf"), pr, mono,
                               stereo, outl, &H, m["rec_init"] != 0);
        const auto Hc = opt.ConstraintPoseImu(H);   // the prior the next frame would receive
        write_bin(dir, "out_Hc", Hc.data(), 225);
    } else {
        n_good = opt.LastKeyFrame(frame, other, read_bin<float>(dir, "preint"), mono, stereo, outl, &H, m["rec_init"] != 0);
    }
    std::vector<double> Rc, tc;
    for (int c = 0; c < C; ++c) Rc.insert(Rc.end(), frame.Rcw[c].begin(), frame.Rcw[c].end()), tc.insert(tc.end(), frame.tcw[c].begin(), frame.tcw[c].end());
    write_bin(dir, "out_Rwb", frame.Rwb.data(), 9), write_bin(dir, "out_twb", frame.twb.data(), 3);
    write_bin(dir, "out_vel", frame.vel.data(), 3), write_bin(dir, "out_bg", frame.bg.data(), 3);
    write_bin(dir, "out_ba", frame.ba.data(), 3), write_bin(dir, "out_Rcw", Rc), write_bin(dir, "out_tcw", tc);
    write_bin(dir, "out_kpo", outl), write_bin(dir, "out_H", H.data(), 225), write_bin(dir, "n_good", &n_good, 1);
    return 0;
}

// Fuse(pKF, vpMapPoints, th, cameraID) for every camera block of one keyframe (one job list per block)
int run_fuse(const std::string &dir) {
    auto m = read_meta(dir);
    const int C = (int)m["C"], cap = (int)m["kp_cap"], J = (int)m["n_jobs"];
    omv_adapt::Fuse fuse(C, cap, (int)m["W"], (int)m["H"], read_bin<float>(dir, "scale_factors"), read_bin<float>(dir, "cams"),
                         read_opt<int32_t>(dir, "cam_model"), (float)m["bf"], (int)m["max_points"]);
    fuse.set_keyframe(read_bin<omv_kp>(dir, "kps"), read_bin<uint8_t>(dir, "desc"), read_bin<int32_t>(dir, "n_kp"),
                      read_bin<float>(dir, "uright"));
    const auto jc = read_bin<int32_t>(dir, "job_cam"), jn = read_bin<int32_t>(dir, "job_count");
    const auto jT = read_bin<float>(dir, "job_Tcw"), jO = read_bin<float>(dir, "job_Ow");
    const auto pos = read_bin<float>(dir, "mp_pos"), nrm = read_bin<float>(dir, "mp_normal");
    const auto mind = read_bin<float>(dir, "mp_min_dist"), maxd = read_bin<float>(dir, "mp_max_dist");
    const auto desc = read_bin<uint8_t>(dir, "mp_desc");
    const auto ils = read_bin<float>(dir, "inv_level_sigma2");
    std::vector<int32_t> all_idx, all_dist, nf;
    size_t at = 0;
    for (int j = 0; j < J; ++j) {
        omv_adapt::FuseMapPoints mp;
        const size_t n = (size_t)jn[j];
        mp.pos.assign(&pos[3 * at], &pos[3 * (at + n)]), mp.normal.assign(&nrm[3 * at], &nrm[3 * (at + n)]);
        mp.min_dist.assign(&mind[at], &mind[at + n]), mp.max_dist.assign(&maxd[at], &maxd[at + n]);
        mp.desc.assign(&desc[32 * at], &desc[32 * (at + n)]);
        std::vector<int32_t> bi, bd;
        const omv_se3f T = se3_of(std::vector<float>(&jT[7 * j], &jT[7 * j + 7]));
        nf.push_back(fuse(mp, jc[j], T, {jO[3 * j], jO[3 * j + 1], jO[3 * j + 2]}, (float)m["th"], ils, bi, bd));
        all_idx.insert(all_idx.end(), bi.begin(), bi.end()), all_dist.insert(all_dist.end(), bd.begin(), bd.end());
        at += n;
    }
    write_bin(dir, "best_idx", all_idx), write_bin(dir, "best_dist", all_dist), write_bin(dir, "n_fused", nf);
    return 0;
}

// ---- Optimizer::PoseOptimization(Frame*) on one frame
int run_posopt(const std::string &dir) {
    auto m = read_meta(dir);
    const int C = (int)m["n_cams"], cap = (int)m["kp_cap"];
    const auto cams = read_bin<float>(dir, "cams");
    const auto model = read_opt<int32_t>(dir, "cam_model");
    const auto rq = read_bin<double>(dir, "rig_q"), rt = read_bin<double>(dir, "rig_t");
    std::vector<std::array<double, 4>> rig_q(C);
    std::vector<std::array<double, 3>> rig_t(C);
    for (int c = 0; c < C; ++c) {
        for (int q = 0; q < 4; ++q) rig_q[c][q] = rq[4 * c + q];
        for (int q = 0; q < 3; ++q) rig_t[c][q] = rt[3 * c + q];
    }
    omv_adapt::PoseOptimization po(C, cams, model, (float)m["bf"], rig_q, rig_t);
    const auto mc = read_opt<int32_t>(dir, "mono_cam"), mk = read_opt<int32_t>(dir, "mono_kp");
    const auto mo = read_opt<double>(dir, "mono_obs");
    const auto mw = read_opt<float>(dir, "mono_w"), mx = read_opt<float>(dir, "mono_xw");
    const auto sk = read_opt<int32_t>(dir, "stereo_kp");
    const auto so = read_opt<double>(dir, "stereo_obs");
    const auto sw = read_opt<float>(dir, "stereo_w"), sx = read_opt<float>(dir, "stereo_xw");
    std::vector<omv_adapt::PoseOptimization::Mono> mono(mc.size());
    for (size_t e = 0; e < mc.size(); ++e)
        mono[e] = {mc[e], mk[e], mo[2 * e], mo[2 * e + 1], mw[e], {mx[3 * e], mx[3 * e + 1], mx[3 * e + 2]}};
    std::vector<omv_adapt::PoseOptimization::Stereo> stereo(sk.size());
    for (size_t e = 0; e < sk.size(); ++e)
        stereo[e] = {sk[e], so[3 * e], so[3 * e + 1], so[3 * e + 2], sw[e], {sx[3 * e], sx[3 * e + 1], sx[3 * e + 2]}};
    const auto q0 = read_bin<double>(dir, "pose_q"), t0 = read_bin<double>(dir, "pose_t");
    std::array<double, 4> q{q0[0], q0[1], q0[2], q0[3]};
    std::array<double, 3> t{t0[0], t0[1], t0[2]};
    std::vector<uint8_t> outl(cap, 255);
    const int n_good = po(q, t, mono, stereo, outl);
    write_bin(dir, "q", q.data(), 4), write_bin(dir, "t", t.data(), 3), write_bin(dir, "kpo", outl);
    write_bin(dir, "n_good", &n_good, 1);
    return 0;
}

// ---- LocalMapping::CreateNewMapPoints: keyframe k's arrays are DIR/kf<k>_*.bin (k = 0 the current keyframe)
omv_adapt::CnmpKeyFrame read_cnmp_kf(const std::string &dir, int k) {
    const std::string p = "kf" + std::to_string(k) + "_";
    omv_adapt::CnmpKeyFrame f;
    const auto ints = read_bin<int32_t>(dir, p + "ints");   // N NLeft NRight NSideLeft
    f.view.N = ints[0], f.view.NLeft = ints[1], f.view.NRight = ints[2], f.view.NSideLeft = ints[3];
    f.view.keys = read_bin<omv_kp>(dir, p + "keys");
    f.view.descriptors = read_bin<uint8_t>(dir, p + "desc");
    f.view.has_map_point = read_bin<uint8_t>(dir, p + "has_mp");
    f.view.feat_node = read_bin<uint32_t>(dir, p + "node_id");
    f.view.feat_start = read_bin<int32_t>(dir, p + "node_start");
    f.view.feat_idx = read_bin<int32_t>(dir, p + "node_idx");
    const auto sg = read_bin<float>(dir, p + "sigma2");
    std::copy(sg.begin(), sg.begin() + 16, f.view.level_sigma2.begin());
    const auto T = read_bin<float>(dir, p + "Tcw"), O = read_bin<float>(dir, p + "Ow");
    for (int c = 0; c < 4; ++c) {
        std::copy(&T[12 * c], &T[12 * c + 12], f.Tcw[c].begin());
        std::copy(&O[3 * c], &O[3 * c + 3], f.Ow[c].begin());
    }
    const auto g = read_bin<float>(dir, p + "geom");   // Rwc[9] twc[3] fx fy cx cy invfx invfy mb mbf
    std::copy(&g[0], &g[9], f.Rwc.begin()), std::copy(&g[9], &g[12], f.twc.begin());
    f.fx = g[12], f.fy = g[13], f.cx = g[14], f.cy = g[15], f.invfx = g[16], f.invfy = g[17], f.mb = g[18], f.mbf = g[19];
    f.uright = read_bin<float>(dir, p + "uright"), f.depth = read_bin<float>(dir, p + "depth");
    const auto sf = read_bin<float>(dir, p + "scale");
    std::copy(sf.begin(), sf.begin() + 16, f.scale_factors.begin());
    return f;
}

int run_cnmp(const std::string &dir) {
    auto m = read_meta(dir);
    const int n_nb = (int)m["n_nb"], split = (int)m["split"];
    omv_adapt::CreateNewMapPoints cnmp(read_bin<float>(dir, "cams"), read_bin<int32_t>(dir, "cam_model"), (int)m["n_cams"],
                                       m["inertial"] != 0, m["monocular"] != 0, m["far"] != 0, (float)m["th_far"]);
    const omv_adapt::CnmpKeyFrame kf1 = read_cnmp_kf(dir, 0);
    std::vector<omv_adapt::CnmpKeyFrame> nbs;
    for (int k = 1; k <= n_nb; ++k) nbs.push_back(read_cnmp_kf(dir, k));
    const auto Tall = read_bin<float>(dir, "T");
    std::vector<std::array<std::array<float, 12>, OMV_TRI_PAIRS>> T(n_nb);
    for (int j = 0; j < n_nb; ++j)
        for (int q = 0; q < OMV_TRI_PAIRS; ++q) std::copy(&Tall[(j * OMV_TRI_PAIRS + q) * 12], &Tall[(j * OMV_TRI_PAIRS + q) * 12 + 12], T[j][q].begin());
    const auto skip = read_bin<int32_t>(dir, "skip");
    std::vector<int> sk(skip.begin(), skip.end());
    std::vector<uint8_t> has_mp1 = kf1.view.has_map_point;
    // the neighbours in two calls (a CheckNewKeyFrames() boundary after `split`), side 1 carried over
    std::vector<omv_adapt::NewMapPoint> pts;
    std::vector<int> nm_all, nm;
    for (int part = 0; part < 2; ++part) {
        const size_t lo = part == 0 ? 0 : (size_t)split, hi = part == 0 ? (size_t)split : (size_t)n_nb;
        auto p = cnmp(kf1, has_mp1, nbs, T, sk, m["coarse"] != 0, (float)m["scale_factor"], lo, hi, part == 0, &nm);
        pts.insert(pts.end(), p.begin(), p.end());
        nm_all.insert(nm_all.end(), nm.begin(), nm.end());
    }
    std::vector<int32_t> rec;   // per new point: neighbour idx1 idx2 stereo
    std::vector<float> x;
    for (const auto &p : pts) {
        rec.insert(rec.end(), {p.neighbour, (int32_t)p.idx1, (int32_t)p.idx2, p.stereo ? 1 : 0});
        x.insert(x.end(), p.x3D.begin(), p.x3D.end());
    }
    write_bin(dir, "points", rec), write_bin(dir, "x3d", x), write_bin(dir, "has_mp1", has_mp1);
    std::vector<int32_t> nmv(nm_all.begin(), nm_all.end());
    write_bin(dir, "n_matches", nmv);
    return 0;
}

// ---- MapPoint::ComputeDistinctiveDescriptors / UpdateNormalAndDepth
int run_mprefresh(const std::string &dir) {
    omv_adapt::MapPointRefresh r;
    std::vector<uint8_t> dout;
    const auto best = r.distinctive(read_bin<int32_t>(dir, "desc_start"), read_bin<int32_t>(dir, "desc_row"),
                                    read_bin<uint8_t>(dir, "desc"), dout);
    write_bin(dir, "best", best), write_bin(dir, "desc_out", dout);
    auto normal = read_bin<float>(dir, "normal_in");
    auto mn = read_bin<float>(dir, "min_in"), mx = read_bin<float>(dir, "max_in");
    r.normal_depth(read_bin<int32_t>(dir, "obs_start"), read_bin<float>(dir, "obs_center"), read_bin<float>(dir, "pos"),
                   read_bin<float>(dir, "ref_center"), read_bin<float>(dir, "ref_level_scale"),
                   read_bin<float>(dir, "ref_max_scale"), normal, mn, mx);
    write_bin(dir, "normal", normal), write_bin(dir, "min_dist", mn), write_bin(dir, "max_dist", mx);
    return 0;
}

// ---- LocalMapping::SearchInNeighbors' fuse sequence
int run_fuseseq(const std::string &dir) {
    auto m = read_meta(dir);
    omv_adapt::FuseGraphView g;
    g.n_kf = (int)m["n_kf"], g.n_cams = (int)m["n_cams"], g.kp_cap = (int)m["kp_cap"];
    g.width = (int)m["width"], g.height = (int)m["height"], g.bf = (float)m["bf"], g.th = (float)m["th"];
    g.scale_factors = read_bin<float>(dir, "scale"), g.cams = read_bin<float>(dir, "cams");
    g.kps = read_bin<omv_kp>(dir, "kps"), g.desc = read_bin<uint8_t>(dir, "desc"), g.n_kp = read_bin<int32_t>(dir, "n_kp");
    g.uright = read_bin<float>(dir, "uright"), g.n_blocks = read_bin<int32_t>(dir, "n_blocks");
    g.Tcw = read_bin<omv_se3f>(dir, "Tcw"), g.Ow = read_bin<float>(dir, "Ow"), g.kf_mps = read_bin<int32_t>(dir, "kf_mps");
    g.pos = read_bin<float>(dir, "pos"), g.normal = read_bin<float>(dir, "normal");
    g.min_dist = read_bin<float>(dir, "min_dist"), g.max_dist = read_bin<float>(dir, "max_dist");
    g.mp_desc = read_bin<uint8_t>(dir, "mp_desc"), g.bad = read_bin<int32_t>(dir, "bad"), g.n_obs = read_bin<int32_t>(dir, "n_obs");
    g.obs_start = read_bin<int32_t>(dir, "obs_start"), g.obs_kf = read_bin<int32_t>(dir, "obs_kf");
    g.obs_idx = read_bin<int32_t>(dir, "obs_idx");
    omv_adapt::SearchInNeighborsFuse f;
    const auto nf = f(g, (int)m["current"], read_bin<int32_t>(dir, "targets"), read_bin<float>(dir, "inv_sigma2"));
    write_bin(dir, "out_kf_mps", g.kf_mps), write_bin(dir, "out_bad", g.bad), write_bin(dir, "out_n_obs", g.n_obs);
    write_bin(dir, "out_replaced", g.replaced), write_bin(dir, "out_obs_start", g.obs_start);
    write_bin(dir, "out_obs_kf", g.obs_kf), write_bin(dir, "out_obs_idx", g.obs_idx), write_bin(dir, "out_log", g.log);
    write_bin(dir, "out_desc", g.mp_desc), write_bin(dir, "out_n_fused", nf);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s orb|frame|lba|lastframe|tri|pose|fuse|posopt|cnmp|mprefresh|fuseseq DIR\n", argv[0]);
        return 2;
    }
    try {
        const std::string mode = argv[1], dir = argv[2];
        if (mode == "orb") return run_orb(dir);
        if (mode == "frame") return run_frame(dir);
        if (mode == "lba") return run_lba(dir);
        if (mode == "lastframe") return run_lastframe(dir);
        if (mode == "tri") return run_tri(dir);
        if (mode == "pose") return run_pose(dir);
        if (mode == "fuse") return run_fuse(dir);
        if (mode == "posopt") return run_posopt(dir);
        if (mode == "cnmp") return run_cnmp(dir);
        if (mode == "mprefresh") return run_mprefresh(dir);
        if (mode == "fuseseq") return run_fuseseq(dir);
        std::fprintf(stderr, "unknown mode %s\n", argv[1]);
        return 2;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "omv_consumer: %s\n", e.what());
        return 1;
    }
}
