// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for the Hamming matchers. Never linked into the product.
//
// Scalar restatement of
//   Frame::AssignFeaturesToGrid / PosInGrid         src/Frame.cc:541-582, :969-978
//   Frame::GetFeaturesInArea                         src/Frame.cc:890-967
//   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
//                                                    src/ORBmatcher.cc:23-340 (+ RadiusByViewingCos :342-347)
//   ORBmatcher::DescriptorDistance                   src/ORBmatcher.cc:2577-2591
//   Frame::isInFrustum / isInFrustumChecks           src/Frame.cc:736-826, :1529-1653 (multi-camera branch)
//     + MapPoint::PredictScale                       src/MapPoint.cc:624-637
//     + KannalaBrandt8::project(Eigen::Vector3f)     src/CameraModels/KannalaBrandt8.cpp:48-67
//   ORBmatcher::SearchByProjection(Frame&, const Frame& LastFrame, th, bMono)
//                                                    src/ORBmatcher.cc:1985-2413 (+ ComputeThreeMaxima :2537-2573)
//   ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, S12, th)
//                                                    src/ORBmatcher.cc:1771-1983
//   cv::BFMatcher(NORM_HAMMING).knnMatch(k = 2)      as called by Frame::ComputeMultiFishEyeMatches,
//                                                    src/Frame.cc:1483 (OpenCV batchDistance K = 2:
//                                                    strict '<' insertion, first train index wins ties)
// generalised from the reference's 4 camera blocks (L, R, SL, SR) to n_cams blocks: block 0 behaves as
// the left camera, block 1 as the right camera, blocks >= 2 as side cameras.  Multi-camera frames only
// (Nleft != -1); the monocular mvuRight branch is not part of this path.
//
// Data layout (shared with the C ABI): keypoints/descriptors padded per camera, [cam][kp_cap];
// kp_to_mp / occ_init indexed by slot = cam * kp_cap + i (F.mvpMapPoints in padded form).
// Parity status: no reference test pins these functions; parity is to this restatement.
// =====================================================================================================
#include <array>
#include <cmath>
#include <map>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

const int kGridCols = 64, kGridRows = 48;   // FRAME_GRID_COLS / FRAME_GRID_ROWS (include/Frame.h:24-25)
const int TH_HIGH = 100;

struct KP {
    float x, y, size, angle, response;
    int32_t octave;
};

struct FrameGeom {   // omv_frame_geom
    int n_cams;
    float min_x, max_x, min_y, max_y;
    int nlevels;
    float scale_factors[16];
    int cam_model[8];   // 0 KannalaBrandt8, 1 Pinhole per camera block
};

int descriptor_distance(const uint8_t *a, const uint8_t *b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        uint32_t v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24;
    }
    return dist;
}

struct Grid {   // per camera: cells[ix][iy] -> ascending keypoint indices
    std::vector<std::vector<int>> cells;
    Grid() : cells(kGridCols * kGridRows) {}
    std::vector<int> &at(int ix, int iy) { return cells[ix * kGridRows + iy]; }
    const std::vector<int> &at(int ix, int iy) const { return cells[ix * kGridRows + iy]; }
};

struct View {
    const FrameGeom *g;
    float invW, invH;
    std::vector<Grid> grids;
    const KP *kps;
    int kp_cap;
    const int *n_kp;
};

bool pos_in_grid(const View &v, const KP &kp, int &px, int &py) {
    px = (int)std::round((kp.x - v.g->min_x) * v.invW);
    py = (int)std::round((kp.y - v.g->min_y) * v.invH);
    return !(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows);
}

void build_grids(View &v) {
    v.invW = (float)kGridCols / (v.g->max_x - v.g->min_x);
    v.invH = (float)kGridRows / (v.g->max_y - v.g->min_y);
    v.grids.assign(v.g->n_cams, Grid());
    for (int c = 0; c < v.g->n_cams; ++c)
        for (int i = 0; i < v.n_kp[c]; ++i) {
            int px, py;
            if (pos_in_grid(v, v.kps[(size_t)c * v.kp_cap + i], px, py)) v.grids[c].at(px, py).push_back(i);
        }
}

std::vector<int> features_in_area(const View &v, float x, float y, float r, int minLevel, int maxLevel, int cam) {
    std::vector<int> out;
    const int nMinCellX = std::max(0, (int)std::floor((x - v.g->min_x - r) * v.invW));
    if (nMinCellX >= kGridCols) return out;
    const int nMaxCellX = std::min(kGridCols - 1, (int)std::ceil((x - v.g->min_x + r) * v.invW));
    if (nMaxCellX < 0) return out;
    const int nMinCellY = std::max(0, (int)std::floor((y - v.g->min_y - r) * v.invH));
    if (nMinCellY >= kGridRows) return out;
    const int nMaxCellY = std::min(kGridRows - 1, (int)std::ceil((y - v.g->min_y + r) * v.invH));
    if (nMaxCellY < 0) return out;
    const bool checkLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
        for (int iy = nMinCellY; iy <= nMaxCellY; ++iy)
            for (int i : v.grids[cam].at(ix, iy)) {
                const KP &k = v.kps[(size_t)cam * v.kp_cap + i];
                if (checkLevels) {
                    if (k.octave < minLevel) continue;
                    if (maxLevel >= 0 && k.octave > maxLevel) continue;
                }
                const float dx = k.x - x, dy = k.y - y;
                if (std::fabs(dx) < r && std::fabs(dy) < r) out.push_back(i);
            }
    return out;
}

}  // namespace

extern "C" {

// Grid of one camera: cell_start[64*48+1] (cell = ix*48+iy) and idx[] in cell order.
int oracle_grid(const FrameGeom *g, const KP *kps, int kp_cap, const int *n_kp, int cam, int32_t *cell_start,
                int32_t *idx) {
    View v{g, 0, 0, {}, kps, kp_cap, n_kp};
    build_grids(v);
    int pos = 0;
    for (int c = 0; c < kGridCols * kGridRows; ++c) {
        cell_start[c] = pos;
        for (int i : v.grids[cam].cells[c]) idx[pos++] = i;
    }
    cell_start[kGridCols * kGridRows] = pos;
    return pos;
}

// GetFeaturesInArea on one camera block; returns count written to out (up to cap).
int oracle_features_in_area(const FrameGeom *g, const KP *kps, int kp_cap, const int *n_kp, float x, float y,
                            float r, int minLevel, int maxLevel, int cam, int32_t *out, int cap) {
    View v{g, 0, 0, {}, kps, kp_cap, n_kp};
    build_grids(v);
    std::vector<int> r_ = features_in_area(v, x, y, r, minLevel, maxLevel, cam);
    for (size_t i = 0; i < r_.size() && (int)i < cap; ++i) out[i] = r_[i];
    return (int)r_.size();
}

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints).
// Map point arrays: desc [M][32]; proj_x/proj_y/view_cos/level/in_view [M][n_cams];
// track_depth/is_bad/has_obs [M].  kp_to_mp [n_cams*kp_cap] in/out, occ_init [n_cams*kp_cap].
int oracle_search_by_projection(const FrameGeom *g, const KP *kps, const uint8_t *desc, int kp_cap,
                                const int *n_kp, const uint8_t *mp_desc, const float *proj_x,
                                const float *proj_y, const float *view_cos, const int32_t *level,
                                const uint8_t *in_view, const float *track_depth, const uint8_t *is_bad,
                                const uint8_t *has_obs, int M, float th, int bFarPoints, float thFarPoints,
                                float nnratio, const int32_t *l2r, const int32_t *r2l, const uint8_t *occ_init,
                                int32_t *kp_to_mp) {
    View v{g, 0, 0, {}, kps, kp_cap, n_kp};
    build_grids(v);
    const int C = g->n_cams;
    const bool bFactor = th != 1.0;
    // "F.mvpMapPoints[idx] && F.mvpMapPoints[idx]->Observations() > 0"
    std::vector<uint8_t> blocked(occ_init, occ_init + (size_t)C * kp_cap);
    auto assign = [&](int slot, int mp) {
        kp_to_mp[slot] = mp;
        blocked[slot] = has_obs[mp] ? 1 : 0;
    };
    int nmatches = 0;
    for (int m = 0; m < M; ++m) {
        bool any = false;
        for (int c = 0; c < C; ++c) any = any || in_view[(size_t)m * C + c];
        if (!any) continue;
        if (bFarPoints && track_depth[m] > thFarPoints) continue;
        if (is_bad[m]) continue;
        const uint8_t *dmp = mp_desc + (size_t)m * 32;
        for (int c = 0; c < C; ++c) {
            const size_t mc = (size_t)m * C + c;
            if (!in_view[mc]) continue;
            const int lvl = level[mc];
            if (c > 0 && lvl == -1) continue;
            float r = view_cos[mc] > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos
            if (c == 0 && bFactor) r *= th;                 // th scales the left block only
            const std::vector<int> cand =
                features_in_area(v, proj_x[mc], proj_y[mc], r * g->scale_factors[lvl], lvl - 1, lvl, c);
            if (cand.empty()) continue;
            int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
            for (int idx : cand) {
                const int slot = c * kp_cap + idx;
                if (blocked[slot]) continue;
                const int dist = descriptor_distance(dmp, desc + (size_t)slot * 32);
                const int oct = kps[slot].octave;
                if (dist < bestDist) {
                    bestDist2 = bestDist, bestDist = dist;
                    bestLevel2 = bestLevel, bestLevel = oct;
                    bestIdx = idx;
                } else if (dist < bestDist2) {
                    bestLevel2 = oct, bestDist2 = dist;
                }
            }
            if (bestDist <= TH_HIGH) {
                if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) goto next_mp;   // `continue`
                if (c == 0) {
                    assign(bestIdx, m);
                    if (C > 1 && l2r[bestIdx] != -1) {
                        assign(kp_cap + l2r[bestIdx], m);
                        nmatches++;
                    }
                    nmatches++;
                } else if (c == 1) {
                    if (r2l[bestIdx] != -1) {
                        assign(r2l[bestIdx], m);
                        nmatches++;
                    }
                    assign(kp_cap + bestIdx, m);
                    nmatches++;
                } else {
                    assign(c * kp_cap + bestIdx, m);
                    nmatches++;
                }
            }
        }
    next_mp:;
    }
    return nmatches;
}

// knnMatch(k = 2), NORM_HAMMING.  idx2/dist2 [nq][2]; -1 / INT32_MAX where fewer trains exist.
void oracle_bf_knn2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *idx2, int32_t *dist2) {
    for (int i = 0; i < nq; ++i) {
        int d[2] = {INT32_MAX, INT32_MAX}, id[2] = {-1, -1};
        for (int j = 0; j < nt; ++j) {
            const int dd = descriptor_distance(q + (size_t)i * 32, t + (size_t)j * 32);
            if (dd < d[1]) {
                int k = 0;
                for (k = 0; k >= 0 && d[k] > dd; --k) d[k + 1] = d[k], id[k + 1] = id[k];
                d[k + 1] = dd, id[k + 1] = j;
            }
        }
        idx2[2 * i] = id[0], idx2[2 * i + 1] = id[1];
        dist2[2 * i] = d[0], dist2[2 * i + 1] = d[1];
    }
}

int oracle_descriptor_distance(const uint8_t *a, const uint8_t *b) { return descriptor_distance(a, b); }

// ---- ORBmatcher::SearchByProjection(Frame&, const Frame& LastFrame, th, bMono) (multi-camera) ----------
// Sophus::SE3f * p = q._transformVector(p) + t with Eigen's formula uv = 2 (q.vec x p),
// p + w uv + q.vec x uv (Quaternion.h), in float without contraction.
struct SE3F {
    float q[4];   // x y z w
    float t[3];
};
static void cross3f(const float *a, const float *b, float *r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}
static void quat_rotate(const float *q, const float *v, float *r) {
    float uv[3], c[3];
    cross3f(q, v, uv);
    for (int i = 0; i < 3; ++i) uv[i] = uv[i] + uv[i];
    cross3f(q, uv, c);
    for (int i = 0; i < 3; ++i) r[i] = v[i] + q[3] * uv[i] + c[i];
}
static void se3_apply(const SE3F &T, const float *p, float *r) {
    quat_rotate(T.q, p, r);
    for (int i = 0; i < 3; ++i) r[i] = r[i] + T.t[i];
}
static void kb8_project_f(const float *k, const float *X, float &u, float &v);
static void pinhole_project_f(const float *k, const float *X, float &u, float &v);
// GeometricCamera::project(const Eigen::Vector3f&), dispatched on the block's camera type
static void cam_project_f(int model, const float *k, const float *X, float &u, float &v) {
    if (model == 1) pinhole_project_f(k, X, u, v);   // OMV_CAM_PINHOLE
    else kb8_project_f(k, X, u, v);
}

}  // extern "C"

extern "C" {

// cur_*: the current frame (kps/desc [C][kp_cap], n_kp [C]), its pose Tcw, the rig (R_cl/t_cl unused here:
// Trl is passed as SE3), last_*: per LastFrame keypoint slot s = cam * last_cap + i: the tracked map point's
// world position / descriptor / Observations() > 0, validity (mvpMapPoints[s] && !mvbOutlier[s]) and the
// keypoint itself (octave, angle).  kp_to_mp [C * kp_cap] in/out receives last-frame slots.
int oracle_search_last_frame(const FrameGeom *g, const KP *kps, const uint8_t *desc, int kp_cap, const int *n_kp,
                             const float *cams /* [C][8] */, const SE3F *Tcw, const SE3F *Tlw, const SE3F *Trl,
                             const float *last_pos, const uint8_t *last_desc, const uint8_t *last_valid,
                             const uint8_t *last_obs, const KP *last_kps, int S_last, float th, int bMono, float mb,
                             int check_ori, const uint8_t *occ_init, int32_t *kp_to_mp) {
    View v{g, 0, 0, {}, kps, kp_cap, n_kp};
    build_grids(v);
    const int C = g->n_cams;
    const int HISTO_LENGTH = 30;
    const float factor = 1.0f / HISTO_LENGTH;
    std::vector<std::vector<int>> rotHist(HISTO_LENGTH);
    std::vector<uint8_t> blocked(occ_init, occ_init + (size_t)C * kp_cap);
    // twc = Tcw.inverse().translation() = -(q^-1 * t); tlc = Tlw * twc
    SE3F inv{{-Tcw->q[0], -Tcw->q[1], -Tcw->q[2], Tcw->q[3]}, {0, 0, 0}};
    float twc[3], tlc[3];
    quat_rotate(inv.q, Tcw->t, twc);
    for (int i = 0; i < 3; ++i) twc[i] = -twc[i];
    se3_apply(*Tlw, twc, tlc);
    const bool bForward = tlc[2] > mb && !bMono;
    const bool bBackward = -tlc[2] > mb && !bMono;
    int nmatches = 0;
    for (int s = 0; s < S_last; ++s) {
        if (!last_valid[s]) continue;
        float x3Dc[3];
        se3_apply(*Tcw, last_pos + 3 * (size_t)s, x3Dc);
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0) continue;
        float u, vv;
        cam_project_f(g->cam_model[0], cams, x3Dc, u, vv);   // CurrentFrame.mpCamera->project (:2022)
        if (u < g->min_x || u > g->max_x) continue;
        if (vv < g->min_y || vv > g->max_y) continue;
        const int oct = last_kps[s].octave;
        const float radius = th * g->scale_factors[oct];
        const uint8_t *dmp = last_desc + (size_t)s * 32;
        auto window = [&](float x, float y, int cam) {
            if (bForward) return features_in_area(v, x, y, radius, oct, -1, cam);
            if (bBackward) return features_in_area(v, x, y, radius, 0, oct, cam);
            return features_in_area(v, x, y, radius, oct - 1, oct + 1, cam);
        };
        auto search = [&](float x, float y, int cam) {
            int bestDist = 256, bestIdx = -1;
            for (int i2 : window(x, y, cam)) {
                const int slot = cam * kp_cap + i2;
                if (blocked[slot]) continue;
                const int dist = descriptor_distance(dmp, desc + (size_t)slot * 32);
                if (dist < bestDist) bestDist = dist, bestIdx = i2;
            }
            if (bestDist <= TH_HIGH) {
                const int slot = cam * kp_cap + bestIdx;
                kp_to_mp[slot] = s;
                blocked[slot] = last_obs[s] ? 1 : 0;
                nmatches++;
                if (check_ori) {
                    float rot = last_kps[s].angle - kps[slot].angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)std::round(rot * factor);
                    if (bin == HISTO_LENGTH) bin = 0;
                    rotHist[bin].push_back(slot);
                }
            }
        };
        search(u, vv, 0);
        if (C > 1) {   // right block: Trl * x3Dc projected with the LEFT camera model, no bounds check
            float x3Dr[3], ur, vr;
            se3_apply(*Trl, x3Dc, x3Dr);
            cam_project_f(g->cam_model[0], cams, x3Dr, ur, vr);   // CurrentFrame.mpCamera->project (:2134)
            search(ur, vr, 1);
        }
        for (int cam = 2; cam < C; ++cam) search(u, vv, cam);   // side blocks search at the LEFT projection
    }
    if (check_ori) {   // ComputeThreeMaxima + removal of every push outside the three top bins
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < HISTO_LENGTH; i++) {
            const int sz = (int)rotHist[i].size();
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
        for (int i = 0; i < HISTO_LENGTH; i++)
            if (i != ind1 && i != ind2 && i != ind3)
                for (int slot : rotHist[i]) kp_to_mp[slot] = -1, nmatches--;
    }
    return nmatches;
}

}  // extern "C"

extern "C" {
// ---- Frame::isInFrustum, multi-camera branch (one frame) ----------------------------------------------
// Float arithmetic in Eigen's evaluation order without contraction: 3x3 products and dot products sum
// left to right, norm() = sqrt((x*x + y*y) + z*z).  KannalaBrandt8.cpp and MapPoint.cc have no
// `using namespace std`, so cos(float) / sin(float) / log(float) there resolve to the C double
// functions: the float argument is promoted and the double result feeds the float expression.
struct RigF {
    int n_cams;
    float cam[8][8];
    float R_cl[8][9], t_cl[8][3];   // camera block c from camera 0 (mTrl / mTsll / mTsrl)
    float t_lc[8][3];               // translation of the inverse (mTlr / mTlsl / mTlsr)
    float min_x, max_x, min_y, max_y;
    float log_scale_factor;         // mfLogScaleFactor = (float)log(mfScaleFactor)
    int n_levels;
    int model[8];                   // 0 KannalaBrandt8, 1 Pinhole
};
struct PoseF {
    float Rcw[9], tcw[3], Rwc[9], Ow[3];
};

static void mat3f(const float *a, const float *b, float *r) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
static void matvec3f(const float *a, const float *x, float *r) {
    for (int i = 0; i < 3; ++i) r[i] = a[3 * i] * x[0] + a[3 * i + 1] * x[1] + a[3 * i + 2] * x[2];
}

// KannalaBrandt8::project(const Eigen::Vector3f&)
static void kb8_project_f(const float *k, const float *X, float &u, float &v) {
    const float x2y2 = X[0] * X[0] + X[1] * X[1];
    const float theta = atan2f(sqrtf(x2y2), X[2]);
    const float psi = atan2f(X[1], X[0]);
    const float t2 = theta * theta, t3 = theta * t2, t5 = t3 * t2, t7 = t5 * t2, t9 = t7 * t2;
    const float r = theta + k[4] * t3 + k[5] * t5 + k[6] * t7 + k[7] * t9;
    u = (float)(k[0] * r * std::cos((double)psi) + k[2]);
    v = (float)(k[1] * r * std::sin((double)psi) + k[3]);
}

// Pinhole::project(const Eigen::Vector3f&) (Pinhole.cpp:26-32): fx * x / z + cx, float, left to right
static void pinhole_project_f(const float *k, const float *X, float &u, float &v) {
    u = k[0] * X[0] / X[2] + k[2];
    v = k[1] * X[1] / X[2] + k[3];
}

int oracle_frustum(const RigF *rig, const PoseF *pose, const float *pos, const float *normal, const float *min_d,
                   const float *max_d, int M, float cos_limit, float *proj_x, float *proj_y, float *view_cos,
                   int32_t *level, uint8_t *in_view, float *track_depth) {
    const int C = rig->n_cams;
    float Rc[8][9], tc[8][3], twc[8][3];
    for (int c = 0; c < C; ++c) {
        if (c == 0) {
            std::memcpy(Rc[0], pose->Rcw, 36), std::memcpy(tc[0], pose->tcw, 12), std::memcpy(twc[0], pose->Ow, 12);
            continue;
        }
        mat3f(rig->R_cl[c], pose->Rcw, Rc[c]);         // mR = Rrl * mRcw
        float t[3];
        matvec3f(rig->R_cl[c], pose->tcw, t);          // mt = Rrl * mtcw + trl
        for (int i = 0; i < 3; ++i) tc[c][i] = t[i] + rig->t_cl[c][i];
        matvec3f(pose->Rwc, rig->t_lc[c], t);          // twc = mRwc * mTlr.translation() + mOw
        for (int i = 0; i < 3; ++i) twc[c][i] = t[i] + pose->Ow[i];
    }
    int n_any = 0;
    for (int i = 0; i < M; ++i) {
        const float *P = pos + 3 * i, *Pn = normal + 3 * i;
        bool any = false;
        for (int c = 0; c < C; ++c) {   // isInFrustum resets the projections and levels first
            proj_x[i * C + c] = -1, proj_y[i * C + c] = -1, level[i * C + c] = -1, in_view[i * C + c] = 0;
        }
        for (int c = 0; c < C; ++c) {
            float Pc[3];
            matvec3f(Rc[c], P, Pc);
            for (int q = 0; q < 3; ++q) Pc[q] = Pc[q] + tc[c][q];
            const float Pc_dist = std::sqrt(Pc[0] * Pc[0] + Pc[1] * Pc[1] + Pc[2] * Pc[2]);
            if (Pc[2] < 0.0f) continue;
            float u, v;   // mpCamera{,2,3,4}->project(Pc) (Frame.cc:1577-1592)
            if (rig->model[c] == 1) pinhole_project_f(rig->cam[c], Pc, u, v);
            else kb8_project_f(rig->cam[c], Pc, u, v);
            if (u < rig->min_x || u > rig->max_x) continue;
            if (v < rig->min_y || v > rig->max_y) continue;
            const float maxD = 1.2f * max_d[i], minD = 0.8f * min_d[i];
            const float PO[3] = {P[0] - twc[c][0], P[1] - twc[c][1], P[2] - twc[c][2]};
            const float dist = std::sqrt(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
            if (dist < minD || dist > maxD) continue;
            const float vc = (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) / dist;
            if (vc < cos_limit) continue;
            const float ratio = max_d[i] / dist;   // PredictScale
            int ns = (int)std::ceil(std::log((double)ratio) / (double)rig->log_scale_factor);
            if (ns < 0) ns = 0;
            else if (ns >= rig->n_levels) ns = rig->n_levels - 1;
            proj_x[i * C + c] = u, proj_y[i * C + c] = v, level[i * C + c] = ns, view_cos[i * C + c] = vc;
            in_view[i * C + c] = 1;
            if (c == 0) track_depth[i] = Pc_dist;
            any = true;
        }
        n_any += any;
    }
    return n_any;
}

}  // extern "C"

// ---- Keyframe-side projection searches -------------------------------------------------------------------
//   ORBmatcher::Fuse(KF, vpMapPoints, th, cameraID)                    src/ORBmatcher.cc:1458-1647
//   ORBmatcher::Fuse(KF, Scw, vpPoints, th, vpReplacePoint)            src/ORBmatcher.cc:1649-1769
//   ORBmatcher::SearchByProjection(KF, Siw, vpPoints, vpMatched, ...)  src/ORBmatcher.cc:668-776, 778-893
//   ORBmatcher::SearchByProjection(Frame&, KF, sAlreadyFound, th, ORBdist)  src/ORBmatcher.cc:2415-2535
//   KeyFrame::GetFeaturesInArea / IsInImage                            src/KeyFrame.cc:771-838
//   MapPoint::Get{Min,Max}DistanceInvariance / PredictScale(KF)       src/MapPoint.cc:598-622
// Each job is the reference's loop over its map points, literally; the map mutations the reference makes
// after a Fuse decision (Replace / AddObservation) are the caller's, so Fuse reports the decision per point.
#include "../include/omv.h"

extern "C" {

int oracle_search_kf(const FrameGeom *g, const KP *kps, const uint8_t *desc, int kp_cap, const int *n_kp, int n_kf,
                     int n_jobs, const omv_kf_search_job *jobs, const int32_t *mp_list, const float *pos,
                     const float *normal, const float *min_d, const float *max_d, const uint8_t *mp_desc,
                     const omv_kf_search_params *p, int32_t *kp_match, int32_t *best_idx, int32_t *best_dist,
                     int32_t *n_matches) {
    const int C = g->n_cams;
    const int mode = p->mode;
    const bool claim = mode == OMV_KF_SBP_SIM3 || mode == OMV_KF_SBP_FRAME;
    std::vector<View> views(n_kf);
    std::vector<bool> built(n_kf, false);
    const int HISTO_LENGTH = 30;
    const float factor = 1.0f / HISTO_LENGTH;
    for (int j = 0; j < n_jobs; ++j) {
        const omv_kf_search_job &J = jobs[j];
        const int kf = J.kf, cam = J.cam;
        if (!built[kf]) {
            views[kf] = View{g, 0, 0, {}, kps + (size_t)kf * C * kp_cap, kp_cap, n_kp + (size_t)kf * C};
            build_grids(views[kf]);
            built[kf] = true;
        }
        const View &v = views[kf];
        int32_t *claims = claim ? kp_match + (size_t)kf * C * kp_cap : nullptr;
        const KP *kk = kps + (size_t)kf * C * kp_cap;
        const uint8_t *dd = desc + (size_t)kf * C * kp_cap * 32;
        int off = 0;   // the keyframe's N-index of the block's first keypoint
        for (int c = 0; c < cam; ++c) off += n_kp[(size_t)kf * C + c];
        SE3F T;
        std::memcpy(T.q, J.Tcw.q, 16), std::memcpy(T.t, J.Tcw.t, 12);
        std::vector<std::vector<int>> rotHist(HISTO_LENGTH);
        int nm = 0;
        for (int e = J.mp_start; e < J.mp_start + J.mp_count; ++e) {
            best_idx[e] = -1, best_dist[e] = -1;
            const int mp = mp_list[e];
            const float *P = pos + 3 * (size_t)mp, *Pn = normal + 3 * (size_t)mp;
            float Pc[3];
            se3_apply(T, P, Pc);
            if (mode != OMV_KF_SBP_FRAME && Pc[2] < 0.0f) continue;   // depth must be positive
            float u, vv;
            cam_project_f(g->cam_model[cam], p->cams[cam], Pc, u, vv);   // pCamera / GetCamera(camId) (:1536, :1710)
            if (mode == OMV_KF_SBP_FRAME) {   // CurrentFrame.mnMinX .. mnMaxX, inclusive (:2445-2448)
                if (u < g->min_x || u > g->max_x) continue;
                if (vv < g->min_y || vv > g->max_y) continue;
            } else if (!(u >= g->min_x && u < g->max_x && vv >= g->min_y && vv < g->max_y)) {   // IsInImage
                continue;
            }
            const float invz = 1 / Pc[2];
            const float ur = u - p->bf * invz;
            const float maxDistance = 1.2f * max_d[mp], minDistance = 0.8f * min_d[mp];
            const float PO[3] = {P[0] - J.Ow[0], P[1] - J.Ow[1], P[2] - J.Ow[2]};
            const float dist3D = std::sqrt(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
            if (mode != OMV_KF_FUSE_SIM3 && (dist3D < minDistance || dist3D > maxDistance)) continue;
            if ((mode == OMV_KF_FUSE || mode == OMV_KF_SBP_SIM3) &&
                PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2] < 0.5 * dist3D)   // viewing angle < 60 deg
                continue;
            int pred = (int)std::ceil(std::log((double)(max_d[mp] / dist3D)) / (double)p->log_scale_factor);
            if (pred < 0) pred = 0;
            else if (pred >= p->n_levels) pred = p->n_levels - 1;
            const float radius = p->th * g->scale_factors[pred];
            const std::vector<int> win = mode == OMV_KF_SBP_FRAME
                                             ? features_in_area(v, u, vv, radius, pred - 1, pred + 1, cam)
                                             : features_in_area(v, u, vv, radius, 0, -1, cam);   // KeyFrame version
            if (win.empty()) continue;
            const uint8_t *dmp = mp_desc + (size_t)mp * 32;
            int bestDist = mode == OMV_KF_FUSE_SIM3 ? INT32_MAX : 256, bestIdx = -1;
            for (int i : win) {
                const int slot = cam * kp_cap + i;
                if (claim && claims[slot] >= 0) continue;   // vpMatched[idx] / CurrentFrame.mvpMapPoints[i2]
                const KP &kp = kk[slot];
                if (mode != OMV_KF_SBP_FRAME && (kp.octave < pred - 1 || kp.octave > pred)) continue;
                if (mode == OMV_KF_FUSE) {   // reprojection gate (:1594-1615)
                    const float ex = u - kp.x, ey = vv - kp.y;
                    if (cam == 0 && p->uright[(size_t)kf * kp_cap + i] >= 0) {
                        const float er = ur - p->uright[(size_t)kf * kp_cap + i];
                        const float e2 = ex * ex + ey * ey + er * er;
                        if (e2 * p->inv_level_sigma2[kp.octave] > 7.8) continue;
                    } else {
                        const float e2 = ex * ex + ey * ey;
                        if (e2 * p->inv_level_sigma2[kp.octave] > 5.99) continue;
                    }
                }
                const int d = descriptor_distance(dmp, dd + (size_t)slot * 32);
                if (d < bestDist) bestDist = d, bestIdx = i;
            }
            // bestIdx >= 0: with the reference's thresholds (< 256) an empty scan is never accepted
            const bool ok = bestIdx >= 0 && (float)bestDist <= p->max_dist;
            if (!claim) {
                if (bestIdx >= 0) best_idx[e] = off + bestIdx, best_dist[e] = bestDist;
                if (ok) ++nm;
                continue;
            }
            if (!ok) continue;
            const int slot = cam * kp_cap + bestIdx;
            claims[slot] = mp;
            best_idx[e] = off + bestIdx, best_dist[e] = bestDist;
            ++nm;
            if (mode == OMV_KF_SBP_FRAME && p->check_ori) {
                float rot = p->mp_angle[e] - kk[slot].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(e);
            }
        }
        if (mode == OMV_KF_SBP_FRAME && p->check_ori) {   // ComputeThreeMaxima (:2537-2573) + removal
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO_LENGTH; i++) {
                const int sz = (int)rotHist[i].size();
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
            for (int i = 0; i < HISTO_LENGTH; i++)
                if (i != ind1 && i != ind2 && i != ind3)
                    for (int e : rotHist[i]) {
                        claims[cam * kp_cap + (best_idx[e] - off)] = -1;
                        best_idx[e] = -1, best_dist[e] = -1;
                        --nm;
                    }
        }
        n_matches[j] = nm;
    }
    return 0;
}

// ---- ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, S12, th)            src/ORBmatcher.cc:1771-1983
// Sophus Sim3f * p = RxSO3 * p + t (sim3.hpp:226-229) with RxSO3 * p = s p + (w 2(v x p) + v x 2(v x p))
// (rxso3.hpp:265-272, s = the caller's S.scale()).  Side lists: the keypoints whose map point the reference
// projects (mapped, not vbAlreadyMatched, not bad), in index order; vnMatch1 / vnMatch2 are the reference's
// per-keypoint arrays.
static void sim3_apply(const omv_sim3f &S, const float *p, float *r) {
    float two[3], c[3];
    cross3f(S.q, p, two);
    for (int i = 0; i < 3; ++i) two[i] = two[i] + two[i];
    cross3f(S.q, two, c);
    for (int i = 0; i < 3; ++i) r[i] = (S.scale * p[i] + (S.q[3] * two[i] + c[i])) + S.t[i];
}

int oracle_search_by_sim3(const FrameGeom *g, const KP *kps, const uint8_t *desc, int kp_cap, const int *n_kp,
                          int n_kf, int n_jobs, const omv_sim3_job *jobs, const int32_t *kp1, const int32_t *mp1,
                          const int32_t *kp2, const int32_t *mp2, const float *pos, const float *min_d,
                          const float *max_d, const uint8_t *mp_desc, float th, float log_scale_factor, int n_levels,
                          int32_t *match12, int32_t *n_found) {
    const int C = g->n_cams;
    std::vector<View> views(n_kf);
    for (int kf = 0; kf < n_kf; ++kf) {
        views[kf] = View{g, 0, 0, {}, kps + (size_t)kf * C * kp_cap, kp_cap, n_kp + (size_t)kf * C};
        build_grids(views[kf]);
    }
    const int N = C * kp_cap;   // N-index bound (GetMapPointMatches().size() <= N)
    for (int j = 0; j < n_jobs; ++j) {
        const omv_sim3_job &J = jobs[j];
        // one direction: the points of a side projected through T then S into keyframe `tgt`
        auto pass = [&](const int32_t *kpl, const int32_t *mpl, int start, int count, const omv_se3f &Tw,
                        const omv_sim3f &S, int tgt, std::vector<int> &vnMatch) {
            SE3F T;
            std::memcpy(T.q, Tw.q, 16), std::memcpy(T.t, Tw.t, 12);
            const View &v = views[tgt];
            const KP *kk = kps + (size_t)tgt * C * kp_cap;
            const uint8_t *dd = desc + (size_t)tgt * C * kp_cap * 32;
            for (int e = start; e < start + count; ++e) {
                const int mp = mpl[e];
                const float *P = pos + 3 * (size_t)mp;
                float p3Dc1[3], p3Dc2[3];
                se3_apply(T, P, p3Dc1);
                sim3_apply(S, p3Dc1, p3Dc2);
                if (p3Dc2[2] < 0.0) continue;   // depth must be positive
                const float invz = 1.0 / p3Dc2[2];
                const float x = p3Dc2[0] * invz;
                const float y = p3Dc2[1] * invz;
                const float u = J.fx * x + J.cx;
                const float vv = J.fy * y + J.cy;
                if (!(u >= g->min_x && u < g->max_x && vv >= g->min_y && vv < g->max_y)) continue;   // IsInImage
                const float maxDistance = 1.2f * max_d[mp], minDistance = 0.8f * min_d[mp];
                const float dist3D = std::sqrt(p3Dc2[0] * p3Dc2[0] + p3Dc2[1] * p3Dc2[1] + p3Dc2[2] * p3Dc2[2]);
                if (dist3D < minDistance || dist3D > maxDistance) continue;
                int pred = (int)std::ceil(std::log((double)(max_d[mp] / dist3D)) / (double)log_scale_factor);
                if (pred < 0) pred = 0;
                else if (pred >= n_levels) pred = n_levels - 1;
                const float radius = th * g->scale_factors[pred];
                const std::vector<int> win = features_in_area(v, u, vv, radius, 0, -1, 0);   // KeyFrame version
                if (win.empty()) continue;
                const uint8_t *dMP = mp_desc + (size_t)mp * 32;
                int bestDist = INT32_MAX, bestIdx = -1;
                for (int idx : win) {
                    const KP &kp = kk[idx];
                    if (kp.octave < pred - 1 || kp.octave > pred) continue;
                    const int dist = descriptor_distance(dMP, dd + (size_t)idx * 32);
                    if (dist < bestDist) bestDist = dist, bestIdx = idx;
                }
                if (bestDist <= TH_HIGH) vnMatch[kpl[e]] = bestIdx;
            }
        };
        std::vector<int> vnMatch1(N, -1), vnMatch2(N, -1);
        pass(kp1, mp1, J.start1, J.count1, J.T1w, J.S21, J.kf2, vnMatch1);
        pass(kp2, mp2, J.start2, J.count2, J.T2w, J.S12, J.kf1, vnMatch2);
        int nFound = 0;   // check agreement
        for (int e = J.start1; e < J.start1 + J.count1; ++e) {
            const int i1 = kp1[e];
            const int idx2 = vnMatch1[i1];
            match12[e] = -1;
            if (idx2 >= 0 && vnMatch2[idx2] == i1) {
                match12[e] = idx2;
                nFound++;
            }
        }
        n_found[j] = nFound;
    }
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------
// ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
//                                                    src/ORBmatcher.cc:895-1004 (+ ComputeThreeMaxima :2537-2573)
// Single-camera frames (F.Nleft == -1): GetFeaturesInArea on F2's mGrid of mvKeysUn with levels [0, 0].
// The rotation histogram keeps every push, including F1 keypoints whose F2 keypoint a later, better F1
// keypoint took over (their removal then finds vnMatches12 < 0 and changes nothing), as the reference.
namespace {
const int TH_LOW_INIT = 50, HISTO_INIT = 30;
void three_maxima_init(const int *cnt, int &ind1, int &ind2, int &ind3) {   // ComputeThreeMaxima
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_INIT; i++) {
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
}
}  // namespace

extern "C" {

// F1: n1 keypoints / descriptors; F2: n2 keypoints / descriptors with geometry g (n_cams ignored: one block);
// prev [n1][2] in/out (vbPrevMatched); m12 [n1] out.  Returns nmatches.
int oracle_search_for_initialization(const FrameGeom *g, const KP *kps1, const uint8_t *desc1, int n1, const KP *kps2,
                                     const uint8_t *desc2, int n2, float *prev, int window, float nnratio,
                                     int check_ori, int32_t *m12) {
    FrameGeom g1 = *g;
    g1.n_cams = 1;
    View v{&g1, 0, 0, {}, kps2, n2, &n2};
    build_grids(v);
    int nmatches = 0;
    for (int i = 0; i < n1; ++i) m12[i] = -1;
    std::vector<int> rotHist[HISTO_INIT];
    const float factor = 1.0f / HISTO_INIT;
    std::vector<int> vMatchedDistance(n2, INT32_MAX), vnMatches21(n2, -1);
    for (int i1 = 0; i1 < n1; i1++) {
        const KP kp1 = kps1[i1];
        const int level1 = kp1.octave;
        if (level1 > 0) continue;
        const std::vector<int> vIndices2 =
            features_in_area(v, prev[2 * i1], prev[2 * i1 + 1], (float)window, level1, level1, 0);
        if (vIndices2.empty()) continue;
        const uint8_t *d1 = desc1 + 32 * (size_t)i1;
        int bestDist = INT32_MAX, bestDist2 = INT32_MAX, bestIdx2 = -1;
        for (int i2 : vIndices2) {
            const int dist = descriptor_distance(d1, desc2 + 32 * (size_t)i2);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW_INIT) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    m12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                m12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (check_ori) {
                    float rot = kps1[i1].angle - kps2[bestIdx2].angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)std::round(rot * factor);
                    if (bin == HISTO_INIT) bin = 0;
                    rotHist[bin].push_back(i1);
                }
            }
        }
    }
    if (check_ori) {
        int cnt[HISTO_INIT], ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < HISTO_INIT; ++i) cnt[i] = (int)rotHist[i].size();
        three_maxima_init(cnt, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_INIT; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx1 : rotHist[i])
                if (m12[idx1] >= 0) {
                    m12[idx1] = -1;
                    nmatches--;
                }
        }
    }
    for (int i1 = 0; i1 < n1; i1++)
        if (m12[i1] >= 0) prev[2 * i1] = kps2[m12[i1]].x, prev[2 * i1 + 1] = kps2[m12[i1]].y;
    return nmatches;
}

}  // extern "C"

// ---- LocalMapping::SearchInNeighbors' fuse sequence                     src/LocalMapping.cc:837-889
//   ORBmatcher::Fuse(pKF, vpMapPoints, th, cameraID)                       src/ORBmatcher.cc:1458-1647
//   MapPoint::AddObservation / Replace / ComputeDistinctiveDescriptors    src/MapPoint.cc:199-226, :316-380, :405-483
//   KeyFrame::AddMapPoint / ReplaceMapPointMatch / EraseMapPointMatch / GetMapPoint (mvpMapPoints[idx])
// Written literally: every decision reads the map as the previous decisions left it, every window search runs when the
// loop reaches the point (with its descriptor of that moment).  mObservations is a std::map keyed by KeyFrame*: keyed
// here by keyframe index (the adapter numbers keyframes in pointer order).  No mnFuseTargetForKF / covisibility: the
// target list is the caller's; phase C (:891-900) is not part of this restatement.
extern "C" void oracle_distinctive_descriptors(int n_points, const int32_t *desc_start, const int32_t *desc_row,
                                               const uint8_t *desc, int32_t *best_row);
namespace {
struct FuseMap {
    const FrameGeom *g;
    const KP *kps;
    const uint8_t *desc;
    const int *n_kp;
    int kp_cap, C;
    omv_fuse_graph *G;
    const float *pos, *normal, *min_d, *max_d;
    uint8_t *mp_desc;
    const omv_kf_search_params *p;
    std::vector<View> views;
    std::vector<std::map<int, std::array<int, 4>>> obs;
    int n_log = 0;

    int N(int kf) const {
        int n = 0;
        for (int c = 0; c < C; ++c) n += n_kp[(size_t)kf * C + c];
        return n;
    }
    int *mvp(int kf) { return G->kf_mps + (size_t)kf * C * kp_cap; }
    const uint8_t *row_desc(int kf, int idx) const {   // pKF->mDescriptors.row(idx)
        int c = 0, off = 0;
        while (c + 1 < C && idx >= off + n_kp[(size_t)kf * C + c]) off += n_kp[(size_t)kf * C + c], ++c;
        return desc + (((size_t)kf * C + c) * kp_cap + (idx - off)) * 32;
    }
    void log(int a, int b, int c, int d) {
        if (n_log < G->log_cap) {
            int32_t *r = G->log + 4 * (size_t)n_log;
            r[0] = a, r[1] = b, r[2] = c, r[3] = d;
        }
        ++n_log;
    }
    bool IsInKeyFrame(int mp, int kf) const { return obs[mp].count(kf) > 0; }
    void AddObservation(int mp, int kf, int idx) {
        std::array<int, 4> indexes = {-1, -1, -1, -1};
        if (obs[mp].count(kf)) indexes = obs[mp][kf];
        const int NLeft = G->n_blocks[kf] == 1 ? -1 : n_kp[(size_t)kf * C];
        const int NRight = C > 1 ? n_kp[(size_t)kf * C + 1] : 0, NSideLeft = C > 2 ? n_kp[(size_t)kf * C + 2] : 0;
        if (NLeft == -1) indexes[0] = idx;
        else if (idx < NLeft) indexes[0] = idx;
        else if (idx >= NLeft && idx < NLeft + NRight) indexes[1] = idx;
        else if (idx >= NLeft + NRight && idx < NLeft + NRight + NSideLeft) indexes[2] = idx;
        else indexes[3] = idx;
        obs[mp][kf] = indexes;
        if (NLeft == -1 && G->uright && G->uright[(size_t)kf * kp_cap + idx] >= 0) G->n_obs[mp] += 2;   // !mpCamera2
        else G->n_obs[mp]++;
    }
    void ComputeDistinctiveDescriptors(int mp) {
        if (G->bad[mp]) return;
        if (obs[mp].empty()) return;
        std::vector<int32_t> rows;
        std::vector<uint8_t> stack;
        for (auto &kv : obs[mp])
            for (int s = 0; s < 4; ++s)
                if (kv.second[s] != -1) {
                    const uint8_t *d = row_desc(kv.first, kv.second[s]);
                    stack.insert(stack.end(), d, d + 32);
                }
        if (stack.empty()) return;
        const int n = (int)(stack.size() / 32);
        for (int i = 0; i < n; ++i) rows.push_back(i);
        const int32_t start[2] = {0, n};
        int32_t best = -1;
        oracle_distinctive_descriptors(1, start, rows.data(), stack.data(), &best);
        std::memcpy(mp_desc + (size_t)mp * 32, stack.data() + (size_t)best * 32, 32);
    }
    void Replace(int self, int pMP) {
        log(1, self, pMP, -1);
        if (pMP == self) return;
        std::map<int, std::array<int, 4>> o = obs[self];
        obs[self].clear();
        G->bad[self] = 1;
        G->replaced[self] = pMP;
        for (auto &kv : o) {
            const int pKF = kv.first;
            if (!IsInKeyFrame(pMP, pKF)) {
                for (int s = 0; s < 4; ++s)
                    if (kv.second[s] != -1) {
                        mvp(pKF)[kv.second[s]] = pMP;   // ReplaceMapPointMatch
                        AddObservation(pMP, pKF, kv.second[s]);
                    }
            } else {
                for (int s = 0; s < 4; ++s)
                    if (kv.second[s] != -1) mvp(pKF)[kv.second[s]] = -1;   // EraseMapPointMatch
            }
        }
        ComputeDistinctiveDescriptors(pMP);
    }
    // ORBmatcher::Fuse(pKF, vpMapPoints, th, cameraID)
    int Fuse(int pKF, const std::vector<int> &vpMapPoints, int cameraID) {
        if (views[pKF].g == nullptr) {
            views[pKF] = View{g, 0, 0, {}, kps + (size_t)pKF * C * kp_cap, kp_cap, n_kp + (size_t)pKF * C};
            build_grids(views[pKF]);
        }
        const View &v = views[pKF];
        SE3F Tcw;
        std::memcpy(Tcw.q, G->Tcw[(size_t)pKF * C + cameraID].q, 16);
        std::memcpy(Tcw.t, G->Tcw[(size_t)pKF * C + cameraID].t, 12);
        const float *Ow = G->Ow + ((size_t)pKF * C + cameraID) * 3;
        const KP *kk = kps + (size_t)pKF * C * kp_cap;
        int off = 0;
        for (int c = 0; c < cameraID; ++c) off += n_kp[(size_t)pKF * C + c];
        int nFused = 0;
        for (int pMP : vpMapPoints) {
            if (pMP < 0) continue;
            if (G->bad[pMP]) continue;
            else if (IsInKeyFrame(pMP, pKF)) continue;
            const float *P = pos + 3 * (size_t)pMP, *Pn = normal + 3 * (size_t)pMP;
            float Pc[3];
            se3_apply(Tcw, P, Pc);
            if (Pc[2] < 0.0f) continue;
            const float invz = 1 / Pc[2];
            float u, vv;
            cam_project_f(g->cam_model[cameraID], p->cams[cameraID], Pc, u, vv);
            if (!(u >= g->min_x && u < g->max_x && vv >= g->min_y && vv < g->max_y)) continue;   // IsInImage
            const float ur = u - p->bf * invz;
            const float maxDistance = 1.2f * max_d[pMP], minDistance = 0.8f * min_d[pMP];
            const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
            const float dist3D = std::sqrt(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
            if (dist3D < minDistance || dist3D > maxDistance) continue;
            if (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2] < 0.5 * dist3D) continue;
            int nPredictedLevel = (int)std::ceil(std::log((double)(max_d[pMP] / dist3D)) / (double)p->log_scale_factor);
            if (nPredictedLevel < 0) nPredictedLevel = 0;
            else if (nPredictedLevel >= p->n_levels) nPredictedLevel = p->n_levels - 1;
            const float radius = p->th * g->scale_factors[nPredictedLevel];
            const std::vector<int> vIndices = features_in_area(v, u, vv, radius, 0, -1, cameraID);
            if (vIndices.empty()) continue;
            const uint8_t *dMP = mp_desc + (size_t)pMP * 32;
            int bestDist = 256, bestIdx = -1;
            for (int i : vIndices) {
                const int slot = cameraID * kp_cap + i;
                const KP &kp = kk[slot];
                const int kpLevel = kp.octave;
                if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
                const float ex = u - kp.x, ey = vv - kp.y;
                if (cameraID == 0 && p->uright[(size_t)pKF * kp_cap + i] >= 0) {
                    const float er = ur - p->uright[(size_t)pKF * kp_cap + i];
                    const float e2 = ex * ex + ey * ey + er * er;
                    if (e2 * p->inv_level_sigma2[kpLevel] > 7.8) continue;
                } else {
                    const float e2 = ex * ex + ey * ey;
                    if (e2 * p->inv_level_sigma2[kpLevel] > 5.99) continue;
                }
                const int dist = descriptor_distance(dMP, desc + ((size_t)pKF * C * kp_cap + slot) * 32);
                if (dist < bestDist) bestDist = dist, bestIdx = off + i;
            }
            if (bestDist <= 50) {   // TH_LOW
                const int pMPinKF = mvp(pKF)[bestIdx];
                if (pMPinKF >= 0) {
                    if (!G->bad[pMPinKF]) {
                        if (G->n_obs[pMPinKF] > G->n_obs[pMP]) Replace(pMP, pMPinKF);
                        else Replace(pMPinKF, pMP);
                    }
                } else {
                    log(0, pMP, pKF, bestIdx);
                    AddObservation(pMP, pKF, bestIdx);
                    mvp(pKF)[bestIdx] = pMP;   // pKF->AddMapPoint(pMP, bestIdx)
                }
                nFused++;
            }
        }
        return nFused;
    }
};
}  // namespace

extern "C" int oracle_search_in_neighbors_fuse(const FrameGeom *g, const KP *kps, const uint8_t *desc, const int *n_kp,
                                               int kp_cap, omv_fuse_graph *G, int current, int n_targets,
                                               const int32_t *targets, const float *pos, const float *normal,
                                               const float *min_d, const float *max_d, uint8_t *mp_desc,
                                               const omv_kf_search_params *p, int32_t *n_fused) {
    const int C = g->n_cams;
    FuseMap M{g, kps, desc, n_kp, kp_cap, C, G, pos, normal, min_d, max_d, mp_desc, p, {}, {}, 0};
    M.views.assign(G->n_kf, View{});
    for (auto &v : M.views) v.g = nullptr;
    M.obs.resize(G->n_mps);
    for (int mp = 0; mp < G->n_mps; ++mp) {
        G->replaced[mp] = -1;
        for (int r = G->obs_start[mp]; r < G->obs_start[mp + 1]; ++r)
            M.obs[mp][G->obs_kf[r]] = {G->obs_idx[4 * r], G->obs_idx[4 * r + 1], G->obs_idx[4 * r + 2], G->obs_idx[4 * r + 3]};
    }
    for (int t = 0; t < n_targets * C + C; ++t) n_fused[t] = 0;
    // vector<MapPoint*> vpMapPointMatches = mpCurrentKeyFrame->GetMapPointMatches();  (:839)
    const std::vector<int> vpMapPointMatches(M.mvp(current), M.mvp(current) + M.N(current));
    for (int t = 0; t < n_targets; ++t) {   // (:840-853)
        const int pKFi = targets[t];
        n_fused[t * C + 0] = M.Fuse(pKFi, vpMapPointMatches, 0);
        if (G->n_blocks[pKFi] >= 2) n_fused[t * C + 1] = M.Fuse(pKFi, vpMapPointMatches, 1);
        if (G->n_blocks[pKFi] == 4) {
            n_fused[t * C + 2] = M.Fuse(pKFi, vpMapPointMatches, 2);
            n_fused[t * C + 3] = M.Fuse(pKFi, vpMapPointMatches, 3);
        }
    }
    // vpFuseCandidates (:859-881)
    std::vector<int> vpFuseCandidates;
    std::vector<char> cand(G->n_mps, 0);   // mnFuseCandidateForKF
    for (int t = 0; t < n_targets; ++t) {
        const int pKFi = targets[t];
        for (int i = 0; i < M.N(pKFi); ++i) {
            const int pMP = M.mvp(pKFi)[i];
            if (pMP < 0) continue;
            if (G->bad[pMP] || cand[pMP]) continue;
            cand[pMP] = 1;
            vpFuseCandidates.push_back(pMP);
        }
    }
    n_fused[n_targets * C + 0] = M.Fuse(current, vpFuseCandidates, 0);   // (:883-889)
    if (G->n_blocks[current] >= 2) n_fused[n_targets * C + 1] = M.Fuse(current, vpFuseCandidates, 1);
    if (G->n_blocks[current] == 4) {
        n_fused[n_targets * C + 2] = M.Fuse(current, vpFuseCandidates, 2);
        n_fused[n_targets * C + 3] = M.Fuse(current, vpFuseCandidates, 3);
    }
    int rows = 0;
    for (int mp = 0; mp < G->n_mps; ++mp) {
        G->out_obs_start[mp] = rows;
        for (auto &kv : M.obs[mp]) {
            if (rows < G->obs_cap) {
                G->out_obs_kf[rows] = kv.first;
                for (int s = 0; s < 4; ++s) G->out_obs_idx[4 * (size_t)rows + s] = kv.second[s];
            }
            ++rows;
        }
    }
    G->out_obs_start[G->n_mps] = rows;
    G->n_log = M.n_log;
    return (M.n_log > G->log_cap || rows > G->obs_cap) ? 1 : 0;
}
