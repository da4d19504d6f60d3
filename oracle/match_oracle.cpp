// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for the Hamming matchers. Never linked into the product.
//
// Scalar restatement of
//   Frame::AssignFeaturesToGrid / PosInGrid         src/Frame.cc:541-582, :969-978
//   Frame::GetFeaturesInArea                         src/Frame.cc:890-967
//   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
//                                                    src/ORBmatcher.cc:23-340 (+ RadiusByViewingCos :342-347)
//   ORBmatcher::DescriptorDistance                   src/ORBmatcher.cc:2577-2591
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
#include <cmath>
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

struct FrameGeom {
    int n_cams;
    float min_x, max_x, min_y, max_y;
    int nlevels;
    float scale_factors[16];
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

}  // extern "C"
