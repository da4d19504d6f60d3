// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for ORBmatcher::SearchByBoW. Never linked into the product.
//
// Scalar restatement of
//   ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F, vector<MapPoint*> &vpMapPointMatches)
//                                                    src/ORBmatcher.cc:349-666 (+ ComputeThreeMaxima :2537-2573)
//   ORBmatcher::SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, vector<MapPoint*> &vpMatches12)
//                                                    src/ORBmatcher.cc:1006-1129
//   ORBmatcher::DescriptorDistance                   src/ORBmatcher.cc:2577-2591
// The DBoW2 FeatureVector walk (std::map iterators advanced together on equal node ids, lower_bound on the
// smaller side) visits exactly the node ids both vectors hold, ascending: restated as that merge.
// Kept from the reference literally:
//   - (KF, F): the right / side blocks are only searched when the left block's best passes TH_LOW (they sit
//     inside `if (bestDist1 <= TH_LOW)`), and their ratio test is `... || true` (always passes); a frame
//     keypoint matched earlier in the call is skipped (vpMapPointMatches[realIdxF] != NULL); F.Nleft == -1
//     (single-camera frame) searches one block;
//   - (KF1, KF2): acceptance at bestDist1 < TH_LOW (strict), vbMatched2 claims, the `idx >= N` skips;
//   - the rotation histogram's 13 effective bins (round(rot / 30)), ComputeThreeMaxima's 10 % rule, and the
//     removal of every match pushed outside the three top bins.
// The MapPoint pointers become keypoint indices: (KF, F) reports per frame keypoint the keyframe keypoint
// whose point it received (vpMapPointMatches[i] = vpMapPointsKF[match[i]]); (KF1, KF2) per pKF1 keypoint the
// pKF2 keypoint (vpMatches12[i] = vpMapPoints2[match[i]]).  has_mp = (GetMapPoint(idx) && !isBad()).
// Parity status: no reference test pins these functions; the device path is bit-exact to THIS
// restatement.
// =====================================================================================================
#include <cmath>
#include <cstdint>
#include <vector>

#include "../include/omv.h"

namespace {

const int TH_LOW = 50;
const int HISTO_LENGTH = 30;

int hamming(const uint8_t *a, const uint8_t *b) {
    int d = 0;
    for (int k = 0; k < 32; ++k) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
    return d;
}

// ComputeThreeMaxima (ORBmatcher.cc:2537-2573)
void three_maxima(const int *cnt, int &ind1, int &ind2, int &ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
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

int rot_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// best / second of one block, the reference's update order
struct Best {
    int d1 = 256, idx = -1, d2 = 256;
    void add(int dist, int i) {
        if (dist < d1) {
            d2 = d1, d1 = dist, idx = i;
        } else if (dist < d2) {
            d2 = dist;
        }
    }
};

void remove_outside_top3(const std::vector<int> *hist, int32_t *match, int &nmatches) {
    int cnt[HISTO_LENGTH], ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < HISTO_LENGTH; ++i) cnt[i] = (int)hist[i].size();
    three_maxima(cnt, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (int idx : hist[i]) match[idx] = -1, nmatches--;
    }
}

}  // namespace

extern "C" {

// One job (host pointers in the views); mode OMV_BOW_KF_FRAME or OMV_BOW_KF_KF.  Writes job->match and returns
// the reference's nmatches.
int oracle_search_by_bow(const omv_bow_job *J, int mode, float nnratio, int check_ori) {
    const omv_kf_view &K = J->kf, &O = J->other;
    std::vector<int> hist[HISTO_LENGTH];
    int nmatches = 0;
    const int n_out = mode == OMV_BOW_KF_FRAME ? O.n : K.n;
    for (int i = 0; i < n_out; ++i) J->match[i] = -1;
    std::vector<uint8_t> matched2(O.n, 0);   // (KF1, KF2): vbMatched2
    int a = 0, b = 0;
    while (a < K.n_nodes && b < O.n_nodes) {
        if (K.node_id[a] == O.node_id[b]) {
            for (int i1 = K.node_start[a]; i1 < K.node_start[a + 1]; ++i1) {
                const int idx1 = K.node_idx[i1];
                if (mode == OMV_BOW_KF_KF && K.n_left != -1 && idx1 >= K.n) continue;
                if (!K.has_mp[idx1]) continue;
                const uint8_t *d1 = K.desc + 32 * (size_t)idx1;
                if (mode == OMV_BOW_KF_FRAME) {
                    // blocks by the frame's ranges: L [0, Nleft), R [Nleft, +Nright), SL, SR
                    const int nl = O.n_left, nr = O.n_right, nsl = O.n_sideleft;
                    const bool sides = nsl >= 0;
                    Best B[4];
                    for (int i2 = O.node_start[b]; i2 < O.node_start[b + 1]; ++i2) {
                        const int idxF = O.node_idx[i2];
                        if (J->match[idxF] >= 0) continue;
                        const int dist = hamming(d1, O.desc + 32 * (size_t)idxF);
                        if (nl == -1) {
                            B[0].add(dist, idxF);
                        } else if (idxF < nl) {
                            B[0].add(dist, idxF);
                        } else if (idxF < nl + nr) {
                            B[1].add(dist, idxF);
                        } else if (sides && idxF < nl + nr + nsl) {
                            B[2].add(dist, idxF);
                        } else if (sides && idxF < O.n) {
                            B[3].add(dist, idxF);
                        }
                    }
                    if (B[0].d1 <= TH_LOW) {
                        for (int c = 0; c < 4; ++c) {
                            if (B[c].d1 > TH_LOW) continue;
                            // left: the nnratio test; right / side: `... || true`
                            if (c == 0 && !((float)B[0].d1 < nnratio * (float)B[0].d2)) continue;
                            J->match[B[c].idx] = idx1;
                            if (check_ori) hist[rot_bin(K.kps[idx1].angle, O.kps[B[c].idx].angle)].push_back(B[c].idx);
                            nmatches++;
                        }
                    }
                } else {
                    Best B;
                    for (int i2 = O.node_start[b]; i2 < O.node_start[b + 1]; ++i2) {
                        const int idx2 = O.node_idx[i2];
                        if (O.n_left != -1 && idx2 >= O.n) continue;
                        if (matched2[idx2] || !O.has_mp[idx2]) continue;
                        B.add(hamming(d1, O.desc + 32 * (size_t)idx2), idx2);
                    }
                    if (B.d1 < TH_LOW && (float)B.d1 < nnratio * (float)B.d2) {
                        J->match[idx1] = B.idx;
                        matched2[B.idx] = 1;
                        if (check_ori) hist[rot_bin(K.kps[idx1].angle, O.kps[B.idx].angle)].push_back(idx1);
                        nmatches++;
                    }
                }
            }
            ++a, ++b;
        } else if (K.node_id[a] < O.node_id[b]) {
            ++a;
        } else {
            ++b;
        }
    }
    if (check_ori) remove_outside_top3(hist, J->match, nmatches);
    return nmatches;
}

}  // extern "C"
