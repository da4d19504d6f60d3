// =====================================================================================================
// TEST INFRASTRUCTURE ONLY — CPU oracle for the DBoW2 vocabulary transform. Never linked into the product.
//
// Scalar restatement of DBoW2 (Thirdparty/DBoW2, vendored in the reference) as ORB-SLAM3 calls it from
// Frame::ComputeBoW / KeyFrame::ComputeBoW (src/KeyFrame.cc:207-214: transform(desc, mBowVec, mFeatVec, 4)):
//   TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)   TemplatedVocabulary.h:1127-1194
//   TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)          TemplatedVocabulary.h:1217-1259
//   FORB::distance                                                                   FORB.cpp:81-101
//   BowVector::addWeight / addIfNotExist / normalize                                 BowVector.cpp
//   FeatureVector::addFeature                                                        FeatureVector.cpp:31-45
//   ScoringObject mustNormalize (L1, L2, chi-square, KL, Bhattacharyya: yes; dot product: no)
// with std::map exactly as the reference uses it.  ORBvoc.txt is not in the container: parity is to this
// restatement on synthetic vocabularies ("parity unpinned" against the real vocabulary file).
// =====================================================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "../include/omv.h"

namespace {

int forb_distance(const uint8_t *a, const uint8_t *b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        unsigned int v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

// transform(feature, word_id, weight, nid, levelsup): the descent, first child wins distance ties.
void transform1(const omv_vocab *v, const uint8_t *f, int levelsup, int &word, double &weight, int &nid) {
    const int nid_level = v->L - levelsup;
    if (nid_level <= 0) nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int c0 = v->child_start[final_id], c1 = v->child_start[final_id + 1];
        final_id = v->child_ids[c0];
        double best_d = forb_distance(f, v->desc + 32 * (size_t)final_id);
        for (int c = c0 + 1; c < c1; ++c) {
            const int id = v->child_ids[c];
            const double d = forb_distance(f, v->desc + 32 * (size_t)id);
            if (d < best_d) best_d = d, final_id = id;
        }
        if (level == nid_level) nid = final_id;
    } while (v->child_start[final_id] != v->child_start[final_id + 1]);
    word = v->word_id[final_id];
    weight = v->weight[final_id];
}

}  // namespace

extern "C" {

// One descriptor set (a frame's / keyframe's N rows).  Per feature: word [N], wval [N], node [N] (the
// FeatureVector node; -1 if the descent never reached the FeatureVector level).  BowVector: bow_word /
// bow_value [*bow_n] ascending; FeatureVector: fv_node [*fv_n] ascending, fv_start [*fv_n + 1], fv_idx.
int oracle_bow_transform(const omv_vocab *v, const uint8_t *desc, int N, int levelsup, int32_t *word, double *wval,
                         int32_t *node, int32_t *bow_word, double *bow_value, int32_t *bow_n, int32_t *fv_node,
                         int32_t *fv_start, int32_t *fv_idx, int32_t *fv_n) {
    std::map<unsigned, double> bow;
    std::map<unsigned, std::vector<unsigned>> fv;
    if (v->n_words > 0) {
        const int sc = v->scoring;
        const bool must = sc != 5;            // DOT_PRODUCT does not normalise
        const bool l2 = sc == 1;              // L2_NORM normalises with L2, the others with L1
        const bool tf = v->weighting == 0 || v->weighting == 1;   // TF_IDF, TF: addWeight
        for (int i = 0; i < N; ++i) {
            int w, nid = -1;
            double wt;
            transform1(v, desc + 32 * (size_t)i, levelsup, w, wt, nid);
            word[i] = w, wval[i] = wt, node[i] = nid;
            if (!(wt > 0)) continue;   // stopped
            if (tf) {
                auto it = bow.lower_bound((unsigned)w);
                if (it != bow.end() && !(bow.key_comp()((unsigned)w, it->first))) it->second += wt;
                else bow.insert(it, {(unsigned)w, wt});
            } else {
                auto it = bow.lower_bound((unsigned)w);
                if (it == bow.end() || bow.key_comp()((unsigned)w, it->first)) bow.insert(it, {(unsigned)w, wt});
            }
            fv[(unsigned)nid].push_back((unsigned)i);
        }
        if (tf && !bow.empty() && !must) {
            const double nd = bow.size();
            for (auto &p : bow) p.second /= nd;
        }
        if (must) {
            double norm = 0.0;
            if (!l2) {
                for (auto &p : bow) norm += std::fabs(p.second);
            } else {
                for (auto &p : bow) norm += p.second * p.second;
                norm = std::sqrt(norm);
            }
            if (norm > 0.0)
                for (auto &p : bow) p.second /= norm;
        }
    } else {
        for (int i = 0; i < N; ++i) word[i] = -1, wval[i] = 0, node[i] = -1;
    }
    int k = 0;
    for (auto &p : bow) bow_word[k] = (int32_t)p.first, bow_value[k] = p.second, ++k;
    *bow_n = k;
    k = 0;
    int pos = 0;
    for (auto &p : fv) {
        fv_node[k] = (int32_t)p.first;
        fv_start[k] = pos;
        for (unsigned i : p.second) fv_idx[pos++] = (int32_t)i;
        ++k;
    }
    fv_start[k] = pos;
    *fv_n = k;
    return 0;
}

}  // extern "C"
