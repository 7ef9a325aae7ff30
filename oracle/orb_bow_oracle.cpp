// ORACLE -- TEST INFRASTRUCTURE ONLY.  CPU restatement of DBoW2's TemplatedVocabulary::transform
// (reference Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1260) with the FORB distance
// (DBoW2/FORB.cpp:81-100), BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84),
// FeatureVector::addFeature (FeatureVector.cpp) and the ScoringObject normalisation rules
// (ScoringObject.h: L1/L2/ChiSquare/KL/Bhattacharyya normalise, DotProduct does not).  std::map
// holds the vectors, so iteration (and the L1/L2 sums) run in ascending id order exactly as DBoW2's.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "../include/orbgpu.h"

namespace {

int forb_distance(const uint8_t* a, const uint8_t* b) {  // FORB::distance (== DescriptorDistance)
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

// transform(feature, word_id, weight, nid, levelsup), TemplatedVocabulary.h:1213-1260.  The
// reference leaves *nid untouched when the leaf is reached above level L - levelsup (then read
// uninitialised by the caller); here it is the leaf.
void descend(const orb_vocabulary_view_t& V, const uint8_t* f, int levelsup, int& word, double& w, int& nid) {
    const int nid_level = V.L - levelsup;
    nid = -1;
    if (nid_level <= 0) nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int cb = V.child_begin[final_id], ce = V.child_begin[final_id + 1];
        final_id = V.child_idx[cb];
        double best_d = forb_distance(f, V.desc + 32 * (size_t)final_id);
        for (int c = cb + 1; c < ce; ++c) {
            const int id = V.child_idx[c];
            const double d = forb_distance(f, V.desc + 32 * (size_t)id);
            if (d < best_d) {
                best_d = d;
                final_id = id;
            }
        }
        if (level == nid_level) nid = final_id;
    } while (V.child_begin[final_id + 1] > V.child_begin[final_id] && level < 64);
    if (nid < 0) nid = final_id;
    word = V.word_id[final_id];
    w = V.weight[final_id];
}

}  // namespace

extern "C" int oracle_bow_transform(const orb_vocabulary_view_t* V, const uint8_t* desc, int n, int levelsup,
                                    int32_t* bow_word, double* bow_value, int32_t* n_words, int32_t* fv_node,
                                    int32_t* fv_begin, int32_t* fv_feat, int32_t* n_nodes) {
    std::map<int, double> v;
    std::map<int, std::vector<int>> fv;
    *n_words = *n_nodes = 0;
    if (V->n_nodes <= 1 || V->child_begin[1] <= V->child_begin[0]) {  // empty(): nothing
        fv_begin[0] = 0;
        return 0;
    }
    const bool must = V->scoring != 5;          // DotProductScoring does not normalise
    const bool l1 = V->scoring != 1;            // L2Scoring uses L2, the others L1
    const bool tf = V->weighting == 0 || V->weighting == 1;
    for (int i = 0; i < n; ++i) {
        int word, nid;
        double w;
        descend(*V, desc + 32 * (size_t)i, levelsup, word, w, nid);
        if (w > 0) {
            if (tf) {
                auto it = v.lower_bound(word);
                if (it != v.end() && !(word < it->first)) it->second += w;
                else v.insert(it, {word, w});
            } else {
                if (!v.count(word)) v[word] = w;
            }
            fv[nid].push_back(i);
        }
    }
    if (tf && !v.empty() && !must) {
        const double nd = v.size();
        for (auto& kv : v) kv.second /= nd;
    }
    if (must) {  // BowVector::normalize
        double norm = 0.0;
        if (l1) {
            for (auto& kv : v) norm += std::fabs(kv.second);
        } else {
            for (auto& kv : v) norm += kv.second * kv.second;
            norm = std::sqrt(norm);
        }
        if (norm > 0.0)
            for (auto& kv : v) kv.second /= norm;
    }
    int k = 0;
    for (auto& kv : v) {
        bow_word[k] = kv.first;
        bow_value[k] = kv.second;
        ++k;
    }
    *n_words = k;
    int m = 0, off = 0;
    for (auto& kv : fv) {
        fv_node[m] = kv.first;
        fv_begin[m] = off;
        for (int i : kv.second) fv_feat[off++] = i;
        ++m;
    }
    fv_begin[m] = off;
    *n_nodes = m;
    return 0;
}
