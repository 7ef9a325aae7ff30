// ORACLE -- TEST INFRASTRUCTURE ONLY.  CPU restatement of ORBmatcher::SearchForTriangulation
// (reference src/ORBmatcher.cc:1046-1324) with Pinhole::epipolarConstrain
// (src/CameraModels/Pinhole.cpp:186-216) and ComputeThreeMaxima (src/ORBmatcher.cc:2336-2378),
// for one keyframe pair at a time, written as the reference's sequential loop over a std::map.
// Only tests/ and bench.py's cpu_baseline use it; the product path never does.
//
// Float rounding follows the reference build (g++ -O3 -march=native on an FMA machine): a*b + c*d
// becomes fma(a, b, c*d) (checked with g++ 11 on this image).  F12's Eigen evaluation is restated
// as Eigen 3.x's closed-form 3x3 inverse and unrolled 3x3 products with those contractions.
// Parity with the real reference's F12 bits is unpinned (Eigen is absent); everything downstream of
// F12 is the reference's arithmetic.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "../include/orbgpu.h"

namespace {

constexpr int TH_LOW = 50;        // src/ORBmatcher.cc:37
constexpr int HISTO_LENGTH = 30;  // src/ORBmatcher.cc:38

struct Mat3 {
    float v[3][3];
};

Mat3 mul(const Mat3& a, const Mat3& b) {
    Mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            // Eigen's lazy product: ((a0*b0 + a1*b1) + a2*b2), contracted by g++
            float s = std::fma(a.v[i][0], b.v[0][j], a.v[i][1] * b.v[1][j]);
            r.v[i][j] = std::fma(a.v[i][2], b.v[2][j], s);
        }
    return r;
}

float cofactor(const Mat3& m, int i, int j) {  // Eigen cofactor_3x3<M, i, j>
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return std::fma(m.v[i1][j1], m.v[i2][j2], -(m.v[i1][j2] * m.v[i2][j1]));
}

Mat3 inverse(const Mat3& m) {  // Eigen compute_inverse<.., 3>
    float c[3] = {cofactor(m, 0, 0), cofactor(m, 1, 0), cofactor(m, 2, 0)};
    float det = std::fma(c[2], m.v[2][0], std::fma(c[0], m.v[0][0], c[1] * m.v[1][0]));
    float invdet = 1.0f / det;
    Mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.v[i][j] = cofactor(m, j, i) * invdet;
    return r;
}

Mat3 toK(const orb_kf_view_t& k) {  // Pinhole::toK_ (Pinhole.cpp:168-173)
    Mat3 K = {{{k.fx, 0.f, k.cx}, {0.f, k.fy, k.cy}, {0.f, 0.f, 1.f}}};
    return K;
}

Mat3 transpose(const Mat3& m) {
    Mat3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.v[i][j] = m.v[j][i];
    return r;
}

// Pinhole::epipolarConstrain
bool epipolar_constrain(const orb_kf_view_t& k1, const orb_kf_view_t& k2, const orb_keypoint_t& kp1,
                        const orb_keypoint_t& kp2, const orb_kf_pair_geom_t& g, float unc) {
    Mat3 R12;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R12.v[i][j] = g.R12[3 * i + j];
    const float* t = g.t12;
    Mat3 t12x = {{{0.f, -t[2], t[1]}, {t[2], 0.f, -t[0]}, {-t[1], t[0], 0.f}}};
    Mat3 F12 = mul(mul(mul(inverse(transpose(toK(k1))), t12x), R12), inverse(toK(k2)));
    const float a = std::fma(kp1.x, F12.v[0][0], kp1.y * F12.v[1][0]) + F12.v[2][0];
    const float b = std::fma(kp1.x, F12.v[0][1], kp1.y * F12.v[1][1]) + F12.v[2][1];
    const float c = std::fma(kp1.x, F12.v[0][2], kp1.y * F12.v[1][2]) + F12.v[2][2];
    const float num = std::fma(a, kp2.x, b * kp2.y) + c;
    const float den = std::fma(a, a, b * b);
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * unc;
}

int descriptor_distance(const uint8_t* a, const uint8_t* b) {  // src/ORBmatcher.cc:2384-2404
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        uint32_t v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s; ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

std::map<uint32_t, std::vector<int>> feature_vector(const orb_kf_view_t& k) {
    std::map<uint32_t, std::vector<int>> fv;
    for (int i = 0; i < k.n_nodes; ++i)
        fv[k.fv_node[i]] = std::vector<int>(k.fv_index + k.fv_offset[i], k.fv_index + k.fv_offset[i + 1]);
    return fv;
}

}  // namespace

extern "C" int oracle_search_for_triangulation(const orb_kf_view_t* pKF1, const orb_kf_view_t* pKF2,
                                               const orb_kf_pair_geom_t* geom, int bOnlyStereo, int bCoarse,
                                               int mbCheckOrientation, int32_t* vMatches12out) {
    const auto vFeatVec1 = feature_vector(*pKF1);
    const auto vFeatVec2 = feature_vector(*pKF2);
    const float* ep = geom->ep;
    auto hasMP = [](const orb_kf_view_t* k, int i) { return k->has_mappoint && k->has_mappoint[i]; };
    auto uR = [](const orb_kf_view_t* k, int i) { return k->u_right ? k->u_right[i] : -1.0f; };

    int nmatches = 0;
    std::vector<bool> vbMatched2(pKF2->n, false);
    std::vector<int> vMatches12(pKF1->n, -1);
    std::vector<int> rotHist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;

    auto f1it = vFeatVec1.begin(), f2it = vFeatVec2.begin();
    auto f1end = vFeatVec1.end(), f2end = vFeatVec2.end();
    while (f1it != f1end && f2it != f2end) {
        if (f1it->first == f2it->first) {
            for (size_t i1 = 0, iend1 = f1it->second.size(); i1 < iend1; i1++) {
                const size_t idx1 = f1it->second[i1];
                if (hasMP(pKF1, idx1)) continue;
                const bool bStereo1 = uR(pKF1, idx1) >= 0;
                if (bOnlyStereo && !bStereo1) continue;
                const orb_keypoint_t& kp1 = pKF1->kps_un[idx1];
                const uint8_t* d1 = pKF1->desc + 32 * idx1;
                int bestDist = TH_LOW;
                int bestIdx2 = -1;
                for (size_t i2 = 0, iend2 = f2it->second.size(); i2 < iend2; i2++) {
                    size_t idx2 = f2it->second[i2];
                    if (vbMatched2[idx2] || hasMP(pKF2, idx2)) continue;
                    const bool bStereo2 = uR(pKF2, idx2) >= 0;
                    if (bOnlyStereo && !bStereo2) continue;
                    const int dist = descriptor_distance(d1, pKF2->desc + 32 * idx2);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const orb_keypoint_t& kp2 = pKF2->kps_un[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ep[0] - kp2.x;
                        const float distey = ep[1] - kp2.y;
                        if (std::fma(distex, distex, distey * distey) < 100 * pKF2->scale_factors[kp2.octave])
                            continue;
                    }
                    if (bCoarse || epipolar_constrain(*pKF1, *pKF2, kp1, kp2, *geom, pKF2->level_sigma2[kp2.octave])) {
                        bestIdx2 = (int)idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    const orb_keypoint_t& kp2 = pKF2->kps_un[bestIdx2];
                    vMatches12[idx1] = bestIdx2;
                    nmatches++;
                    if (mbCheckOrientation) {
                        float rot = kp1.angle - kp2.angle;
                        if (rot < 0.0) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        rotHist[bin].push_back((int)idx1);
                    }
                }
            }
            f1it++;
            f2it++;
        } else if (f1it->first < f2it->first) {
            f1it = vFeatVec1.lower_bound(f2it->first);
        } else {
            f2it = vFeatVec2.lower_bound(f1it->first);
        }
    }
    if (mbCheckOrientation) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (size_t j = 0, jend = rotHist[i].size(); j < jend; j++) {
                vbMatched2[vMatches12[rotHist[i][j]]] = false;
                vMatches12[rotHist[i][j]] = -1;
                nmatches--;
            }
        }
    }
    for (int i = 0; i < pKF1->n; ++i) vMatches12out[i] = vMatches12[i];
    return nmatches;
}

// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:438-529) for n_points points: point p's
// descriptors are rows [offsets[p], offsets[p+1]) of desc.  best[p] = BestIdx, or -1 when the point has
// no descriptor (the reference returns before choosing).  Written as the reference: a float N x N
// matrix, each row copied into vector<int>, std::sort, median at index 0.5*(N-1) (size_t truncation),
// the first strictly smaller median wins.
extern "C" void oracle_compute_distinctive_descriptors(const uint8_t* desc, const int32_t* offsets, int n_points,
                                                      int32_t* best) {
    for (int p = 0; p < n_points; ++p) {
        const int o = offsets[p];
        const size_t N = (size_t)(offsets[p + 1] - o);
        if (N == 0) {
            best[p] = -1;
            continue;
        }
        std::vector<float> Distances(N * N);
        for (size_t i = 0; i < N; i++) {
            Distances[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                const int distij = descriptor_distance(desc + 32 * (size_t)(o + i), desc + 32 * (size_t)(o + j));
                Distances[i * N + j] = distij;
                Distances[j * N + i] = distij;
            }
        }
        int BestMedian = INT_MAX;
        int BestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> vDists(Distances.begin() + i * N, Distances.begin() + (i + 1) * N);
            std::sort(vDists.begin(), vDists.end());
            const int median = vDists[0.5 * (N - 1)];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best[p] = BestIdx;
    }
}

// Best / second-best Hamming scan of every query over the train set in index order, the update rule
// of the ORBmatcher loops (a strictly smaller distance replaces the best, otherwise a smaller one the
// second; src/ORBmatcher.cc:1160-1175).  257 = none.
extern "C" void oracle_hamming_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* best_idx,
                                   int32_t* best_dist, int32_t* second_dist) {
    for (int i = 0; i < nq; ++i) {
        int best = 257, second = 257, bi = -1;
        for (int j = 0; j < nt; ++j) {
            const int d = descriptor_distance(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (d < best) {
                second = best;
                best = d;
                bi = j;
            } else if (d < second) {
                second = d;
            }
        }
        best_idx[i] = bi;
        best_dist[i] = best;
        second_dist[i] = second;
    }
}
