// ORACLE (test infrastructure only; never linked into the product): CPU restatement of
// Frame::ComputeStereoMatches (reference src/Frame.cc:1102-1358) for rectified stereo pairs.
//
// Inputs are the two extractors' outputs (keypoints in cv::KeyPoint layout, 32-byte descriptors)
// and their image pyramids (padded planes with the 19-px REFLECT_101 frame; mvImagePyramid[l] is
// the view at (19, 19)).  Outputs mvuRight / mvDepth.  Float semantics follow the reference:
//   - vRowIndices[(size_t)vL]                                   src/Frame.cc:1134-1152, :1176
//   - coarse search: first strict minimum over ascending iR, TH_HIGH start   :1190-1226
//   - SAD refinement (11x11 window, +-5 px), float distances, strict <       :1236-1280
//   - parabola fit, disparity range, 0.01 clamp (double literal)              :1286-1328
//   - median cull: 1.5f*1.4f*median over the sorted (dist, iL) pairs          :1334-1352
// Every value entering a float expression here is an integer below 2^24 or a product the
// reference also rounds once, so g++'s -march=native contractions cannot change a result (see
// DESIGN.md); the file is compiled with -ffp-contract=off regardless.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace {

struct KeyPoint {  // cv::KeyPoint layout (28 bytes)
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

int descriptor_distance(const uint8_t* a, const uint8_t* b) {  // src/ORBmatcher.cc:2384-2404
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

struct Level {  // one side's pyramid level: view origin inside the padded plane
    const uint8_t* view;
    int pitch, w, h;
    uint8_t at(int y, int x) const { return view[(long long)y * pitch + x]; }
};

constexpr int kThHigh = 100, kThLow = 50;  // ORBmatcher::TH_HIGH / TH_LOW, src/ORBmatcher.cc:36-37

}  // namespace

extern "C" {

// planes_l/planes_r: per level, the padded plane of that level ((w+38) x (h+38), row pitch `pitch`).
// Returns the number of keypoints with a stereo match after the cull (mvuRight >= 0).
int oracle_compute_stereo_matches(const void* kps_l, int n_l, const uint8_t* desc_l, const void* kps_r, int n_r,
                                  const uint8_t* desc_r, const uint8_t* const* planes_l,
                                  const uint8_t* const* planes_r, const int* pitch, const int* w, const int* h,
                                  int nlevels, const float* scale, const float* inv_scale, float bf, float b,
                                  float* u_right, float* depth) {
    const KeyPoint* KL = (const KeyPoint*)kps_l;
    const KeyPoint* KR = (const KeyPoint*)kps_r;
    std::vector<Level> LL(nlevels), LR(nlevels);
    for (int l = 0; l < nlevels; ++l) {
        LL[l] = {planes_l[l] + 19 * pitch[l] + 19, pitch[l], w[l], h[l]};
        LR[l] = {planes_r[l] + 19 * pitch[l] + 19, pitch[l], w[l], h[l]};
    }
    for (int i = 0; i < n_l; ++i) u_right[i] = depth[i] = -1.0f;  // :1119-1120
    const int thOrbDist = (kThHigh + kThLow) / 2;                 // :1123
    const int nRows = h[0];                                       // :1126
    // Step 1: row table, :1134-1152
    std::vector<std::vector<size_t>> rows(nRows);
    for (int iR = 0; iR < n_r; ++iR) {
        const float kpY = KR[iR].y;
        const float r = 2.0f * scale[KR[iR].octave];
        const int maxr = (int)std::ceil(kpY + r);
        const int minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; ++yi)
            if (yi >= 0 && yi < nRows) rows[yi].push_back(iR);  // (always in range for real keypoints)
    }
    // search limits, :1160-1163
    const float minZ = b;
    const float minD = 0;
    const float maxD = bf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    for (int iL = 0; iL < n_l; ++iL) {
        const KeyPoint& kpL = KL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const size_t row = (size_t)vL;
        if (row >= (size_t)nRows) continue;
        const std::vector<size_t>& cand = rows[row];
        if (cand.empty()) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = kThHigh;
        size_t bestIdxR = 0;
        for (size_t iR : cand) {  // :1195-1220
            const KeyPoint& kpR = KR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = descriptor_distance(desc_l + 32 * (size_t)iL, desc_r + 32 * iR);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist >= thOrbDist) continue;
        // subpixel match by correlation, :1228-1280
        const float uR0 = KR[bestIdxR].x;
        const float scaleFactor = inv_scale[kpL.octave];
        const float scaleduL = std::round(kpL.x * scaleFactor);
        const float scaledvL = std::round(kpL.y * scaleFactor);
        const float scaleduR0 = std::round(uR0 * scaleFactor);
        const int wS = 5, L = 5;
        const Level& IL = LL[kpL.octave];
        const Level& IR = LR[kpL.octave];
        const int cuL = (int)scaleduL, cvL = (int)scaledvL, cuR = (int)scaleduR0;
        const float iniu = scaleduR0 + L - wS;
        const float endu = scaleduR0 + L + wS + 1;
        if (iniu < 0 || endu >= IR.w) continue;
        // the reference would throw (cv::Mat::colRange) for windows leaving the view on the left or
        // at the top/bottom; keypoints never get there (>= 19 px inside every level)
        if (cuR - L - wS < 0 || cvL - wS < 0 || cvL + wS >= IL.h || cuL - wS < 0 || cuL + wS >= IL.w) continue;
        int bestDistS = INT_MAX;
        int bestincR = 0;
        float vDists[2 * L + 1];
        for (int incR = -L; incR <= L; ++incR) {
            int sad = 0;
            for (int y = -wS; y <= wS; ++y)
                for (int x = -wS; x <= wS; ++x)
                    sad += std::abs((int)IL.at(cvL + y, cuL + x) - (int)IR.at(cvL + y, cuR + incR + x));
            const float dist = (float)sad;  // cv::norm(NORM_L1) -> double -> float, exact
            if (dist < bestDistS) {
                bestDistS = (int)dist;
                bestincR = incR;
            }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;
        // parabola, :1302-1308
        const float dist1 = vDists[L + bestincR - 1];
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[iL] = bf / disparity;
            u_right[iL] = bestuR;
            vDistIdx.push_back(std::pair<int, int>(bestDistS, iL));
        }
    }
    // Step 6: outlier cull, :1334-1352 (the reference indexes vDistIdx[0] even when it is empty)
    if (vDistIdx.empty()) return 0;
    std::sort(vDistIdx.begin(), vDistIdx.end());
    const float median = vDistIdx[vDistIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    int kept = (int)vDistIdx.size();
    for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
        if (vDistIdx[i].first < thDist) break;
        u_right[vDistIdx[i].second] = -1;
        depth[vDistIdx[i].second] = -1;
        --kept;
    }
    return kept;
}

}  // extern "C"
