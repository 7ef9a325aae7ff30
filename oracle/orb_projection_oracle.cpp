// ORACLE -- TEST INFRASTRUCTURE ONLY.  CPU restatement of
// ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, th, bMono)
// (reference src/ORBmatcher.cc:1951-2185) for pinhole frames (Nleft == -1), with
// Frame::AssignFeaturesToGrid / PosInGrid (src/Frame.cc:469-504, 970-978) and
// Frame::GetFeaturesInArea (src/Frame.cc:859-951).  Sequential, like the reference: a current
// keypoint that already holds a map point with observations is skipped by later points.
//
// Float arithmetic: g++ -O3 -march=native contracts `a*b + c*d` into fma(a, b, c*d) and `a - b*c`
// into fma(-b, c, a).  The poses are 3x4 matrices here; the reference applies Sophus quaternions,
// so the projected coordinates agree with the real reference only up to float rounding
// ("parity unpinned" at the ulp level).  Everything downstream (windows, distances, ties,
// histogram) is the reference's logic.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/orbgpu.h"

namespace {

constexpr int GRID_COLS = 64, GRID_ROWS = 48;  // include/Frame.h:44-45
constexpr int TH_HIGH = 100, HISTO_LENGTH = 30;

int dist256(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

// y = R x + t with the rows contracted as g++ does: fma(r2, x2, fma(r0, x0, r1 * x1)) + t
void transform(const float T[12], const float x[3], float y[3]) {
    for (int i = 0; i < 3; ++i)
        y[i] = std::fma(T[4 * i + 2], x[2], std::fma(T[4 * i], x[0], T[4 * i + 1] * x[1])) + T[4 * i + 3];
}

struct Grid {
    std::vector<int> cell[GRID_COLS][GRID_ROWS];
};

void build_grid(const orb_frame_view_t& F, Grid& G) {  // Frame::AssignFeaturesToGrid
    for (int i = 0; i < F.n; ++i) {
        const orb_keypoint_t& kp = F.kps_un[i];
        const int px = (int)std::round((kp.x - F.min_x) * F.grid_inv_w);
        const int py = (int)std::round((kp.y - F.min_y) * F.grid_inv_h);
        if (px < 0 || px >= GRID_COLS || py < 0 || py >= GRID_ROWS) continue;
        G.cell[px][py].push_back(i);
    }
}

std::vector<int> features_in_area(const orb_frame_view_t& F, const Grid& G, float x, float y, float r, int minLevel,
                                  int maxLevel) {  // Frame::GetFeaturesInArea
    std::vector<int> v;
    const float factorX = r, factorY = r;
    const int nMinCellX = std::max(0, (int)std::floor((x - F.min_x - factorX) * F.grid_inv_w));
    if (nMinCellX >= GRID_COLS) return v;
    const int nMaxCellX = std::min(GRID_COLS - 1, (int)std::ceil((x - F.min_x + factorX) * F.grid_inv_w));
    if (nMaxCellX < 0) return v;
    const int nMinCellY = std::max(0, (int)std::floor((y - F.min_y - factorY) * F.grid_inv_h));
    if (nMinCellY >= GRID_ROWS) return v;
    const int nMaxCellY = std::min(GRID_ROWS - 1, (int)std::ceil((y - F.min_y + factorY) * F.grid_inv_h));
    if (nMaxCellY < 0) return v;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
            for (int j : G.cell[ix][iy]) {
                const orb_keypoint_t& kp = F.kps_un[j];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = kp.x - x, disty = kp.y - y;
                if (std::fabs(distx) < factorX && std::fabs(disty) < factorY) v.push_back(j);
            }
    return v;
}

void three_maxima(const std::vector<int>* histo, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
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
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) ind3 = -1;
}

}  // namespace

extern "C" int oracle_search_by_projection_frame(const orb_frame_view_t* cur, const orb_last_points_t* last, float th,
                                                 int bMono, int mbCheckOrientation, int32_t* match_out) {
    const orb_frame_view_t& F = *cur;
    Grid* G = new Grid();
    build_grid(F, *G);
    std::vector<int> mp(F.n, -1);  // CurrentFrame.mvpMapPoints as LastFrame indices
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    const float factor = 1.0f / HISTO_LENGTH;
    // twc = Tcw.inverse().translation() = -R^T t;  tlc = Tlw * twc
    float twc[3], tlc[3];
    for (int i = 0; i < 3; ++i)
        twc[i] = -std::fma(F.Tcw[8 + i], F.Tcw[11], std::fma(F.Tcw[i], F.Tcw[3], F.Tcw[4 + i] * F.Tcw[7]));
    transform(last->Tcw, twc, tlc);
    const bool bForward = tlc[2] > F.b && !bMono;
    const bool bBackward = -tlc[2] > F.b && !bMono;
    for (int i = 0; i < last->n; i++) {
        if (!last->valid[i]) continue;
        float x3Dc[3];
        transform(F.Tcw, last->xyz + 3 * i, x3Dc);
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0) continue;
        const float u = F.fx * x3Dc[0] / x3Dc[2] + F.cx;
        const float v = F.fy * x3Dc[1] / x3Dc[2] + F.cy;
        if (u < F.min_x || u > F.max_x) continue;
        if (v < F.min_y || v > F.max_y) continue;
        const int nLastOctave = last->kps_un[i].octave;
        const float radius = th * F.scale_factors[nLastOctave];
        std::vector<int> vIndices2;
        if (bForward) vIndices2 = features_in_area(F, *G, u, v, radius, nLastOctave, -1);
        else if (bBackward) vIndices2 = features_in_area(F, *G, u, v, radius, 0, nLastOctave);
        else vIndices2 = features_in_area(F, *G, u, v, radius, nLastOctave - 1, nLastOctave + 1);
        if (vIndices2.empty()) continue;
        const uint8_t* dMP = last->desc + 32 * i;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : vIndices2) {
            if (mp[i2] >= 0 && last->observed[mp[i2]]) continue;
            if (F.u_right && F.u_right[i2] > 0) {
                const float ur = std::fma(-F.bf, invzc, u);
                const float er = std::fabs(ur - F.u_right[i2]);
                if (er > radius) continue;
            }
            const int dist = dist256(dMP, F.desc + 32 * i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            mp[bestIdx2] = i;
            nmatches++;
            if (mbCheckOrientation) {
                float rot = last->kps_un[i].angle - F.kps_un[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (mbCheckOrientation) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i != ind1 && i != ind2 && i != ind3) {
                for (int j : rotHist[i]) {
                    mp[j] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i = 0; i < F.n; ++i) match_out[i] = mp[i];
    delete G;
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame &F, const vector<MapPoint*> &vpMapPoints, th, bFarPoints,
// thFarPoints), src/ORBmatcher.cc:46-240 (Nleft == -1), with RadiusByViewingCos (src:243-250).
extern "C" int oracle_search_by_projection_local(const orb_frame_view_t* Fv, const uint8_t* frame_taken,
                                                 const orb_local_points_t* pts, float th, int bFarPoints,
                                                 float thFarPoints, float mfNNratio, int32_t* match_out) {
    const orb_frame_view_t& F = *Fv;
    Grid* G = new Grid();
    build_grid(F, *G);
    std::vector<int> owner_obs(F.n, 0), match(F.n, -1);
    if (frame_taken)
        for (int i = 0; i < F.n; ++i) owner_obs[i] = frame_taken[i];
    int nmatches = 0;
    const bool bFactor = th != 1.0;
    for (int iMP = 0; iMP < pts->n; iMP++) {
        if (!pts->track_in_view[iMP]) continue;
        if (bFarPoints && pts->track_depth[iMP] > thFarPoints) continue;
        if (pts->is_bad[iMP]) continue;
        const int nPredictedLevel = pts->track_level[iMP];
        float r = (pts->track_view_cos[iMP] > 0.998) ? 2.5 : 4.0;
        if (bFactor) r *= th;
        const std::vector<int> vIndices =
            features_in_area(F, *G, pts->track_proj[3 * iMP], pts->track_proj[3 * iMP + 1],
                             r * F.scale_factors[nPredictedLevel], nPredictedLevel - 1, nPredictedLevel);
        if (vIndices.empty()) continue;
        const uint8_t* MPdescriptor = pts->desc + 32 * iMP;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int idx : vIndices) {
            if (owner_obs[idx]) continue;  // F.mvpMapPoints[idx] && ->Observations() > 0
            if (F.u_right && F.u_right[idx] > 0) {
                const float er = std::fabs(pts->track_proj[3 * iMP + 2] - F.u_right[idx]);
                if (er > r * F.scale_factors[nPredictedLevel]) continue;
            }
            const int dist = dist256(MPdescriptor, F.desc + 32 * idx);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = F.kps_un[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = F.kps_un[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > mfNNratio * bestDist2) continue;
            if (bestLevel != bestLevel2 || bestDist <= mfNNratio * bestDist2) {
                match[bestIdx] = iMP;
                owner_obs[bestIdx] = pts->observed[iMP];
                nmatches++;
            }
        }
    }
    for (int i = 0; i < F.n; ++i) match_out[i] = match[i];
    delete G;
    return nmatches;
}
