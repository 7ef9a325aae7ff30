// ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, th, bMono) on MI355X
// (reference src/ORBmatcher.cc:1951-2185; Frame::GetFeaturesInArea src/Frame.cc:859-951).
//
// The reference loop is sequential in one respect only: once a current keypoint holds a map point
// with observations, later last-frame points skip it (src:2050-2052).  Everything else -- the
// projection, the grid window, the level range, the stereo check, the Hamming distances -- is
// independent per point, so:
//   k_proj_candidates  one thread per last-frame point: project, walk the 64 x 48 grid window in the
//                      reference's cell order and keep (keypoint, distance) of every candidate that
//                      passes the static tests, plus the first minimum (the unconstrained best).
//   k_proj_resolve     one wave, points in index order: if the unconstrained best is still free it
//                      is the answer; otherwise the wave re-scans that point's candidates with the
//                      claimed ones masked out (first minimum again).  Then the rotation histogram /
//                      ComputeThreeMaxima filter (src:2158-2181).
//   k_lmp_candidates / k_lmp_resolve: the same scheme for SearchByProjection(Frame, local map points)
//                      (src:46-240) with the best / second-best ratio test.
// Float arithmetic follows the reference build's contractions (see oracle/orb_projection_oracle.cpp);
// this file is compiled with -ffp-contract=off and every fma is explicit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kGridCols = 64, kGridRows = 48;  // include/Frame.h:44-45
constexpr int kThHigh = 100, kHisto = 30;
constexpr int kMaxLevels = 12;

struct ProjParams {
    float Tcw[12];
    float min_x, max_x, min_y, max_y, inv_w, inv_h, fx, fy, cx, cy, bf, th;
    float scale[kMaxLevels];
    int n_cur, n_last, has_ur, bForward, bBackward, cap, check_ori;
};

struct Cand {
    int32_t i2;
    int32_t dist;
};

__device__ __forceinline__ int hamming(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(256) void k_proj_candidates(const ProjParams* __restrict__ pp, const uint8_t* __restrict__ valid,
                                                         const float* __restrict__ xyz, const uint4* __restrict__ mp_desc,
                                                         const int32_t* __restrict__ last_octave,
                                                         const float4* __restrict__ cur_kp,  // x, y, angle, octave bits
                                                         const float* __restrict__ cur_ur, const uint4* __restrict__ cur_desc,
                                                         const int32_t* __restrict__ cell_off, const int32_t* __restrict__ cell_idx,
                                                         Cand* __restrict__ cands, int32_t* __restrict__ ncand,
                                                         int32_t* __restrict__ best_c, int32_t* __restrict__ overflow) {
    const ProjParams& P = *pp;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P.n_last) return;
    ncand[i] = 0;
    best_c[i] = -1;
    if (!valid[i]) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    float c[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
        c[r] = __fmaf_rn(P.Tcw[4 * r + 2], z, __fmaf_rn(P.Tcw[4 * r], x, P.Tcw[4 * r + 1] * y)) + P.Tcw[4 * r + 3];
    const float invzc = (float)(1.0 / (double)c[2]);
    if (invzc < 0) return;
    const float u = P.fx * c[0] / c[2] + P.cx;
    const float v = P.fy * c[1] / c[2] + P.cy;
    if (u < P.min_x || u > P.max_x || v < P.min_y || v > P.max_y) return;
    const int oct = last_octave[i];
    const float radius = P.th * P.scale[oct];
    int minLevel, maxLevel;
    if (P.bForward) { minLevel = oct; maxLevel = -1; }
    else if (P.bBackward) { minLevel = 0; maxLevel = oct; }
    else { minLevel = oct - 1; maxLevel = oct + 1; }
    const int nMinCellX = max(0, (int)floorf((u - P.min_x - radius) * P.inv_w));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((u - P.min_x + radius) * P.inv_w));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((v - P.min_y - radius) * P.inv_h));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((v - P.min_y + radius) * P.inv_h));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const uint4 d0 = mp_desc[2 * (size_t)i], d1 = mp_desc[2 * (size_t)i + 1];
    const float ur = __fmaf_rn(-P.bf, invzc, u);
    Cand* out = cands + (size_t)i * P.cap;
    int n = 0, best = 256, bc = -1;
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int cell = ix * kGridRows + iy;
            for (int k = cell_off[cell]; k < cell_off[cell + 1]; ++k) {
                const int j = cell_idx[k];
                const float4 kp = cur_kp[j];
                const int koct = __float_as_int(kp.w);
                if (bCheckLevels) {
                    if (koct < minLevel) continue;
                    if (maxLevel >= 0 && koct > maxLevel) continue;
                }
                const float distx = kp.x - u, disty = kp.y - v;
                if (!(fabsf(distx) < radius && fabsf(disty) < radius)) continue;
                if (P.has_ur && cur_ur[j] > 0) {
                    const float er = fabsf(ur - cur_ur[j]);
                    if (er > radius) continue;
                }
                const int dist = hamming(d0, d1, cur_desc[2 * (size_t)j], cur_desc[2 * (size_t)j + 1]);
                if (n < P.cap) out[n] = Cand{j, dist};
                if (dist < best) { best = dist; bc = n; }
                ++n;
            }
        }
    ncand[i] = n;
    best_c[i] = bc;
    if (n > P.cap) atomicMax(overflow, n);
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {
    float rot = a1 - a2;
    if ((double)rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / kHisto));
    if (bin == kHisto) bin = 0;
    return bin;
}

// One wave: the reference's in-order assignment, then the orientation filter.
// mp[i2] = last-frame index assigned to current keypoint i2 (-1: none).
__global__ __launch_bounds__(64) void k_proj_resolve(const ProjParams* __restrict__ pp, const Cand* __restrict__ cands,
                                                     const int32_t* __restrict__ ncand, const int32_t* __restrict__ best_c,
                                                     const uint8_t* __restrict__ observed,
                                                     const float* __restrict__ last_angle,
                                                     const float4* __restrict__ cur_kp, int32_t* __restrict__ mp,
                                                     int32_t* __restrict__ match_i2, int32_t* __restrict__ match_bin,
                                                     int32_t* __restrict__ out_n) {
    const ProjParams& P = *pp;
    const int lane = threadIdx.x;
    __shared__ int hist[kHisto];
    for (int k = lane; k < P.n_cur; k += 64) mp[k] = -1;
    if (lane < kHisto) hist[lane] = 0;
    __syncthreads();
    int nm = 0;
    for (int i = 0; i < P.n_last; ++i) {
        const int n = ncand[i];
        if (n == 0) continue;
        const Cand* C = cands + (size_t)i * P.cap;
        int bi2 = -1, bd = 256;
        {
            const Cand c = C[best_c[i]];
            const int owner = mp[c.i2];
            if (owner < 0 || !observed[owner]) {
                bi2 = c.i2;
                bd = c.dist;
            } else {  // the unconstrained best is claimed: first minimum among the free candidates
                unsigned long long key = ~0ull;
                for (int k = lane; k < n; k += 64) {
                    const Cand q = C[k];
                    const int o = mp[q.i2];
                    if (o < 0 || !observed[o]) {
                        const unsigned long long kk = ((unsigned long long)q.dist << 32) | (unsigned)k;
                        key = kk < key ? kk : key;
                    }
                }
                for (int off = 32; off > 0; off >>= 1) {
                    const unsigned long long o = __shfl_xor(key, off, 64);
                    key = o < key ? o : key;
                }
                if (key != ~0ull) {
                    bd = (int)(key >> 32);
                    bi2 = C[(int)(key & 0xffffffffu)].i2;
                }
            }
        }
        __syncthreads();
        if (bi2 >= 0 && bd <= kThHigh) {
            if (lane == 0) {
                mp[bi2] = i;
                match_i2[nm] = bi2;
                const int bin = P.check_ori ? rot_bin(last_angle[i], cur_kp[bi2].z) : 0;
                match_bin[nm] = bin;
                if (P.check_ori) hist[bin]++;
            }
            ++nm;
        }
        __syncthreads();
    }
    int removed = 0;
    if (P.check_ori) {
        __shared__ int keep[3];
        if (lane == 0) {  // ComputeThreeMaxima (src:2336-2378)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int b = 0; b < kHisto; ++b) {
                const int s = hist[b];
                if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = b; }
                else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = b; }
                else if (s > max3) { max3 = s; ind3 = b; }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) ind3 = -1;
            keep[0] = ind1; keep[1] = ind2; keep[2] = ind3;
        }
        __syncthreads();
        for (int k = lane; k < nm; k += 64) {
            const int b = match_bin[k];
            if (b != keep[0] && b != keep[1] && b != keep[2]) {
                mp[match_i2[k]] = -1;
                ++removed;
            }
        }
        for (int off = 32; off > 0; off >>= 1) removed += __shfl_xor(removed, off, 64);
    }
    if (lane == 0) *out_n = nm - removed;
}

// ---- SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints, thFarPoints), src:46-240 -------

struct LocalParams {
    float min_x, min_y, inv_w, inv_h, th, th_far, nnratio;
    float scale[kMaxLevels];
    int n_cur, n_pts, has_ur, far, nlevels, cap;
};

// best / second best of the reference's update rule (src:121-138) = the first and second
// lexicographic minima of (dist, order) among candidates with dist < 256
struct Best2 {
    int c1, c2;  // candidate positions, -1 if none
};

__global__ __launch_bounds__(256) void k_lmp_candidates(const LocalParams* __restrict__ pp, const uint8_t* __restrict__ in_view,
                                                        const uint8_t* __restrict__ bad, const float* __restrict__ proj,
                                                        const float* __restrict__ view_cos, const float* __restrict__ depth,
                                                        const int32_t* __restrict__ level, const uint4* __restrict__ mp_desc,
                                                        const float4* __restrict__ cur_kp, const float* __restrict__ cur_ur,
                                                        const uint4* __restrict__ cur_desc, const int32_t* __restrict__ cell_off,
                                                        const int32_t* __restrict__ cell_idx, Cand* __restrict__ cands,
                                                        int32_t* __restrict__ ncand, Best2* __restrict__ best,
                                                        int32_t* __restrict__ overflow) {
    const LocalParams& P = *pp;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P.n_pts) return;
    ncand[i] = 0;
    best[i] = Best2{-1, -1};
    if (!in_view[i]) return;
    if (P.far && depth[i] > P.th_far) return;
    if (bad[i]) return;
    const int lvl = level[i];
    float r = ((double)view_cos[i] > 0.998) ? 2.5f : 4.0f;  // RadiusByViewingCos (src:243-250)
    if (P.th != 1.0f) r *= P.th;
    const float radius = r * P.scale[lvl];
    const float x = proj[3 * i], y = proj[3 * i + 1], xr = proj[3 * i + 2];
    const int minLevel = lvl - 1, maxLevel = lvl;
    const int nMinCellX = max(0, (int)floorf((x - P.min_x - radius) * P.inv_w));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - P.min_x + radius) * P.inv_w));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - P.min_y - radius) * P.inv_h));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - P.min_y + radius) * P.inv_h));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const uint4 d0 = mp_desc[2 * (size_t)i], d1 = mp_desc[2 * (size_t)i + 1];
    Cand* out = cands + (size_t)i * P.cap;
    int n = 0, b1 = 256, b2 = 256, c1 = -1, c2 = -1;
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int cell = ix * kGridRows + iy;
            for (int k = cell_off[cell]; k < cell_off[cell + 1]; ++k) {
                const int j = cell_idx[k];
                const float4 kp = cur_kp[j];
                const int koct = __float_as_int(kp.w);
                if (bCheckLevels) {
                    if (koct < minLevel) continue;
                    if (maxLevel >= 0 && koct > maxLevel) continue;
                }
                if (!(fabsf(kp.x - x) < radius && fabsf(kp.y - y) < radius)) continue;
                if (P.has_ur && cur_ur[j] > 0) {
                    const float er = fabsf(xr - cur_ur[j]);
                    if (er > r * P.scale[lvl]) continue;
                }
                const int dist = hamming(d0, d1, cur_desc[2 * (size_t)j], cur_desc[2 * (size_t)j + 1]);
                if (n < P.cap) out[n] = Cand{j, dist};
                if (dist < b1) { b2 = b1; c2 = c1; b1 = dist; c1 = n; }
                else if (dist < b2) { b2 = dist; c2 = n; }
                ++n;
            }
        }
    ncand[i] = n;
    best[i] = Best2{c1, c2};
    if (n > P.cap) atomicMax(overflow, n);
}

__global__ __launch_bounds__(64) void k_lmp_resolve(const LocalParams* __restrict__ pp, const Cand* __restrict__ cands,
                                                    const int32_t* __restrict__ ncand, const Best2* __restrict__ best,
                                                    const uint8_t* __restrict__ observed, const uint8_t* __restrict__ taken0,
                                                    const float4* __restrict__ cur_kp, int32_t* __restrict__ owner_obs,
                                                    int32_t* __restrict__ match, int32_t* __restrict__ out_n) {
    const LocalParams& P = *pp;
    const int lane = threadIdx.x;
    for (int k = lane; k < P.n_cur; k += 64) {
        owner_obs[k] = taken0 ? taken0[k] : 0;
        match[k] = -1;
    }
    __syncthreads();
    int nm = 0;
    for (int i = 0; i < P.n_pts; ++i) {
        const int n = ncand[i];
        if (n == 0) continue;
        const Cand* C = cands + (size_t)i * P.cap;
        const Best2 B = best[i];
        int d1 = 256, d2 = 256, j1 = -1, l1 = -1, l2 = -1;
        const bool t1 = B.c1 >= 0 && owner_obs[C[B.c1].i2];
        const bool t2 = B.c2 >= 0 && owner_obs[C[B.c2].i2];
        if (!t1 && !t2) {  // claimed candidates elsewhere in the list change neither minimum
            if (B.c1 >= 0) { d1 = C[B.c1].dist; j1 = C[B.c1].i2; l1 = __float_as_int(cur_kp[j1].w); }
            if (B.c2 >= 0) { d2 = C[B.c2].dist; l2 = __float_as_int(cur_kp[C[B.c2].i2].w); }
        } else {  // first and second minima among the free candidates
            unsigned long long k1 = ~0ull, k2 = ~0ull;
            for (int k = lane; k < n; k += 64) {
                const Cand q = C[k];
                if (q.dist < 256 && !owner_obs[q.i2]) {
                    const unsigned long long kk = ((unsigned long long)q.dist << 32) | (unsigned)k;
                    if (kk < k1) { k2 = k1; k1 = kk; }
                    else if (kk < k2) k2 = kk;
                }
            }
            for (int off = 32; off > 0; off >>= 1) {  // merge (k1, k2) pairs across lanes
                const unsigned long long o1 = __shfl_xor(k1, off, 64), o2 = __shfl_xor(k2, off, 64);
                const unsigned long long m1 = o1 < k1 ? o1 : k1;
                const unsigned long long hi = o1 < k1 ? k1 : o1;
                const unsigned long long lo2 = o2 < k2 ? o2 : k2;
                k2 = hi < lo2 ? hi : lo2;
                k1 = m1;
            }
            if (k1 != ~0ull) {
                d1 = (int)(k1 >> 32);
                j1 = C[(int)(k1 & 0xffffffffu)].i2;
                l1 = __float_as_int(cur_kp[j1].w);
            }
            if (k2 != ~0ull) {
                d2 = (int)(k2 >> 32);
                l2 = __float_as_int(cur_kp[C[(int)(k2 & 0xffffffffu)].i2].w);
            }
        }
        __syncthreads();
        if (j1 >= 0 && d1 <= kThHigh) {
            const bool ratio_fail = (l1 == l2) && ((float)d1 > P.nnratio * (float)d2);  // src:146-148
            if (!ratio_fail) {
                if (lane == 0) {
                    match[j1] = i;
                    owner_obs[j1] = observed[i];
                }
                ++nm;
            }
        }
        __syncthreads();
    }
    if (lane == 0) *out_n = nm;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

// Defined in orb_triangulation.hip: the matcher handle's staging buffers and ratio.
int orbgpu_matcher_reserve(orb_matcher_t m, size_t bytes, char** d_buf, char** h_buf, hipStream_t* stream,
                           int* check_ori);
float orbgpu_matcher_nnratio(orb_matcher_t m);

extern "C" int orb_search_by_projection_frame(orb_matcher_t m, const orb_frame_view_t* cur, const orb_last_points_t* last,
                                              float th, int mono, int32_t* match, int32_t* n_matches) {
    if (!m || !cur || !last || !match || !n_matches || cur->n < 0 || last->n < 0 || cur->nlevels <= 0 ||
        cur->nlevels > kMaxLevels || (cur->n && (!cur->kps_un || !cur->desc)) ||
        (last->n && (!last->valid || !last->observed || !last->xyz || !last->desc || !last->kps_un)) ||
        !cur->scale_factors || !(cur->grid_inv_w > 0) || !(cur->grid_inv_h > 0))
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection arguments");
    for (int i = 0; i < last->n; ++i)
        if (last->valid[i] && (last->kps_un[i].octave < 0 || last->kps_un[i].octave >= cur->nlevels))
            return orbgpu_fail(ORB_ERR_ARG, "last-frame octave out of range");
    const int n = cur->n, nl = last->n;
    // Frame::AssignFeaturesToGrid: cell (round((x - mnMinX) * inv_w), round((y - mnMinY) * inv_h)),
    // keypoints in index order inside each cell
    std::vector<int32_t> cell_off(kGridCols * kGridRows + 1, 0), cell_idx;
    std::vector<int32_t> cell_of(n, -1);
    for (int i = 0; i < n; ++i) {
        const orb_keypoint_t& kp = cur->kps_un[i];
        const int px = (int)std::round((kp.x - cur->min_x) * cur->grid_inv_w);
        const int py = (int)std::round((kp.y - cur->min_y) * cur->grid_inv_h);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
        cell_of[i] = px * kGridRows + py;
        cell_off[cell_of[i] + 1]++;
    }
    for (int c = 0; c < kGridCols * kGridRows; ++c) cell_off[c + 1] += cell_off[c];
    cell_idx.resize(cell_off.back());
    {
        std::vector<int32_t> fill(cell_off.begin(), cell_off.end() - 1);
        for (int i = 0; i < n; ++i)
            if (cell_of[i] >= 0) cell_idx[fill[cell_of[i]]++] = i;
    }
    ProjParams P{};
    memcpy(P.Tcw, cur->Tcw, sizeof(P.Tcw));
    P.min_x = cur->min_x; P.max_x = cur->max_x; P.min_y = cur->min_y; P.max_y = cur->max_y;
    P.inv_w = cur->grid_inv_w; P.inv_h = cur->grid_inv_h;
    P.fx = cur->fx; P.fy = cur->fy; P.cx = cur->cx; P.cy = cur->cy; P.bf = cur->bf; P.th = th;
    for (int l = 0; l < cur->nlevels; ++l) P.scale[l] = cur->scale_factors[l];
    P.n_cur = n; P.n_last = nl; P.has_ur = cur->u_right != nullptr;
    {   // twc = -R^T t, tlc = Tlw * twc (src:1960-1968)
        const float* T = cur->Tcw;
        float twc[3], tlc[3];
        for (int i = 0; i < 3; ++i) twc[i] = -std::fma(T[8 + i], T[11], std::fma(T[i], T[3], T[4 + i] * T[7]));
        for (int i = 0; i < 3; ++i)
            tlc[i] = std::fma(last->Tcw[4 * i + 2], twc[2], std::fma(last->Tcw[4 * i], twc[0], last->Tcw[4 * i + 1] * twc[1])) +
                     last->Tcw[4 * i + 3];
        P.bForward = tlc[2] > cur->b && !mono;
        P.bBackward = -tlc[2] > cur->b && !mono;
    }
    P.cap = 128;
    // packed inputs: params | cur kp (float4) | cur ur | cur desc | cells | last valid | observed | xyz |
    // mp desc | last octave | last angle | outputs (cands, ncand, best_c, overflow, mp, match lists, n)
    for (int attempt = 0; attempt < 3; ++attempt) {
        char* d = nullptr;
        char* h = nullptr;
        hipStream_t s = nullptr;
        int check_ori = 0;
        size_t off = 0;
        const size_t o_p = off; off = align256(off + sizeof(ProjParams));
        const size_t o_kp = off; off = align256(off + (size_t)n * 16);
        const size_t o_ur = off; off = align256(off + (size_t)n * 4);
        const size_t o_cd = off; off = align256(off + (size_t)n * 32);
        const size_t o_co = off; off = align256(off + cell_off.size() * 4);
        const size_t o_ci = off; off = align256(off + cell_idx.size() * 4);
        const size_t o_va = off; off = align256(off + (size_t)nl);
        const size_t o_ob = off; off = align256(off + (size_t)nl);
        const size_t o_xyz = off; off = align256(off + (size_t)nl * 12);
        const size_t o_md = off; off = align256(off + (size_t)nl * 32);
        const size_t o_lo = off; off = align256(off + (size_t)nl * 4);
        const size_t o_la = off; off = align256(off + (size_t)nl * 4);
        const size_t in_bytes = off;
        const size_t o_cand = off; off = align256(off + (size_t)nl * P.cap * sizeof(Cand));
        const size_t o_nc = off; off = align256(off + (size_t)nl * 4);
        const size_t o_bc = off; off = align256(off + (size_t)nl * 4);
        const size_t o_ovf = off; off = align256(off + 16);
        const size_t o_mp = off; off = align256(off + (size_t)std::max(n, 1) * 4);
        const size_t o_mi = off; off = align256(off + (size_t)std::max(nl, 1) * 4);
        const size_t o_mb = off; off = align256(off + (size_t)std::max(nl, 1) * 4);
        if (int rc = orbgpu_matcher_reserve(m, off, &d, &h, &s, &check_ori)) return rc;
        P.check_ori = check_ori;
        memcpy(h + o_p, &P, sizeof(P));
        float* kp4 = reinterpret_cast<float*>(h + o_kp);
        for (int i = 0; i < n; ++i) {
            kp4[4 * i] = cur->kps_un[i].x;
            kp4[4 * i + 1] = cur->kps_un[i].y;
            kp4[4 * i + 2] = cur->kps_un[i].angle;
            memcpy(&kp4[4 * i + 3], &cur->kps_un[i].octave, 4);
        }
        if (cur->u_right) memcpy(h + o_ur, cur->u_right, (size_t)n * 4);
        if (n) memcpy(h + o_cd, cur->desc, (size_t)n * 32);
        memcpy(h + o_co, cell_off.data(), cell_off.size() * 4);
        if (!cell_idx.empty()) memcpy(h + o_ci, cell_idx.data(), cell_idx.size() * 4);
        if (nl) {
            memcpy(h + o_va, last->valid, nl);
            memcpy(h + o_ob, last->observed, nl);
            memcpy(h + o_xyz, last->xyz, (size_t)nl * 12);
            memcpy(h + o_md, last->desc, (size_t)nl * 32);
        }
        int32_t* lo = reinterpret_cast<int32_t*>(h + o_lo);
        float* la = reinterpret_cast<float*>(h + o_la);
        for (int i = 0; i < nl; ++i) {
            lo[i] = last->kps_un[i].octave;
            la[i] = last->kps_un[i].angle;
        }
        bool ok = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s) == hipSuccess;
        ok = ok && hipMemsetAsync(d + o_ovf, 0, 16, s) == hipSuccess;
        if (ok && nl > 0)
            hipLaunchKernelGGL(k_proj_candidates, dim3((nl + 255) / 256), dim3(256), 0, s, (const ProjParams*)(d + o_p),
                               (const uint8_t*)(d + o_va), (const float*)(d + o_xyz), (const uint4*)(d + o_md),
                               (const int32_t*)(d + o_lo), (const float4*)(d + o_kp), (const float*)(d + o_ur),
                               (const uint4*)(d + o_cd), (const int32_t*)(d + o_co), (const int32_t*)(d + o_ci),
                               (Cand*)(d + o_cand), (int32_t*)(d + o_nc), (int32_t*)(d + o_bc), (int32_t*)(d + o_ovf));
        int32_t ovf = 0;
        ok = ok && hipMemcpyAsync(&ovf, d + o_ovf, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection candidate pass failed");
        if (ovf > P.cap) {  // a point had more candidates than the capacity: redo with room for all
            P.cap = (ovf + 63) & ~63;
            continue;
        }
        hipLaunchKernelGGL(k_proj_resolve, dim3(1), dim3(64), 0, s, (const ProjParams*)(d + o_p), (const Cand*)(d + o_cand),
                           (const int32_t*)(d + o_nc), (const int32_t*)(d + o_bc), (const uint8_t*)(d + o_ob),
                           (const float*)(d + o_la), (const float4*)(d + o_kp), (int32_t*)(d + o_mp),
                           (int32_t*)(d + o_mi), (int32_t*)(d + o_mb), (int32_t*)(d + o_ovf + 4));
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(h + o_mp, d + o_mp, (size_t)std::max(n, 1) * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipMemcpyAsync(h + o_ovf, d + o_ovf, 16, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection resolve failed");
        if (n) memcpy(match, h + o_mp, (size_t)n * 4);
        memcpy(n_matches, h + o_ovf + 4, 4);
        return ORB_OK;
    }
    return orbgpu_fail(ORB_ERR_INTERNAL, "SearchByProjection candidate capacity");
}

extern "C" int orb_search_by_projection_local(orb_matcher_t m, const orb_frame_view_t* F, const uint8_t* frame_taken,
                                              const orb_local_points_t* pts, float th, int far_points, float th_far_points,
                                              int32_t* match, int32_t* n_matches) {
    if (!m || !F || !pts || !match || !n_matches || F->n < 0 || pts->n < 0 || F->nlevels <= 0 ||
        F->nlevels > kMaxLevels || (F->n && (!F->kps_un || !F->desc)) || !F->scale_factors ||
        (pts->n && (!pts->track_in_view || !pts->is_bad || !pts->observed || !pts->track_proj || !pts->track_view_cos ||
                    !pts->track_depth || !pts->track_level || !pts->desc)) ||
        !(F->grid_inv_w > 0) || !(F->grid_inv_h > 0))
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection(local map) arguments");
    for (int i = 0; i < pts->n; ++i)
        if (pts->track_in_view[i] && (pts->track_level[i] < 0 || pts->track_level[i] >= F->nlevels))
            return orbgpu_fail(ORB_ERR_ARG, "predicted level out of range");
    const int n = F->n, np = pts->n;
    std::vector<int32_t> cell_off(kGridCols * kGridRows + 1, 0), cell_idx, cell_of(n, -1);
    for (int i = 0; i < n; ++i) {  // Frame::AssignFeaturesToGrid
        const int px = (int)std::round((F->kps_un[i].x - F->min_x) * F->grid_inv_w);
        const int py = (int)std::round((F->kps_un[i].y - F->min_y) * F->grid_inv_h);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
        cell_of[i] = px * kGridRows + py;
        cell_off[cell_of[i] + 1]++;
    }
    for (int c = 0; c < kGridCols * kGridRows; ++c) cell_off[c + 1] += cell_off[c];
    cell_idx.resize(cell_off.back());
    {
        std::vector<int32_t> fill(cell_off.begin(), cell_off.end() - 1);
        for (int i = 0; i < n; ++i)
            if (cell_of[i] >= 0) cell_idx[fill[cell_of[i]]++] = i;
    }
    LocalParams P{};
    P.min_x = F->min_x; P.min_y = F->min_y; P.inv_w = F->grid_inv_w; P.inv_h = F->grid_inv_h;
    P.th = th; P.th_far = th_far_points;
    for (int l = 0; l < F->nlevels; ++l) P.scale[l] = F->scale_factors[l];
    P.n_cur = n; P.n_pts = np; P.has_ur = F->u_right != nullptr; P.far = far_points ? 1 : 0; P.nlevels = F->nlevels;
    P.cap = 128;
    for (int attempt = 0; attempt < 3; ++attempt) {
        char *d = nullptr, *h = nullptr;
        hipStream_t s = nullptr;
        int check_ori = 0;
        size_t off = 0;
        const size_t o_p = off; off = align256(off + sizeof(LocalParams));
        const size_t o_kp = off; off = align256(off + (size_t)n * 16);
        const size_t o_ur = off; off = align256(off + (size_t)n * 4);
        const size_t o_cd = off; off = align256(off + (size_t)n * 32);
        const size_t o_tk = off; off = align256(off + (size_t)n);
        const size_t o_co = off; off = align256(off + cell_off.size() * 4);
        const size_t o_ci = off; off = align256(off + cell_idx.size() * 4);
        const size_t o_iv = off; off = align256(off + (size_t)np);
        const size_t o_bd = off; off = align256(off + (size_t)np);
        const size_t o_ob = off; off = align256(off + (size_t)np);
        const size_t o_pj = off; off = align256(off + (size_t)np * 12);
        const size_t o_vc = off; off = align256(off + (size_t)np * 4);
        const size_t o_dp = off; off = align256(off + (size_t)np * 4);
        const size_t o_lv = off; off = align256(off + (size_t)np * 4);
        const size_t o_md = off; off = align256(off + (size_t)np * 32);
        const size_t in_bytes = off;
        const size_t o_cand = off; off = align256(off + (size_t)np * P.cap * sizeof(Cand));
        const size_t o_nc = off; off = align256(off + (size_t)np * 4);
        const size_t o_b2 = off; off = align256(off + (size_t)np * sizeof(Best2));
        const size_t o_ovf = off; off = align256(off + 16);
        const size_t o_own = off; off = align256(off + (size_t)std::max(n, 1) * 4);
        const size_t o_m = off; off = align256(off + (size_t)std::max(n, 1) * 4);
        if (int rc = orbgpu_matcher_reserve(m, off, &d, &h, &s, &check_ori)) return rc;
        P.nnratio = orbgpu_matcher_nnratio(m);
        memcpy(h + o_p, &P, sizeof(P));
        float* kp4 = reinterpret_cast<float*>(h + o_kp);
        for (int i = 0; i < n; ++i) {
            kp4[4 * i] = F->kps_un[i].x;
            kp4[4 * i + 1] = F->kps_un[i].y;
            kp4[4 * i + 2] = F->kps_un[i].angle;
            memcpy(&kp4[4 * i + 3], &F->kps_un[i].octave, 4);
        }
        if (F->u_right) memcpy(h + o_ur, F->u_right, (size_t)n * 4);
        if (n) memcpy(h + o_cd, F->desc, (size_t)n * 32);
        if (frame_taken && n) memcpy(h + o_tk, frame_taken, n);
        memcpy(h + o_co, cell_off.data(), cell_off.size() * 4);
        if (!cell_idx.empty()) memcpy(h + o_ci, cell_idx.data(), cell_idx.size() * 4);
        if (np) {
            memcpy(h + o_iv, pts->track_in_view, np);
            memcpy(h + o_bd, pts->is_bad, np);
            memcpy(h + o_ob, pts->observed, np);
            memcpy(h + o_pj, pts->track_proj, (size_t)np * 12);
            memcpy(h + o_vc, pts->track_view_cos, (size_t)np * 4);
            memcpy(h + o_dp, pts->track_depth, (size_t)np * 4);
            memcpy(h + o_lv, pts->track_level, (size_t)np * 4);
            memcpy(h + o_md, pts->desc, (size_t)np * 32);
        }
        bool ok = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s) == hipSuccess &&
                  hipMemsetAsync(d + o_ovf, 0, 16, s) == hipSuccess;
        if (ok && np > 0)
            hipLaunchKernelGGL(k_lmp_candidates, dim3((np + 255) / 256), dim3(256), 0, s, (const LocalParams*)(d + o_p),
                               (const uint8_t*)(d + o_iv), (const uint8_t*)(d + o_bd), (const float*)(d + o_pj),
                               (const float*)(d + o_vc), (const float*)(d + o_dp), (const int32_t*)(d + o_lv),
                               (const uint4*)(d + o_md), (const float4*)(d + o_kp), (const float*)(d + o_ur),
                               (const uint4*)(d + o_cd), (const int32_t*)(d + o_co), (const int32_t*)(d + o_ci),
                               (Cand*)(d + o_cand), (int32_t*)(d + o_nc), (Best2*)(d + o_b2), (int32_t*)(d + o_ovf));
        int32_t ovf = 0;
        ok = ok && hipMemcpyAsync(&ovf, d + o_ovf, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection(local) candidate pass failed");
        if (ovf > P.cap) {
            P.cap = (ovf + 63) & ~63;
            continue;
        }
        hipLaunchKernelGGL(k_lmp_resolve, dim3(1), dim3(64), 0, s, (const LocalParams*)(d + o_p), (const Cand*)(d + o_cand),
                           (const int32_t*)(d + o_nc), (const Best2*)(d + o_b2), (const uint8_t*)(d + o_ob),
                           frame_taken ? (const uint8_t*)(d + o_tk) : nullptr, (const float4*)(d + o_kp),
                           (int32_t*)(d + o_own), (int32_t*)(d + o_m), (int32_t*)(d + o_ovf + 4));
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(h + o_m, d + o_m, (size_t)std::max(n, 1) * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipMemcpyAsync(h + o_ovf, d + o_ovf, 16, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection(local) resolve failed");
        if (n) memcpy(match, h + o_m, (size_t)n * 4);
        memcpy(n_matches, h + o_ovf + 4, 4);
        return ORB_OK;
    }
    return orbgpu_fail(ORB_ERR_INTERNAL, "SearchByProjection(local) candidate capacity");
}
