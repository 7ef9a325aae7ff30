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

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

// Defined in orb_triangulation.hip: the matcher handle's staging buffers.
int orbgpu_matcher_reserve(orb_matcher_t m, size_t bytes, char** d_buf, char** h_buf, hipStream_t* stream,
                           int* check_ori);

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
