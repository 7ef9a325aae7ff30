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
//   k_lmp_candidates   the same for SearchByProjection(Frame, local map points) (src:46-240).
//   k_resolve_rounds   one workgroup: the in-order assignment of both overloads (ratio test for the
//                      local map), decided in parallel rounds (below), then the rotation histogram /
//                      ComputeThreeMaxima filter (src:2158-2181).
// Float arithmetic follows the reference build's contractions (see oracle/orb_projection_oracle.cpp);
// this file is compiled with -ffp-contract=off and every fma is explicit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <cstdlib>

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

// After a point's candidates are written: the wave (lanes over its list) records, for every usable
// candidate keypoint (distance < 256, not already taken), the earliest observed point listing it
// (`lister`, initialised to 0x7f7f7f7f).  k_resolve_init uses it to find the points whose answer no
// earlier point can change.
__device__ __forceinline__ void record_listers(int lane, int i, int n, int cap, const Cand* __restrict__ c_i,
                                               const uint8_t* __restrict__ taken0, int32_t* __restrict__ lister) {
    if (n > cap) return;  // overflow: the call is redone with a larger capacity
    for (int k = lane; k < n; k += 64) {
        const Cand c = c_i[k];
        if (c.dist < 256 && !(taken0 && taken0[c.i2])) atomicMin(&lister[c.i2], i);
    }
}

__device__ __forceinline__ int hamming(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// One wave scans one point's grid window (Frame::GetFeaturesInArea, src/Frame.cc:859-951) in the
// reference's order -- cells ix outer, iy inner, keypoints of a cell in index order -- with the lanes
// spread over the window: 64 cells at a time, a wave prefix sum of the cells' keypoint counts, then
// 64 keypoints at a time (lane -> cell by binary search of the prefix), `test(j)` -> Hamming distance
// or -1, and an order-preserving ballot compaction into out[0 .. cap).  Returns the candidate count
// (wave-uniform; counted beyond cap).
template <class Test>
__device__ __forceinline__ int window_candidates(int lane, int* __restrict__ pre, int* __restrict__ beg,
                                                 const int32_t* __restrict__ cell_off, const int32_t* __restrict__ cell_idx,
                                                 int x0, int x1, int y0, int y1, Cand* __restrict__ out, int cap,
                                                 Test test) {
    const int ny = y1 - y0 + 1, ncells = (x1 - x0 + 1) * ny;
    int n = 0;
    for (int c0 = 0; c0 < ncells; c0 += 64) {
        const int t = c0 + lane;
        int b = 0, cnt = 0;
        if (t < ncells) {
            const int cell = (x0 + t / ny) * kGridRows + (y0 + t % ny);
            b = cell_off[cell];
            cnt = cell_off[cell + 1] - b;
        }
        int incl = cnt;  // inclusive prefix over the lanes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        const int total = __shfl(incl, 63, 64);
        pre[lane] = incl - cnt;
        beg[lane] = b;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        for (int i0 = 0; i0 < total; i0 += 64) {
            const int it = i0 + lane;
            int j = -1, dist = -1;
            if (it < total) {
                int lo = 0, hi = 63;  // the last cell lane whose prefix is <= it
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (pre[mid] <= it) lo = mid;
                    else hi = mid - 1;
                }
                j = cell_idx[beg[lo] + it - pre[lo]];
                dist = test(j);
            }
            const unsigned long long m = __ballot(dist >= 0);
            const int pos = n + (int)__popcll(m & ((1ull << lane) - 1ull));
            if (dist >= 0 && pos < cap) out[pos] = Cand{j, dist};
            n += (int)__popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    return n;
}

constexpr int kCandWaves = 4;

// one wave per last-frame point (src:1978-2062 up to the minimum): project with the current pose,
// the window by forward / backward motion (src:2019-2024), the stereo u_R test, distances
__device__ __forceinline__ void k_proj_candidates_body(const ProjParams P, const int32_t* __restrict__ n_dev,
                                                         const uint8_t* __restrict__ valid,
                                                         const float* __restrict__ xyz, const uint4* __restrict__ mp_desc,
                                                         const int32_t* __restrict__ last_octave,
                                                         const float4* __restrict__ cur_kp,  // x, y, angle, octave bits
                                                         const float* __restrict__ cur_ur, const uint4* __restrict__ cur_desc,
                                                         const int32_t* __restrict__ cell_off, const int32_t* __restrict__ cell_idx,
                                                         Cand* __restrict__ cands, int32_t* __restrict__ ncand,
                                                         int32_t* __restrict__ overflow, const uint8_t* __restrict__ observed,
                                                         int32_t* __restrict__ lister) {
    __shared__ int pre_s[kCandWaves][64], beg_s[kCandWaves][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = blockIdx.x * kCandWaves + w;
    if (i >= (n_dev ? *n_dev : P.n_last)) return;  // (device forms: the count the prep kernel clamped)
    int n = 0;
    if (valid[i]) {
        const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        float c[3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            c[r] = __fmaf_rn(P.Tcw[4 * r + 2], z, __fmaf_rn(P.Tcw[4 * r], x, P.Tcw[4 * r + 1] * y)) + P.Tcw[4 * r + 3];
        const float invzc = (float)(1.0 / (double)c[2]);
        const float u = P.fx * c[0] / c[2] + P.cx;
        const float v = P.fy * c[1] / c[2] + P.cy;
        if (!(invzc < 0) && !(u < P.min_x || u > P.max_x || v < P.min_y || v > P.max_y)) {
            const int oct = last_octave[i];
            const float radius = P.th * P.scale[oct];
            int minLevel, maxLevel;
            if (P.bForward) { minLevel = oct; maxLevel = -1; }
            else if (P.bBackward) { minLevel = 0; maxLevel = oct; }
            else { minLevel = oct - 1; maxLevel = oct + 1; }
            const int x0 = max(0, (int)floorf((u - P.min_x - radius) * P.inv_w));
            const int x1 = min(kGridCols - 1, (int)ceilf((u - P.min_x + radius) * P.inv_w));
            const int y0 = max(0, (int)floorf((v - P.min_y - radius) * P.inv_h));
            const int y1 = min(kGridRows - 1, (int)ceilf((v - P.min_y + radius) * P.inv_h));
            if (x0 < kGridCols && x1 >= 0 && y0 < kGridRows && y1 >= 0) {
                const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
                const uint4 d0 = mp_desc[2 * (size_t)i], d1 = mp_desc[2 * (size_t)i + 1];
                const float ur = __fmaf_rn(-P.bf, invzc, u);
                n = window_candidates(lane, pre_s[w], beg_s[w], cell_off, cell_idx, x0, x1, y0, y1,
                                      cands + (size_t)i * P.cap, P.cap, [&](int j) -> int {
                                          const float4 kp = cur_kp[j];
                                          const int koct = __float_as_int(kp.w);
                                          if (bCheckLevels) {
                                              if (koct < minLevel) return -1;
                                              if (maxLevel >= 0 && koct > maxLevel) return -1;
                                          }
                                          const float distx = kp.x - u, disty = kp.y - v;
                                          if (!(fabsf(distx) < radius && fabsf(disty) < radius)) return -1;
                                          if (P.has_ur && cur_ur[j] > 0) {
                                              const float er = fabsf(ur - cur_ur[j]);
                                              if (er > radius) return -1;
                                          }
                                          return hamming(d0, d1, cur_desc[2 * (size_t)j], cur_desc[2 * (size_t)j + 1]);
                                      });
            }
        }
    }
    if (lane == 0) {
        ncand[i] = n;
        if (n > P.cap) atomicMax(overflow, n);
    }
    __threadfence_block();  // the wave's own candidate stores, read back across lanes
    if (observed[i]) record_listers(lane, i, n, P.cap, cands + (size_t)i * P.cap, nullptr, lister);
}
__global__ __launch_bounds__(64 * kCandWaves) void k_proj_candidates(const ProjParams P, const int32_t* __restrict__ n_dev,
                                                         const uint8_t* __restrict__ valid,
                                                         const float* __restrict__ xyz, const uint4* __restrict__ mp_desc,
                                                         const int32_t* __restrict__ last_octave,
                                                         const float4* __restrict__ cur_kp,  // x, y, angle, octave bits
                                                         const float* __restrict__ cur_ur, const uint4* __restrict__ cur_desc,
                                                         const int32_t* __restrict__ cell_off, const int32_t* __restrict__ cell_idx,
                                                         Cand* __restrict__ cands, int32_t* __restrict__ ncand,
                                                         int32_t* __restrict__ overflow, const uint8_t* __restrict__ observed,
                                                         int32_t* __restrict__ lister) {
    k_proj_candidates_body(P, n_dev, valid, xyz, mp_desc, last_octave, cur_kp, cur_ur, cur_desc, cell_off, cell_idx,
                           cands, ncand, overflow, observed, lister);
}
struct k_proj_candidates_args {
    ProjParams P;
    const int32_t* n_dev;
    const uint8_t* valid;
    const float* xyz;
    const uint4* mp_desc;
    const int32_t* last_octave;
    const float4* cur_kp;
    const float* cur_ur;
    const uint4* cur_desc;
    const int32_t* cell_off;
    const int32_t* cell_idx;
    Cand* cands;
    int32_t* ncand;
    int32_t* overflow;
    const uint8_t* observed;
    int32_t* lister;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(64 * kCandWaves) void k_proj_candidates_b(const k_proj_candidates_args* __restrict__ a) {
    const k_proj_candidates_args& A = a[blockIdx.y];
    k_proj_candidates_body(A.P, A.n_dev, A.valid, A.xyz, A.mp_desc, A.last_octave, A.cur_kp, A.cur_ur, A.cur_desc,
                           A.cell_off, A.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.lister);
}

// The same candidate lists with one THREAD per point (round 5): a window holds a handful of cells and
// keypoints, so a wave per point spent most of its time on the 64-lane prefix and compaction machinery;
// a thread walks its window's cells (ix outer, iy inner) and their keypoints in index order, which is
// window_candidates' order, and writes the same list.
template <class Test, class CO = const int32_t*, class CI = const int32_t*>
__device__ __forceinline__ int window_candidates_serial(CO cell_off, CI cell_idx, int x0, int x1, int y0,
                                                        int y1, Cand* __restrict__ out, int cap, Test test) {
    int n = 0;
    for (int ix = x0; ix <= x1; ++ix)
        for (int iy = y0; iy <= y1; ++iy) {
            const int cell = ix * kGridRows + iy;
            const int b = cell_off[cell], e = cell_off[cell + 1];
            for (int k = b; k < e; ++k) {
                const int j = cell_idx[k];
                const int dist = test(j);
                if (dist >= 0) {
                    if (n < cap) out[n] = Cand{j, dist};
                    ++n;
                }
            }
        }
    return n;
}
__device__ __forceinline__ void record_listers_serial(int i, int n, int cap, const Cand* __restrict__ c_i,
                                                      const uint8_t* __restrict__ taken0, int32_t* __restrict__ lister) {
    if (n > cap) return;  // overflow: the call is redone with a larger capacity
    for (int k = 0; k < n; ++k) {
        const Cand c = c_i[k];
        if (c.dist < 256 && !(taken0 && taken0[c.i2])) atomicMin(&lister[c.i2], i);
    }
}

constexpr int kCandThreads = 256;

// (KP / UR / DS / CO / CI: the current frame's records, global pointers or, in the LDS-staged form, LDS ones)
template <class KP = const float4*, class UR = const float*, class DS = const uint4*, class CO = const int32_t*,
          class CI = const int32_t*>
__device__ __forceinline__ void k_proj_candidates_t_body(int i, const ProjParams P, const int32_t* __restrict__ n_dev,
                                                         const uint8_t* __restrict__ valid,
                                                         const float* __restrict__ xyz, const uint4* __restrict__ mp_desc,
                                                         const int32_t* __restrict__ last_octave,
                                                         KP cur_kp, UR cur_ur, DS cur_desc, CO cell_off, CI cell_idx,
                                                         Cand* __restrict__ cands, int32_t* __restrict__ ncand,
                                                         int32_t* __restrict__ overflow, const uint8_t* __restrict__ observed,
                                                         int32_t* __restrict__ lister) {
    if (i >= (n_dev ? *n_dev : P.n_last)) return;
    int n = 0;
    Cand* const out = cands + (size_t)i * P.cap;
    if (valid[i]) {
        const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        float c[3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
            c[r] = __fmaf_rn(P.Tcw[4 * r + 2], z, __fmaf_rn(P.Tcw[4 * r], x, P.Tcw[4 * r + 1] * y)) + P.Tcw[4 * r + 3];
        const float invzc = (float)(1.0 / (double)c[2]);
        const float u = P.fx * c[0] / c[2] + P.cx;
        const float v = P.fy * c[1] / c[2] + P.cy;
        if (!(invzc < 0) && !(u < P.min_x || u > P.max_x || v < P.min_y || v > P.max_y)) {
            const int oct = last_octave[i];
            const float radius = P.th * P.scale[oct];
            int minLevel, maxLevel;
            if (P.bForward) { minLevel = oct; maxLevel = -1; }
            else if (P.bBackward) { minLevel = 0; maxLevel = oct; }
            else { minLevel = oct - 1; maxLevel = oct + 1; }
            const int x0 = max(0, (int)floorf((u - P.min_x - radius) * P.inv_w));
            const int x1 = min(kGridCols - 1, (int)ceilf((u - P.min_x + radius) * P.inv_w));
            const int y0 = max(0, (int)floorf((v - P.min_y - radius) * P.inv_h));
            const int y1 = min(kGridRows - 1, (int)ceilf((v - P.min_y + radius) * P.inv_h));
            if (x0 < kGridCols && x1 >= 0 && y0 < kGridRows && y1 >= 0) {
                const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
                const uint4 d0 = mp_desc[2 * (size_t)i], d1 = mp_desc[2 * (size_t)i + 1];
                const float ur = __fmaf_rn(-P.bf, invzc, u);
                n = window_candidates_serial(cell_off, cell_idx, x0, x1, y0, y1, out, P.cap, [&](int j) -> int {
                    const float4 kp = cur_kp[j];
                    const int koct = __float_as_int(kp.w);
                    if (bCheckLevels) {
                        if (koct < minLevel) return -1;
                        if (maxLevel >= 0 && koct > maxLevel) return -1;
                    }
                    const float distx = kp.x - u, disty = kp.y - v;
                    if (!(fabsf(distx) < radius && fabsf(disty) < radius)) return -1;
                    if (P.has_ur && cur_ur[j] > 0) {
                        const float er = fabsf(ur - cur_ur[j]);
                        if (er > radius) return -1;
                    }
                    return hamming(d0, d1, cur_desc[2 * (size_t)j], cur_desc[2 * (size_t)j + 1]);
                });
            }
        }
    }
    ncand[i] = n;
    if (n > P.cap) atomicMax(overflow, n);
    if (observed[i]) record_listers_serial(i, n, P.cap, out, nullptr, lister);
}
__global__ __launch_bounds__(kCandThreads) void k_proj_candidates_t(const k_proj_candidates_args A) {
    k_proj_candidates_t_body(blockIdx.x * kCandThreads + threadIdx.x, A.P, A.n_dev, A.valid, A.xyz, A.mp_desc, A.last_octave, A.cur_kp, A.cur_ur, A.cur_desc,
                             A.cell_off, A.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.lister);
}
__global__ __launch_bounds__(kCandThreads) void k_proj_candidates_t_b(const k_proj_candidates_args* __restrict__ a) {
    const k_proj_candidates_args& A = a[blockIdx.y];
    k_proj_candidates_t_body(blockIdx.x * kCandThreads + threadIdx.x, A.P, A.n_dev, A.valid, A.xyz, A.mp_desc, A.last_octave, A.cur_kp, A.cur_ur, A.cur_desc,
                             A.cell_off, A.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.lister);
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {
    float rot = a1 - a2;
    if ((double)rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / kHisto));
    if (bin == kHisto) bin = 0;
    return bin;
}

// ---- SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints, thFarPoints), src:46-240 -------

struct LocalParams {
    float min_x, min_y, inv_w, inv_h, th, th_far, nnratio;
    float scale[kMaxLevels];
    int n_cur, n_pts, has_ur, far, nlevels, cap;
};

// one wave per local map point (src:54-143 up to the minima): RadiusByViewingCos, the window at the
// predicted level (levels level-1 .. level), the stereo u_R test, distances
__device__ __forceinline__ void k_lmp_candidates_body(const LocalParams P, const uint8_t* __restrict__ in_view,
                                                        const uint8_t* __restrict__ bad, const float* __restrict__ proj,
                                                        const float* __restrict__ view_cos, const float* __restrict__ depth,
                                                        const int32_t* __restrict__ level, const uint4* __restrict__ mp_desc,
                                                        const float4* __restrict__ cur_kp, const float* __restrict__ cur_ur,
                                                        const uint4* __restrict__ cur_desc, const int32_t* __restrict__ cell_off,
                                                        const int32_t* __restrict__ cell_idx, Cand* __restrict__ cands,
                                                        int32_t* __restrict__ ncand, int32_t* __restrict__ overflow,
                                                        const uint8_t* __restrict__ observed, const uint8_t* __restrict__ taken0,
                                                        int32_t* __restrict__ lister) {
    __shared__ int pre_s[kCandWaves][64], beg_s[kCandWaves][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = blockIdx.x * kCandWaves + w;
    if (i >= P.n_pts) return;
    int n = 0;
    if (in_view[i] && !(P.far && depth[i] > P.th_far) && !bad[i]) {
        const int lvl = level[i];
        float r = ((double)view_cos[i] > 0.998) ? 2.5f : 4.0f;  // RadiusByViewingCos (src:243-250)
        if (P.th != 1.0f) r *= P.th;
        const float radius = r * P.scale[lvl];
        const float x = proj[3 * i], y = proj[3 * i + 1], xr = proj[3 * i + 2];
        const int minLevel = lvl - 1, maxLevel = lvl;
        const int x0 = max(0, (int)floorf((x - P.min_x - radius) * P.inv_w));
        const int x1 = min(kGridCols - 1, (int)ceilf((x - P.min_x + radius) * P.inv_w));
        const int y0 = max(0, (int)floorf((y - P.min_y - radius) * P.inv_h));
        const int y1 = min(kGridRows - 1, (int)ceilf((y - P.min_y + radius) * P.inv_h));
        if (x0 < kGridCols && x1 >= 0 && y0 < kGridRows && y1 >= 0) {
            const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
            const uint4 d0 = mp_desc[2 * (size_t)i], d1 = mp_desc[2 * (size_t)i + 1];
            n = window_candidates(lane, pre_s[w], beg_s[w], cell_off, cell_idx, x0, x1, y0, y1, cands + (size_t)i * P.cap,
                                  P.cap, [&](int j) -> int {
                                      const float4 kp = cur_kp[j];
                                      const int koct = __float_as_int(kp.w);
                                      if (bCheckLevels) {
                                          if (koct < minLevel) return -1;
                                          if (maxLevel >= 0 && koct > maxLevel) return -1;
                                      }
                                      if (!(fabsf(kp.x - x) < radius && fabsf(kp.y - y) < radius)) return -1;
                                      if (P.has_ur && cur_ur[j] > 0) {
                                          const float er = fabsf(xr - cur_ur[j]);
                                          if (er > r * P.scale[lvl]) return -1;
                                      }
                                      return hamming(d0, d1, cur_desc[2 * (size_t)j], cur_desc[2 * (size_t)j + 1]);
                                  });
        }
    }
    if (lane == 0) {
        ncand[i] = n;
        if (n > P.cap) atomicMax(overflow, n);
    }
    __threadfence_block();  // the wave's own candidate stores, read back across lanes
    if (observed[i]) record_listers(lane, i, n, P.cap, cands + (size_t)i * P.cap, taken0, lister);
}
__global__ __launch_bounds__(64 * kCandWaves) void k_lmp_candidates(const LocalParams P, const uint8_t* __restrict__ in_view,
                                                        const uint8_t* __restrict__ bad, const float* __restrict__ proj,
                                                        const float* __restrict__ view_cos, const float* __restrict__ depth,
                                                        const int32_t* __restrict__ level, const uint4* __restrict__ mp_desc,
                                                        const float4* __restrict__ cur_kp, const float* __restrict__ cur_ur,
                                                        const uint4* __restrict__ cur_desc, const int32_t* __restrict__ cell_off,
                                                        const int32_t* __restrict__ cell_idx, Cand* __restrict__ cands,
                                                        int32_t* __restrict__ ncand, int32_t* __restrict__ overflow,
                                                        const uint8_t* __restrict__ observed, const uint8_t* __restrict__ taken0,
                                                        int32_t* __restrict__ lister) {
    k_lmp_candidates_body(P, in_view, bad, proj, view_cos, depth, level, mp_desc, cur_kp, cur_ur, cur_desc, cell_off,
                          cell_idx, cands, ncand, overflow, observed, taken0, lister);
}
struct k_lmp_candidates_args {
    LocalParams P;
    const uint8_t* in_view;
    const uint8_t* bad;
    const float* proj;
    const float* view_cos;
    const float* depth;
    const int32_t* level;
    const uint4* mp_desc;
    const float4* cur_kp;
    const float* cur_ur;
    const uint4* cur_desc;
    const int32_t* cell_off;
    const int32_t* cell_idx;
    Cand* cands;
    int32_t* ncand;
    int32_t* overflow;
    const uint8_t* observed;
    const uint8_t* taken0;
    int32_t* lister;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(64 * kCandWaves) void k_lmp_candidates_b(const k_lmp_candidates_args* __restrict__ a) {
    const k_lmp_candidates_args& A = a[blockIdx.y];
    k_lmp_candidates_body(A.P, A.in_view, A.bad, A.proj, A.view_cos, A.depth, A.level, A.mp_desc, A.cur_kp, A.cur_ur,
                          A.cur_desc, A.cell_off, A.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.taken0,
                          A.lister);
}

template <class KP = const float4*, class UR = const float*, class DS = const uint4*, class CO = const int32_t*,
          class CI = const int32_t*>
__device__ __forceinline__ void k_lmp_candidates_t_body(int i, const LocalParams P, const uint8_t* __restrict__ in_view,
                                                        const uint8_t* __restrict__ bad, const float* __restrict__ proj,
                                                        const float* __restrict__ view_cos, const float* __restrict__ depth,
                                                        const int32_t* __restrict__ level, const uint4* __restrict__ mp_desc,
                                                        KP cur_kp, UR cur_ur, DS cur_desc, CO cell_off, CI cell_idx,
                                                        Cand* __restrict__ cands,
                                                        int32_t* __restrict__ ncand, int32_t* __restrict__ overflow,
                                                        const uint8_t* __restrict__ observed, const uint8_t* __restrict__ taken0,
                                                        int32_t* __restrict__ lister) {
    if (i >= P.n_pts) return;
    int n = 0;
    Cand* const out = cands + (size_t)i * P.cap;
    if (in_view[i] && !(P.far && depth[i] > P.th_far) && !bad[i]) {
        const int lvl = level[i];
        float r = ((double)view_cos[i] > 0.998) ? 2.5f : 4.0f;  // RadiusByViewingCos (src:243-250)
        if (P.th != 1.0f) r *= P.th;
        const float radius = r * P.scale[lvl];
        const float x = proj[3 * i], y = proj[3 * i + 1], xr = proj[3 * i + 2];
        const int minLevel = lvl - 1, maxLevel = lvl;
        const int x0 = max(0, (int)floorf((x - P.min_x - radius) * P.inv_w));
        const int x1 = min(kGridCols - 1, (int)ceilf((x - P.min_x + radius) * P.inv_w));
        const int y0 = max(0, (int)floorf((y - P.min_y - radius) * P.inv_h));
        const int y1 = min(kGridRows - 1, (int)ceilf((y - P.min_y + radius) * P.inv_h));
        if (x0 < kGridCols && x1 >= 0 && y0 < kGridRows && y1 >= 0) {
            const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
            const uint4 d0 = mp_desc[2 * (size_t)i], d1 = mp_desc[2 * (size_t)i + 1];
            n = window_candidates_serial(cell_off, cell_idx, x0, x1, y0, y1, out, P.cap, [&](int j) -> int {
                const float4 kp = cur_kp[j];
                const int koct = __float_as_int(kp.w);
                if (bCheckLevels) {
                    if (koct < minLevel) return -1;
                    if (maxLevel >= 0 && koct > maxLevel) return -1;
                }
                if (!(fabsf(kp.x - x) < radius && fabsf(kp.y - y) < radius)) return -1;
                if (P.has_ur && cur_ur[j] > 0) {
                    const float er = fabsf(xr - cur_ur[j]);
                    if (er > r * P.scale[lvl]) return -1;
                }
                return hamming(d0, d1, cur_desc[2 * (size_t)j], cur_desc[2 * (size_t)j + 1]);
            });
        }
    }
    ncand[i] = n;
    if (n > P.cap) atomicMax(overflow, n);
    if (observed[i]) record_listers_serial(i, n, P.cap, out, taken0, lister);
}
__global__ __launch_bounds__(kCandThreads) void k_lmp_candidates_t(const k_lmp_candidates_args A) {
    k_lmp_candidates_t_body(blockIdx.x * kCandThreads + threadIdx.x, A.P, A.in_view, A.bad, A.proj, A.view_cos, A.depth, A.level, A.mp_desc, A.cur_kp, A.cur_ur,
                            A.cur_desc, A.cell_off, A.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.taken0,
                            A.lister);
}
__global__ __launch_bounds__(kCandThreads) void k_lmp_candidates_t_b(const k_lmp_candidates_args* __restrict__ a) {
    const k_lmp_candidates_args& A = a[blockIdx.y];
    k_lmp_candidates_t_body(blockIdx.x * kCandThreads + threadIdx.x, A.P, A.in_view, A.bad, A.proj, A.view_cos, A.depth, A.level, A.mp_desc, A.cur_kp, A.cur_ur,
                            A.cur_desc, A.cell_off, A.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.taken0,
                            A.lister);
}

// LDS-staged batch forms (round 6).  The thread forms above walk a window as a chain of dependent
// global loads per candidate (cell offsets -> keypoint index -> keypoint record -> descriptor); with a
// batch those records are spread over hundreds of frames and miss the caches.  Here one 1024-thread
// workgroup per frame first copies the frame's grid (cell offsets, cell index list) and its keypoint
// records (x, y, angle, octave; u_R; descriptors: all `cap` rows, the frame's padding included) into
// LDS, then every thread walks its points' windows with the same code -- the same lists in the same
// order, the chain now on LDS.  LDS: 56 B per keypoint + the 3,073 cell offsets (cap <= kCandLdsCap).
constexpr int kCandLdsThreads = 1024;
constexpr int kCandLdsCap = (160 * 1024 - 4 * (kGridCols * kGridRows + 1)) / 56;
__host__ __device__ constexpr size_t cand_lds_bytes(int cap) {
    return (size_t)cap * (32 + 16 + 4 + 4) + 4 * (size_t)(kGridCols * kGridRows + 1);
}
// Readers of the staged records through address-space-3 pointers, so that the walk issues ds_read
// (the compiler does not infer the address space through the generic pointers otherwise: flat loads)
#define ORB_LDS __attribute__((address_space(3)))
struct LdsF4 {
    const ORB_LDS float* p;
    __device__ float4 operator[](int j) const { const ORB_LDS float* q = p + 4 * j; return make_float4(q[0], q[1], q[2], q[3]); }
};
struct LdsU4 {
    const ORB_LDS uint32_t* p;
    __device__ uint4 operator[](size_t j) const { const ORB_LDS uint32_t* q = p + 4 * j; return make_uint4(q[0], q[1], q[2], q[3]); }
};
template <class T>
struct LdsArr {
    const ORB_LDS T* p;
    __device__ T operator[](int k) const { return p[k]; }
};
struct CandLds {
    LdsU4 desc;
    LdsF4 kp;
    LdsArr<float> ur;
    LdsArr<int32_t> cell_idx;
    LdsArr<int32_t> cell_off;
};
// descriptors | keypoint records | u_R | cell index list | cell offsets (16-B aligned sections); the
// first `rows` keypoint rows are staged (the cell offsets always)
__device__ __forceinline__ CandLds stage_frame_lds(uint8_t* smem, int cap, const float4* __restrict__ kp,
                                                   const float* __restrict__ ur, const uint4* __restrict__ desc,
                                                   const int32_t* __restrict__ cell_off, const int32_t* __restrict__ cell_idx,
                                                   int rows) {
    uint4* s_desc = reinterpret_cast<uint4*>(smem);
    float4* s_kp = reinterpret_cast<float4*>(smem + 32 * (size_t)cap);
    float* s_ur = reinterpret_cast<float*>(smem + 48 * (size_t)cap);
    int32_t* s_idx = reinterpret_cast<int32_t*>(smem + 52 * (size_t)cap);
    int32_t* s_off = reinterpret_cast<int32_t*>(smem + 56 * (size_t)cap);
    const int t = threadIdx.x;
    for (int k = t; k < 2 * rows; k += kCandLdsThreads) s_desc[k] = desc[k];
    for (int k = t; k < rows; k += kCandLdsThreads) {
        s_kp[k] = kp[k];
        s_idx[k] = cell_idx[k];
        if (ur) s_ur[k] = ur[k];
    }
    for (int k = t; k <= kGridCols * kGridRows; k += kCandLdsThreads) s_off[k] = cell_off[k];
    __syncthreads();
    // (u_R is read only when the frame has it, ProjParams / LocalParams has_ur)
    return CandLds{LdsU4{(const ORB_LDS uint32_t*)s_desc}, LdsF4{(const ORB_LDS float*)s_kp}, LdsArr<float>{(const ORB_LDS float*)s_ur},
                   LdsArr<int32_t>{(const ORB_LDS int32_t*)s_idx}, LdsArr<int32_t>{(const ORB_LDS int32_t*)s_off}};
}
// ---- the in-order assignment, resolved by parallel fixed-point rounds ----------------------------
// Both SearchByProjection loops visit the points in index order, and point i only sees the state the
// earlier points left: a current keypoint that holds a map point with observations is skipped
// (src:103-105, src:2040-2042).  That state changes once per keypoint -- the first successful
// assignment by an observed point -- so point i's answer is a function f_i of which of its candidates
// earlier observed points claimed:
//   A(i) = f_i({ j : some k < i, observed(k), A(k) = j }).
// One workgroup iterates this map on all points at once (Jacobi): every round computes claimMin[j] =
// the smallest observed point whose current answer is j, then every point re-derives its answer with
// the candidates claimed by an earlier point excluded.  A fixed point is the sequential answer (by
// induction on i), and after round r the first r points are final, so the iteration ends; in practice
// after a few rounds more than the longest chain of actual claim conflicts.  The results are then
// exactly those of the sequential loop:
//   mp[j]  = the last point assigned to keypoint j (a later unobserved-free assignment overwrites an
//            earlier one, src:156 / :2067), or -1;
//   count  = every successful assignment (the reference's nmatches++ per assignment), minus, for
//            SearchByProjection(Frame, Frame) with checkOri, every assignment in a rotation bin outside
//            ComputeThreeMaxima's top three, whose keypoint is then cleared (src:2160-2181).
// The candidate kernels store each point's candidates in the reference's scan order (the order key of
// a candidate is its list position) with their Hamming distances; the first / second minimum of the
// reference's update rules (src:126-142, :2057-2061) are the lexicographic (distance, order) minima.
constexpr int kResolveThreads = 1024, kResolveLdsKeypoints = 16384;
constexpr unsigned long long kNone = ~0ull;
constexpr int kTop = 8;  // best usable candidates kept per point for the rounds

struct ResolveArgs {
    int n_pts, n_cur, cap;
    int local;          // 1: best + second best with the ratio test (src:145-167); 0: best only (src:2064-2068)
    int check_ori;      // rotation histogram (SearchByProjection(Frame, Frame) only)
    float nnratio;
    const Cand* cands;
    const int32_t* ncand;
    const uint8_t* observed;   // per point: its map point has Observations() > 0
    const uint8_t* taken0;     // per keypoint: holds a map point with observations before the call (may be null)
    const float4* cur_kp;      // x, y, angle, octave bits
    const float* last_angle;   // per point (rotation bins)
    const int32_t* overflow;   // the candidate pass's overflow (> cap: results not written)
    int32_t* st;               // per point: the current answer, -1 no match, j >= 0 keypoint j
    int lds_keypoints;         // 1: claimMin in LDS (dynamic, 4 B per keypoint)
    int32_t* claimMin;         // per keypoint (when not in LDS)
    const int32_t* lister;     // per keypoint: the first observed point listing it (candidate kernels)
    int32_t* fixed;            // per keypoint: the smallest final (unaffected) observed claimant (0x7f.. none)
    int32_t* work;             // the points whose answer can change (the rounds' list), count in out_n[2]
    int4* top;                 // per point: its kTop best usable candidates as (dist, i2) pairs, by (dist, order)
    int32_t* nusable;          // per point: its usable candidate count
    int32_t* last;             // per keypoint
    int32_t* removed;          // per keypoint
    int32_t* mp;               // out: per keypoint
    int32_t* out_n;            // out: [0] count, [1] rounds
    int32_t* out_user;         // out (device forms, may be null): the count, for the caller
    const int32_t* dims;       // device forms: [0] n_pts, [1] n_cur read on the device (NULL: the fields above)
};

// a candidate resolve_point can take (the lister pass counts exactly these)
__device__ __forceinline__ bool usable(const ResolveArgs& a, const Cand& c) {
    return c.dist < 256 && !(a.taken0 && a.taken0[c.i2]);
}

// Visit point i's usable candidates in list order, fn(candidate, position).  The list is read 8
// entries at a time (and their taken0 bytes 8 at a time), so a thread keeps 8 loads in flight instead
// of one dependent round trip per candidate.
template <class Fn>
__device__ __forceinline__ void for_each_usable(const ResolveArgs& a, int i, Fn fn) {
    const Cand* C = a.cands + (size_t)i * a.cap;
    const int n = a.ncand[i];
    for (int k0 = 0; k0 < n; k0 += 8) {
        Cand cs[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) cs[u] = k0 + u < n ? C[k0 + u] : Cand{0, 256};
        bool tk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) tk[u] = a.taken0 && cs[u].dist < 256 && a.taken0[cs[u].i2];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (cs[u].dist < 256 && !tk[u]) fn(cs[u], k0 + u);  // dist >= 256: never below the initial 256
    }
}

// point i's answer given claimMin (candidates claimed by an earlier point excluded): the first and
// second minimum of (distance, list position), the reference's update order
__device__ __forceinline__ int resolve_point(const ResolveArgs& a, const int32_t* claimMin, int i) {
    unsigned long long m1 = kNone, m2 = kNone;
    int j1 = -1, j2 = -1;
    for_each_usable(a, i, [&](const Cand& c, int k) {  // (selects, no branches: the state stays in registers)
        const bool ok = claimMin[c.i2] >= i;
        const unsigned long long key = ((unsigned long long)c.dist << 32) | (unsigned)k;
        const bool lt1 = ok && key < m1, lt2 = ok && key < m2;
        m2 = lt1 ? m1 : (lt2 ? key : m2);
        j2 = lt1 ? j1 : (lt2 ? c.i2 : j2);
        m1 = lt1 ? key : m1;
        j1 = lt1 ? c.i2 : j1;
    });
    if (m1 == kNone) return -1;
    const int d1 = (int)(m1 >> 32);
    if (d1 > kThHigh) return -1;
    if (a.local) {  // src:148-155
        const int l1 = __float_as_int(a.cur_kp[j1].w);
        const int l2 = m2 != kNone ? __float_as_int(a.cur_kp[j2].w) : -1;
        const int d2 = m2 != kNone ? (int)(m2 >> 32) : 256;
        if (l1 == l2 && (float)d1 > a.nnratio * (float)d2) return -1;
    }
    return j1;
}

// The answer rules (src:145-167 / :2064-2068) given the first and second unclaimed candidates.
__device__ __forceinline__ int decide(const ResolveArgs& a, int d1, int j1, int d2, int j2) {
    if (j1 < 0 || d1 > kThHigh) return -1;
    if (a.local) {  // src:148-155
        const int l1 = __float_as_int(a.cur_kp[j1].w);
        const int l2 = j2 >= 0 ? __float_as_int(a.cur_kp[j2].w) : -1;
        if (l1 == l2 && (float)d1 > a.nnratio * (float)(j2 >= 0 ? d2 : 256)) return -1;
    }
    return j1;
}

// Points that cannot be affected are taken out of the rounds: point i can only lose a candidate j to
// an observed point k < i that has j among its usable candidates, so if every usable candidate of i
// has no such earlier lister, i's unconstrained answer is final, and its claim is fixed.
// k_resolve_init (one thread per point, over the whole chip): the unconstrained answer, the point's
// kTop best usable candidates in (distance, order), the classification, the work list and the fixed
// claims.  k_resolve_rounds (one workgroup) then iterates only the work list, each point re-deciding
// from its kTop best (a full scan only when too many of them are claimed).
__device__ __forceinline__ void resolve_init_point(const ResolveArgs& a, int i) {
    unsigned long long t[kTop];
    int ti[kTop];
#pragma unroll
    for (int q = 0; q < kTop; ++q) { t[q] = kNone; ti[q] = -1; }
    int nu = 0;
    bool affected = false;
    for_each_usable(a, i, [&](const Cand& c, int k) {
        ++nu;
        affected |= a.lister[c.i2] < i;
        unsigned long long key = ((unsigned long long)c.dist << 32) | (unsigned)k;
        int j = c.i2;
#pragma unroll
        for (int q = 0; q < kTop; ++q) {  // insertion into the sorted kTop (selects only)
            const bool lt = key < t[q];
            const unsigned long long tk = t[q];
            const int tj = ti[q];
            t[q] = lt ? key : tk;
            ti[q] = lt ? j : tj;
            key = lt ? tk : key;
            j = lt ? tj : j;
        }
    });
    const int st = decide(a, (int)(t[0] >> 32), ti[0], (int)(t[1] >> 32), ti[1]);
    a.st[i] = st;
#pragma unroll
    for (int q = 0; q < kTop; q += 2)
        a.top[(size_t)i * (kTop / 2) + q / 2] = make_int4((int)(t[q] >> 32), ti[q], (int)(t[q + 1] >> 32), ti[q + 1]);
    a.nusable[i] = nu;
    if (affected) a.work[atomicAdd(&a.out_n[2], 1)] = i;
    else if (st >= 0 && a.observed[i]) atomicMin(&a.fixed[st], i);
}
__device__ __forceinline__ void k_resolve_init_body(ResolveArgs a) {
    if (a.dims) {
        a.n_pts = a.dims[0];
        a.n_cur = a.dims[1];
    }
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n_pts || *a.overflow > a.cap) return;
    resolve_init_point(a, i);
}
__global__ __launch_bounds__(256) void k_resolve_init(ResolveArgs a) {
    k_resolve_init_body(a);
}
struct k_resolve_init_args {
    ResolveArgs a;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(256) void k_resolve_init_b(const k_resolve_init_args* __restrict__ a) {
    const k_resolve_init_args& A = a[blockIdx.y];
    k_resolve_init_body(A.a);
}

// The LDS-staged candidate passes of a batch (one workgroup per frame).  (Running k_resolve_init's
// per-point pass in the same launch, after the frame's listers are final, was measured slower: 2.14 ->
// 2.62 ms per 512-frame call -- one CU per frame instead of the whole chip.)
__global__ __launch_bounds__(kCandLdsThreads) void k_proj_candidates_l_b(const k_proj_candidates_args* __restrict__ a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t cand_smem[];
    const k_proj_candidates_args& A = a[blockIdx.x];
    const int np = A.n_dev ? *A.n_dev : A.P.n_last;
    if (np == 0) return;  // (a frame the motion gate turned off: nothing to stage)
    const CandLds S = stage_frame_lds(cand_smem, A.P.cap, A.cur_kp, A.cur_ur, A.cur_desc, A.cell_off, A.cell_idx, A.P.cap);
    for (int i = threadIdx.x; i < np; i += kCandLdsThreads)
        k_proj_candidates_t_body(i, A.P, A.n_dev, A.valid, A.xyz, A.mp_desc, A.last_octave, S.kp, S.ur, S.desc, S.cell_off,
                                 S.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.lister);
}
__global__ __launch_bounds__(kCandLdsThreads) void k_lmp_candidates_l_b(const k_lmp_candidates_args* __restrict__ a,
                                                                        const k_resolve_init_args* __restrict__ ri) {
    extern __shared__ __attribute__((aligned(16))) uint8_t cand_smem[];
    const k_lmp_candidates_args& A = a[blockIdx.x];
    const ResolveArgs& R = ri[blockIdx.x].a;
    if (A.P.n_pts == 0) return;
    // a frame without keypoints (the motion gate's failed frames) stages only its (empty) grid
    const CandLds S = stage_frame_lds(cand_smem, A.P.cap, A.cur_kp, A.cur_ur, A.cur_desc, A.cell_off, A.cell_idx,
                                      R.dims && R.dims[1] == 0 ? 0 : A.P.cap);
    for (int i = threadIdx.x; i < A.P.n_pts; i += kCandLdsThreads)
        k_lmp_candidates_t_body(i, A.P, A.in_view, A.bad, A.proj, A.view_cos, A.depth, A.level, A.mp_desc, S.kp, S.ur,
                                S.desc, S.cell_off, S.cell_idx, A.cands, A.ncand, A.overflow, A.observed, A.taken0,
                                A.lister);
}

// point i's answer in a round, from its kTop best (claims by earlier points excluded)
__device__ __forceinline__ int resolve_top(const ResolveArgs& a, const int32_t* claimMin, int i) {
    int d1 = 0, j1 = -1, d2 = 0, j2 = -1, found = 0;
#pragma unroll
    for (int q = 0; q < kTop; q += 2) {
        const int4 e = a.top[(size_t)i * (kTop / 2) + q / 2];
        const int d[2] = {e.x, e.z}, j[2] = {e.y, e.w};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (j[u] < 0 || claimMin[j[u]] < i) continue;
            if (found == 0) { d1 = d[u]; j1 = j[u]; }
            else if (found == 1) { d2 = d[u]; j2 = j[u]; }
            ++found;
        }
    }
    const int need = a.local ? 2 : 1;
    if (found < need && a.nusable[i] > kTop) return resolve_point(a, claimMin, i);
    return decide(a, d1, j1, d2, j2);
}

// A work point's round state in registers: its kTop best (keypoint, distance, level), usable count,
// index, observed flag and current answer; the rounds then touch only LDS.
struct WorkPoint {
    int i, st, nu, obs;
    uint32_t e[kTop];  // keypoint (16 bits) | distance << 16 (8 bits) | (level + 1) << 24; 0xffffffff: none
};
constexpr int kWorkPerThread = 2;

__device__ __forceinline__ void load_work(const ResolveArgs& a, int i, WorkPoint& p) {
    p.i = i;
    p.st = a.st[i];
    p.nu = a.nusable[i];
    p.obs = a.observed[i];
    int d[kTop], j[kTop];
#pragma unroll
    for (int q = 0; q < kTop; q += 2) {
        const int4 t = a.top[(size_t)i * (kTop / 2) + q / 2];
        d[q] = t.x; j[q] = t.y; d[q + 1] = t.z; j[q + 1] = t.w;
    }
#pragma unroll
    for (int q = 0; q < kTop; ++q) {  // octaves are 0 .. 11, distances < 256, keypoints < 65536
        const int l1 = (a.local && j[q] >= 0) ? __float_as_int(a.cur_kp[j[q]].w) + 1 : 0;
        p.e[q] = j[q] < 0 ? 0xffffffffu : (uint32_t)j[q] | (uint32_t)d[q] << 16 | (uint32_t)l1 << 24;
    }
}

// resolve_top on a register-resident work point (same rules; the full scan when its kTop best run out)
__device__ __forceinline__ int resolve_reg(const ResolveArgs& a, const int32_t* claimMin, const WorkPoint& p) {
    uint32_t e1 = 0xffffffffu, e2 = 256u << 16;  // (e2 default: distance 256, level -1)
    int found = 0;
#pragma unroll
    for (int q = 0; q < kTop; ++q) {
        const bool ok = p.e[q] != 0xffffffffu && claimMin[p.e[q] & 0xffffu] >= p.i;
        if (ok && found == 0) e1 = p.e[q];
        else if (ok && found == 1) e2 = p.e[q];
        found += ok ? 1 : 0;
    }
    if (found < (a.local ? 2 : 1) && p.nu > kTop) return resolve_point(a, claimMin, p.i);
    if (found == 0) return -1;
    const int j1 = (int)(e1 & 0xffffu), d1 = (int)((e1 >> 16) & 0xffu), l1 = (int)(e1 >> 24) - 1;
    const int d2 = found > 1 ? (int)((e2 >> 16) & 0xffu) : 256, l2 = found > 1 ? (int)(e2 >> 24) - 1 : -1;
    if (d1 > kThHigh) return -1;
    if (a.local && l1 == l2 && (float)d1 > a.nnratio * (float)d2) return -1;  // src:148-155
    return j1;
}

__device__ __forceinline__ void k_resolve_rounds_body(ResolveArgs a) {
    if (a.dims) {
        a.n_pts = a.dims[0];
        a.n_cur = a.dims[1];
    }
    const int tid = threadIdx.x;
    __shared__ int hist[kHisto], keep[3], cnt[2];
    extern __shared__ int32_t kp_lds[];
    int32_t* const claimMin = a.lds_keypoints ? kp_lds : a.claimMin;
    if (*a.overflow > a.cap) {  // the host re-runs with a larger capacity
        if (tid == 0) *a.out_n = -1;
        return;
    }
    for (int j = tid; j < a.n_cur; j += kResolveThreads) {
        a.last[j] = -1;
        a.removed[j] = 0;
    }
    if (tid < kHisto) hist[tid] = 0;
    if (tid < 2) cnt[tid] = 0;
    const int nw = a.out_n[2];
    int rounds = 1;
    if (nw <= kWorkPerThread * kResolveThreads && a.n_cur <= 65536) {
        // the usual case: every work point in registers, the fixed claims in LDS next to claimMin
        int32_t* const fixedL = a.lds_keypoints ? kp_lds + a.n_cur : a.fixed;
        WorkPoint wp[kWorkPerThread];
#pragma unroll
        for (int q = 0; q < kWorkPerThread; ++q) {
            const int w = tid + q * kResolveThreads;
            wp[q].i = -1;
            if (w < nw) load_work(a, a.work[w], wp[q]);
        }
        if (a.lds_keypoints)
            for (int j = tid; j < a.n_cur; j += kResolveThreads) fixedL[j] = a.fixed[j];
        for (;; ++rounds) {
            __syncthreads();
            for (int j = tid; j < a.n_cur; j += kResolveThreads) claimMin[j] = fixedL[j];
            __syncthreads();
#pragma unroll
            for (int q = 0; q < kWorkPerThread; ++q)
                if (wp[q].i >= 0 && wp[q].st >= 0 && wp[q].obs) atomicMin(&claimMin[wp[q].st], wp[q].i);
            __syncthreads();
            int changed = 0;
#pragma unroll
            for (int q = 0; q < kWorkPerThread; ++q) {
                if (wp[q].i < 0) continue;
                const int r = resolve_reg(a, claimMin, wp[q]);
                changed += r != wp[q].st;
                wp[q].st = r;
            }
            if (__syncthreads_count(changed) == 0 || rounds > a.n_pts) break;
        }
#pragma unroll
        for (int q = 0; q < kWorkPerThread; ++q)
            if (wp[q].i >= 0) a.st[wp[q].i] = wp[q].st;
        __syncthreads();  // (global st: visible to the workgroup's results pass below)
    } else {
        for (;; ++rounds) {
            __syncthreads();
            for (int j = tid; j < a.n_cur; j += kResolveThreads) claimMin[j] = a.fixed[j];
            __syncthreads();
            for (int w = tid; w < nw; w += kResolveThreads) {
                const int i = a.work[w], j = a.st[i];
                if (j >= 0 && a.observed[i]) atomicMin(&claimMin[j], i);
            }
            __syncthreads();
            int changed = 0;
            for (int w = tid; w < nw; w += kResolveThreads) {
                const int i = a.work[w];
                const int r = resolve_top(a, claimMin, i);
                if (r != a.st[i]) {
                    a.st[i] = r;
                    ++changed;
                }
            }
            if (__syncthreads_count(changed) == 0 || rounds > a.n_pts) break;
        }
    }
    // results
    int nsucc = 0;
    for (int i = tid; i < a.n_pts; i += kResolveThreads) {
        const int j = a.st[i];
        if (j < 0) continue;
        ++nsucc;
        atomicMax(&a.last[j], i);
        if (a.check_ori) atomicAdd(&hist[rot_bin(a.last_angle[i], a.cur_kp[j].z)], 1);
    }
    atomicAdd(&cnt[0], nsucc);
    __syncthreads();
    if (a.check_ori) {
        if (tid == 0) {  // ComputeThreeMaxima (src:2336-2378)
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
        int nrem = 0;
        for (int i = tid; i < a.n_pts; i += kResolveThreads) {
            const int j = a.st[i];
            if (j < 0) continue;
            const int b = rot_bin(a.last_angle[i], a.cur_kp[j].z);
            if (b != keep[0] && b != keep[1] && b != keep[2]) {
                a.removed[j] = 1;
                ++nrem;
            }
        }
        atomicAdd(&cnt[1], nrem);
        __syncthreads();
    }
    for (int j = tid; j < a.n_cur; j += kResolveThreads) a.mp[j] = a.removed[j] ? -1 : a.last[j];
    if (tid == 0) {
        a.out_n[0] = cnt[0] - cnt[1];
        a.out_n[1] = rounds;
        a.out_n[2] = nw;
        if (a.out_user) a.out_user[0] = cnt[0] - cnt[1];
    }
}
__global__ __launch_bounds__(kResolveThreads) void k_resolve_rounds(ResolveArgs a) {
    k_resolve_rounds_body(a);
}
struct k_resolve_rounds_args {
    ResolveArgs a;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(kResolveThreads) void k_resolve_rounds_b(const k_resolve_rounds_args* __restrict__ a) {
    const k_resolve_rounds_args& A = a[blockIdx.y];
    k_resolve_rounds_body(A.a);
}

// ---- device-resident forms: the frame's grid and packed keypoints built on the device ------------

// scratch initialisation done by k_frame_prep (the device forms launch no fills): fill_7f (lister /
// fixed claims) with 0x7f7f7f7f, fill_m1 (the match array) with -1, the 4 overflow / counter words
// zero, and dims[0] = dims0 when dims0 >= 0 (the local-map form's point count)
struct ScratchInit {
    int32_t* fill_7f;
    int n_7f;
    int32_t* fill_m1;
    int n_m1;
    int32_t* zero4;
    int32_t* dims;
    int dims0;
};

// Frame::AssignFeaturesToGrid (src/Frame.cc:1418-1440) on a device frame, one workgroup: cell
// (round((x - mnMinX) inv_w), round((y - mnMinY) inv_h)), keypoints in index order inside each cell
// (counting sort, then each cell's few entries put back in index order); the (x, y, angle, octave) float4
// rows the candidate kernels read; the clamped count into n_out[0] and n_out[1].  The counts, offsets
// and (up to kPrepLds keypoints) the cell lists are built in LDS and written out once; a thread keeps its
// keypoints' cells in registers.
constexpr int kPrepThreads = 1024, kCells = kGridCols * kGridRows, kPrepLds = 8192;
constexpr int kPrepPer = 16;  // keypoints per thread: cap <= 16384
__device__ __forceinline__ void k_frame_prep_body(const orb_keypoint_t* __restrict__ kps,
                                                             const int32_t* __restrict__ n_ptr, int cap, float min_x,
                                                             float min_y, float inv_w, float inv_h,
                                                             float4* __restrict__ kp4, int32_t* __restrict__ cell_off,
                                                             int32_t* __restrict__ cell_idx, int32_t* __restrict__ cell_of,
                                                             int32_t* n_out0, int32_t* n_out1, ScratchInit z) {
    __shared__ int cnt[kCells];       // counts, then fill cursors
    __shared__ int off[kCells + 1];   // cell offsets
    __shared__ int wtot[kPrepThreads / 64];
    __shared__ int sidx[kPrepLds];    // the cell lists (n <= kPrepLds)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = min(max(*n_ptr, 0), cap);
    const bool lds = n <= kPrepLds;
    int* const idx = lds ? sidx : cell_idx;
    // the call's scratch words, in place of fill launches (the later kernels of the call read them)
    for (int i = tid; i < z.n_7f; i += kPrepThreads) z.fill_7f[i] = 0x7f7f7f7f;
    for (int i = tid; i < z.n_m1; i += kPrepThreads) z.fill_m1[i] = -1;
    if (tid < 4) z.zero4[tid] = 0;
    if (tid == 0 && z.dims0 >= 0) z.dims[0] = z.dims0;
    for (int c = tid; c < kCells; c += kPrepThreads) cnt[c] = 0;
    __syncthreads();
    int mine[kPrepPer];
#pragma unroll
    for (int k = 0; k < kPrepPer; ++k) {
        const int i = tid + k * kPrepThreads;
        int cell = -1;
        if (i < n) {
            const orb_keypoint_t kp = kps[i];
            kp4[i] = make_float4(kp.x, kp.y, kp.angle, __int_as_float(kp.octave));
            const int px = (int)roundf((kp.x - min_x) * inv_w);
            const int py = (int)roundf((kp.y - min_y) * inv_h);
            if (px >= 0 && px < kGridCols && py >= 0 && py < kGridRows) {
                cell = px * kGridRows + py;
                atomicAdd(&cnt[cell], 1);
            }
            cell_of[i] = cell;
        }
        mine[k] = cell;
    }
    __syncthreads();
    // exclusive scan of the 3072 counts: three cells per thread, a wave scan, the wave totals
    constexpr int kPer = kCells / kPrepThreads;
    static_assert(kCells % kPrepThreads == 0, "cells per thread");
    int loc[kPer], sum = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        loc[q] = sum;
        sum += cnt[tid * kPer + q];
    }
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int w = 0; w < wv; ++w) base += wtot[w];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        off[tid * kPer + q] = base + loc[q];
        cnt[tid * kPer + q] = base + loc[q];  // becomes the fill cursor
    }
    if (tid == kPrepThreads - 1) off[kCells] = base + sum;
    if (tid == 0) {
        *n_out0 = n;
        if (n_out1) *n_out1 = n;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPrepPer; ++k)
        if (mine[k] >= 0) idx[atomicAdd(&cnt[mine[k]], 1)] = tid + k * kPrepThreads;
    __threadfence_block();
    __syncthreads();
    for (int c = tid; c < kCells; c += kPrepThreads) {  // index order inside each cell (insertion sort)
        const int b = off[c], e = off[c + 1];
        for (int a = b + 1; a < e; ++a) {
            const int v = idx[a];
            int k = a;
            for (; k > b && idx[k - 1] > v; --k) idx[k] = idx[k - 1];
            idx[k] = v;
        }
    }
    for (int c = tid; c <= kCells; c += kPrepThreads) cell_off[c] = off[c];
    if (lds) {
        __syncthreads();
        for (int i = tid; i < n; i += kPrepThreads) cell_idx[i] = sidx[i];
    }
}
__global__ __launch_bounds__(kPrepThreads) void k_frame_prep(const orb_keypoint_t* __restrict__ kps,
                                                             const int32_t* __restrict__ n_ptr, int cap, float min_x,
                                                             float min_y, float inv_w, float inv_h,
                                                             float4* __restrict__ kp4, int32_t* __restrict__ cell_off,
                                                             int32_t* __restrict__ cell_idx, int32_t* __restrict__ cell_of,
                                                             int32_t* n_out0, int32_t* n_out1, ScratchInit z) {
    k_frame_prep_body(kps, n_ptr, cap, min_x, min_y, inv_w, inv_h, kp4, cell_off, cell_idx, cell_of, n_out0, n_out1, z);
}
struct k_frame_prep_args {
    const orb_keypoint_t* kps;
    const int32_t* n_ptr;
    int cap;
    float min_x;
    float min_y;
    float inv_w;
    float inv_h;
    float4* kp4;
    int32_t* cell_off;
    int32_t* cell_idx;
    int32_t* cell_of;
    int32_t* n_out0;
    int32_t* n_out1;
    ScratchInit z;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(kPrepThreads) void k_frame_prep_b(const k_frame_prep_args* __restrict__ a) {
    const k_frame_prep_args& A = a[blockIdx.y];
    k_frame_prep_body(A.kps, A.n_ptr, A.cap, A.min_x, A.min_y, A.inv_w, A.inv_h, A.kp4, A.cell_off, A.cell_idx,
                      A.cell_of, A.n_out0, A.n_out1, A.z);
}

// the last frame's per-point inputs of k_proj_candidates / the rotation bins: a point whose octave is
// outside the pyramid is not valid (the host form rejects the call instead)
__device__ __forceinline__ void k_last_prep_body(const orb_keypoint_t* __restrict__ kps, const uint8_t* __restrict__ valid,
                                                   const int32_t* __restrict__ n_ptr, int cap, int nlevels,
                                                   uint8_t* __restrict__ valid2, int32_t* __restrict__ octave,
                                                   float* __restrict__ angle, int32_t* n_out0, int32_t* n_out1) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = min(max(*n_ptr, 0), cap);
    if (i == 0) {
        *n_out0 = n;
        if (n_out1) *n_out1 = n;
    }
    if (i >= n) return;
    const orb_keypoint_t kp = kps[i];
    octave[i] = kp.octave;
    angle[i] = kp.angle;
    valid2[i] = valid[i] && kp.octave >= 0 && kp.octave < nlevels;
}
__global__ __launch_bounds__(256) void k_last_prep(const orb_keypoint_t* __restrict__ kps, const uint8_t* __restrict__ valid,
                                                   const int32_t* __restrict__ n_ptr, int cap, int nlevels,
                                                   uint8_t* __restrict__ valid2, int32_t* __restrict__ octave,
                                                   float* __restrict__ angle, int32_t* n_out0, int32_t* n_out1) {
    k_last_prep_body(kps, valid, n_ptr, cap, nlevels, valid2, octave, angle, n_out0, n_out1);
}
struct k_last_prep_args {
    const orb_keypoint_t* kps;
    const uint8_t* valid;
    const int32_t* n_ptr;
    int cap;
    int nlevels;
    uint8_t* valid2;
    int32_t* octave;
    float* angle;
    int32_t* n_out0;
    int32_t* n_out1;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(256) void k_last_prep_b(const k_last_prep_args* __restrict__ a) {
    const k_last_prep_args& A = a[blockIdx.y];
    k_last_prep_body(A.kps, A.valid, A.n_ptr, A.cap, A.nlevels, A.valid2, A.octave, A.angle, A.n_out0, A.n_out1);
}

// local map points: a predicted level outside the pyramid leaves the point out
__device__ __forceinline__ void k_local_prep_body(const uint8_t* __restrict__ in_view, const int32_t* __restrict__ level,
                                                    int n, int nlevels, uint8_t* __restrict__ in_view2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) in_view2[i] = in_view[i] && level[i] >= 0 && level[i] < nlevels;
}
__global__ __launch_bounds__(256) void k_local_prep(const uint8_t* __restrict__ in_view, const int32_t* __restrict__ level,
                                                    int n, int nlevels, uint8_t* __restrict__ in_view2) {
    k_local_prep_body(in_view, level, n, nlevels, in_view2);
}
struct k_local_prep_args {
    const uint8_t* in_view;
    const int32_t* level;
    int n;
    int nlevels;
    uint8_t* in_view2;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(256) void k_local_prep_b(const k_local_prep_args* __restrict__ a) {
    const k_local_prep_args& A = a[blockIdx.y];
    k_local_prep_body(A.in_view, A.level, A.n, A.nlevels, A.in_view2);
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// k_resolve_rounds keeps claimMin and the fixed claims in dynamic LDS (8 B per keypoint, up to 128 KB)
bool resolve_lds_ready() {
    static const bool ok = hipFuncSetAttribute((const void*)k_resolve_rounds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               8 * kResolveLdsKeypoints) == hipSuccess;
    return ok;
}

// Device forms' candidate pass: one wave per point or one thread per point; both write the same lists.
// A single frame's few thousand points leave the chip mostly idle, and a wave's parallel window scan
// has the shorter latency (0.51 vs 0.65 ms per tracked frame); a batch fills the chip, and threads
// carry far less per-point machinery (256 frames: 3.2 -> 1.5 ms per call).  ORBGPU_CAND_MODE=wave /
// thread forces one form everywhere (A/B).
int cand_forced_mode() {
    static const int forced = [] {
        const char* c = getenv("ORBGPU_CAND_MODE");
        return !c ? -1 : strcmp(c, "lds") == 0 ? 2 : strcmp(c, "thread") == 0 ? 1 : strcmp(c, "wave") == 0 ? 0 : -1;
    }();
    return forced;
}
bool cand_thread_mode(bool batch) {
    const int forced = cand_forced_mode();
    return forced >= 0 ? forced >= 1 : batch;
}
// A batch's candidate pass in the LDS-staged form (k_*_candidates_l_b) unless a form is forced
// (ORBGPU_CAND_MODE=thread / wave) or the frame's records do not fit one workgroup's LDS.
bool cand_lds_mode(int cap) {
    const int forced = cand_forced_mode();
    if (!(forced == -1 || forced == 2) || cap > kCandLdsCap) return false;
    static const bool ready = [] {
        return hipFuncSetAttribute((const void*)k_proj_candidates_l_b, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)cand_lds_bytes(kCandLdsCap)) == hipSuccess &&
               hipFuncSetAttribute((const void*)k_lmp_candidates_l_b, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)cand_lds_bytes(kCandLdsCap)) == hipSuccess;
    }();
    return ready;
}

}  // namespace

// Defined in orb_triangulation.hip: the matcher handle's staging buffers and ratio.
int orbgpu_matcher_reserve(orb_matcher_t m, size_t bytes, char** d_buf, char** h_buf, hipStream_t* stream,
                           int* check_ori);
float orbgpu_matcher_nnratio(orb_matcher_t m);
int orbgpu_matcher_check_ori(orb_matcher_t m);

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
        // initialised with the inputs (one upload, no fills): the lister / fixed claims (0x7f..) and
        // the overflow word + counters (0), which the one download then reads back with the matches
        const size_t o_lf = off; off = align256(off + (size_t)std::max(n, 1) * 8);
        const size_t o_ovf = off; off = align256(off + 16);
        const size_t in_bytes = off;
        const size_t o_mp = off; off = align256(off + (size_t)std::max(n, 1) * 4);
        const size_t o_cand = off; off = align256(off + (size_t)nl * P.cap * sizeof(Cand));
        const size_t o_nc = off; off = align256(off + (size_t)nl * 4);
        const size_t o_st = off; off = align256(off + (size_t)std::max(nl, 1) * 4);
        const size_t o_kw = off; off = align256(off + (size_t)std::max(n, 1) * 12);  // claimMin, last, removed
        const size_t o_wl = off; off = align256(off + (size_t)std::max(nl, 1) * 4);  // resolve work list
        const size_t o_top = off; off = align256(off + (size_t)std::max(nl, 1) * 68);  // 8 best (64 B) + usable count
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
        memset(h + o_lf, 0x7f, (size_t)std::max(n, 1) * 8);
        memset(h + o_ovf, 0, 16);
        bool ok = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s) == hipSuccess;
        if (ok && nl > 0)
            hipLaunchKernelGGL(k_proj_candidates, dim3((nl + kCandWaves - 1) / kCandWaves), dim3(64 * kCandWaves), 0, s, P,
                               (const int32_t*)nullptr,
                               (const uint8_t*)(d + o_va), (const float*)(d + o_xyz), (const uint4*)(d + o_md),
                               (const int32_t*)(d + o_lo), (const float4*)(d + o_kp), (const float*)(d + o_ur),
                               (const uint4*)(d + o_cd), (const int32_t*)(d + o_co), (const int32_t*)(d + o_ci),
                               (Cand*)(d + o_cand), (int32_t*)(d + o_nc), (int32_t*)(d + o_ovf), (const uint8_t*)(d + o_ob),
                               (int32_t*)(d + o_lf));
        ResolveArgs ra{};
        ra.n_pts = nl; ra.n_cur = n; ra.cap = P.cap; ra.local = 0; ra.check_ori = check_ori; ra.nnratio = 0.f;
        ra.cands = (const Cand*)(d + o_cand); ra.ncand = (const int32_t*)(d + o_nc); ra.observed = (const uint8_t*)(d + o_ob);
        ra.taken0 = nullptr; ra.cur_kp = (const float4*)(d + o_kp); ra.last_angle = (const float*)(d + o_la);
        ra.overflow = (const int32_t*)(d + o_ovf); ra.st = (int32_t*)(d + o_st);
        int32_t* kw = (int32_t*)(d + o_kw);
        const size_t nk = (size_t)std::max(n, 1);
        ra.claimMin = kw; ra.last = kw + nk; ra.removed = kw + 2 * nk;
        ra.lister = (int32_t*)(d + o_lf); ra.fixed = (int32_t*)(d + o_lf) + nk;
        ra.work = (int32_t*)(d + o_wl);
        ra.top = (int4*)(d + o_top); ra.nusable = (int32_t*)(d + o_top + (size_t)std::max(nl, 1) * 64);
        ra.lds_keypoints = n <= kResolveLdsKeypoints && resolve_lds_ready() ? 1 : 0;
        ra.mp = (int32_t*)(d + o_mp); ra.out_n = (int32_t*)(d + o_ovf) + 1;
        // candidates and the rounds back to back, one synchronisation; an overflowing candidate pass
        // (a point with more candidates than the capacity) makes the resolve a no-op and is re-run
        if (ok) {
            if (ra.n_pts > 0) hipLaunchKernelGGL(k_resolve_init, dim3((ra.n_pts + 255) / 256), dim3(256), 0, s, ra);
            hipLaunchKernelGGL(k_resolve_rounds, dim3(1), dim3(kResolveThreads), ra.lds_keypoints ? 8 * (size_t)n : 0,
                               s, ra);
        }
        ok = ok && hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(h + o_ovf, d + o_ovf, o_mp - o_ovf + (size_t)std::max(n, 1) * 4, hipMemcpyDeviceToHost, s) ==
                 hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection failed");
        int32_t ovf = 0;
        memcpy(&ovf, h + o_ovf, 4);
        if (ovf > P.cap) {  // a point had more candidates than the capacity: redo with room for all
            P.cap = (ovf + 63) & ~63;
            continue;
        }
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
        const size_t o_lf = off; off = align256(off + (size_t)std::max(n, 1) * 8);  // lister, fixed (0x7f..)
        const size_t o_ovf = off; off = align256(off + 16);                          // overflow + counters (0)
        const size_t in_bytes = off;
        const size_t o_m = off; off = align256(off + (size_t)std::max(n, 1) * 4);
        const size_t o_cand = off; off = align256(off + (size_t)np * P.cap * sizeof(Cand));
        const size_t o_nc = off; off = align256(off + (size_t)np * 4);
        const size_t o_st = off; off = align256(off + (size_t)std::max(np, 1) * 4);
        const size_t o_kw = off; off = align256(off + (size_t)std::max(n, 1) * 12);  // claimMin, last, removed
        const size_t o_wl = off; off = align256(off + (size_t)std::max(np, 1) * 4);  // resolve work list
        const size_t o_top = off; off = align256(off + (size_t)std::max(np, 1) * 68);  // 8 best (64 B) + usable count
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
        memset(h + o_lf, 0x7f, (size_t)std::max(n, 1) * 8);
        memset(h + o_ovf, 0, 16);
        bool ok = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s) == hipSuccess;
        if (ok && np > 0)
            hipLaunchKernelGGL(k_lmp_candidates, dim3((np + kCandWaves - 1) / kCandWaves), dim3(64 * kCandWaves), 0, s, P,
                               (const uint8_t*)(d + o_iv), (const uint8_t*)(d + o_bd), (const float*)(d + o_pj),
                               (const float*)(d + o_vc), (const float*)(d + o_dp), (const int32_t*)(d + o_lv),
                               (const uint4*)(d + o_md), (const float4*)(d + o_kp), (const float*)(d + o_ur),
                               (const uint4*)(d + o_cd), (const int32_t*)(d + o_co), (const int32_t*)(d + o_ci),
                               (Cand*)(d + o_cand), (int32_t*)(d + o_nc), (int32_t*)(d + o_ovf), (const uint8_t*)(d + o_ob),
                               frame_taken ? (const uint8_t*)(d + o_tk) : nullptr, (int32_t*)(d + o_lf));
        ResolveArgs ra{};
        ra.n_pts = np; ra.n_cur = n; ra.cap = P.cap; ra.local = 1; ra.check_ori = 0; ra.nnratio = P.nnratio;
        ra.cands = (const Cand*)(d + o_cand); ra.ncand = (const int32_t*)(d + o_nc); ra.observed = (const uint8_t*)(d + o_ob);
        ra.taken0 = frame_taken ? (const uint8_t*)(d + o_tk) : nullptr; ra.cur_kp = (const float4*)(d + o_kp);
        ra.last_angle = nullptr; ra.overflow = (const int32_t*)(d + o_ovf); ra.st = (int32_t*)(d + o_st);
        int32_t* kw = (int32_t*)(d + o_kw);
        const size_t nk = (size_t)std::max(n, 1);
        ra.claimMin = kw; ra.last = kw + nk; ra.removed = kw + 2 * nk;
        ra.lister = (int32_t*)(d + o_lf); ra.fixed = (int32_t*)(d + o_lf) + nk;
        ra.work = (int32_t*)(d + o_wl);
        ra.top = (int4*)(d + o_top); ra.nusable = (int32_t*)(d + o_top + (size_t)std::max(np, 1) * 64);
        ra.lds_keypoints = n <= kResolveLdsKeypoints && resolve_lds_ready() ? 1 : 0;
        ra.mp = (int32_t*)(d + o_m); ra.out_n = (int32_t*)(d + o_ovf) + 1;
        if (ok) {
            if (ra.n_pts > 0) hipLaunchKernelGGL(k_resolve_init, dim3((ra.n_pts + 255) / 256), dim3(256), 0, s, ra);
            hipLaunchKernelGGL(k_resolve_rounds, dim3(1), dim3(kResolveThreads), ra.lds_keypoints ? 8 * (size_t)n : 0,
                               s, ra);
        }
        ok = ok && hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(h + o_ovf, d + o_ovf, o_m - o_ovf + (size_t)std::max(n, 1) * 4, hipMemcpyDeviceToHost, s) ==
                 hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection(local) failed");
        int32_t ovf = 0;
        memcpy(&ovf, h + o_ovf, 4);
        if (ovf > P.cap) {
            P.cap = (ovf + 63) & ~63;
            continue;
        }
        if (n) memcpy(match, h + o_m, (size_t)n * 4);
        memcpy(n_matches, h + o_ovf + 4, 4);
        return ORB_OK;
    }
    return orbgpu_fail(ORB_ERR_INTERNAL, "SearchByProjection(local) candidate capacity");
}

namespace {

// the stream-ordered scratch of one device call
struct DevScratch {
    char* base = nullptr;
    size_t off = 0;
    template <class T>
    T* take(size_t count) {
        T* p = reinterpret_cast<T*>(base + off);
        off = align256(off + std::max<size_t>(count, 1) * sizeof(T));
        return p;
    }
};

bool frame_device_ok(const orb_frame_device_t* F) {
    return F && F->kps_un && F->desc && F->n && F->cap > 0 && F->cap <= kResolveLdsKeypoints && F->nlevels > 0 &&
           F->nlevels <= kMaxLevels && F->scale_factors && F->grid_inv_w > 0 && F->grid_inv_h > 0 &&
           (reinterpret_cast<uintptr_t>(F->desc) & 15) == 0;
}

}  // namespace

size_t orbgpu_sbp_frame_scratch_bytes(int C, int NL) {
    DevScratch z;
    z.take<int32_t>(2); z.take<float4>(C); z.take<int32_t>(kCells + 1); z.take<int32_t>(C);
    z.take<int32_t>(C); z.take<uint8_t>(NL); z.take<int32_t>(NL); z.take<float>(NL); z.take<int32_t>(2 * (size_t)C);
    z.take<int32_t>(4); z.take<Cand>((size_t)NL * C); z.take<int32_t>(NL); z.take<int32_t>(NL);
    z.take<int32_t>(3 * (size_t)C); z.take<int32_t>(NL); z.take<int4>((kTop / 2) * (size_t)NL); z.take<int32_t>(NL);
    return z.off;
}

extern "C" int orb_search_by_projection_frame_device(orb_matcher_t m, const orb_frame_device_t* cur,
                                                     const orb_last_points_device_t* last, float th, int mono,
                                                     int32_t* d_match, int32_t* d_n_matches, void* stream) {
    return orbgpu_sbp_frame_device_scratch(m, cur, last, th, mono, d_match, d_n_matches, stream, nullptr);
}

namespace {

// One frame's launches of a device SearchByProjection form, as argument blocks (the single-frame call
// launches them by value, the batch copies them to the device and launches one grid row per frame).
struct SbpFramePlan {
    k_frame_prep_args prep;
    k_last_prep_args lprep;
    k_proj_candidates_args cand;
    k_resolve_init_args init;
    k_resolve_rounds_args rounds;
    int C, NL;
};

bool sbp_frame_args_ok(orb_matcher_t m, const orb_frame_device_t* cur, const orb_last_points_device_t* last,
                       const int32_t* d_match, const int32_t* d_n_matches) {
    return m && frame_device_ok(cur) && last && d_match && d_n_matches && last->n && last->cap >= 0 &&
           (last->cap == 0 || (last->valid && last->observed && last->xyz && last->desc && last->kps_un)) &&
           (reinterpret_cast<uintptr_t>(last->desc) & 15) == 0;
}

void sbp_frame_plan(orb_matcher_t m, const orb_frame_device_t* cur, const orb_last_points_device_t* last, float th,
                    int mono, int32_t* d_match, int32_t* d_n_matches, char* base, SbpFramePlan& pl) {
    const int C = cur->cap, NL = last->cap;
    pl.C = C;
    pl.NL = NL;
    ProjParams P{};
    memcpy(P.Tcw, cur->Tcw, sizeof(P.Tcw));
    P.min_x = cur->min_x; P.max_x = cur->max_x; P.min_y = cur->min_y; P.max_y = cur->max_y;
    P.inv_w = cur->grid_inv_w; P.inv_h = cur->grid_inv_h;
    P.fx = cur->fx; P.fy = cur->fy; P.cx = cur->cx; P.cy = cur->cy; P.bf = cur->bf; P.th = th;
    for (int l = 0; l < cur->nlevels; ++l) P.scale[l] = cur->scale_factors[l];
    P.n_cur = 0; P.n_last = 0; P.has_ur = cur->u_right != nullptr;
    {   // twc = -R^T t, tlc = Tlw * twc (src:1960-1968), as the host form computes them
        const float* T = cur->Tcw;
        float twc[3], tlc[3];
        for (int i = 0; i < 3; ++i) twc[i] = -std::fma(T[8 + i], T[11], std::fma(T[i], T[3], T[4 + i] * T[7]));
        for (int i = 0; i < 3; ++i)
            tlc[i] = std::fma(last->Tcw[4 * i + 2], twc[2], std::fma(last->Tcw[4 * i], twc[0], last->Tcw[4 * i + 1] * twc[1])) +
                     last->Tcw[4 * i + 3];
        P.bForward = tlc[2] > cur->b && !mono;
        P.bBackward = -tlc[2] > cur->b && !mono;
    }
    P.cap = C;  // a point's candidates are distinct current keypoints: never more than the frame holds
    P.check_ori = orbgpu_matcher_check_ori(m);
    // scratch: dims | kp4 | cells | cell_of | last prep | lister + fixed | overflow block | candidates |
    // ncand | st | claimMin, last, removed | work list | top
    DevScratch z;
    z.base = base;
    int32_t* dims = z.take<int32_t>(2);
    float4* kp4 = z.take<float4>(C);
    int32_t* cell_off = z.take<int32_t>(kCells + 1);
    int32_t* cell_idx = z.take<int32_t>(C);
    int32_t* cell_of = z.take<int32_t>(C);
    uint8_t* valid2 = z.take<uint8_t>(NL);
    int32_t* loct = z.take<int32_t>(NL);
    float* lang = z.take<float>(NL);
    int32_t* lf = z.take<int32_t>(2 * (size_t)C);
    int32_t* ovf = z.take<int32_t>(4);
    Cand* cands = z.take<Cand>((size_t)NL * C);
    int32_t* nc = z.take<int32_t>(NL);
    int32_t* st = z.take<int32_t>(NL);
    int32_t* kw = z.take<int32_t>(3 * (size_t)C);
    int32_t* wl = z.take<int32_t>(NL);
    int4* top = z.take<int4>((kTop / 2) * (size_t)NL);
    int32_t* nus = z.take<int32_t>(NL);
    const ScratchInit zi{lf, 2 * C, d_match, C, ovf, dims, NL > 0 ? -1 : 0};
    pl.prep = k_frame_prep_args{cur->kps_un, cur->n, C, cur->min_x, cur->min_y, cur->grid_inv_w, cur->grid_inv_h, kp4,
                                cell_off, cell_idx, cell_of, dims + 1, nullptr, zi};
    pl.lprep = k_last_prep_args{last->kps_un, last->valid, last->n, NL, cur->nlevels, valid2, loct, lang, dims, nullptr};
    pl.cand = k_proj_candidates_args{P, dims, valid2, last->xyz, (const uint4*)last->desc, loct, kp4, cur->u_right,
                                     (const uint4*)cur->desc, cell_off, cell_idx, cands, nc, ovf, last->observed, lf};
    ResolveArgs ra{};
    ra.n_pts = NL; ra.n_cur = C; ra.cap = C; ra.local = 0; ra.check_ori = P.check_ori; ra.nnratio = 0.f;
    ra.cands = cands; ra.ncand = nc; ra.observed = last->observed; ra.taken0 = nullptr; ra.cur_kp = kp4;
    ra.last_angle = lang; ra.overflow = ovf; ra.st = st;
    ra.claimMin = kw; ra.last = kw + C; ra.removed = kw + 2 * (size_t)C;
    ra.lister = lf; ra.fixed = lf + C; ra.work = wl; ra.top = top; ra.nusable = nus;
    ra.lds_keypoints = resolve_lds_ready() ? 1 : 0;
    ra.mp = d_match; ra.out_n = ovf + 1; ra.dims = dims; ra.out_user = d_n_matches;
    pl.init.a = ra;
    pl.rounds.a = ra;
}

// Argument blocks of B frames into one host block (each kernel's B blocks contiguous, 256-B aligned),
// copied once; pointers of each kernel's array on the device.
struct ArgPacker {
    std::vector<char> host;
    template <class T>
    size_t add(const std::vector<T>& v) {
        const size_t off = align256(host.size());
        host.resize(off + v.size() * sizeof(T));
        memcpy(host.data() + off, v.data(), v.size() * sizeof(T));
        return off;
    }
};

}  // namespace

int orbgpu_sbp_frame_device_scratch(orb_matcher_t m, const orb_frame_device_t* cur, const orb_last_points_device_t* last,
                                    float th, int mono, int32_t* d_match, int32_t* d_n_matches, void* stream,
                                    void* scratch) {
    if (!sbp_frame_args_ok(m, cur, last, d_match, d_n_matches))
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection device arguments");
    hipStream_t s = (hipStream_t)stream;
    const int C = cur->cap, NL = last->cap;
    char* base = static_cast<char*>(scratch);  // the caller's (orbgpu_sbp_frame_scratch_bytes), else stream-ordered
    if (!base && hipMallocAsync(reinterpret_cast<void**>(&base), orbgpu_sbp_frame_scratch_bytes(C, NL), s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    SbpFramePlan pl;
    sbp_frame_plan(m, cur, last, th, mono, d_match, d_n_matches, base, pl);
    const k_frame_prep_args& fp = pl.prep;
    hipLaunchKernelGGL(k_frame_prep, dim3(1), dim3(kPrepThreads), 0, s, fp.kps, fp.n_ptr, fp.cap, fp.min_x, fp.min_y,
                       fp.inv_w, fp.inv_h, fp.kp4, fp.cell_off, fp.cell_idx, fp.cell_of, fp.n_out0, fp.n_out1, fp.z);
    if (NL > 0) {
        const k_last_prep_args& lp = pl.lprep;
        hipLaunchKernelGGL(k_last_prep, dim3((NL + 255) / 256), dim3(256), 0, s, lp.kps, lp.valid, lp.n_ptr, lp.cap,
                           lp.nlevels, lp.valid2, lp.octave, lp.angle, lp.n_out0, lp.n_out1);
        const k_proj_candidates_args& c = pl.cand;
        if (cand_thread_mode(false))
            hipLaunchKernelGGL(k_proj_candidates_t, dim3((NL + kCandThreads - 1) / kCandThreads), dim3(kCandThreads), 0,
                               s, c);
        else
            hipLaunchKernelGGL(k_proj_candidates, dim3((NL + kCandWaves - 1) / kCandWaves), dim3(64 * kCandWaves), 0, s,
                               c.P, c.n_dev, c.valid, c.xyz, c.mp_desc, c.last_octave, c.cur_kp, c.cur_ur, c.cur_desc,
                               c.cell_off, c.cell_idx, c.cands, c.ncand, c.overflow, c.observed, c.lister);
        hipLaunchKernelGGL(k_resolve_init, dim3((NL + 255) / 256), dim3(256), 0, s, pl.init.a);
    }
    hipLaunchKernelGGL(k_resolve_rounds, dim3(1), dim3(kResolveThreads), pl.rounds.a.lds_keypoints ? 8 * (size_t)C : 0, s,
                       pl.rounds.a);
    bool ok = hipGetLastError() == hipSuccess;
    if (!scratch && hipFreeAsync(base, s) != hipSuccess) ok = false;
    return ok ? ORB_OK : orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection device failed");
}

int orbgpu_sbp_frame_batch(orb_matcher_t m, int B, const orb_frame_device_t* const* cur,
                           const orb_last_points_device_t* const* last, float th, int mono, int32_t* const* d_match,
                           int32_t* const* d_n_matches, char* scratch, size_t stride, void* d_args, void* h_args,
                           size_t args_cap, void* stream) {
    if (B <= 0 || !scratch || !d_args || !h_args) return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection batch arguments");
    hipStream_t s = (hipStream_t)stream;
    std::vector<k_frame_prep_args> fp(B);
    std::vector<k_last_prep_args> lp(B);
    std::vector<k_proj_candidates_args> ca(B);
    std::vector<k_resolve_init_args> ri(B);
    std::vector<k_resolve_rounds_args> rr(B);
    int C = -1, maxNL = 0;
    for (int b = 0; b < B; ++b) {
        if (!sbp_frame_args_ok(m, cur[b], last[b], d_match[b], d_n_matches[b]) || (C >= 0 && cur[b]->cap != C) ||
            orbgpu_sbp_frame_scratch_bytes(cur[b]->cap, last[b]->cap) > stride)
            return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection batch frame (caps must agree, scratch stride)");
        C = cur[b]->cap;
        SbpFramePlan pl;
        sbp_frame_plan(m, cur[b], last[b], th, mono, d_match[b], d_n_matches[b], scratch + (size_t)b * stride, pl);
        fp[b] = pl.prep; lp[b] = pl.lprep; ca[b] = pl.cand; ri[b] = pl.init; rr[b] = pl.rounds;
        maxNL = std::max(maxNL, pl.NL);
    }
    ArgPacker pk;
    const size_t o_fp = pk.add(fp), o_lp = pk.add(lp), o_ca = pk.add(ca), o_ri = pk.add(ri), o_rr = pk.add(rr);
    if (pk.host.size() > args_cap) return orbgpu_fail(ORB_ERR_ARG, "SearchByProjection batch: argument area too small");
    char* d = static_cast<char*>(d_args);
    memcpy(h_args, pk.host.data(), pk.host.size());  // pinned staging: the copy reads it when the stream runs it
    if (hipMemcpyAsync(d, h_args, pk.host.size(), hipMemcpyHostToDevice, s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
    hipLaunchKernelGGL(k_frame_prep_b, dim3(1, B), dim3(kPrepThreads), 0, s, (const k_frame_prep_args*)(d + o_fp));
    if (maxNL > 0) {  // grids sized for the largest frame; the kernels bound themselves by their own counts
        hipLaunchKernelGGL(k_last_prep_b, dim3((maxNL + 255) / 256, B), dim3(256), 0, s,
                           (const k_last_prep_args*)(d + o_lp));
        if (cand_lds_mode(C))
            hipLaunchKernelGGL(k_proj_candidates_l_b, dim3(B), dim3(kCandLdsThreads), cand_lds_bytes(C), s,
                               (const k_proj_candidates_args*)(d + o_ca));
        else if (cand_thread_mode(true))
            hipLaunchKernelGGL(k_proj_candidates_t_b, dim3((maxNL + kCandThreads - 1) / kCandThreads, B), dim3(kCandThreads), 0,
                               s, (const k_proj_candidates_args*)(d + o_ca));
        else
            hipLaunchKernelGGL(k_proj_candidates_b, dim3((maxNL + kCandWaves - 1) / kCandWaves, B), dim3(64 * kCandWaves), 0, s,
                               (const k_proj_candidates_args*)(d + o_ca));
        hipLaunchKernelGGL(k_resolve_init_b, dim3((maxNL + 255) / 256, B), dim3(256), 0, s,
                           (const k_resolve_init_args*)(d + o_ri));
    }
    hipLaunchKernelGGL(k_resolve_rounds_b, dim3(1, B), dim3(kResolveThreads), rr[0].a.lds_keypoints ? 8 * (size_t)C : 0, s,
                       (const k_resolve_rounds_args*)(d + o_rr));
    return hipGetLastError() == hipSuccess ? ORB_OK : orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection batch launch failed");
}

size_t orbgpu_sbp_local_scratch_bytes(int C, int np) {
    DevScratch z;
    z.take<int32_t>(2); z.take<float4>(C); z.take<int32_t>(kCells + 1); z.take<int32_t>(C);
    z.take<int32_t>(C); z.take<uint8_t>(np); z.take<int32_t>(2 * (size_t)C); z.take<int32_t>(4);
    z.take<Cand>((size_t)np * C); z.take<int32_t>(np); z.take<int32_t>(np); z.take<int32_t>(3 * (size_t)C);
    z.take<int32_t>(np); z.take<int4>((kTop / 2) * (size_t)np); z.take<int32_t>(np);
    return z.off;
}

extern "C" int orb_search_by_projection_local_device(orb_matcher_t m, const orb_frame_device_t* F,
                                                     const uint8_t* d_frame_taken, const orb_local_points_device_t* pts,
                                                     float th, int far_points, float th_far_points, int32_t* d_match,
                                                     int32_t* d_n_matches, void* stream) {
    return orbgpu_sbp_local_device_scratch(m, F, d_frame_taken, pts, th, far_points, th_far_points, d_match, d_n_matches,
                                           stream, nullptr);
}

namespace {

struct SbpLocalPlan {
    k_frame_prep_args prep;
    k_local_prep_args lprep;
    k_lmp_candidates_args cand;
    k_resolve_init_args init;
    k_resolve_rounds_args rounds;
    int C, np;
};

bool sbp_local_args_ok(orb_matcher_t m, const orb_frame_device_t* F, const orb_local_points_device_t* pts,
                       const int32_t* d_match, const int32_t* d_n_matches) {
    return m && frame_device_ok(F) && pts && pts->n >= 0 && d_match && d_n_matches &&
           (pts->n == 0 || (pts->track_in_view && pts->is_bad && pts->observed && pts->track_proj && pts->track_view_cos &&
                            pts->track_depth && pts->track_level && pts->desc)) &&
           (reinterpret_cast<uintptr_t>(pts->desc) & 15) == 0;
}

void sbp_local_plan(orb_matcher_t m, const orb_frame_device_t* F, const uint8_t* d_frame_taken,
                    const orb_local_points_device_t* pts, float th, int far_points, float th_far_points, int32_t* d_match,
                    int32_t* d_n_matches, char* base, SbpLocalPlan& pl) {
    const int C = F->cap, np = pts->n;
    pl.C = C;
    pl.np = np;
    LocalParams P{};
    P.min_x = F->min_x; P.min_y = F->min_y; P.inv_w = F->grid_inv_w; P.inv_h = F->grid_inv_h;
    P.th = th; P.th_far = th_far_points;
    for (int l = 0; l < F->nlevels; ++l) P.scale[l] = F->scale_factors[l];
    P.n_cur = 0; P.n_pts = np; P.has_ur = F->u_right != nullptr; P.far = far_points ? 1 : 0; P.nlevels = F->nlevels;
    P.cap = C;
    P.nnratio = orbgpu_matcher_nnratio(m);
    DevScratch z;
    z.base = base;
    int32_t* dims = z.take<int32_t>(2);
    float4* kp4 = z.take<float4>(C);
    int32_t* cell_off = z.take<int32_t>(kCells + 1);
    int32_t* cell_idx = z.take<int32_t>(C);
    int32_t* cell_of = z.take<int32_t>(C);
    uint8_t* iv2 = z.take<uint8_t>(np);
    int32_t* lf = z.take<int32_t>(2 * (size_t)C);
    int32_t* ovf = z.take<int32_t>(4);
    Cand* cands = z.take<Cand>((size_t)np * C);
    int32_t* nc = z.take<int32_t>(np);
    int32_t* st = z.take<int32_t>(np);
    int32_t* kw = z.take<int32_t>(3 * (size_t)C);
    int32_t* wl = z.take<int32_t>(np);
    int4* top = z.take<int4>((kTop / 2) * (size_t)np);
    int32_t* nus = z.take<int32_t>(np);
    const ScratchInit zi{lf, 2 * C, d_match, C, ovf, dims, np};
    pl.prep = k_frame_prep_args{F->kps_un, F->n, C, F->min_x, F->min_y, F->grid_inv_w, F->grid_inv_h, kp4, cell_off,
                                cell_idx, cell_of, dims + 1, nullptr, zi};
    pl.lprep = k_local_prep_args{pts->track_in_view, pts->track_level, np, F->nlevels, iv2};
    pl.cand = k_lmp_candidates_args{P, iv2, pts->is_bad, pts->track_proj, pts->track_view_cos, pts->track_depth,
                                    pts->track_level, (const uint4*)pts->desc, kp4, F->u_right, (const uint4*)F->desc,
                                    cell_off, cell_idx, cands, nc, ovf, pts->observed, d_frame_taken, lf};
    ResolveArgs ra{};
    ra.n_pts = np; ra.n_cur = C; ra.cap = C; ra.local = 1; ra.check_ori = 0; ra.nnratio = P.nnratio;
    ra.cands = cands; ra.ncand = nc; ra.observed = pts->observed; ra.taken0 = d_frame_taken; ra.cur_kp = kp4;
    ra.last_angle = nullptr; ra.overflow = ovf; ra.st = st;
    ra.claimMin = kw; ra.last = kw + C; ra.removed = kw + 2 * (size_t)C;
    ra.lister = lf; ra.fixed = lf + C; ra.work = wl; ra.top = top; ra.nusable = nus;
    ra.lds_keypoints = resolve_lds_ready() ? 1 : 0;
    ra.mp = d_match; ra.out_n = ovf + 1; ra.dims = dims; ra.out_user = d_n_matches;
    pl.init.a = ra;
    pl.rounds.a = ra;
}

}  // namespace

int orbgpu_sbp_local_device_scratch(orb_matcher_t m, const orb_frame_device_t* F, const uint8_t* d_frame_taken,
                                    const orb_local_points_device_t* pts, float th, int far_points, float th_far_points,
                                    int32_t* d_match, int32_t* d_n_matches, void* stream, void* scratch) {
    if (!sbp_local_args_ok(m, F, pts, d_match, d_n_matches))
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection(local map) device arguments");
    hipStream_t s = (hipStream_t)stream;
    const int C = F->cap, np = pts->n;
    char* base = static_cast<char*>(scratch);  // the caller's (orbgpu_sbp_local_scratch_bytes), else stream-ordered
    if (!base && hipMallocAsync(reinterpret_cast<void**>(&base), orbgpu_sbp_local_scratch_bytes(C, np), s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    SbpLocalPlan pl;
    sbp_local_plan(m, F, d_frame_taken, pts, th, far_points, th_far_points, d_match, d_n_matches, base, pl);
    const k_frame_prep_args& fp = pl.prep;
    hipLaunchKernelGGL(k_frame_prep, dim3(1), dim3(kPrepThreads), 0, s, fp.kps, fp.n_ptr, fp.cap, fp.min_x, fp.min_y,
                       fp.inv_w, fp.inv_h, fp.kp4, fp.cell_off, fp.cell_idx, fp.cell_of, fp.n_out0, fp.n_out1, fp.z);
    if (np > 0) {
        const k_local_prep_args& lp = pl.lprep;
        hipLaunchKernelGGL(k_local_prep, dim3((np + 255) / 256), dim3(256), 0, s, lp.in_view, lp.level, lp.n, lp.nlevels,
                           lp.in_view2);
        const k_lmp_candidates_args& c = pl.cand;
        if (cand_thread_mode(false))
            hipLaunchKernelGGL(k_lmp_candidates_t, dim3((np + kCandThreads - 1) / kCandThreads), dim3(kCandThreads), 0,
                               s, c);
        else
            hipLaunchKernelGGL(k_lmp_candidates, dim3((np + kCandWaves - 1) / kCandWaves), dim3(64 * kCandWaves), 0, s,
                               c.P, c.in_view, c.bad, c.proj, c.view_cos, c.depth, c.level, c.mp_desc, c.cur_kp, c.cur_ur,
                               c.cur_desc, c.cell_off, c.cell_idx, c.cands, c.ncand, c.overflow, c.observed, c.taken0,
                               c.lister);
        hipLaunchKernelGGL(k_resolve_init, dim3((np + 255) / 256), dim3(256), 0, s, pl.init.a);
    }
    hipLaunchKernelGGL(k_resolve_rounds, dim3(1), dim3(kResolveThreads), pl.rounds.a.lds_keypoints ? 8 * (size_t)C : 0, s,
                       pl.rounds.a);
    bool ok = hipGetLastError() == hipSuccess;
    if (!scratch && hipFreeAsync(base, s) != hipSuccess) ok = false;
    return ok ? ORB_OK : orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection(local) device failed");
}

int orbgpu_sbp_local_batch(orb_matcher_t m, int B, const orb_frame_device_t* const* F, const uint8_t* const* d_frame_taken,
                           const orb_local_points_device_t* const* pts, float th, int far_points, float th_far_points,
                           int32_t* const* d_match, int32_t* const* d_n_matches, char* scratch, size_t stride,
                           void* d_args, void* h_args, size_t args_cap, void* stream) {
    if (B <= 0 || !scratch || !d_args || !h_args)
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection(local) batch arguments");
    hipStream_t s = (hipStream_t)stream;
    std::vector<k_frame_prep_args> fp(B);
    std::vector<k_local_prep_args> lp(B);
    std::vector<k_lmp_candidates_args> ca(B);
    std::vector<k_resolve_init_args> ri(B);
    std::vector<k_resolve_rounds_args> rr(B);
    int C = -1, maxNp = 0;
    for (int b = 0; b < B; ++b) {
        if (!sbp_local_args_ok(m, F[b], pts[b], d_match[b], d_n_matches[b]) || (C >= 0 && F[b]->cap != C) ||
            orbgpu_sbp_local_scratch_bytes(F[b]->cap, pts[b]->n) > stride)
            return orbgpu_fail(ORB_ERR_ARG, "bad SearchByProjection(local) batch frame (caps must agree, scratch stride)");
        C = F[b]->cap;
        SbpLocalPlan pl;
        sbp_local_plan(m, F[b], d_frame_taken[b], pts[b], th, far_points, th_far_points, d_match[b], d_n_matches[b],
                       scratch + (size_t)b * stride, pl);
        fp[b] = pl.prep; lp[b] = pl.lprep; ca[b] = pl.cand; ri[b] = pl.init; rr[b] = pl.rounds;
        maxNp = std::max(maxNp, pl.np);
    }
    ArgPacker pk;
    const size_t o_fp = pk.add(fp), o_lp = pk.add(lp), o_ca = pk.add(ca), o_ri = pk.add(ri), o_rr = pk.add(rr);
    if (pk.host.size() > args_cap)
        return orbgpu_fail(ORB_ERR_ARG, "SearchByProjection(local) batch: argument area too small");
    char* d = static_cast<char*>(d_args);
    memcpy(h_args, pk.host.data(), pk.host.size());  // pinned staging: the copy reads it when the stream runs it
    if (hipMemcpyAsync(d, h_args, pk.host.size(), hipMemcpyHostToDevice, s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
    hipLaunchKernelGGL(k_frame_prep_b, dim3(1, B), dim3(kPrepThreads), 0, s, (const k_frame_prep_args*)(d + o_fp));
    if (maxNp > 0) {
        hipLaunchKernelGGL(k_local_prep_b, dim3((maxNp + 255) / 256, B), dim3(256), 0, s,
                           (const k_local_prep_args*)(d + o_lp));
        if (cand_lds_mode(C))  // (the frame's keypoint count, for the gated frames: the init block's dims)
            hipLaunchKernelGGL(k_lmp_candidates_l_b, dim3(B), dim3(kCandLdsThreads), cand_lds_bytes(C), s,
                               (const k_lmp_candidates_args*)(d + o_ca), (const k_resolve_init_args*)(d + o_ri));
        else if (cand_thread_mode(true))
            hipLaunchKernelGGL(k_lmp_candidates_t_b, dim3((maxNp + kCandThreads - 1) / kCandThreads, B), dim3(kCandThreads), 0,
                               s, (const k_lmp_candidates_args*)(d + o_ca));
        else
            hipLaunchKernelGGL(k_lmp_candidates_b, dim3((maxNp + kCandWaves - 1) / kCandWaves, B), dim3(64 * kCandWaves), 0, s,
                               (const k_lmp_candidates_args*)(d + o_ca));
        hipLaunchKernelGGL(k_resolve_init_b, dim3((maxNp + 255) / 256, B), dim3(256), 0, s,
                           (const k_resolve_init_args*)(d + o_ri));
    }
    hipLaunchKernelGGL(k_resolve_rounds_b, dim3(1, B), dim3(kResolveThreads), rr[0].a.lds_keypoints ? 8 * (size_t)C : 0, s,
                       (const k_resolve_rounds_args*)(d + o_rr));
    return hipGetLastError() == hipSuccess ? ORB_OK
                                           : orbgpu_fail(ORB_ERR_DEVICE, "SearchByProjection(local) batch launch failed");
}
