// MI355X (gfx950) ORB extraction: ORBextractor::operator() (reference src/ORBextractor.cc:1557-1682)
// as five batched HIP kernels over B frames:
//
//   k_pyramid_level  per level: padded level plane (INTER_LINEAR from the previous level, 19-px
//                    REFLECT_101 frame) + its 7x7 sigma-2 Gaussian (for rBRIEF), one LDS tile pass
//   k_fast_cells     one wave per (frame, FAST cell): threshold-independent FAST-9 score, 3x3 NMS
//                    inside the cell window, iniTh/minTh choice, row-major candidate emission
//   k_quadtree       one wave per (frame, level): DistributeOctTree, exact list/sort semantics
//   k_place          one wave per frame: level-0 scaling and vLappingArea output placement
//   k_describe       one wave per keypoint: IC_Angle (31-px disc) + steered rBRIEF (256 tests)
//
// No MFMA anywhere: this is byte / integer / popcount work.  All float arithmetic that reaches an
// output (resize coefficients are host tables; fastAtan2; pattern steering) is compiled with
// -ffp-contract=off and uses explicit fmaf() exactly where the reference's g++ -march=native build
// contracts (see orb_hd.h / orb_sincos.h and DESIGN.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "orb_extract_geom.h"
#include "orb_hd.h"
#include "orb_sincos.h"
#include "orbgpu.h"
#include "orbgpu_internal.h"

using namespace orbgpu;

namespace {

__constant__ int c_pattern[1024] = {
#include "orb_pattern31.inc"
};

__constant__ uint32_t c_sincos_exc[][3] = {
#include "orb_sincos_exceptions.inc"
};
constexpr int kNumSincosExc = sizeof(c_sincos_exc) / sizeof(c_sincos_exc[0]);

// 8-fraction-bit GaussianBlur(7x7, sigma=2) kernel of OpenCV's bit-exact 8U path
// (getGaussianKernelBitExact + error-diffusion fixed point): sums to 256.
__device__ __forceinline__ int blur_tap(int k) {
    return k == 3 ? 56 : (k == 2 || k == 4) ? 48 : (k == 1 || k == 5) ? 34 : 18;
}

__device__ __forceinline__ int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int rank_in(unsigned long long m) {  // set lanes below this one
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ================================================================================================
// 1. pyramid level: padded plane + blurred view, src:1687-1740 and src:1629-1637
// ================================================================================================
constexpr int kTileW = 64, kTileH = 16, kHalo = 3;
constexpr int kLW = kTileW + 2 * kHalo, kLH = kTileH + 2 * kHalo;  // 70 x 22

// cv::resize INTER_LINEAR 8U value of level pixel (vx, vy) from the previous level view S
__device__ __forceinline__ int resize_px(const uint8_t* __restrict__ S, int sstride, int sw, int vx, int vy,
                                         const int2* __restrict__ xt, const int4* __restrict__ yt, int simd_end) {
    const int2 X = xt[vx];
    const int4 Y = yt[vy];
    const int sx = X.x, sx1 = min(sx + 1, sw - 1);
    const int a0 = X.y & 0xffff, a1 = X.y >> 16;
    const uint8_t* R0 = S + (size_t)Y.x * sstride;
    const uint8_t* R1 = S + (size_t)Y.y * sstride;
    const int h0 = R0[sx] * a0 + R0[sx1] * a1;
    const int h1 = R1[sx] * a0 + R1[sx1] * a1;
    int v;
    if (vx < simd_end) {  // VResizeLinearVec_32s8u: v_mul_hi on (S >> 4), then rounding shift by 2
        const int t0 = min(h0 >> 4, 32767), t1 = min(h1 >> 4, 32767);
        v = (((t0 * Y.z) >> 16) + ((t1 * Y.w) >> 16) + 2) >> 2;
    } else {              // FixedPtCast<int, uchar, 22>
        v = (h0 * Y.z + h1 * Y.w + (1 << 21)) >> 22;
    }
    return min(max(v, 0), 255);
}

template <bool kLevel0>
__global__ __launch_bounds__(256) void k_pyramid_level(KernelGeom g, int level, const uint8_t* __restrict__ in,
                                                       long long in_frame_stride, int in_stride,
                                                       uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                       const int2* __restrict__ xtab, const int4* __restrict__ ytab) {
    __shared__ uint8_t tile[kLH][kLW + 2];
    __shared__ int hsum[kLH][kTileW];
    const int f = blockIdx.z;
    const LevelGeom& L = g.lv[level];
    const int X0 = blockIdx.x * kTileW, Y0 = blockIdx.y * kTileH;
    uint8_t* plane = pyr + (size_t)f * g.pyr_frame_bytes + L.plane_off;
    uint8_t* bplane = blur + (size_t)f * g.pyr_frame_bytes + L.plane_off;
    const uint8_t* src;
    int sstride, sw = 0;
    if (kLevel0) {
        src = in + (size_t)f * in_frame_stride;
        sstride = in_stride;
    } else {
        const LevelGeom& P = g.lv[level - 1];
        src = pyr + (size_t)f * g.pyr_frame_bytes + P.plane_off + (size_t)kEdge * P.pitch + kEdge;
        sstride = P.pitch;
        sw = P.w;
    }
    const int2* xt = xtab + (kLevel0 ? 0 : L.xtab_off);
    const int4* yt = ytab + (kLevel0 ? 0 : L.ytab_off);
    for (int i = threadIdx.x; i < kLH * kLW; i += 256) {
        const int ty = i / kLW, tx = i - ty * kLW;
        const int vx = reflect101(X0 - kHalo + tx - kEdge, L.w);
        const int vy = reflect101(Y0 - kHalo + ty - kEdge, L.h);
        int v;
        if (kLevel0) v = src[(size_t)vy * sstride + vx];
        else v = resize_px(src, sstride, sw, vx, vy, xt, yt, L.simd_end);
        tile[ty][tx] = (uint8_t)v;
    }
    __syncthreads();
    // padded plane: 4 consecutive pixels per thread
    {
        const int r = threadIdx.x >> 4, c = (threadIdx.x & 15) * 4;
        const int py = Y0 + r, px = X0 + c;
        if (py < L.ph) {
            uint8_t* dst = plane + (size_t)py * L.pitch + px;
            if (px + 3 < L.pw) {
                const uint32_t w = tile[r + kHalo][c + kHalo] | (tile[r + kHalo][c + kHalo + 1] << 8) |
                                   (tile[r + kHalo][c + kHalo + 2] << 16) | ((uint32_t)tile[r + kHalo][c + kHalo + 3] << 24);
                *reinterpret_cast<uint32_t*>(dst) = w;
            } else {
                for (int k = 0; k < 4 && px + k < L.pw; ++k) dst[k] = tile[r + kHalo][c + kHalo + k];
            }
        }
    }
    // does this tile touch the view at all?
    if (X0 + kTileW <= kEdge || X0 >= kEdge + L.w || Y0 + kTileH <= kEdge || Y0 >= kEdge + L.h) return;
    // horizontal 7-tap pass over all 22 rows (exact in 16 bits, kept as int)
    for (int i = threadIdx.x; i < kLH * kTileW; i += 256) {
        const int ty = i / kTileW, tx = i - ty * kTileW;
        int acc = 0;
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += blur_tap(k) * tile[ty][tx + k];
        hsum[ty][tx] = acc;
    }
    __syncthreads();
    {
        const int r = threadIdx.x >> 4, c = (threadIdx.x & 15) * 4;
        const int py = Y0 + r;
        const int vy = py - kEdge;
        if (vy >= 0 && vy < L.h) {
            uint32_t word = 0;
            int acc4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                int acc = 0;
#pragma unroll
                for (int k = 0; k < 7; ++k) acc += blur_tap(k) * hsum[r + k][c + q];
                acc4[q] = min((acc + (1 << 15)) >> 16, 255);
                word |= (uint32_t)acc4[q] << (8 * q);
            }
            const int px = X0 + c;
            uint8_t* dst = bplane + (size_t)py * L.pitch + px;
            if (px >= kEdge && px + 3 < kEdge + L.w) {
                *reinterpret_cast<uint32_t*>(dst) = word;
            } else {
                for (int q = 0; q < 4; ++q)
                    if (px + q >= kEdge && px + q < kEdge + L.w) dst[q] = (uint8_t)acc4[q];
            }
        }
    }
}

// ================================================================================================
// 2. FAST cells: src:1098-1166 (cell loop) + OpenCV FAST_t<16>/cornerScore<16> semantics
// ================================================================================================
// score(p) = max over the 16 9-pixel arcs and both polarities of the arc minimum of |I(p)-I(q)|,
// minus 1.  corner(t) <=> score >= t, and for corners this equals cornerScore<16>.  OpenCV's NMS
// (a candidate survives iff its score beats the 8 neighbours' *thresholded* scores inside the
// window) is then equivalent to: score >= t && score > score(n) for every neighbour n inside the
// window's detectable region (neighbours below t can never beat a corner).
__device__ __forceinline__ int fast_score(const uint8_t* __restrict__ p, const int (&off)[16]) {
    const int v = p[0];
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - (int)p[off[k]];
    int mn2[16], mx2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { mn2[k] = min(d[k], d[(k + 1) & 15]); mx2[k] = max(d[k], d[(k + 1) & 15]); }
    int mn4[16], mx4[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { mn4[k] = min(mn2[k], mn2[(k + 2) & 15]); mx4[k] = max(mx2[k], mx2[(k + 2) & 15]); }
    int best_dark = -1000, best_bright = 1000;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int mn8 = min(mn4[k], mn4[(k + 4) & 15]), mx8 = max(mx4[k], mx4[(k + 4) & 15]);
        best_dark = max(best_dark, min(mn8, d[(k + 8) & 15]));
        best_bright = min(best_bright, max(mx8, d[(k + 8) & 15]));
    }
    return max(best_dark, -best_bright) - 1;
}

__device__ __forceinline__ bool is_local_max(const uint8_t* __restrict__ sc, int stride, int idx, int s) {
    const uint8_t* q = sc + idx;
    return s > q[-stride - 1] && s > q[-stride] && s > q[-stride + 1] && s > q[-1] && s > q[1] &&
           s > q[stride - 1] && s > q[stride] && s > q[stride + 1];
}

__device__ __forceinline__ uint32_t pack_key(int x, int y, int score) {
    return (uint32_t)score | ((uint32_t)x << 8) | ((uint32_t)y << 20);
}
__device__ __forceinline__ int key_x(uint32_t k) { return (int)((k >> 8) & 0xfff); }
__device__ __forceinline__ int key_y(uint32_t k) { return (int)(k >> 20); }
__device__ __forceinline__ int key_score(uint32_t k) { return (int)(k & 0xff); }

__global__ __launch_bounds__(256) void k_fast_cells(KernelGeom g, const CellDesc* __restrict__ cells, int win_cap,
                                                    const uint8_t* __restrict__ pyr, uint32_t* __restrict__ cand,
                                                    int32_t* __restrict__ cell_count, uint8_t* __restrict__ cell_thr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cid = blockIdx.x * 4 + wave;
    const int f = blockIdx.y;
    if (cid >= g.ncells) return;
    const CellDesc C = cells[cid];
    const LevelGeom& L = g.lv[C.level];
    const uint8_t* view = pyr + (size_t)f * g.pyr_frame_bytes + L.plane_off + (size_t)kEdge * L.pitch + kEdge;
    uint8_t* win = smem + (size_t)wave * 2 * win_cap;
    uint8_t* sc = win + win_cap;
    const int ww = C.win_w, wh = C.win_h, n = ww * wh;
    const uint8_t* src = view + (size_t)C.ini_y * L.pitch + C.ini_x;
    for (int i = lane; i < n; i += 64) {
        const int r = i / ww, c = i - r * ww;
        win[i] = src[(size_t)r * L.pitch + c];
        sc[i] = 0;
    }
    wave_sync();
    const int dw = ww - 6, dh = wh - 6, nd = max(dw, 0) * max(dh, 0);
    int off[16];
    {
        const int cx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
        const int cy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
#pragma unroll
        for (int k = 0; k < 16; ++k) off[k] = cx[k] + cy[k] * ww;
    }
    for (int i = lane; i < nd; i += 64) {
        const int r = 3 + i / dw, c = 3 + (i - (i / dw) * dw);
        const int s = fast_score(win + r * ww + c, off);
        sc[r * ww + c] = (uint8_t)min(max(s, 0), 255);
    }
    wave_sync();
    const int ini = g.ini_th, mint = g.min_th;
    bool any = false;
    for (int i = lane; i < nd; i += 64) {
        const int r = 3 + i / dw, c = 3 + (i - (i / dw) * dw);
        const int idx = r * ww + c, s = sc[idx];
        any |= (s >= ini) && is_local_max(sc, ww, idx, s);
    }
    const int t = ballot(any) ? ini : mint;
    uint32_t* out = cand + (size_t)f * g.cand_frame_cap + L.cand_off + C.slot;
    int count = 0;
    for (int i0 = 0; i0 < nd; i0 += 64) {
        const int i = i0 + lane;
        bool keep = false;
        int r = 0, c = 0, s = 0;
        if (i < nd) {
            r = 3 + i / dw;
            c = 3 + (i - (i / dw) * dw);
            const int idx = r * ww + c;
            s = sc[idx];
            keep = (s >= t) && is_local_max(sc, ww, idx, s);
        }
        const unsigned long long m = ballot(keep);
        if (keep) {
            const int pos = count + rank_in(m);
            if (pos < C.cap) out[pos] = pack_key(C.off_x + c, C.off_y + r, s);
        }
        count += __popcll(m);
    }
    if (lane == 0) {
        cell_count[(size_t)f * g.ncells + cid] = min(count, (int)C.cap);
        cell_thr[(size_t)f * g.ncells + cid] = (uint8_t)t;
    }
}

// ================================================================================================
// 3. DistributeOctTree, src:711-1057, one wave per (frame, level)
// ================================================================================================
// The reference keeps the nodes in a std::list: every non-leaf node is divided and its non-empty
// children pushed to the FRONT in the order n1..n4, the parent erased.  A pass therefore yields
// list = reverse(children in push order) ++ (leaf nodes in old order).  In the "careful" phase the
// children of the last pass are std::sort-ed with compareNodes and divided from the largest until
// the list reaches N; parents are erased from wherever they are.  We keep the list as an array that
// is re-materialised after every pass / careful round, node keys as contiguous ranges of packed
// keys that are stably 4-way partitioned between two buffers on every division, and port the
// libstdc++ introsort exactly (orb_hd.h) because compareNodes has ties.
struct QTree {
    uint32_t* keys[2];
    // node arrays (NCAP)
    int16_t *x0, *y0, *x1, *y1;
    int32_t *kstart, *kcount;
    uint8_t *kbuf, *leaf, *erased;
    uint16_t* freelist;
    // list arrays (LCAP)
    uint16_t *list, *list2, *stack, *surv, *split, *prev, *pending;
    int ncap, lcap;
};

__device__ __forceinline__ size_t qt_node_bytes(int ncap) { return (size_t)ncap * (4 * 2 + 2 * 4 + 3 + 2); }
__device__ __forceinline__ size_t qt_list_bytes(int lcap) { return (size_t)lcap * 2 * 7; }

__device__ inline void qt_carve(QTree& t, uint8_t* p, int ncap, int lcap) {
    t.ncap = ncap; t.lcap = lcap;
    t.kstart = (int32_t*)p; p += 4 * ncap;
    t.kcount = (int32_t*)p; p += 4 * ncap;
    t.x0 = (int16_t*)p; p += 2 * ncap;
    t.y0 = (int16_t*)p; p += 2 * ncap;
    t.x1 = (int16_t*)p; p += 2 * ncap;
    t.y1 = (int16_t*)p; p += 2 * ncap;
    t.freelist = (uint16_t*)p; p += 2 * ncap;
    t.list = (uint16_t*)p; p += 2 * lcap;
    t.list2 = (uint16_t*)p; p += 2 * lcap;
    t.stack = (uint16_t*)p; p += 2 * lcap;
    t.surv = (uint16_t*)p; p += 2 * lcap;
    t.split = (uint16_t*)p; p += 2 * lcap;
    t.prev = (uint16_t*)p; p += 2 * lcap;
    t.pending = (uint16_t*)p; p += 2 * lcap;
    t.kbuf = p; p += ncap;
    t.leaf = p; p += ncap;
    t.erased = p; p += ncap;
}

struct QState {  // wave-uniform scalars (every lane holds the same values)
    int nfree;
    int nstack, nsplit;
    int npending;     // parents divided in a careful round; recycled after the list is rebuilt
    bool overflow;
};

// Divide `node`: stable 4-way partition of its keys into the other buffer, children pushed to
// `stack` (order n1, n2, n3, n4), the splittable ones (> 1 key) appended to `split`.
// Returns the number of children created.
__device__ inline int qt_divide(QTree& t, QState& s, int node, int lane, bool defer_free) {
    const int x0 = t.x0[node], y0 = t.y0[node], x1 = t.x1[node], y1 = t.y1[node];
    const int ks = uniform(t.kstart[node]), kn = uniform(t.kcount[node]), kb = uniform(t.kbuf[node]);
    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;  // ceil((float)(d)/2), src:608-609
    const int sx = x0 + hx, sy = y0 + hy;
    const uint32_t* src = t.keys[kb] + ks;
    uint32_t* dst = t.keys[kb ^ 1] + ks;
    int cnt[4] = {0, 0, 0, 0};
    for (int b = 0; b < kn; b += 64) {
        const int i = b + lane;
        int q = -1;
        if (i < kn) {
            const uint32_t k = src[i];
            q = (key_x(k) >= sx ? 1 : 0) + (key_y(k) >= sy ? 2 : 0);  // src:651-661
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) cnt[qq] += __popcll(ballot(q == qq));
    }
    int base[4];
    base[0] = 0; base[1] = cnt[0]; base[2] = cnt[0] + cnt[1]; base[3] = base[2] + cnt[2];
    for (int b = 0; b < kn; b += 64) {
        const int i = b + lane;
        int q = -1;
        uint32_t k = 0;
        if (i < kn) {
            k = src[i];
            q = (key_x(k) >= sx ? 1 : 0) + (key_y(k) >= sy ? 2 : 0);
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const unsigned long long m = ballot(q == qq);
            if (q == qq) dst[base[qq] + rank_in(m)] = k;
            base[qq] += __popcll(m);
        }
    }
    // children rectangles, src:614-640
    const int cx0[4] = {x0, sx, x0, sx}, cy0[4] = {y0, y0, sy, sy};
    const int cx1[4] = {sx, x1, sx, x1}, cy1[4] = {sy, sy, y1, y1};
    int start = ks, made = 0;
    // the parent's id is recycled after its children are allocated (it is no longer referenced)
    for (int qq = 0; qq < 4; ++qq) {
        const int n = cnt[qq];
        if (n > 0) {
            if (s.nfree == 0 || s.nstack >= t.lcap) { s.overflow = true; return made; }
            const int id = t.freelist[--s.nfree];
            if (lane == 0) {
                t.x0[id] = (int16_t)cx0[qq]; t.y0[id] = (int16_t)cy0[qq];
                t.x1[id] = (int16_t)cx1[qq]; t.y1[id] = (int16_t)cy1[qq];
                t.kstart[id] = start; t.kcount[id] = n;
                t.kbuf[id] = (uint8_t)(kb ^ 1);
                t.leaf[id] = n == 1;
                t.erased[id] = 0;
                t.stack[s.nstack] = (uint16_t)id;
                if (n > 1) t.split[s.nsplit] = (uint16_t)id;
            }
            s.nstack++;
            if (n > 1) {
                if (s.nsplit >= t.lcap) { s.overflow = true; return made; }
                s.nsplit++;
            }
            made++;
        }
        start += n;
    }
    // a careful round still scans the old list (and its erased flags) after this division, so the
    // parent's id must not be handed out again before the list is rebuilt
    if (defer_free) {
        if (lane == 0) { t.pending[s.npending] = (uint16_t)node; t.erased[node] = 1; }
        s.npending++;
    } else {
        if (lane == 0) t.freelist[s.nfree] = (uint16_t)node;
        s.nfree++;
    }
    wave_sync();
    return made;
}

template <bool kKeysInLds>
__device__ void qt_run(QTree& t, int K, int N, int nroots, float root_w, int span_x, int span_y,
                       const uint32_t* __restrict__ cand_level, const CellDesc* __restrict__ cells, int cell_begin,
                       int cell_count, const int32_t* __restrict__ ccount, uint32_t* __restrict__ sel_out,
                       int sel_cap, int* n_sel, int* status) {
    const int lane = lane_id();
    QState s{};
    s.nfree = 0;
    // free list: ids ncap-1 .. 0 so that allocation order is 0, 1, 2, ...
    for (int i = lane; i < t.ncap; i += 64) t.freelist[i] = (uint16_t)(t.ncap - 1 - i);
    s.nfree = t.ncap;
    // ---- gather candidates in cell order into keys[1], counting per root (src:756-764)
    int rcount[kMaxRoots];
#pragma unroll
    for (int r = 0; r < kMaxRoots; ++r) rcount[r] = 0;
    {
        int pos = 0;
        for (int c = 0; c < cell_count; ++c) {
            const int n = uniform(ccount[c]);
            const uint32_t* src = cand_level + cells[cell_begin + c].slot;
            for (int b = 0; b < n; b += 64) {
                const int i = b + lane;
                int root = -1;
                if (i < n) {
                    const uint32_t k = src[i];
                    t.keys[1][pos + i] = k;
                    root = (int)((float)key_x(k) / root_w);
                }
#pragma unroll
                for (int r = 0; r < kMaxRoots; ++r)
                    if (r < nroots) rcount[r] += __popcll(ballot(root == r));
            }
            pos += n;
        }
    }
    wave_sync();
    // stable partition by root into keys[0]
    {
        int base[kMaxRoots];
        int acc = 0;
#pragma unroll
        for (int r = 0; r < kMaxRoots; ++r) { base[r] = acc; acc += r < nroots ? rcount[r] : 0; }
        for (int b = 0; b < K; b += 64) {
            const int i = b + lane;
            int root = -1;
            uint32_t k = 0;
            if (i < K) { k = t.keys[1][i]; root = (int)((float)key_x(k) / root_w); }
#pragma unroll
            for (int r = 0; r < kMaxRoots; ++r) {
                if (r >= nroots) break;
                const unsigned long long m = ballot(root == r);
                if (root == r) t.keys[0][base[r] + rank_in(m)] = k;
                base[r] += __popcll(m);
            }
        }
    }
    // ---- roots (src:733-786): empty roots erased, single-key roots are leaves
    int nlist = 0;
    {
        int start = 0;
        for (int r = 0; r < nroots; ++r) {
            const int n = rcount[r];
            if (n > 0) {
                const int id = t.freelist[--s.nfree];
                if (lane == 0) {
                    t.x0[id] = (int16_t)(int)(root_w * (float)r);
                    t.x1[id] = (int16_t)(int)(root_w * (float)(r + 1));
                    t.y0[id] = 0;
                    t.y1[id] = (int16_t)span_y;
                    t.kstart[id] = start; t.kcount[id] = n; t.kbuf[id] = 0;
                    t.leaf[id] = n == 1; t.erased[id] = 0;
                    t.list[nlist] = (uint16_t)id;
                }
                nlist++;
            }
            start += n;
        }
    }
    wave_sync();
    (void)span_x;
    bool done = false;
    while (!done && !s.overflow) {
        // ---------------- regular pass (src:802-918)
        const int prev_size = nlist;
        int nsurv = 0, to_expand = 0;
        s.nstack = 0;
        s.nsplit = 0;
        for (int i = 0; i < nlist && !s.overflow; ++i) {
            const int node = uniform(t.list[i]);
            if (t.leaf[node]) {
                if (lane == 0) t.surv[nsurv] = (uint16_t)node;
                nsurv++;
                continue;
            }
            const int before = s.nsplit;
            qt_divide(t, s, node, lane, false);
            to_expand += s.nsplit - before;
        }
        if (s.overflow) break;
        wave_sync();
        nlist = s.nstack + nsurv;
        if (nlist > t.lcap) { s.overflow = true; break; }
        for (int i = lane; i < nlist; i += 64)
            t.list2[i] = i < s.nstack ? t.stack[s.nstack - 1 - i] : t.surv[i - s.nstack];
        wave_sync();
        for (int i = lane; i < nlist; i += 64) t.list[i] = t.list2[i];
        wave_sync();
        if (nlist >= N || nlist == prev_size) {
            done = true;
        } else if (nlist + to_expand * 3 > N) {
            // ---------------- careful rounds (src:932-1016)
            while (!done && !s.overflow) {
                const int round_prev = nlist;
                const int nprev = s.nsplit;
                for (int i = lane; i < nprev; i += 64) t.prev[i] = t.split[i];
                wave_sync();
                if (lane == 0) {
                    const int16_t* x0a = t.x0;
                    const int32_t* kc = t.kcount;
                    orb_std_sort(t.prev, nprev, [&](uint16_t a, uint16_t b) {
                        const int ca = kc[a], cb = kc[b];
                        return ca < cb || (ca == cb && x0a[a] < x0a[b]);
                    });
                }
                wave_sync();
                s.nstack = 0;
                s.nsplit = 0;
                s.npending = 0;
                int size = nlist;
                for (int j = nprev - 1; j >= 0; --j) {
                    const int node = uniform(t.prev[j]);
                    const int made = qt_divide(t, s, node, lane, true);
                    if (s.overflow) break;
                    size += made - 1;
                    if (size >= N) break;
                }
                if (s.overflow) break;
                wave_sync();
                // list = reverse(stack) ++ (old list minus erased)
                int w = s.nstack;
                for (int b = 0; b < nlist; b += 64) {
                    const int i = b + lane;
                    bool keep = false;
                    int id = 0;
                    if (i < nlist) { id = t.list[i]; keep = !t.erased[id]; }
                    const unsigned long long m = ballot(keep);
                    if (keep && w + rank_in(m) < t.lcap) t.list2[w + rank_in(m)] = (uint16_t)id;
                    w += __popcll(m);
                }
                if (w > t.lcap) { s.overflow = true; break; }
                for (int i = lane; i < s.nstack; i += 64) t.list2[i] = t.stack[s.nstack - 1 - i];
                wave_sync();
                nlist = w;
                for (int i = lane; i < nlist; i += 64) t.list[i] = t.list2[i];
                for (int i = lane; i < s.npending; i += 64) t.freelist[s.nfree + i] = t.pending[i];
                s.nfree += s.npending;
                s.npending = 0;
                wave_sync();
                if (nlist >= N || nlist == round_prev) done = true;
            }
        }
    }
    if (s.overflow || nlist > sel_cap) {
        if (lane == 0) { *n_sel = 0; atomicMax(status, 1); }
        return;
    }
    // ---- keep the first max-response key of every node, in list order (src:1028-1053)
    for (int i = lane; i < nlist; i += 64) {
        const int id = t.list[i];
        const uint32_t* kk = t.keys[t.kbuf[id]] + t.kstart[id];
        const int n = t.kcount[id];
        uint32_t best = kk[0];
        for (int q = 1; q < n; ++q)
            if (key_score(kk[q]) > key_score(best)) best = kk[q];
        sel_out[i] = best;
    }
    if (lane == 0) *n_sel = nlist;
}

__global__ __launch_bounds__(64) void k_quadtree(KernelGeom g, const CellDesc* __restrict__ cells,
                                                 const uint32_t* __restrict__ cand, const int32_t* __restrict__ cell_count,
                                                 uint32_t* __restrict__ key_scratch, uint32_t* __restrict__ sel,
                                                 int32_t* __restrict__ sel_count, int lds_bytes, int* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int level = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
    const LevelGeom& L = g.lv[level];
    const int32_t* cc = cell_count + (size_t)f * g.ncells + L.cell_begin;
    int K = 0;
    for (int c = lane; c < L.cell_count; c += 64) K += cc[c];
    K = wave_sum(K);
    K = uniform(K);
    const int N = L.nfeat;
    const int lcap = L.sel_cap + 64, ncap = 2 * lcap + 8;
    QTree t;
    size_t meta = qt_node_bytes(ncap) + qt_list_bytes(lcap);
    meta = (meta + 15) & ~(size_t)15;
    qt_carve(t, smem, ncap, lcap);
    uint32_t* sel_out = sel + (size_t)f * g.sel_frame_cap + L.sel_off;
    int32_t* n_sel = sel_count + (size_t)f * g.nlevels + level;
    const uint32_t* cand_level = cand + (size_t)f * g.cand_frame_cap + L.cand_off;
    const size_t key_bytes = (size_t)K * 4 * 2;
    if (meta + key_bytes <= (size_t)lds_bytes) {
        t.keys[0] = (uint32_t*)(smem + meta);
        t.keys[1] = t.keys[0] + K;
        qt_run<true>(t, K, N, L.n_roots, L.root_w, L.maxBX - L.minB, L.maxBY - L.minB, cand_level, cells,
                     L.cell_begin, L.cell_count, cc, sel_out, L.sel_cap, n_sel, status);
    } else {
        uint32_t* scratch = key_scratch + ((size_t)f * g.cand_frame_cap + L.cand_off) * 2;
        t.keys[0] = scratch;
        t.keys[1] = scratch + L.cand_cap;
        qt_run<false>(t, K, N, L.n_roots, L.root_w, L.maxBX - L.minB, L.maxBY - L.minB, cand_level, cells,
                      L.cell_begin, L.cell_count, cc, sel_out, L.sel_cap, n_sel, status);
    }
}

// ================================================================================================
// 4. output placement by vLappingArea, src:1613-1681
// ================================================================================================
__global__ __launch_bounds__(64) void k_place(KernelGeom g, const uint32_t* __restrict__ sel,
                                              const int32_t* __restrict__ sel_count, int32_t* __restrict__ dst_index,
                                              int lap0, int lap1, int cap, int32_t* __restrict__ counts) {
    const int f = blockIdx.x, lane = threadIdx.x;
    int total = 0;
    for (int l = 0; l < g.nlevels; ++l) total += sel_count[(size_t)f * g.nlevels + l];
    int mono = 0, stereo = 0;
    for (int l = 0; l < g.nlevels; ++l) {
        const LevelGeom& L = g.lv[l];
        const int n = sel_count[(size_t)f * g.nlevels + l];
        const uint32_t* s = sel + (size_t)f * g.sel_frame_cap + L.sel_off;
        int32_t* d = dst_index + (size_t)f * g.sel_frame_cap + L.sel_off;
        for (int b = 0; b < n; b += 64) {
            const int i = b + lane;
            bool valid = i < n, lap = false;
            if (valid) {
                float x = (float)(key_x(s[i]) + L.minB);
                if (l != 0) x = x * L.scale;
                lap = x >= (float)lap0 && x <= (float)lap1;
            }
            const unsigned long long ml = ballot(valid && lap), mm = ballot(valid && !lap);
            if (valid) d[i] = lap ? total - 1 - (stereo + rank_in(ml)) : mono + rank_in(mm);
            stereo += __popcll(ml);
            mono += __popcll(mm);
        }
    }
    if (lane == 0) {
        counts[2 * f] = total;
        counts[2 * f + 1] = total > cap ? ORB_ERR_CAPACITY : mono;
    }
}

// ================================================================================================
// 5. IC_Angle + steered rBRIEF, src:91-138, 150-203, 1534-1547, 1656-1676
// ================================================================================================
__device__ __forceinline__ void steer_sincos(float ang, float* s, float* c) {
    orb_det_sincosf(ang, s, c);
    const uint32_t bits = __float_as_uint(ang);
    int lo = 0, hi = kNumSincosExc - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const uint32_t m = c_sincos_exc[mid][0];
        if (m == bits) { *c = __uint_as_float(c_sincos_exc[mid][1]); *s = __uint_as_float(c_sincos_exc[mid][2]); return; }
        if (m < bits) lo = mid + 1; else hi = mid - 1;
    }
}

__global__ __launch_bounds__(256) void k_describe(KernelGeom g, const uint8_t* __restrict__ pyr,
                                                  const uint8_t* __restrict__ blur, const uint32_t* __restrict__ sel,
                                                  const int32_t* __restrict__ sel_count,
                                                  const int32_t* __restrict__ dst_index, const int32_t* __restrict__ counts,
                                                  int cap, orb_keypoint_t* __restrict__ kps, uint8_t* __restrict__ desc) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int slot = blockIdx.x * 4 + wave, level = blockIdx.y, f = blockIdx.z;
    const int n = sel_count[(size_t)f * g.nlevels + level];
    if (slot >= n) return;
    if (counts[2 * f + 1] < 0) return;  // frame exceeded the caller's capacity
    const LevelGeom& L = g.lv[level];
    const uint32_t key = sel[(size_t)f * g.sel_frame_cap + L.sel_off + slot];
    const int x = key_x(key) + L.minB, y = key_y(key) + L.minB;
    // ---- IC_Angle on the unblurred level: lane = (side, u); side 0 rows +v, side 1 rows -v
    const uint8_t* center = pyr + (size_t)f * g.pyr_frame_bytes + L.plane_off + (size_t)(y + kEdge) * L.pitch + (x + kEdge);
    const int side = lane >> 5, u = (lane & 31) - kHalfPatch;
    const bool col_ok = (lane & 31) < 2 * kHalfPatch + 1;
    int m10 = 0, m01 = 0;
    if (col_ok && side == 0) m10 += u * center[u];
#pragma unroll
    for (int v = 1; v <= kHalfPatch; ++v) {
        const int d = g.umax[v];
        if (col_ok && u >= -d && u <= d) {
            const int sv = side ? -v : v;
            const int val = center[u + sv * L.pitch];
            m10 += u * val;
            m01 += sv * val;
        }
    }
    m10 = wave_sum(m10);
    m01 = wave_sum(m01);
    const float angle = orb_fast_atan2((float)m01, (float)m10);
    // ---- steered BRIEF on the blurred level
    const float ang = angle * (float)(3.14159265358979323846 / 180.f);
    float a, b;
    steer_sincos(ang, &b, &a);  // a = cos, b = sin
    const uint8_t* bc = blur + (size_t)f * g.pyr_frame_bytes + L.plane_off + (size_t)(y + kEdge) * L.pitch + (x + kEdge);
    unsigned long long words[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int j = 64 * m + lane;  // test j = byte j/8, bit j%8 (src:173-199)
        int t[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float px = (float)c_pattern[4 * j + 2 * e], py = (float)c_pattern[4 * j + 2 * e + 1];
            const int r = (int)__builtin_rintf(__builtin_fmaf(px, b, py * a));
            const int c = (int)__builtin_rintf(__builtin_fmaf(px, a, -(py * b)));
            t[e] = bc[r * L.pitch + c];
        }
        words[m] = ballot(t[0] < t[1]);
    }
    const int dst = dst_index[(size_t)f * g.sel_frame_cap + L.sel_off + slot];
    if (lane < 4) {
        unsigned long long* dd = reinterpret_cast<unsigned long long*>(desc + ((size_t)f * cap + dst) * 32);
        dd[lane] = words[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
    }
    if (lane == 0) {
        orb_keypoint_t k;
        float fx = (float)x, fy = (float)y;
        if (level != 0) { fx = fx * L.scale; fy = fy * L.scale; }
        k.x = fx; k.y = fy;
        k.size = (float)L.patch_size;
        k.angle = angle;
        k.response = (float)key_score(key);
        k.octave = level;
        k.class_id = -1;
        kps[(size_t)f * cap + dst] = k;
    }
}

}  // namespace

// ================================================================================================
// host side
// ================================================================================================
namespace orbgpu {

struct Extractor {
    Params P;
    int max_w = 0, max_h = 0, max_batch = 0;
    int cur_w = -1, cur_h = -1;
    Geometry geo;
    bool geo_ok = false;
    // device buffers
    CellDesc* d_cells = nullptr; size_t cells_cap = 0;
    int2* d_xtab = nullptr; size_t xtab_cap = 0;
    int4* d_ytab = nullptr; size_t ytab_cap = 0;
    uint8_t* d_pyr = nullptr; size_t pyr_cap = 0;
    uint8_t* d_blur = nullptr; size_t blur_cap = 0;
    uint32_t* d_cand = nullptr; size_t cand_cap = 0;
    uint32_t* d_scratch = nullptr; size_t scratch_cap = 0;
    int32_t* d_cell_count = nullptr; size_t cell_count_cap = 0;
    uint8_t* d_cell_thr = nullptr; size_t cell_thr_cap = 0;
    uint32_t* d_sel = nullptr; size_t sel_cap = 0;
    int32_t* d_dst = nullptr; size_t dst_cap = 0;
    int32_t* d_sel_count = nullptr; size_t selcount_cap = 0;
    int* d_status = nullptr;
    // synchronous path staging
    uint8_t* d_img = nullptr; size_t img_cap = 0;
    orb_keypoint_t* d_kps = nullptr; uint8_t* d_desc = nullptr; int32_t* d_counts = nullptr; size_t out_cap = 0;
    hipStream_t stream = nullptr;
    int last_n = 0;
    int qt_lds = 0;
    // optional per-stage timing: HIP events recorded on the launch stream between the stages
    bool profile = false;
    std::vector<hipEvent_t> events;   // kStages + 1 per profiled launch
    int ev_used = 0;                  // launches recorded since the last read
    long long frames_profiled = 0;
};

}  // namespace orbgpu

using orbgpu::Extractor;

namespace {

template <class T>
int grow(T*& p, size_t& cap, size_t need) {
    if (need <= cap && p) return ORB_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (need == 0) need = 1;
    if (hipMalloc(&p, need * sizeof(T)) != hipSuccess) { p = nullptr; return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed"); }
    cap = need;
    return ORB_OK;
}

int prepare(Extractor* e, int w, int h, int n) {
    if (w != e->cur_w || h != e->cur_h) {
        orbgpu::Geometry g;
        if (!orbgpu::build_geometry(e->P, w, h, g)) return orbgpu_fail(ORB_ERR_ARG, "image too small for the pyramid/cell grid");
        e->geo = g;
        e->cur_w = w;
        e->cur_h = h;
        int rc;
        if ((rc = grow(e->d_cells, e->cells_cap, g.cells.size())) != ORB_OK) return rc;
        if ((rc = grow(e->d_xtab, e->xtab_cap, std::max<size_t>(1, g.xtab.size() / 2))) != ORB_OK) return rc;
        if ((rc = grow(e->d_ytab, e->ytab_cap, std::max<size_t>(1, g.ytab.size() / 4))) != ORB_OK) return rc;
        if (hipMemcpy(e->d_cells, g.cells.data(), g.cells.size() * sizeof(orbgpu::CellDesc), hipMemcpyHostToDevice) != hipSuccess ||
            (!g.xtab.empty() && hipMemcpy(e->d_xtab, g.xtab.data(), g.xtab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
            (!g.ytab.empty() && hipMemcpy(e->d_ytab, g.ytab.data(), g.ytab.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
            return orbgpu_fail(ORB_ERR_DEVICE, "table upload failed");
        e->geo_ok = true;
    }
    const orbgpu::KernelGeom& k = e->geo.k;
    int rc;
    if ((rc = grow(e->d_pyr, e->pyr_cap, (size_t)k.pyr_frame_bytes * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_blur, e->blur_cap, (size_t)k.pyr_frame_bytes * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_cand, e->cand_cap, (size_t)k.cand_frame_cap * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_scratch, e->scratch_cap, (size_t)k.cand_frame_cap * n * 2)) != ORB_OK) return rc;
    if ((rc = grow(e->d_cell_count, e->cell_count_cap, (size_t)k.ncells * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_cell_thr, e->cell_thr_cap, (size_t)k.ncells * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_sel, e->sel_cap, (size_t)k.sel_frame_cap * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_dst, e->dst_cap, (size_t)k.sel_frame_cap * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_sel_count, e->selcount_cap, (size_t)k.nlevels * n)) != ORB_OK) return rc;
    return ORB_OK;
}

int launch_batch(Extractor* e, const uint8_t* d_images, int n, int w, int h, int stride, size_t frame_stride,
                 int lap0, int lap1, orb_keypoint_t* d_kps, uint8_t* d_desc, int cap, int32_t* d_counts,
                 hipStream_t st) {
    const orbgpu::Geometry& G = e->geo;
    const orbgpu::KernelGeom& k = G.k;
    hipEvent_t* ev = nullptr;
    if (e->profile) {
        const size_t need = (size_t)(e->ev_used + 1) * (orbgpu::kStages + 1);
        while (e->events.size() < need) {
            hipEvent_t x;
            if (hipEventCreate(&x) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipEventCreate failed");
            e->events.push_back(x);
        }
        ev = &e->events[(size_t)e->ev_used * (orbgpu::kStages + 1)];
        e->ev_used++;
        e->frames_profiled += n;
    }
    auto mark = [&](int i) { if (ev) hipEventRecord(ev[i], st); };
    hipMemsetAsync(e->d_status, 0, sizeof(int), st);
    mark(0);
    for (int l = 0; l < k.nlevels; ++l) {
        const orbgpu::LevelGeom& L = k.lv[l];
        dim3 grid((L.pw + kTileW - 1) / kTileW, (L.ph + kTileH - 1) / kTileH, n);
        if (l == 0)
            hipLaunchKernelGGL(k_pyramid_level<true>, grid, dim3(256), 0, st, k, 0, d_images, (long long)frame_stride,
                               stride, e->d_pyr, e->d_blur, e->d_xtab, e->d_ytab);
        else
            hipLaunchKernelGGL(k_pyramid_level<false>, grid, dim3(256), 0, st, k, l, nullptr, 0LL, 0, e->d_pyr,
                               e->d_blur, e->d_xtab, e->d_ytab);
    }
    mark(1);
    const int win_cap = (G.max_win + 15) & ~15;
    hipLaunchKernelGGL(k_fast_cells, dim3((k.ncells + 3) / 4, n), dim3(256), 4 * 2 * win_cap, st, k, e->d_cells,
                       win_cap, e->d_pyr, e->d_cand, e->d_cell_count, e->d_cell_thr);
    mark(2);
    hipLaunchKernelGGL(k_quadtree, dim3(k.nlevels, n), dim3(64), e->qt_lds, st, k, e->d_cells, e->d_cand,
                       e->d_cell_count, e->d_scratch, e->d_sel, e->d_sel_count, e->qt_lds, e->d_status);
    mark(3);
    hipLaunchKernelGGL(k_place, dim3(n), dim3(64), 0, st, k, e->d_sel, e->d_sel_count, e->d_dst, lap0, lap1, cap,
                       d_counts);
    mark(4);
    hipLaunchKernelGGL(k_describe, dim3((G.max_sel + 3) / 4, k.nlevels, n), dim3(256), 0, st, k, e->d_pyr, e->d_blur,
                       e->d_sel, e->d_sel_count, e->d_dst, d_counts, cap, d_kps, d_desc);
    mark(5);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "kernel launch failed");
    e->last_n = n;
    return ORB_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
extern "C" {

int orb_extractor_create(const orb_params_t* p, int max_width, int max_height, int max_batch, orb_extractor_t* out) {
    if (!p || !out || max_width <= 0 || max_height <= 0 || max_batch <= 0 || p->nlevels <= 0 ||
        p->nlevels > orbgpu::kMaxLevels || p->nfeatures < 0 || !(p->scale_factor > 1.0f) || max_width > 4095 ||
        max_height > 4095)
        return orbgpu_fail(ORB_ERR_ARG, "invalid extractor parameters");
    if (orb_device_count() <= 0) return orbgpu_fail(ORB_ERR_DEVICE, "no HIP device visible");
    Extractor* e = new Extractor();
    e->P = orbgpu::make_params(p->nfeatures, p->scale_factor, p->nlevels, p->ini_th_fast, p->min_th_fast);
    e->max_w = max_width;
    e->max_h = max_height;
    e->max_batch = max_batch;
    e->qt_lds = 80 * 1024;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&e->d_status, sizeof(int)) != hipSuccess) {
        delete e;
        return orbgpu_fail(ORB_ERR_DEVICE, "stream/status allocation failed");
    }
    hipFuncSetAttribute((const void*)k_quadtree, hipFuncAttributeMaxDynamicSharedMemorySize, e->qt_lds);
    *out = reinterpret_cast<orb_extractor_t>(e);
    return ORB_OK;
}

int orb_extractor_destroy(orb_extractor_t h) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e) return ORB_ERR_ARG;
    if (e->stream) hipStreamSynchronize(e->stream);
    void* bufs[] = {e->d_cells, e->d_xtab, e->d_ytab, e->d_pyr, e->d_blur, e->d_cand, e->d_scratch,
                    e->d_cell_count, e->d_cell_thr, e->d_sel, e->d_dst, e->d_sel_count, e->d_status,
                    e->d_img, e->d_kps, e->d_desc, e->d_counts};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t x : e->events) (void)hipEventDestroy(x);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
    return ORB_OK;
}

int orb_extractor_scales(orb_extractor_t h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                         int32_t* per_level) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e) return orbgpu_fail(ORB_ERR_ARG, "null handle");
    for (int l = 0; l < e->P.nlevels; ++l) {
        if (scale) scale[l] = e->P.scale[l];
        if (inv_scale) inv_scale[l] = e->P.inv_scale[l];
        if (sigma2) sigma2[l] = e->P.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = e->P.inv_sigma2[l];
        if (per_level) per_level[l] = e->P.per_level[l];
    }
    return e->P.nlevels;
}

int orb_extract_batch_device(orb_extractor_t h, const uint8_t* d_images, int n, int width, int height, int stride,
                             size_t frame_stride, int lap_x0, int lap_x1, orb_keypoint_t* d_kps, uint8_t* d_desc,
                             int cap, int32_t* d_counts, void* stream) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !d_images || !d_kps || !d_desc || !d_counts || n <= 0 || cap < 0)
        return orbgpu_fail(ORB_ERR_ARG, "null pointer or bad count");
    if (width <= 0 || height <= 0) return ORB_ERR_EMPTY;
    if (width > e->max_w || height > e->max_h || n > e->max_batch || stride < width)
        return orbgpu_fail(ORB_ERR_ARG, "frame larger than the extractor was created for");
    int rc = prepare(e, width, height, n);
    if (rc != ORB_OK) return rc;
    return launch_batch(e, d_images, n, width, height, stride, frame_stride, lap_x0, lap_x1, d_kps, d_desc, cap,
                        d_counts, (hipStream_t)stream);
}

int orb_extract(orb_extractor_t h, const uint8_t* image, int width, int height, int stride, int lap_x0, int lap_x1,
                orb_keypoint_t* kps, uint8_t* desc, int cap, int* n_kps) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (n_kps) *n_kps = 0;
    if (!e) return orbgpu_fail(ORB_ERR_ARG, "null handle");
    if (!image || width <= 0 || height <= 0) return ORB_ERR_EMPTY;  // src:1561-1562
    if ((cap > 0 && (!kps || !desc)) || cap < 0 || stride < width)
        return orbgpu_fail(ORB_ERR_ARG, "bad output buffers");
    if (width > e->max_w || height > e->max_h) return orbgpu_fail(ORB_ERR_ARG, "frame larger than the extractor");
    int rc = prepare(e, width, height, 1);
    if (rc != ORB_OK) return rc;
    const int dcap = std::max(cap, 1);
    if ((rc = grow(e->d_img, e->img_cap, (size_t)width * height)) != ORB_OK) return rc;
    if (e->out_cap < (size_t)dcap || !e->d_kps) {
        if (e->d_kps) hipFree(e->d_kps);
        if (e->d_desc) hipFree(e->d_desc);
        if (e->d_counts) hipFree(e->d_counts);
        e->d_kps = nullptr; e->d_desc = nullptr; e->d_counts = nullptr; e->out_cap = 0;
        if (hipMalloc(&e->d_kps, sizeof(orb_keypoint_t) * dcap) != hipSuccess ||
            hipMalloc(&e->d_desc, 32 * (size_t)dcap) != hipSuccess || hipMalloc(&e->d_counts, 8) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
        e->out_cap = dcap;
    }
    if (hipMemcpy2DAsync(e->d_img, width, image, stride, width, height, hipMemcpyHostToDevice, e->stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "upload failed");
    rc = launch_batch(e, e->d_img, 1, width, height, width, (size_t)width * height, lap_x0, lap_x1, e->d_kps,
                      e->d_desc, cap, e->d_counts, e->stream);
    if (rc != ORB_OK) return rc;
    int32_t cnt[2] = {0, 0};
    int status = 0;
    if (hipMemcpyAsync(cnt, e->d_counts, 8, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipMemcpyAsync(&status, e->d_status, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "download failed");
    if (status != 0) return orbgpu_fail(ORB_ERR_INTERNAL, "quad-tree capacity guard tripped");
    if (n_kps) *n_kps = cnt[0];
    if (cnt[1] < 0) return orbgpu_fail(ORB_ERR_CAPACITY, "output capacity too small");
    if (cnt[0] > 0) {
        if (hipMemcpy(kps, e->d_kps, sizeof(orb_keypoint_t) * cnt[0], hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(desc, e->d_desc, 32 * (size_t)cnt[0], hipMemcpyDeviceToHost) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "download failed");
    }
    return cnt[1];
}

int orb_extractor_level(orb_extractor_t h, int frame, int level, const uint8_t** d_view, int* width, int* height,
                        int* pitch) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !e->geo_ok || frame < 0 || frame >= e->last_n || level < 0 || level >= e->P.nlevels)
        return orbgpu_fail(ORB_ERR_ARG, "no such level");
    const orbgpu::LevelGeom& L = e->geo.k.lv[level];
    if (d_view)
        *d_view = e->d_pyr + (size_t)frame * e->geo.k.pyr_frame_bytes + L.plane_off + (size_t)orbgpu::kEdge * L.pitch +
                  orbgpu::kEdge;
    if (width) *width = L.w;
    if (height) *height = L.h;
    if (pitch) *pitch = L.pitch;
    return ORB_OK;
}

int orb_extractor_level_download(orb_extractor_t h, int frame, int level, uint8_t* host_padded) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !host_padded || !e->geo_ok || frame < 0 || frame >= e->last_n || level < 0 || level >= e->P.nlevels)
        return orbgpu_fail(ORB_ERR_ARG, "no such level");
    const orbgpu::LevelGeom& L = e->geo.k.lv[level];
    const uint8_t* src = e->d_pyr + (size_t)frame * e->geo.k.pyr_frame_bytes + L.plane_off;
    if (hipStreamSynchronize(e->stream) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy2D(host_padded, L.pw, src, L.pitch, L.pw, L.ph, hipMemcpyDeviceToHost) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "download failed");
    return ORB_OK;
}

// ---- debug / parity hooks (intermediates of the last call, frame `frame`)
int orb_debug_level_candidates(orb_extractor_t h, int frame, int level, uint32_t* out, int cap, uint8_t* thr_out,
                               int thr_cap) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !e->geo_ok || frame < 0 || frame >= e->last_n || level < 0 || level >= e->P.nlevels)
        return orbgpu_fail(ORB_ERR_ARG, "no such level");
    const orbgpu::KernelGeom& k = e->geo.k;
    const orbgpu::LevelGeom& L = k.lv[level];
    hipDeviceSynchronize();
    std::vector<int32_t> cnt(L.cell_count);
    std::vector<uint8_t> thr(L.cell_count);
    hipMemcpy(cnt.data(), e->d_cell_count + (size_t)frame * k.ncells + L.cell_begin, 4 * L.cell_count, hipMemcpyDeviceToHost);
    hipMemcpy(thr.data(), e->d_cell_thr + (size_t)frame * k.ncells + L.cell_begin, L.cell_count, hipMemcpyDeviceToHost);
    std::vector<uint32_t> all((size_t)L.cand_cap);
    hipMemcpy(all.data(), e->d_cand + (size_t)frame * k.cand_frame_cap + L.cand_off, 4 * (size_t)L.cand_cap,
              hipMemcpyDeviceToHost);
    int total = 0;
    for (int c = 0; c < L.cell_count; ++c) {
        const orbgpu::CellDesc& C = e->geo.cells[L.cell_begin + c];
        for (int i = 0; i < cnt[c]; ++i) {
            if (out && total < cap) out[total] = all[C.slot + i];
            total++;
        }
        if (thr_out && c < thr_cap) thr_out[c] = thr[c];
    }
    return total;
}

int orb_debug_level_selected(orb_extractor_t h, int frame, int level, uint32_t* out, int cap) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !e->geo_ok || frame < 0 || frame >= e->last_n || level < 0 || level >= e->P.nlevels)
        return orbgpu_fail(ORB_ERR_ARG, "no such level");
    const orbgpu::KernelGeom& k = e->geo.k;
    const orbgpu::LevelGeom& L = k.lv[level];
    hipDeviceSynchronize();
    int32_t n = 0;
    hipMemcpy(&n, e->d_sel_count + (size_t)frame * k.nlevels + level, 4, hipMemcpyDeviceToHost);
    if (out && n > 0)
        hipMemcpy(out, e->d_sel + (size_t)frame * k.sel_frame_cap + L.sel_off, 4 * (size_t)std::min(n, cap),
                  hipMemcpyDeviceToHost);
    return n;
}

int orb_debug_level_blurred(orb_extractor_t h, int frame, int level, uint8_t* host_view) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !host_view || !e->geo_ok || frame < 0 || frame >= e->last_n || level < 0 || level >= e->P.nlevels)
        return orbgpu_fail(ORB_ERR_ARG, "no such level");
    const orbgpu::LevelGeom& L = e->geo.k.lv[level];
    const uint8_t* src = e->d_blur + (size_t)frame * e->geo.k.pyr_frame_bytes + L.plane_off +
                         (size_t)orbgpu::kEdge * L.pitch + orbgpu::kEdge;
    hipDeviceSynchronize();
    if (hipMemcpy2D(host_view, L.w, src, L.pitch, L.w, L.h, hipMemcpyDeviceToHost) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "download failed");
    return ORB_OK;
}

// Per-stage timing (HIP events on the launch stream).  enable != 0 starts recording (and clears
// what was recorded); orb_extractor_stage_ms waits for the recorded launches and returns the summed
// milliseconds of [pyramid, fast, quadtree, place, describe] and the number of launches / frames.
int orb_extractor_profile(orb_extractor_t h, int enable) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e) return ORB_ERR_ARG;
    e->profile = enable != 0;
    e->ev_used = 0;
    e->frames_profiled = 0;
    return ORB_OK;
}

int orb_extractor_stage_ms(orb_extractor_t h, float* ms, int* launches, long long* frames) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !ms) return ORB_ERR_ARG;
    for (int s = 0; s < orbgpu::kStages; ++s) ms[s] = 0.f;
    for (int i = 0; i < e->ev_used; ++i) {
        hipEvent_t* ev = &e->events[(size_t)i * (orbgpu::kStages + 1)];
        if (hipEventSynchronize(ev[orbgpu::kStages]) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "event sync");
        for (int s = 0; s < orbgpu::kStages; ++s) {
            float t = 0.f;
            hipEventElapsedTime(&t, ev[s], ev[s + 1]);
            ms[s] += t;
        }
    }
    if (launches) *launches = e->ev_used;
    if (frames) *frames = e->frames_profiled;
    return ORB_OK;
}

int orb_debug_status(orb_extractor_t h) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e) return ORB_ERR_ARG;
    int s = 0;
    hipDeviceSynchronize();
    hipMemcpy(&s, e->d_status, 4, hipMemcpyDeviceToHost);
    return s;
}

}  // extern "C"
