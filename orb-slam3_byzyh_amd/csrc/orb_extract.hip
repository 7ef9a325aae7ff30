// MI355X (gfx950) ORB extraction: ORBextractor::operator() (reference src/ORBextractor.cc:1557-1682)
// as five batched HIP kernels over B frames:
//
//   k_pyramid_level  per level: the level view (INTER_LINEAR from the previous level) + a 3-px
//                    REFLECT_101 border inside the 19-px padded plane, one LDS tile pass
//   k_fast_cells     one wave per (frame, FAST cell): threshold-independent FAST-9 score, 3x3 NMS
//                    inside the cell window, iniTh/minTh choice, row-major candidate emission
//   k_quadtree_kp    one 256-thread workgroup per (frame, level): DistributeOctTree with exact list and
//                    std::sort semantics (keys stay put, node ids move), plus each keypoint's
//                    vLappingArea class rank (level-0 scaling, src:1656-1676)
//   k_describe       one half-wave per keypoint: IC_Angle (31-px disc) + steered rBRIEF (256 tests) on
//                    the keypoint's own 7x7 sigma-2 Gaussian, computed from a 43x43 patch in LDS
//
// No MFMA anywhere: this is byte / integer / popcount work.  All float arithmetic that reaches an
// output (resize coefficients are host tables; fastAtan2; pattern steering) is compiled with
// -ffp-contract=off and uses explicit fmaf() exactly where the reference's g++ -march=native build
// contracts (see orb_hd.h / orb_sincos.h and DESIGN.md).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "orb_extract_geom.h"
#include "orb_hd.h"
#include "orb_sincos.h"
#include "orbgpu.h"
#include "orbgpu_internal.h"

using namespace orbgpu;

namespace {

constexpr int kPatternSrc[1024] = {
#include "orb_pattern31.inc"
};
// test j -> one dword of 4 signed bytes (x0, y0, x1, y1); every coordinate is in [-13, 12]
struct PackedPattern { uint32_t w[256]; };
constexpr PackedPattern pack_pattern() {
    PackedPattern p{};
    for (int j = 0; j < 256; ++j)
        for (int c = 0; c < 4; ++c) p.w[j] |= (uint32_t)(uint8_t)(int8_t)kPatternSrc[4 * j + c] << (8 * c);
    return p;
}
__constant__ PackedPattern c_pattern_packed = pack_pattern();

__constant__ uint32_t c_sincos_exc[][3] = {
#include "orb_sincos_exceptions.inc"
};
constexpr int kNumSincosExc = sizeof(c_sincos_exc) / sizeof(c_sincos_exc[0]);

// IC_Angle disc (src:91-138, umax of ORBextractor's constructor, src:484-505) for HALF_PATCH_SIZE 15,
// pinned by tests/test_oracle_kat.py; build_geometry checks the host table against it.
constexpr int kDiscUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
// Per lane r (disc row v = r - 15; lane 31 outside), 8 mask dwords then 8 weight dwords over the 32
// columns u = -15 .. 16 as bytes: mask = [|u| <= umax[|v|]], weight = (u + 16) * mask.
struct DiscTable { uint32_t w[32][16]; };
constexpr DiscTable make_disc_table() {
    DiscTable t{};
    for (int r = 0; r < 31; ++r) {
        const int v = r - 15, U = kDiscUmax[v < 0 ? -v : v];
        for (int j = 0; j < 32; ++j) {
            const int u = j - 15;
            const uint32_t m = (u >= -U && u <= U) ? 1u : 0u;
            t.w[r][j >> 2] |= m << (8 * (j & 3));
            t.w[r][8 + (j >> 2)] |= (m * (uint32_t)(u + 16)) << (8 * (j & 3));
        }
    }
    return t;
}
__constant__ DiscTable c_disc = make_disc_table();

// 8-fraction-bit GaussianBlur(7x7, sigma=2) kernel of OpenCV's bit-exact 8U path
// (getGaussianKernelBitExact + error-diffusion fixed point): sums to 256.
__device__ __forceinline__ int blur_tap(int k) {
    return k == 3 ? 56 : (k == 2 || k == 4) ? 48 : (k == 1 || k == 5) ? 34 : 18;
}

// BORDER_REFLECT_101 index for offsets at most len-1 outside [0, len): one reflection, branch-free.
// Callers stay within the 19-px frame + 3-px blur halo and build_geometry requires len >= 38.
__device__ __forceinline__ int reflect101(int p, int len) {
    p = p < 0 ? -p : p;
    return p >= len ? 2 * len - 2 - p : p;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
// Sum over each 32-lane half of the wave, result in every lane of the half: DPP within the rows of 16
// (quad_perm xor 1 / xor 2, row_ror 4 / 8), then one ds_swizzle (xor 16 inside each 32-lane group),
// instead of five dependent ds_bpermute round trips.
__device__ __forceinline__ int half_wave_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v + __builtin_amdgcn_ds_swizzle(v, 0x401F);                // bitmask mode: lane ^ 16
}
__device__ __forceinline__ int rank_in(unsigned long long m) {  // set lanes below this one
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-wide sum (result uniform): DPP row sums (quad_perm xor 1 / xor 2, row_ror 4 / 8), then the
// four row totals by readlane -- no ds_bpermute round trips.
__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}
// Sum over each 16-lane row, in every lane of the row (DPP only)
__device__ __forceinline__ int row16_isum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v;
}
// Inclusive wave scans (GFX9 DPP): row_shr 1/2/3 on the input, row_shr 4 / 8 under bank masks, then
// row_bcast 15 / 31 across the rows.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    int s = v;
    s += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    s += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    s += __builtin_amdgcn_update_dpp(0, v, 0x113, 0xF, 0xF, false);  // row_shr:3
    s += __builtin_amdgcn_update_dpp(0, s, 0x114, 0xF, 0xE, false);  // row_shr:4, banks 1-3
    s += __builtin_amdgcn_update_dpp(0, s, 0x118, 0xF, 0xC, false);  // row_shr:8, banks 2-3
    s += __builtin_amdgcn_update_dpp(0, s, 0x142, 0xA, 0xF, false);  // row_bcast:15, rows 1, 3
    s += __builtin_amdgcn_update_dpp(0, s, 0x143, 0xC, 0xF, false);  // row_bcast:31, rows 2, 3
    return s;
}
// max-scan (INT_MIN is the identity for the lanes a DPP step leaves out)
__device__ __forceinline__ int wave_incl_max_dpp(int v) {
    constexpr int kId = -2147483647 - 1;
    int s = v;
    s = max(s, __builtin_amdgcn_update_dpp(kId, v, 0x111, 0xF, 0xF, false));
    s = max(s, __builtin_amdgcn_update_dpp(kId, v, 0x112, 0xF, 0xF, false));
    s = max(s, __builtin_amdgcn_update_dpp(kId, v, 0x113, 0xF, 0xF, false));
    s = max(s, __builtin_amdgcn_update_dpp(kId, s, 0x114, 0xF, 0xE, false));
    s = max(s, __builtin_amdgcn_update_dpp(kId, s, 0x118, 0xF, 0xC, false));
    s = max(s, __builtin_amdgcn_update_dpp(kId, s, 0x142, 0xA, 0xF, false));
    s = max(s, __builtin_amdgcn_update_dpp(kId, s, 0x143, 0xC, 0xF, false));
    return s;
}

// ================================================================================================
// 1. pyramid level: src:1687-1740 (ComputePyramid)
// ================================================================================================
constexpr int kBufDword3 = 0x00020000;  // gfx9 buffer resource word 3 (32-bit data format)

// Only the view and a kBorder-px REFLECT_101 border of each padded plane are written: FAST windows
// (src:1098-1166) and IC_Angle stay inside the view, and the one consumer of border pixels is
// k_describe's Gaussian, whose 7x7 taps around a sample <= 18 px from a keypoint at >= 19 px from the
// edge reach 2 px outside (the reference blurs a clone of the view with BORDER_REFLECT_101,
// src:1629-1637).  The rest of the 19-px frame is never read and never written.
constexpr int kBorder = 3;
// A tile is 128 x kTileH plane pixels, one lane per column; tiles start kBorder px before the view.
#ifndef ORBGPU_PYR_TILE_H
#define ORBGPU_PYR_TILE_H 24
#endif
constexpr int kTileW = 128, kTileH = ORBGPU_PYR_TILE_H;
static_assert(kTileH % 2 == 0, "two row halves per tile");
constexpr int kBoxW = 288, kBoxH = 2 * kTileH + 4;  // source box (bytes) for scale factors <= 2
static_assert(kBoxW >= 3 + 2 * kTileW + 2, "box too narrow");
// box for level ratios <= 1.25 (the usual 1.2): 128 * 1.25 + 2 columns + 3 alignment bytes, 24 * 1.25 + 2 rows
constexpr int kSmallBoxW = 176, kSmallBoxH = ((kTileH - 1) * 5 / 4 + 3 + 3) & ~3;
static_assert(kSmallBoxW >= 3 + (kTileW - 1) * 5 / 4 + 3 && kSmallBoxH >= (kTileH - 1) * 5 / 4 + 3, "small box too small");

// 8 bytes from a 4-byte-aligned LDS row at any byte offset, as aligned dword reads + v_alignbyte.
// (Adjacent byte reads would otherwise be merged by the compiler into unaligned ds_read_u16/b64,
// which gfx950 replays: SQ_LDS_UNALIGNED_STALL.)
__device__ __forceinline__ unsigned long long lds_bytes8(const uint8_t* row, int off) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(row) + (off >> 2);
    const unsigned sh = (unsigned)(off & 3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
    return lo | ((unsigned long long)hi << 32);
}

// XCD-aware tile order.  Blocks are dealt round-robin over the 8 XCDs in dispatch order (block b
// and b + 8 share an L2); handing each XCD a contiguous run of tiles keeps vertically adjacent tiles,
// which re-read the same source rows, in one L2.  Performance only: any placement is correct.
__device__ __forceinline__ int xcd_tile(int b, int share) { return (b & 7) * share + (b >> 3); }

// 7-tap GaussianBlur weights as packed u8 (horizontal pass, v_dot4_u32_u8) and u16 pairs (vertical
// pass, v_dot2_u32_u16 over row pairs: even output rows start on a pair, odd ones in its high half)
constexpr uint32_t kBlurK0 = 18u | 34u << 8 | 48u << 16 | 56u << 24, kBlurK1 = 48u | 34u << 8 | 18u << 16;
// the 7 taps shifted by k bytes against three consecutive words (word 0, 1, 2 of output column k)
constexpr uint32_t kBlurS0[4] = {kBlurK0, 18u << 8 | 34u << 16 | 48u << 24, 18u << 16 | 34u << 24, 18u << 24};
constexpr uint32_t kBlurS1[4] = {kBlurK1, 56u | 48u << 8 | 34u << 16 | 18u << 24, 48u | 56u << 8 | 48u << 16 | 34u << 24,
                                 34u | 48u << 8 | 56u << 16 | 48u << 24};
constexpr uint32_t kBlurS2[4] = {0u, 0u, 18u, 34u | 18u << 8};
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 w16(unsigned a, unsigned b) { u16x2 v; v.x = (unsigned short)a; v.y = (unsigned short)b; return v; }
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

// One workgroup = one 128 x kTileH tile of a level's written region (view + kBorder).
// Level 0 copies the input; level l > 0 resizes the previous level view.  The source pixels the tile
// needs are staged in LDS (one round of independent loads), then the resize is written for few VALU
// instructions per pixel (the pyramid is VALU-bound, PMC round 2): lane per tile column,
// wave-uniform rows; the column's INTER_LINEAR coefficients stay in registers, the row coefficients
// are one broadcast LDS read, and every tile row's two source rows are interpolated horizontally.
// Level geometry by value (kernel arguments): no dependent load of the geometry block before the
// source loads can be addressed.
struct PyrArgs {
    long long frame_bytes;         // one frame's pyramid block
    long long plane_off, src_off;  // this level's padded plane; the previous level's view origin
    int w, h, pw, ph, pitch;       // this level
    int sw, sh, spitch;            // previous level view (level > 0)
    int xtab_off, ytab_off, simd_end;
    int tiles_per_frame, share;    // share: tiles of a frame per XCD (blockIdx.x -> tile, pyr_tile)
    int tab_off;                   // this level's tile table (tile_tables)
    int frame_affine;              // 1: every tile of frame f on XCD f % 8 (frames a multiple of 8)
};

template <bool kLevel0, int kBH = kSmallBoxH, int kBW = kSmallBoxW>
__global__ __launch_bounds__(256, 8) void k_pyramid_level(const PyrArgs A, const uint8_t* __restrict__ in,
                                                          long long in_frame_stride, int in_stride,
                                                          uint8_t* __restrict__ pyr,
                                                          const int2* __restrict__ xtab, const int4* __restrict__ ytab,
                                                          const int4* __restrict__ tiletab,
                                                          unsigned long long* __restrict__ stamps,
                                                          int* __restrict__ status_reset) {
    // level 0 clears the batch's error status (read after the quad-tree), instead of a memset launch
    if (kLevel0 && status_reset && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *status_reset = 0;
    // blockIdx.y = frame; blockIdx.x -> tile of the frame, XCD-chunked (xcd_tile).  Frame-affine
    // (round 5): the dispatch deals linear block L to XCD L % 8, so XCD j runs its blocks in the order
    // L >> 3 over all tiles of its frames j, j + 8, ...: a frame's halo re-reads and the next level's
    // reads of this one stay in one L2.
    int t, f;
    if (A.frame_affine) {
        const int L = blockIdx.y * gridDim.x + blockIdx.x, s8 = L >> 3;
        const int q = s8 / A.tiles_per_frame;
        t = s8 - q * A.tiles_per_frame;
        f = (L & 7) + 8 * q;
        if (f >= (int)gridDim.y) return;
    } else {
        t = xcd_tile(blockIdx.x, A.share);
        if (t >= A.tiles_per_frame) return;
        f = blockIdx.y;
    }
    // debug (ORBGPU_PYR_STAMPS): per-block phase clocks, thread 0 of each block
    unsigned long long* stp = stamps ? stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 : nullptr;
    if (stp && threadIdx.x == 0) { stp[6] = wall_clock64(); stp[0] = __builtin_amdgcn_s_memtime(); }
#define PYR_STAMP(k) do { if (stp && threadIdx.x == 0) stp[k] = __builtin_amdgcn_s_memtime(); } while (0)
    // tile record (scalar load): origin, and for level > 0 the previous-level view box it reads
    const int4 T = tiletab[A.tab_off + t];
    constexpr int kBoxWords = kBW / 4;
    __shared__ __attribute__((aligned(16))) uint8_t box[kLevel0 ? 4 : kBH * kBW];
    __shared__ __attribute__((aligned(16))) uint8_t tile[kTileH][kTileW + 8];  // +8: lds_bytes8 over-read
    __shared__ int4 yrow[kLevel0 ? 1 : kTileH];  // per tile row: box row offsets of the two source rows, weights
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uniform(tid >> 6);
    const int X0 = T.x & 0xffff, Y0 = T.x >> 16;
    uint8_t* plane = pyr + (size_t)f * A.frame_bytes + A.plane_off;
    // the written region in plane coordinates, and this lane's tile column (waves 0/1: the upper half
    // of the rows, waves 2/3: the lower half) in view coordinates; columns and rows past the region
    // are clamped to its last one (computed, never stored)
    const int ex = kEdge + A.w + kBorder, ey = kEdge + A.h + kBorder;
    const int tx = (wave & 1) * 64 + lane, r0 = (wave >> 1) * (kTileH / 2);
    const int vx = reflect101(min(X0 + tx, ex - 1) - kEdge, A.w);
    if (kLevel0) {
        // level 0: the written region is the input with REFLECT_101 borders.  Each thread makes 8
        // consecutive plane bytes of a tile row (16 threads per 128-px row, 16 rows per pass) and
        // stores them at once (plane columns of a chunk start 8-aligned).  Interior chunks are two
        // v_alignbyte of three aligned dwords of the input row (buffer loads over the frame rounded up
        // to whole dwords -- an aligned dword never crosses a page -- and 0 past it); chunks that touch
        // the view's left or right edge go byte by byte through reflect101.
        (void)vx; (void)r0;
        const uint8_t* fbase = in + (size_t)f * in_frame_stride;
        const uintptr_t fb = reinterpret_cast<uintptr_t>(fbase);
        const int fmis = uniform((int)(fb & 3));
        const uint64_t fal = (uint64_t)(uint32_t)uniform((int)(uint32_t)(fb - fmis)) |
                             (uint64_t)(uint32_t)uniform((int)(uint32_t)((fb - fmis) >> 32)) << 32;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>(fal), (short)0, uniform((fmis + (A.h - 1) * in_stride + A.w + 3) & ~3), kBufDword3);
        const int c = (tid & 15) * 8, px = X0 + c, x0 = px - kEdge;
        const bool interior = x0 >= 0 && x0 + 8 <= A.w;
        constexpr int kPasses = (kTileH + 15) / 16;
        unsigned long long val[kPasses];
#pragma unroll
        for (int ps = 0; ps < kPasses; ++ps) {
            const int r = (tid >> 4) + 16 * ps;
            const int vy = reflect101(min(Y0 + r, ey - 1) - kEdge, A.h);
            if (interior) {
                const int off = fmis + vy * in_stride + x0, oa = off & ~3, sh = off & 3;
                const uint32_t w0 = __builtin_amdgcn_raw_buffer_load_b32(rs, oa, 0, 0);
                const uint32_t w1 = __builtin_amdgcn_raw_buffer_load_b32(rs, oa, 4, 0);
                const uint32_t w2 = __builtin_amdgcn_raw_buffer_load_b32(rs, oa, 8, 0);
                val[ps] = __builtin_amdgcn_alignbyte(w1, w0, sh) |
                          (unsigned long long)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32;
            } else {
                const uint8_t* srow = fbase + (size_t)vy * in_stride;
                unsigned long long v8 = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    v8 |= (unsigned long long)srow[reflect101(min(px + i, ex - 1) - kEdge, A.w)] << (8 * i);
                val[ps] = v8;
            }
        }
        PYR_STAMP(1);
        PYR_STAMP(2);
#pragma unroll
        for (int ps = 0; ps < kPasses; ++ps) {
            const int r = (tid >> 4) + 16 * ps, py = Y0 + r;
            if (r >= kTileH || py >= ey || px >= ex) continue;
            uint8_t* dst = plane + (size_t)py * A.pitch + px;
            if (px + 7 < ex) {
                *reinterpret_cast<unsigned long long*>(dst) = val[ps];
            } else {
                for (int i = 0; i < 8 && px + i < ex; ++i) dst[i] = (uint8_t)(val[ps] >> (8 * i));
            }
        }
        if (stp) {
            PYR_STAMP(3);
            if (threadIdx.x == 0) { stp[4] = stp[5] = stp[3]; stp[7] = wall_clock64(); }
        }
        return;
    } else {
        const int bx0 = T.y & 0xffff, bw = T.y >> 16, by0 = T.z & 0xffff, bh = T.z >> 16;
        // source box as aligned dwords (over-reads stay inside the previous level's padded plane);
        // src_off and spitch are multiples of 128, so every box row has the same alignment.  Buffer
        // loads: one 32-bit lane offset, the row step in the scalar offset.
        const int shift = (int)((A.src_off + bx0) & 3);  // plane and frame blocks are 256-B aligned
        // The whole kBH x kBW box is loaded (rows and words past the tile's need are never read); the
        // descriptor's range ends with the frame's pyramid block, so reads past it return 0.
        const long long box_off = A.src_off + (long long)by0 * A.spitch + (bx0 - shift);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            pyr + (size_t)f * A.frame_bytes + box_off, (short)0, (int)(A.frame_bytes - box_off), kBufDword3);
        (void)bh;
        uint32_t* boxw = reinterpret_cast<uint32_t*>(box);
        const int rg = tid >> 6;
        // every global load of the block issued before the first LDS store (one round trip): the box,
        // the row coefficients (kTileH lanes) and this lane's column coefficients
        constexpr int kRowPass = kBH / 4, kWordPass = (kBoxWords + 63) / 64;
        uint32_t v[kRowPass][kWordPass];
#pragma unroll
        for (int q = 0; q < kRowPass; ++q)
#pragma unroll
            for (int hx = 0; hx < kWordPass; ++hx) {
                const int w = lane + 64 * hx;
                v[q][hx] = (w < kBoxWords)
                               ? __builtin_amdgcn_raw_buffer_load_b32(rs, rg * A.spitch + 4 * w, 4 * q * A.spitch, 0) : 0u;
            }
        int4 yv = make_int4(0, 0, 0, 0);
        if (tid < kTileH) yv = ytab[A.ytab_off + reflect101(min(Y0 + tid, ey - 1) - kEdge, A.h)];
        const int2 X = xtab[A.xtab_off + vx];
#pragma unroll
        for (int q = 0; q < kRowPass; ++q)
#pragma unroll
            for (int hx = 0; hx < kWordPass; ++hx) {
                const int r = 4 * q + rg, w = lane + 64 * hx;
                if (w < kBoxWords) boxw[r * kBoxWords + w] = v[q][hx];
            }
        // row coefficients pre-shifted by 8 for v_mul_hi_u32_u24 (SIMD path, below)
        if (tid < kTileH) yrow[tid] = make_int4((yv.x - by0) * kBW, (yv.y - by0) * kBW, yv.z << 8, yv.w << 8);
        __syncthreads();
        PYR_STAMP(1);
        // INTER_LINEAR down the column: both source rows of every tile row are interpolated
        // horizontally (no row-to-row dependency, so the unrolled loop keeps many LDS reads in flight).
        // VResizeLinearVec_32s8u (vx < simd_end): v_mul_hi on S >> 4 (S <= 255 * 2049, so S >> 4 <
        // 32767 and the reference's int16 saturation never triggers), rounding shift by 2;
        // else FixedPtCast<int, uchar, 22>.
        // (two separate byte reads: an adjacent pair would be merged into an unaligned ds_read_u16,
        // which gfx950 replays -- measured 5x slower for the whole phase)
        const int sx = X.x - bx0 + shift, sx1 = min(X.x + 1, bx0 + bw - 1) - bx0 + shift;
        const unsigned a0 = X.y & 0xffff, a1 = (unsigned)X.y >> 16;
        const bool simd = vx < A.simd_end;
        auto stream = [&](auto mixed) {
            constexpr bool kMixed = decltype(mixed)::value;
            const int hs = simd ? 4 : 0;
            auto hrow = [&](int off) {
                const int h = (int)(__umul24(box[off + sx], a0) + __umul24(box[off + sx1], a1));
                return kMixed ? h >> hs : h >> 4;
            };
#pragma unroll
            for (int k = 0; k < kTileH / 2; ++k) {
                const int4 Y = yrow[r0 + k];  // LDS broadcast
                const int p0 = (int)__umul24((unsigned)hrow(Y.x), (unsigned)Y.z >> 8);  // < 2^20 * 2^11
                const int p1 = (int)__umul24((unsigned)hrow(Y.y), (unsigned)Y.w >> 8);
                int v = ((p0 >> 16) + (p1 >> 16) + 2) >> 2;  // <= (2 * 1020 + 2) >> 2 = 255
                if (kMixed && !simd) v = min((p0 + p1 + (1 << 21)) >> 22, 255);
                tile[r0 + k][tx] = (uint8_t)v;
            }
        };
        if (__ballot(!simd) == 0) {
            // Every column of the wave on the SIMD path (12 VALU per pixel instead of 16):
            // h = s0 * a0 + s1 * a1 is v_dot2_u32_u16 on the byte pair (one ds_read2 + v_perm), kept
            // as H = (h >> 4) << 8, so that (H * (b << 8)) >> 32 = ((h >> 4) * b) >> 16, the
            // reference's _mm_mulhi_epi16, is one v_mul_hi_u32_u24 (H < 2^23, b << 8 <= 2^19).
            // (Reusing a source row's H for the next tile row, with the rows as scalar loads and the
            // reuse as a scalar branch, saves 2 more VALU per pixel but serialises the LDS reads on
            // the scalar loads' lgkmcnt: measured 15-25 % slower per level.)
            const int sxa = sx & ~3;
            const uint32_t sel = (uint32_t)(sx & 3) | 0x0c00u | (uint32_t)((sx & 3) + 1) << 16 | 0x0c000000u;
            const u16x2 A16 = w16(a0 << 4, a1 << 4);  // 16 * h: the floor of h / 16 is a mask
            auto H = [&](int row_off) -> uint32_t {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(box + row_off + sxa);
                const uint32_t pair = __builtin_amdgcn_perm(p[1], p[0], sel);  // s0 | s1 << 16
                return __builtin_amdgcn_udot2(as_u16x2(pair), A16, 0u, false) & 0xffffff00u;
            };
            uint8_t* out = &tile[r0][tx];
#pragma unroll
            for (int k = 0; k < kTileH / 2; ++k) {
                const int4 Y = yrow[r0 + k];  // LDS broadcast
                const uint32_t HA = H(Y.x), HB = H(Y.y);
                uint32_t m0, m1;
                asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m0) : "v"(HA), "v"(Y.z));
                asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m1) : "v"(HB), "v"(Y.w));
                out[k * (kTileW + 8)] = (uint8_t)((m0 + m1 + 2) >> 2);
            }
        } else {
            stream(std::true_type{});
        }
        __syncthreads();
        PYR_STAMP(2);
    }
    // store: 8 consecutive pixels per thread, 16 rows per pass, clipped to the written region
#pragma unroll
    for (int r = tid >> 4; r < kTileH; r += 16) {
        const int c = (tid & 15) * 8;
        const int py = Y0 + r, px = X0 + c;
        if (py < ey && px < ex) {
            uint8_t* dst = plane + (size_t)py * A.pitch + px;
            if (px + 7 < ex) {
                *reinterpret_cast<unsigned long long*>(dst) = lds_bytes8(tile[r], c);
            } else {
                for (int k = 0; k < 8 && px + k < ex; ++k) dst[k] = tile[r][c + k];
            }
        }
    }
    if (stp) {
        PYR_STAMP(3);
        if (threadIdx.x == 0) { stp[4] = stp[5] = stp[3]; stp[7] = wall_clock64(); }
    }
#undef PYR_STAMP
}

// One lane's output column over kN rows out of an LDS source box: k_pyramid_level's resize in its two
// forms (the SIMD-path form when every lane of the wave is on the 128-bit vertical path, else the mixed
// form).  yr: per output row the two source-row byte offsets into `box` and the row weights << 8;
// sx / sx1: the column's taps relative to a box row, a0 / a1 its weights.  Stores where `ok`.
template <int kN, int kYS = 1>
__device__ __forceinline__ void pyr_resize_col(const uint8_t* __restrict__ box, const int4* __restrict__ yr, int sx,
                                               int sx1, unsigned a0, unsigned a1, bool simd, bool ok,
                                               uint8_t* __restrict__ out, int ostride) {
    if (__ballot(!simd) == 0) {
        const int sxa = sx & ~3;
        const uint32_t sel = (uint32_t)(sx & 3) | 0x0c00u | (uint32_t)((sx & 3) + 1) << 16 | 0x0c000000u;
        const u16x2 A16 = w16(a0 << 4, a1 << 4);
        auto H = [&](int row_off) -> uint32_t {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(box + row_off + sxa);
            const uint32_t pair = __builtin_amdgcn_perm(p[1], p[0], sel);  // s0 | s1 << 16
            return __builtin_amdgcn_udot2(as_u16x2(pair), A16, 0u, false) & 0xffffff00u;
        };
#pragma unroll
        for (int k = 0; k < kN; ++k) {
            const int4 Y = yr[k * kYS];  // LDS broadcast
            const uint32_t HA = H(Y.x), HB = H(Y.y);
            uint32_t m0, m1;
            asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m0) : "v"(HA), "v"(Y.z));
            asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(m1) : "v"(HB), "v"(Y.w));
            if (ok) out[k * ostride] = (uint8_t)((m0 + m1 + 2) >> 2);
        }
    } else {
        const int hs = simd ? 4 : 0;
        auto hrow = [&](int off) { return (int)(__umul24(box[off + sx], a0) + __umul24(box[off + sx1], a1)) >> hs; };
#pragma unroll
        for (int k = 0; k < kN; ++k) {
            const int4 Y = yr[k * kYS];
            const int p0 = (int)__umul24((unsigned)hrow(Y.x), (unsigned)Y.z >> 8);
            const int p1 = (int)__umul24((unsigned)hrow(Y.y), (unsigned)Y.w >> 8);
            int v = ((p0 >> 16) + (p1 >> 16) + 2) >> 2;
            if (!simd) v = min((p0 + p1 + (1 << 21)) >> 22, 255);
            if (ok) out[k * ostride] = (uint8_t)v;
        }
    }
}

// Two levels per pass (round 6).  One workgroup makes a 128 x kTileH tile of level l + 1 -- the tile grid
// and tile records of k_pyramid_level -- and, on the way, the box U of level l that the tile reads:
// INTER_LINEAR from an LDS box C of level l - 1, or for l = 0 the input rows themselves.  It also writes
// the level-l pixels it owns: the level-(l+1) tiles' columns and rows cut level l's written region (view
// + 3-px border) into disjoint shares, each inside its tile's U together with its REFLECT_101 sources.
// Level l is therefore never read back from memory by level l + 1, and a batch's pyramid takes 4
// launches instead of 8.  The arithmetic is k_pyramid_level's; where two tiles' U overlap, both compute
// the same values.
constexpr int kPairUP = 164, kPairUH = 32;  // U: row pitch (>= U width + 8: dword over-read), rows
constexpr int kPairCW = 200, kPairCH = 40;  // C: row pitch (>= C width + 3 alignment + 8), rows (x4)
static_assert(kPairCH * kPairCW >= kTileH * (kTileW + 8), "the tile reuses C's LDS");
static_assert(kPairUH == 4 * 8, "U rows: 8 per wave");

struct PairArgs {
    long long frame_bytes;
    long long plane_l, plane_n;  // padded planes of level l and l + 1
    long long src_off;           // level l - 1 view origin (l > 0)
    int wl, hl, pitch_l, xtab_l, ytab_l, simd_l;  // level l (its tables: the resize from level l - 1)
    int wn, hn, pitch_n, xtab_n, ytab_n, simd_n;  // level l + 1
    int spitch;                                   // level l - 1 row pitch
    int tiles_per_frame, share, tab_off, frame_affine;
};

template <bool kFirst>
__global__ __launch_bounds__(256, 8) void k_pyramid_pair(const PairArgs A, const uint8_t* __restrict__ in,
                                                         long long in_frame_stride, int in_stride,
                                                         uint8_t* __restrict__ pyr, const int2* __restrict__ xtab,
                                                         const int4* __restrict__ ytab,
                                                         const int4* __restrict__ tiletab,
                                                         const int4* __restrict__ pairtab,
                                                         int* __restrict__ status_reset) {
    if (kFirst && status_reset && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *status_reset = 0;
    int t, f;  // tile of level l + 1 and frame, as k_pyramid_level
    if (A.frame_affine) {
        const int L = blockIdx.y * gridDim.x + blockIdx.x, s8 = L >> 3;
        const int q = s8 / A.tiles_per_frame;
        t = s8 - q * A.tiles_per_frame;
        f = (L & 7) + 8 * q;
        if (f >= (int)gridDim.y) return;
    } else {
        t = xcd_tile(blockIdx.x, A.share);
        if (t >= A.tiles_per_frame) return;
        f = blockIdx.y;
    }
    const int4 T = tiletab[A.tab_off + t];
    const int4 P = pairtab[2 * (A.tab_off + t)], O = pairtab[2 * (A.tab_off + t) + 1];
    const int X0 = T.x & 0xffff, Y0 = T.x >> 16;
    const int ux0 = P.x & 0xffff, uw = P.x >> 16, uy0 = P.y & 0xffff, uh = P.y >> 16;
    const int cx0 = P.z & 0xffff, cw = P.z >> 16, cy0 = P.w & 0xffff, ch = P.w >> 16;
    const int ox0 = (int)(int16_t)(O.x & 0xffff), ox1 = O.x >> 16, oy0 = (int)(int16_t)(O.y & 0xffff), oy1 = O.y >> 16;
    // C, then (once U is made) the level-(l+1) tile: one LDS area
    __shared__ __attribute__((aligned(16))) uint8_t cbox[kFirst ? kTileH * (kTileW + 8) : kPairCH * kPairCW];
    __shared__ __attribute__((aligned(16))) uint8_t ubuf[kPairUH * kPairUP];
    uint8_t (*tile)[kTileW + 8] = reinterpret_cast<uint8_t (*)[kTileW + 8]>(cbox);  // +8: lds_bytes8 over-read
    __shared__ int4 yrowU[kPairUH];
    __shared__ int4 yrowT[kTileH];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uniform(tid >> 6);
    uint8_t* plane_l = pyr + (size_t)f * A.frame_bytes + A.plane_l;
    uint8_t* plane_n = pyr + (size_t)f * A.frame_bytes + A.plane_n;
    // the level-(l+1) tile: written region, this lane's column (view coordinates) and its taps in U
    const int ex = kEdge + A.wn + kBorder, ey = kEdge + A.hn + kBorder;
    const int tx = (wave & 1) * 64 + lane, r0 = (wave >> 1) * (kTileH / 2);
    const int vxn = reflect101(min(X0 + tx, ex - 1) - kEdge, A.wn);
    // 1. every global load of the block before the first LDS store
    int2 XU[3] = {make_int2(0, 0), make_int2(0, 0), make_int2(0, 0)};
    int4 yu = make_int4(0, 0, 0, 0);
    int shift = 0;
    if (kFirst) {
        // U = input pixels [ux0, ux0 + uw) x [uy0, uy0 + uh): per row (wave-uniform) the aligned dwords
        // from the row's first byte, realigned by v_alignbyte (buffer loads over the frame rounded up to
        // whole dwords; 0 past it)
        const uint8_t* fbase = in + (size_t)f * in_frame_stride;
        const uintptr_t fb = reinterpret_cast<uintptr_t>(fbase);
        const int fmis = uniform((int)(fb & 3));
        const uint64_t fal = (uint64_t)(uint32_t)uniform((int)(uint32_t)(fb - fmis)) |
                             (uint64_t)(uint32_t)uniform((int)(uint32_t)((fb - fmis) >> 32)) << 32;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>(fal), (short)0, uniform((fmis + (A.hl - 1) * in_stride + A.wl + 3) & ~3), kBufDword3);
        uint32_t w0[8], w1[8];
        int sh[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int y = uy0 + min(wave + 4 * q, uh - 1);
            const int off = uniform(fmis + y * in_stride + ux0), oa = off & ~3;
            sh[q] = off & 3;
            w0[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, oa + 4 * lane, 0, 0);
            w1[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, oa + 4 * lane + 4, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (4 * lane < kPairUP)
                reinterpret_cast<uint32_t*>(ubuf + (wave + 4 * q) * kPairUP)[lane] = __builtin_amdgcn_alignbyte(w1[q], w0[q], sh[q]);
    } else {
        // C = level l - 1 view box [cx0, cx0 + cw) x [cy0, cy0 + ch) as aligned dwords (k_pyramid_level's
        // box load, bounded to the rows and words the resize reads)
        shift = (int)((A.src_off + cx0) & 3);
        const long long box_off = A.src_off + (long long)cy0 * A.spitch + (cx0 - shift);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            pyr + (size_t)f * A.frame_bytes + box_off, (short)0, (int)(A.frame_bytes - box_off), kBufDword3);
        const int cwords = min((cw + shift + 3) / 4 + 1, kPairCW / 4), rg = tid >> 6;
        constexpr int kRowPass = kPairCH / 4;
        uint32_t v[kRowPass];
#pragma unroll
        for (int q = 0; q < kRowPass; ++q)
            v[q] = (4 * q + rg < ch && lane < cwords)
                       ? __builtin_amdgcn_raw_buffer_load_b32(rs, rg * A.spitch + 4 * lane, 4 * q * A.spitch, 0) : 0u;
#pragma unroll
        for (int c = 0; c < 2; ++c) XU[c] = xtab[A.xtab_l + ux0 + min(64 * c + lane, uw - 1)];
        XU[2] = xtab[A.xtab_l + ux0 + min(128 + (lane & 31), uw - 1)];
        if (tid < kPairUH) yu = ytab[A.ytab_l + uy0 + min(tid, uh - 1)];
#pragma unroll
        for (int q = 0; q < kRowPass; ++q)
            if (lane < kPairCW / 4) reinterpret_cast<uint32_t*>(cbox + (4 * q + rg) * kPairCW)[lane] = v[q];
        if (tid < kPairUH)
            yrowU[tid] = make_int4((yu.x - cy0) * kPairCW, (yu.y - cy0) * kPairCW, yu.z << 8, yu.w << 8);
    }
    int4 yv = make_int4(0, 0, 0, 0);
    if (tid < kTileH) yv = ytab[A.ytab_n + reflect101(min(Y0 + tid, ey - 1) - kEdge, A.hn)];
    const int2 XN = xtab[A.xtab_n + vxn];
    if (tid < kTileH) yrowT[tid] = make_int4((yv.x - uy0) * kPairUP, (yv.y - uy0) * kPairUP, yv.z << 8, yv.w << 8);
    __syncthreads();
    // 2. U from C (l > 0): lane per U column, wave per 8 rows -- columns 0-127 in two 64-lane passes,
    //    columns 128.. (at most 28: U is at most kPairUP - 8 wide) as two rows per pass, half-waves on
    //    alternate rows; rows past uh repeat the last one (never read), columns past uw are not stored
    if (!kFirst) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (64 * c >= uw) break;
            const int col = 64 * c + lane, vx = ux0 + min(col, uw - 1);
            const int sx = XU[c].x - cx0 + shift, sx1 = min(XU[c].x + 1, cx0 + cw - 1) - cx0 + shift;
            pyr_resize_col<8>(cbox, &yrowU[8 * wave], sx, sx1, (unsigned)XU[c].y & 0xffffu, (unsigned)XU[c].y >> 16,
                              vx < A.simd_l, col < uw, &ubuf[8 * wave * kPairUP + col], kPairUP);
        }
        if (uw > 128) {
            const int col = 128 + (lane & 31), half = lane >> 5, vx = ux0 + min(col, uw - 1);
            const int sx = XU[2].x - cx0 + shift, sx1 = min(XU[2].x + 1, cx0 + cw - 1) - cx0 + shift;
            pyr_resize_col<4, 2>(cbox, &yrowU[8 * wave + half], sx, sx1, (unsigned)XU[2].y & 0xffffu,
                                 (unsigned)XU[2].y >> 16, vx < A.simd_l, col < uw,
                                 &ubuf[(8 * wave + half) * kPairUP + col], 2 * kPairUP);
        }
        __syncthreads();
    }
    // 3a. the owned share of level l: [ox0, ox1) x [oy0, oy1) in view coordinates (border included), 8
    //     plane bytes per lane (interior chunks by lds_bytes8), nch chunks per row, 64 / nch rows per
    //     wave pass (nch <= 21: the share is at most ~157 bytes wide)
    {
        const int pc0 = (ox0 + kEdge) & ~7;
        const int nch = ((ox1 + kEdge - 1) >> 3) - (pc0 >> 3) + 1;
        const int rpp = 64 / nch, lr = lane / nch, ch = lane - lr * nch;
        const int nrow = oy1 - oy0;
        for (int r0o = rpp * wave; r0o < nrow; r0o += 4 * rpp) {
            const int r = r0o + lr;
            if (lr < rpp && r < nrow) {
                const int y = oy0 + r;
                const uint8_t* urow = ubuf + (reflect101(y, A.hl) - uy0) * kPairUP;
                uint8_t* dst = plane_l + (size_t)(y + kEdge) * A.pitch_l;
                const int pc = pc0 + 8 * ch, x = pc - kEdge;
                if (x >= ox0 && x + 8 <= ox1 && x >= 0 && x + 8 <= A.wl) {
                    *reinterpret_cast<unsigned long long*>(dst + pc) = lds_bytes8(urow, x - ux0);
                } else {
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        if (x + b >= ox0 && x + b < ox1) dst[pc + b] = urow[reflect101(x + b, A.wl) - ux0];
                }
            }
        }
    }
    // 3b. the level-(l+1) tile from U
    {
        const int sx = XN.x - ux0, sx1 = min(XN.x + 1, ux0 + uw - 1) - ux0;
        pyr_resize_col<kTileH / 2>(ubuf, &yrowT[r0], sx, sx1, (unsigned)XN.y & 0xffffu, (unsigned)XN.y >> 16,
                                   vxn < A.simd_n, true, &tile[r0][tx], kTileW + 8);
    }
    __syncthreads();
    // 4. store the tile: 8 consecutive pixels per thread, 16 rows per pass, clipped to the written region
#pragma unroll
    for (int r = tid >> 4; r < kTileH; r += 16) {
        const int c = (tid & 15) * 8;
        const int py = Y0 + r, px = X0 + c;
        if (py < ey && px < ex) {
            uint8_t* dst = plane_n + (size_t)py * A.pitch_n + px;
            if (px + 7 < ex) {
                *reinterpret_cast<unsigned long long*>(dst) = lds_bytes8(tile[r], c);
            } else {
                for (int k = 0; k < 8 && px + k < ex; ++k) dst[k] = tile[r][c + k];
            }
        }
    }
}

// Debug (orb_debug_level_blurred): the reference's GaussianBlur(level.clone(), 7x7, 2, 2,
// BORDER_REFLECT_101) of a whole level view, one thread per pixel, from the stored view (the
// descriptor kernel blurs only its own samples; this is the test hook for that arithmetic).
__global__ __launch_bounds__(256) void k_debug_blur(const uint8_t* __restrict__ view, int pitch, int w, int h,
                                                    uint8_t* __restrict__ out) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= w) return;
    uint32_t acc = 1u << 15;
    for (int i = 0; i < 7; ++i) {
        const uint8_t* row = view + (size_t)reflect101(y + i - 3, h) * pitch;
        uint32_t hs = 0;
        for (int k = 0; k < 7; ++k) hs += (uint32_t)(blur_tap(k) * row[reflect101(x + k - 3, w)]);
        acc += (uint32_t)blur_tap(i) * hs;
    }
    out[(size_t)y * w + x] = (uint8_t)(acc >> 16);
}

// ================================================================================================
// 2. FAST cells: src:1098-1166 (cell loop) + OpenCV FAST_t<16>/cornerScore<16> semantics
// ================================================================================================
// score(p) = max over the 16 9-pixel arcs and both polarities of the arc minimum of |I(p)-I(q)|,
// minus 1.  corner(t) <=> score >= t, and for corners this equals cornerScore<16>.  OpenCV's NMS
// (a candidate survives iff its score beats the 8 neighbours' *thresholded* scores inside the
// window) is then equivalent to: score >= t && score > score(n) for every neighbour n inside the
// window's detectable region (neighbours below t can never beat a corner).
// Packed: the 16 differences d = v - x go into 8 u16 pairs (circle points k, k+8), offset by 256
// (values 1..511, so unsigned v_pk_min/max_u16 order them), and every sliding min / max step works on
// both halves at once; wrapping past point 15 is the pair with its halves swapped.
__device__ __forceinline__ u16x2 swap16(u16x2 a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ int fast_score(const uint8_t* __restrict__ p, const int (&off)[16]) {
    const int v = p[0];
    const u16x2 vv = w16(v + 256, v + 256);
    u16x2 D[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        D[k] = vv - __builtin_bit_cast(u16x2, (uint32_t)p[off[k]] | ((uint32_t)p[off[k + 8]] << 16));
    auto at = [&](const u16x2 (&a)[8], int k) { return k < 8 ? a[k] : swap16(a[k - 8]); };
    u16x2 mn2[8], mx2[8], mn4[8], mx4[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        mn2[k] = __builtin_elementwise_min(D[k], at(D, k + 1));
        mx2[k] = __builtin_elementwise_max(D[k], at(D, k + 1));
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        mn4[k] = __builtin_elementwise_min(mn2[k], at(mn2, k + 2));
        mx4[k] = __builtin_elementwise_max(mx2[k], at(mx2, k + 2));
    }
    // arc k (points k .. k+8) in the low half, arc k+8 in the high half
    u16x2 dark = w16(0, 0), bright = w16(0xffff, 0xffff);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u16x2 mn8 = __builtin_elementwise_min(mn4[k], at(mn4, k + 4));
        const u16x2 mx8 = __builtin_elementwise_max(mx4[k], at(mx4, k + 4));
        dark = __builtin_elementwise_max(dark, __builtin_elementwise_min(mn8, swap16(D[k])));
        bright = __builtin_elementwise_min(bright, __builtin_elementwise_max(mx8, swap16(D[k])));
    }
    const int best_dark = (int)max(dark.x, dark.y) - 256, best_bright = (int)min(bright.x, bright.y) - 256;
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

// The body of one cell for a window row stride known at compile time (kWS > 0: circle, compass and
// neighbour offsets become LDS immediates) or at run time (kWS == 0).
#define FAST_STAMP(k) do { if (stp && lane == 0) stp[k] = __builtin_amdgcn_s_memtime(); } while (0)
template <int kWS, int kSS>
__device__ __forceinline__ void fast_cell(const KernelGeom& g, const CellDesc& C, const LevelGeom& L, int f, int cid,
                                          int lane, uint8_t* win, uint8_t* sc, uint16_t* cl, const uint8_t* src,
                                          int shift, int room, uint32_t* __restrict__ cand, int32_t* __restrict__ cell_count,
                                          uint8_t* __restrict__ cell_thr, unsigned long long* stp) {
    const int ww = C.win_w, wh = C.win_h;
    const int ws = kWS ? kWS : (shift + ww + 3) & ~3, nwr = ws >> 2;
    // score map row stride: the map holds window rows 2 .. wh-3, columns 2 .. ww-3 (candidate list
    // entries are (row << 7 | column) in window coordinates; windows are < 128 pixels wide)
    const int ss = kSS ? kSS : (ww - 4 + 3) & ~3;
    auto sc_at = [&](int e) { return ((e >> 7) - 2) * ss + (e & 127) - 2; };
    const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(src - shift);
    uint32_t* win32 = reinterpret_cast<uint32_t*>(win);
    // lanes = 4 rows x 16 dwords (a second column pass only for windows wider than 16 dwords)
    const int lr = lane >> 4, lw = lane & 15;
    if (nwr <= 16 && wh <= 48) {
        // the usual cell window (<= 64 bytes x 48 rows): every load issued before any LDS store, as
        // raw buffer loads (one lane offset, the row step in the scalar offset; `room` bytes to the
        // end of the frame's pyramid block bound the unconditional over-read, which returns 0 past it)
        // (the window is per wave: make the resource operands wave-uniform, or the compiler wraps
        // every load in a readfirstlane loop)
        const uintptr_t wb = reinterpret_cast<uintptr_t>(wsrc);
        const uint64_t wbu = (uint64_t)(uint32_t)uniform((int)(uint32_t)wb) | (uint64_t)(uint32_t)uniform((int)(uint32_t)(wb >> 32)) << 32;
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(wbu), (short)0, uniform(room), kBufDword3);
        const int pitch = uniform(L.pitch);
        const uint32_t vo = (uint32_t)(lr * pitch + 4 * lw);
        uint32_t v[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b32(rw, vo, 4 * k * pitch, 0);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const int r = 4 * k + lr;
            if (r < wh && lw < nwr) win32[r * nwr + lw] = v[k];
        }
    } else
    for (int w0 = 0; w0 < nwr; w0 += 16) {
        const int w = w0 + lw;
        for (int r0 = 0; r0 < wh; r0 += 16) {
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = r0 + 4 * k + lr;
                v[k] = (r < wh && w < nwr) ? wsrc[(size_t)r * (L.pitch >> 2) + w] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int r = r0 + 4 * k + lr;
                if (r < wh && w < nwr) win32[r * nwr + w] = v[k];
            }
        }
    }
    wave_sync();
    FAST_STAMP(1);
    win += shift;  // window pixel (r, c) is at win[r * ws + c]; its score at sc[sc_at(r << 7 | c)]
    const int dw = ww - 6, dh = wh - 6;
    const int nd = (dw > 0 && dh > 0) ? dw * dh : 0;
    int off[16];
    {
        const int cx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
        const int cy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
#pragma unroll
        for (int k = 0; k < 16; ++k) off[k] = cx[k] + cy[k] * ws;
    }
    const int ini = g.ini_th, mint = g.min_th;
    // 1a. compass filter at minTh: a 9-pixel arc always contains two circle pixels 4 apart among
    //     {0, 4, 8, 12}, so only pixels with such a bright or dark pair can be corners.  Passing
    //     pixels are compacted (row-major) into cl[].
    int nlist = 0;
    if (nd > 0) {
        // Eight pixels per lane (an octet of one detectable row), as u16 pairs: the centre, left (x-3),
        // right (x+3) bytes of the row and the up / down (y-/+3) bytes come from three aligned LDS
        // dwords and two v_alignbyte each, and a bright (dark) adjacent compass pair <=> the largest
        // pairwise minimum exceeds v + t (the smallest pairwise maximum plus t is below v), with
        // v_pk_min/max_u16 and saturating v_pk_sub_u16.  Items are row-major octets, so the compaction
        // (one wave scan per 8 pixels) stays row-major.
        const int no = (dw + 7) >> 3, nitems = dh * no;
        const uint32_t* wrow = reinterpret_cast<const uint32_t*>(win - shift);  // aligned window rows
        const int wsw = ws >> 2;
        const u16x2 tt = w16(mint, mint);
        // bytes [8o + off .. +7] of an aligned row (off includes the row's shift) as two dwords
        auto ext8 = [&](const uint32_t* row, int o, int off, uint32_t& a, uint32_t& b) {
            const int d = 2 * o + (off >> 2);
            const uint32_t w0 = row[d], w1 = row[d + 1], w2 = row[d + 2];
            a = __builtin_amdgcn_alignbyte(w1, w0, off & 3);
            b = __builtin_amdgcn_alignbyte(w2, w1, off & 3);
        };
        auto lo16 = [](uint32_t v) { return as_u16x2(__builtin_amdgcn_perm(v, v, 0x0c010c00u)); };
        auto hi16 = [](uint32_t v) { return as_u16x2(__builtin_amdgcn_perm(v, v, 0x0c030c02u)); };
        // The adjacent compass pairs are exactly the pairs of one vertical point {p0, p8} and one
        // horizontal point {p4, p12}, so the largest pairwise minimum is min(max(p0, p8), max(p4, p12))
        // and the smallest pairwise maximum is max(min(p0, p8), min(p4, p12)): 3 packed ops each.
        auto pass2 = [&](u16x2 v, u16x2 p0, u16x2 p4, u16x2 p8, u16x2 p12) {
            const u16x2 bmax = __builtin_elementwise_min(__builtin_elementwise_max(p0, p8), __builtin_elementwise_max(p4, p12));
            const u16x2 dmin = __builtin_elementwise_max(__builtin_elementwise_min(p0, p8), __builtin_elementwise_min(p4, p12));
            // bright <=> bmax - v > t, dark <=> v - dmin > t (saturating differences of u16 values <= 255)
            const u16x2 m = __builtin_elementwise_max(__builtin_elementwise_sub_sat(bmax, v), __builtin_elementwise_sub_sat(v, dmin));
            // 0 / 1 per pixel (pass <=> m - t, saturated, is non-zero): one v_pk_min_u16 (as written
            // in C the compiler turns the min into two compares, two selects and a v_perm)
            uint32_t r;
            asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(m, tt))), "v"(0x00010001u));
            return r;
        };
        // pass2 results of pixels (0,1), (2,3), (4,5), (6,7) as 0/1 halves, shifted into one word whose
        // low half holds the even pixels' bits and high half the odd ones': bit k = pixel k after
        // folding the high half down by 15
        auto octet_bits = [&](uint32_t C0, uint32_t D0, uint32_t R0, uint32_t U0, uint32_t L0, uint32_t C1,
                              uint32_t D1, uint32_t R1, uint32_t U1, uint32_t L1) {
            const uint32_t p01 = pass2(lo16(C0), lo16(D0), lo16(R0), lo16(U0), lo16(L0));
            const uint32_t p23 = pass2(hi16(C0), hi16(D0), hi16(R0), hi16(U0), hi16(L0));
            const uint32_t p45 = pass2(lo16(C1), lo16(D1), lo16(R1), lo16(U1), lo16(L1));
            const uint32_t p67 = pass2(hi16(C1), hi16(D1), hi16(R1), hi16(U1), hi16(L1));
            const uint32_t t = p01 | (p23 << 2) | (p45 << 4) | (p67 << 6);
            return (t & 0xffu) | (t >> 15);
        };
        // item -> (row, octet): one division here, then a fixed (row, octet) step of 64 items per round
        int r = lane / no, o = lane - (lane / no) * no;
        const int dr = 64 / no, dq = 64 - dr * no;
        for (int i0 = 0; i0 < nitems; i0 += 64) {
            const int it = i0 + lane;
            unsigned bits = 0;
            if (it < nitems) {
                const uint32_t* rc = wrow + (r + 3) * wsw;
                uint32_t L0, L1, C0, C1, R0, R1, U0, U1, D0, D1;
                ext8(rc, o, shift, L0, L1);
                ext8(rc, o, shift + 3, C0, C1);
                ext8(rc, o, shift + 6, R0, R1);
                ext8(rc - 3 * wsw, o, shift + 3, U0, U1);
                ext8(rc + 3 * wsw, o, shift + 3, D0, D1);
                bits = octet_bits(C0, D0, R0, U0, L0, C1, D1, R1, U1, L1);
                const int rem = dw - 8 * o;  // pixels of this octet inside the detectable row
                if (rem < 8) bits &= (1u << rem) - 1u;
            }
            const int row = r, oct = o;
            o += dq;
            r += dr;
            if (o >= no) { o -= no; ++r; }
            const int cnt = __popc(bits);
            const int incl = wave_incl_scan_dpp(cnt);
            int pos = nlist + incl - cnt;
            const int base_idx = ((row + 3) << 7) + 8 * oct + 3;  // (row << 7 | column), window coordinates
            while (bits) {
                const int k = __builtin_ctz(bits);
                bits &= bits - 1u;
                cl[pos++] = (uint16_t)(base_idx + k);
            }
            nlist += __builtin_amdgcn_readlane(incl, 63);
        }
    }
    wave_sync();
    FAST_STAMP(2);
    // 1b. exact score of the filtered pixels: score >= minTh <=> a 9-arc corner at minTh (see
    //     fast_score), so one pass both tests and scores; corners are compacted in place (row-major
    //     order kept: every lane reads its entry before any lane writes, and writes land below j0 + 64)
    //     and their scores go to the map
    int ncand = 0;
    for (int j0 = 0; j0 < nlist; j0 += 64) {
        const int j = j0 + lane;
        int idx = 0, s = -1;
        if (j < nlist) {
            idx = cl[j];
            s = fast_score(win + (idx >> 7) * ws + (idx & 127), off);
        }
        const bool is_c = s >= mint;
        const unsigned long long m = ballot(is_c);
        if (is_c) {
            cl[ncand + rank_in(m)] = (uint16_t)idx;
            sc[sc_at(idx)] = (uint8_t)min(s, 255);
        }
        ncand += __popcll(m);
    }
    wave_sync();
    FAST_STAMP(3);
    FAST_STAMP(4);
    // 3. iniTh first; minTh only if the cell has no corner at iniTh (src:1135-1148).  The local-maximum
    //    test does not depend on the threshold: its result (score + 1, or 0) is kept per candidate in
    //    the window's pixel buffer, which is free once the scores exist.
    uint8_t* lmv = win - shift;
    bool any = false;
    for (int j = lane; j < ncand; j += 64) {
        const int si = sc_at(cl[j]), s = sc[si];
        const bool lm = is_local_max(sc, ss, si, s);
        lmv[j] = lm ? (uint8_t)(s + 1) : (uint8_t)0;  // s <= 254 for a corner (9-arc minimum - 1)
        any |= (s >= ini) && lm;
    }
    const int t = ballot(any) ? ini : mint;
    wave_sync();
    FAST_STAMP(5);
    // 4. emission in row-major order (the candidate list is row-major)
    uint32_t* out = cand + (size_t)f * g.cand_frame_cap + L.cand_off + C.slot;
    int count = 0;
    for (int j0 = 0; j0 < ncand; j0 += 64) {
        const int j = j0 + lane;
        bool keep = false;
        int idx = 0, s = 0;
        if (j < ncand) {
            idx = cl[j];
            const int lv = lmv[j];
            s = lv - 1;
            keep = lv > 0 && s >= t;
        }
        const unsigned long long m = ballot(keep);
        if (keep) {
            const int pos = count + rank_in(m);
            const int r = idx >> 7, c = idx & 127;
            if (pos < C.cap) out[pos] = pack_key(C.off_x + c, C.off_y + r, s);
        }
        count += __popcll(m);
    }
    if (lane == 0) {
        cell_count[(size_t)f * g.ncells + cid] = min(count, (int)C.cap);
        cell_thr[(size_t)f * g.ncells + cid] = (uint8_t)t;
    }
    if (stp && lane == 0) { stp[6] = __builtin_amdgcn_s_memtime(); stp[8] = wall_clock64(); stp[9] = nlist; stp[10] = ncand; }
}


// One wave per FAST cell.  LDS per wave: window | score map | candidate list (u16 pixel indices).
// Pixels with score < minTh can neither be emitted nor beat an emitted neighbour, so the exact score
// is computed only for the pixels that are corners at minTh (compacted list, no divergence).
__global__ __launch_bounds__(256) void k_fast_cells(const KernelGeom* __restrict__ gp, const CellDesc* __restrict__ cells, int win_cap, int sc_cap, int wave_lds,
                                                    const uint8_t* __restrict__ pyr, uint32_t* __restrict__ cand,
                                                    int32_t* __restrict__ cell_count, uint8_t* __restrict__ cell_thr,
                                                    int cell0, int cell_end, unsigned long long* __restrict__ stamps,
                                                    int groups, int nblocks, int share) {
    const KernelGeom& g = *gp;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // XCD-chunked block order (xcd_tile): neighbouring cells, whose windows overlap, share an L2 (the
    // pyramid's frame-affine order measured no fetch change here: the windows miss L2 either way)
    const int tb = xcd_tile(blockIdx.x, share);
    if (tb >= nblocks) return;
    const int f = tb / groups;
    const int cid = cell0 + (tb - f * groups) * 4 + wave;
    if (cid >= cell_end) return;
    // debug (ORBGPU_FAST_STAMPS): per-cell phase clocks of lane 0 (0 start .. 6 end, 7 wall start, 8 wall end,
    // 9 survivors, 10 corners)
    unsigned long long* stp = stamps ? stamps + ((size_t)f * (cell_end - cell0) + (cid - cell0)) * 12 : nullptr;
    if (stp && lane == 0) { stp[7] = wall_clock64(); stp[0] = __builtin_amdgcn_s_memtime(); }
    const CellDesc C = cells[cid];
    const LevelGeom& L = g.lv[C.level];
    const uint8_t* view = pyr + (size_t)f * g.pyr_frame_bytes + L.plane_off + (size_t)kEdge * L.pitch + kEdge;
    uint8_t* win = smem + (size_t)wave * wave_lds;
    uint8_t* sc = win + win_cap;
    uint16_t* cl = reinterpret_cast<uint16_t*>(sc + sc_cap);
    const uint8_t* src = view + (size_t)C.ini_y * L.pitch + C.ini_x;
    // window rows as aligned dwords into an LDS image whose rows start `shift` bytes in (the level's
    // padded plane keeps the over-read inside it); row stride 52 when the window fits (the usual 42-px
    // cell window), else ws = roundup(shift + ww, 4).  52 B = 13 dwords: the compass phase's 32-lane
    // groups (5 octets x ~6.4 rows, 3 dwords each) spread over the 32 banks 2-way instead of the 3-way
    // a 48-B stride gives (rows 12 dwords apart repeat the bank pattern every 8 rows)
    const int shift = (int)((uintptr_t)src & 3);
    const int room = (int)(g.pyr_frame_bytes - (L.plane_off + (long long)(kEdge + C.ini_y) * L.pitch + kEdge + C.ini_x - shift));
    // score map zeroed here (rows 2 .. win_h-3 and columns 2 .. win_w-3 of the window: every
    // detectable pixel and its 3x3 neighbours)
    for (int i = lane; i < (sc_cap >> 4); i += 64) reinterpret_cast<uint4*>(sc)[i] = make_uint4(0u, 0u, 0u, 0u);
    if (shift + C.win_w <= 52 && C.win_h <= 48) {
        if (C.win_w <= 44)
            fast_cell<52, 40>(g, C, L, f, cid, lane, win, sc, cl, src, shift, room, cand, cell_count, cell_thr, stp);
        else
            fast_cell<52, 48>(g, C, L, f, cid, lane, win, sc, cl, src, shift, room, cand, cell_count, cell_thr, stp);
    } else {
        fast_cell<0, 0>(g, C, L, f, cid, lane, win, sc, cl, src, shift, room, cand, cell_count, cell_thr, stp);
    }
}
#undef FAST_STAMP

// ================================================================================================
// 3. DistributeOctTree, src:711-1057, one 256-thread workgroup per (frame, level)
// ================================================================================================
// The reference keeps the nodes in a std::list: every non-leaf node is divided and its non-empty
// children pushed to the FRONT in the order n1..n4, the parent erased.  A pass therefore yields
//   list' = reverse(children in push order) ++ (leaf nodes in old order).
// In the "careful" phase the splittable children of the last pass are std::sort-ed with
// compareNodes and divided from the largest until the list reaches N; parents are erased wherever
// they are, so a round yields list' = reverse(children in push order) ++ (old list minus divided).
// Node records live in list order in two generations (current / next); the positions of children,
// survivors and splittable children come from wave scans (k_quadtree_kp below).
struct QGen {
    int16_t *x0, *y0, *x1, *y1;
    int32_t* kn;  // key count
    uint8_t* leaf;  // bNoMore
};

struct QTree {          // list workspace: generations, sort arrays and index lists
    QGen g0, g1;
    uint16_t *split, *prev;
    uint8_t* divided;
    int* sort_ws;        // introsort stack (kOrbSortStack * 3 ints)
    unsigned long long *sel_el, *sel_tmp;  // sort elements: (count << 16 | UL.x) << 16 | position
    uint16_t *posA, *posB, *bend;          // partition stop lists, leaf-block ends
    int lcap;
};

__device__ __forceinline__ void split_point(const QGen& G, int p, int& sx, int& sy) {
    const int x0 = G.x0[p], y0 = G.y0[p], x1 = G.x1[p], y1 = G.y1[p];
    sx = x0 + ((x1 - x0 + 1) >> 1);  // UL.x + ceil((float)(UR.x-UL.x)/2), src:608
    sy = y0 + ((y1 - y0 + 1) >> 1);
}

__device__ __forceinline__ int wave_incl_scan(int v, int) { return wave_incl_scan_dpp(v); }

__device__ __forceinline__ int wave_incl_max(int v, int) { return wave_incl_max_dpp(v); }

// std::sort(vPrevSizeAndPointerToNode, compareNodes) (src:950) on t.prev[0..n), emulated exactly and
// wave-parallel.  Each libstdc++ partition step (median-of-3 to first, unguarded Hoare partition) is
// computed from two ballot-built stop lists: A = ascending positions with !(a < pivot), B = descending
// positions with !(pivot < a); pairs (A_k, B_k) are swapped while A_k < B_k and the cut is
// min(A_K*, B_K*-1) (tests/native/sort_port_check.cpp checks this against libstdc++).  The final
// insertion sort is stable, so it is a stable rank sort inside each leaf block (<= 16 elements, or
// a heap-sorted range when the depth limit hits, which is then already sorted).
__device__ void qt_sort(QTree& t, const QGen& A, int n, int lane) {
    unsigned long long* el = t.sel_el;
    auto less64 = [](unsigned long long x, unsigned long long y) { return (x >> 16) < (y >> 16); };
    for (int i = lane; i < n; i += 64) {
        const int id = t.prev[i];
        const uint32_t key = ((uint32_t)A.kn[id] << 16) | (uint16_t)A.x0[id];
        el[i] = ((unsigned long long)key << 16) | (unsigned)id;
        t.bend[i] = 0;
    }
    wave_sync();
    if (n <= 1) return;
    if (n > 16) {
        int lg = 0;
        for (int m = n; m > 1; m >>= 1) ++lg;
        int* st = t.sort_ws;
        if (lane == 0) { st[0] = 0; st[1] = n; st[2] = 2 * lg; }
        int sp = 1;
        wave_sync();
        while (sp > 0) {
            --sp;
            const int first = uniform(st[3 * sp]);
            int last = uniform(st[3 * sp + 1]), depth = uniform(st[3 * sp + 2]);
            while (last - first > 16) {
                if (depth == 0) {  // __partial_sort fallback: heap sort, serial (practically never taken)
                    if (lane == 0) orb_heap_sort(el, first, last, less64);
                    wave_sync();
                    break;
                }
                --depth;
                const int mid = first + (last - first) / 2;
                if (lane == 0) orb_move_median_to_first(el, first, first + 1, mid, last - 1, less64);
                wave_sync();
                const unsigned long long p = el[first] >> 16;
                int nA = 0, nB = 0;
                for (int b = first + 1; b < last; b += 64) {
                    const int i = b + lane;
                    const bool fa = i < last && !((el[i] >> 16) < p);
                    const unsigned long long m = ballot(fa);
                    if (fa) t.posA[nA + rank_in(m)] = (uint16_t)i;
                    nA += __popcll(m);
                }
                for (int b = last - 1; b > first; b -= 64) {
                    const int j = b - lane;
                    const bool fb = j > first && !(p < (el[j] >> 16));
                    const unsigned long long m = ballot(fb);
                    if (fb) t.posB[nB + rank_in(m)] = (uint16_t)j;
                    nB += __popcll(m);
                }
                wave_sync();
                const int lim = min(nA, nB);
                int ks = lim;
                for (int b = 0; b < lim; b += 64) {
                    const int k = b + lane;
                    const unsigned long long m = ballot(k < lim && t.posA[k] >= t.posB[k]);
                    if (m) { ks = b + __ffsll((long long)m) - 1; break; }
                }
                ks = uniform(ks);
                const int cut = uniform(min(ks < nA ? (int)t.posA[ks] : 1 << 30, ks > 0 ? (int)t.posB[ks - 1] : 1 << 30));
                for (int k = lane; k < ks; k += 64) {  // disjoint (nested) pairs: no cross-lane hazards
                    const int ia = t.posA[k], ib = t.posB[k];
                    const unsigned long long ea = el[ia], eb = el[ib];
                    el[ia] = eb;
                    el[ib] = ea;
                }
                if (lane == 0) { st[3 * sp] = cut; st[3 * sp + 1] = last; st[3 * sp + 2] = depth; }
                sp++;
                wave_sync();
                last = cut;
            }
            if (lane == 0) t.bend[first] = (uint16_t)last;  // leaf block [first, last)
            wave_sync();
        }
    } else {
        if (lane == 0) t.bend[0] = (uint16_t)n;
        wave_sync();
    }
    // __final_insertion_sort == stable sort; elements never leave their leaf block
    int carry = -1;
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        int v = (i < n && t.bend[i] != 0) ? i : -1;
        v = max(wave_incl_max(v, lane), carry);
        if (i < n) {
            const int s0 = v, e0 = t.bend[v];
            const unsigned long long ki = el[i] >> 16;
            int r = s0;
            for (int j = s0; j < e0; ++j) {
                const unsigned long long kj = el[j] >> 16;
                r += (kj < ki) || (kj == ki && j < i);
            }
            t.sel_tmp[r] = el[i];
        }
        carry = __builtin_amdgcn_readlane(v, 63);
    }
    wave_sync();
    for (int i = lane; i < n; i += 64) t.prev[i] = (uint16_t)(t.sel_tmp[i] & 0xffff);
    wave_sync();
}

// Position of the k-th (0-based) lowest set bit of m (valid for k < popcount(m)): the largest p with
// popcount(m below p) <= k, by a binary search over p.
__device__ __forceinline__ int kth_set_bit(unsigned long long m, int k) {
    int pos = 0;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1)
        if (__popcll(m & ((1ull << (pos + s)) - 1)) <= k) pos += s;
    return pos;
}

// qt_sort for n <= 64 with one element per lane in registers: the same libstdc++ introsort emulation
// (median-of-3 to first, unguarded Hoare partition from the two stop lists, stable sort inside the
// <= 16-element leaf blocks), but the stop lists are ballots, the pair swaps shuffles and the pending
// ranges a bit mask of block starts (ranges are independent, so their order does not matter; each
// block start carries its depth budget).  Returns false, leaving t.prev untouched, if a range would hit
// the depth limit (heap-sort fallback), so the caller runs qt_sort.  Keys: count << 12 | UL.x (callers
// guarantee counts < 2^20).
__device__ bool qt_sort_reg(QTree& t, const QGen& A, int n, int lane) {
    if (n <= 1) return true;
    int id = 0;
    uint32_t key = 0xffffffffu;
    if (lane < n) { id = t.prev[lane]; key = ((uint32_t)A.kn[id] << 12) | (uint32_t)(uint16_t)A.x0[id]; }
    int lg = 0;
    for (int m = n; m > 1; m >>= 1) ++lg;
    uint32_t st_lo = 1u, st_hi = 0u;  // block starts (uniform); a block ends at the next start or n
    int depth = 2 * lg;               // depth budget, meaningful at block starts
    const unsigned long long below = (1ull << lane) - 1, above = lane == 63 ? 0ull : ~((2ull << lane) - 1);
    while (true) {
        int f = -1, l = 0;
        for (unsigned long long b = ((unsigned long long)st_hi << 32) | st_lo; b;) {
            const int s0 = __ffsll((long long)b) - 1;
            b &= b - 1;
            const int e = b ? __ffsll((long long)b) - 1 : n;
            if (e - s0 > 16) { f = s0; l = e; break; }
        }
        f = uniform(f);
        l = uniform(l);
        if (f < 0) break;
        int d = uniform(__builtin_amdgcn_readlane(depth, f));
        if (d == 0) return false;
        --d;
        // __move_median_to_first(first, first + 1, mid, last - 1)
        const int mid = f + (l - f) / 2;
        const uint32_t ka = __builtin_amdgcn_readlane(key, f + 1), kb = __builtin_amdgcn_readlane(key, mid),
                       kc = __builtin_amdgcn_readlane(key, l - 1);
        int sx;
        if (ka < kb) sx = kb < kc ? mid : (ka < kc ? l - 1 : f + 1);
        else sx = ka < kc ? f + 1 : (kb < kc ? l - 1 : mid);
        sx = uniform(sx);
        const uint32_t kf = __builtin_amdgcn_readlane(key, f), ks = __builtin_amdgcn_readlane(key, sx);
        const int idf = __builtin_amdgcn_readlane(id, f), ids = __builtin_amdgcn_readlane(id, sx);
        if (lane == f) { key = ks; id = ids; }
        else if (lane == sx) { key = kf; id = idf; }
        const uint32_t p = ks;
        // __unguarded_partition(first + 1, last, first): stop lists A (ascending, !(a < p)) and
        // B (descending, !(p < a)), ranked by ballots and listed in LDS; pairs (A_k, B_k) swap while
        // A_k < B_k.  An element equal to the pivot is in both lists; it moves at most once (swapped
        // A_k precede every swapped B_k).
        const bool in = lane > f && lane < l;
        const bool inA = in && !(key < p), inB = in && !(p < key);
        const unsigned long long mA = ballot(inA), mB = ballot(inB);
        const int nA = __popcll(mA), nB = __popcll(mB), lim = min(nA, nB);
        const int ra = __popcll(mA & below), rb = __popcll(mB & above);
        if (inA) t.posA[ra] = (uint16_t)lane;
        if (inB) t.posB[rb] = (uint16_t)lane;
        wave_sync();
        const int Ak = lane < nA ? t.posA[lane] : 0, Bk = lane < nB ? t.posB[lane] : 0;
        const int pa = t.posB[min(ra, 63)], pb = t.posA[min(rb, 63)];
        const unsigned long long hit = ballot(lane < lim && Ak >= Bk);
        const int kstop = uniform(hit ? __ffsll((long long)hit) - 1 : lim);
        const int cut = uniform(min(kstop < nA ? __builtin_amdgcn_readlane(Ak, kstop) : 1 << 30,
                                    kstop > 0 ? __builtin_amdgcn_readlane(Bk, kstop - 1) : 1 << 30));
        const int partner = inA && ra < kstop ? pa : (inB && rb < kstop ? pb : lane);
        key = (uint32_t)__shfl((int)key, partner, 64);
        id = __shfl(id, partner, 64);
        wave_sync();  // the lists are rewritten by the next partition
        if (cut < n) {
            if (cut < 32) st_lo |= 1u << cut;
            else st_hi |= 1u << (cut - 32);
        }
        if (lane == f || lane == cut) depth = d;
    }
    const unsigned long long starts = ((unsigned long long)st_hi << 32) | st_lo;
    // __final_insertion_sort: a stable sort inside each block (<= 16 elements); the shuffles stay in
    // uniform control flow
    {
        const int s = 63 - __clzll(starts & (below | (1ull << lane)));
        const unsigned long long up = starts & above;
        const int e = up ? __ffsll((long long)up) - 1 : n;
        int r = s;
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            const int j = s + d;
            const uint32_t kj = (uint32_t)__shfl((int)key, j & 63, 64);
            r += j < e && ((kj < key) || (kj == key && j < lane));
        }
        if (lane < n) t.sel_tmp[r] = (unsigned long long)id;
    }
    wave_sync();
    if (lane < n) t.prev[lane] = (uint16_t)t.sel_tmp[lane];
    wave_sync();
    return true;
}

constexpr int kQtStamps = 12;

struct QPlace {  // vLappingArea classification of the selected keys
    int level, minB, lap0, lap1;
    float scale;
    int32_t* rank_out;
    int32_t* n_lap;
};

// ------------------------------------------------------------------------------------------------
// Key-parallel DistributeOctTree: one 256-thread workgroup per (level, frame).
//
// The keys never move.  They stay in gather order (the reference's vToDistributeKeys order) and
// each carries the list position of its node in the current generation.  Every node's key vector
// in the reference is a subsequence of that order (DivideNode pushes in parent order, src:644-662),
// so "first max-response key of the node" (src:1028-1053) is the max of (score, -gather index),
// and the stable key partition of the wave-per-tree kernel is not needed.  A step is:
//   node phase (wave 0): the list logic of one regular pass (src:802-918) or careful round
//     (src:937-1015) from the child counts, writing the next generation's records, the new
//     positions of every node's children (cmap) and the split points of the nodes whose children
//     the next step needs counted (the splittable children, vSizeAndPointerToNode);
//   key phase (all waves): each key moves to its child's new position and adds itself to the child
//     counts of its new node (LDS atomics), or, after the last step, to its node's best key.
// ------------------------------------------------------------------------------------------------
#ifndef ORB_QT_THREADS
#define ORB_QT_THREADS 256
#endif
constexpr int kQtThreads = ORB_QT_THREADS, kQtWaves = kQtThreads / 64;
constexpr int kQtCtrl = 64;  // ints: [0] fin, [1] overflow, [8..16) root map, [16..24) root counts,
                             // [24..24+W) wave totals, [24+W..24+2W) K partials (W = kQtWaves)
static_assert(kQtThreads % 64 == 0 && 24 + 2 * kQtWaves <= kQtCtrl, "quad-tree control words");

struct QT2 {
    QTree t;                    // list workspace shared with the sort: prev, split, divided, sel_*, pos*, bend
    int32_t* cnt[2];            // [4][lcap] child counts, per generation
    uint32_t* sxy[2];           // split point (sx | sy << 16) of the counted nodes, ~0u for the others
    unsigned long long* cmap;   // [lcap] next-generation positions of a node's children (4 x u16)
    uint32_t* best;             // [lcap] (score << 24) | (0xffffff - key index)
    int* ctrl;
};

__host__ __device__ inline size_t qt2_meta_bytes(int lcap) {
    // u64: cmap; 32-bit: cnt x2, sxy x2, kn x2, best; u16: 2 x (x0 y0 x1 y1), split, prev; u8: 2 x leaf,
    // divided.  The sort's arrays (sel_el, sel_tmp: u64; posA, posB, bend: u16) live in the next
    // generation's counts and in cmap, which no careful round uses until its sort is done (qt2_careful)
    return (size_t)lcap * (8 + 32 + 8 + 8 + 4 + 16 + 4 + 3) + kOrbSortStack * 12 + kQtCtrl * 4 + 64;
}

// The sort's workspace over a counts array that is free while a careful round sorts (16 B per entry:
// sel_el, sel_tmp) and over cmap (8 B per entry: posA, posB, bend)
__device__ __forceinline__ void qt2_sort_space(QT2& T, int32_t* free_cnt) {
    QTree& t = T.t;
    t.sel_el = reinterpret_cast<unsigned long long*>(free_cnt);
    t.sel_tmp = t.sel_el + t.lcap;
    t.posA = reinterpret_cast<uint16_t*>(T.cmap);
    t.posB = t.posA + t.lcap;
    t.bend = t.posB + t.lcap;
}

__device__ inline void qt2_carve(QT2& T, uint8_t* p, int lcap) {
    QTree& t = T.t;
    t.lcap = lcap;
    T.ctrl = (int*)p; p += kQtCtrl * 4;
    t.sort_ws = (int*)p; p += kOrbSortStack * 12;
    T.cmap = (unsigned long long*)p; p += 8 * lcap;
    QGen* gens[2] = {&t.g0, &t.g1};
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        T.cnt[g] = (int32_t*)p; p += 16 * lcap;
        T.sxy[g] = (uint32_t*)p; p += 4 * lcap;
        gens[g]->kn = (int32_t*)p; p += 4 * lcap;
    }
    T.best = (uint32_t*)p; p += 4 * lcap;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        gens[g]->x0 = (int16_t*)p; p += 2 * lcap;
        gens[g]->y0 = (int16_t*)p; p += 2 * lcap;
        gens[g]->x1 = (int16_t*)p; p += 2 * lcap;
        gens[g]->y1 = (int16_t*)p; p += 2 * lcap;
    }
    t.split = (uint16_t*)p; p += 2 * lcap;
    t.prev = (uint16_t*)p; p += 2 * lcap;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        gens[g]->leaf = p; p += lcap;
    }
    t.divided = p;
    qt2_sort_space(T, T.cnt[1]);
}

__device__ __forceinline__ uint32_t qt2_split_word(int x0, int y0, int x1, int y1) {
    return (uint32_t)(x0 + ((x1 - x0 + 1) >> 1)) | ((uint32_t)(y0 + ((y1 - y0 + 1) >> 1)) << 16);  // src:608-609
}
__device__ __forceinline__ int qt2_quadrant(uint32_t k, uint32_t s) {  // ~0u: never splits, quadrant 0
    return (key_x(k) >= (int)(s & 0xffff) ? 1 : 0) + (key_y(k) >= (int)(s >> 16) ? 2 : 0);
}

// next-generation record at `to` for child q (n keys) of node p; counted next step iff `counted`
__device__ __forceinline__ void qt2_write_child(const QT2& T, const QGen& A, QGen& B, int32_t* cB, uint32_t* sB,
                                                int p, int q, int n, int to, bool counted) {
    int sx, sy;
    split_point(A, p, sx, sy);
    const int x0 = (q & 1) ? sx : A.x0[p], x1 = (q & 1) ? A.x1[p] : sx;
    const int y0 = (q & 2) ? sy : A.y0[p], y1 = (q & 2) ? A.y1[p] : sy;
    B.x0[to] = (int16_t)x0; B.x1[to] = (int16_t)x1; B.y0[to] = (int16_t)y0; B.y1[to] = (int16_t)y1;
    B.kn[to] = n;
    B.leaf[to] = n == 1;
    sB[to] = counted ? qt2_split_word(x0, y0, x1, y1) : ~0u;
    const int lcap = T.t.lcap;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) cB[qq * lcap + to] = 0;
    T.best[to] = 0;
}

__device__ __forceinline__ void qt2_copy_node(const QT2& T, const QGen& A, QGen& B, int32_t* cB, uint32_t* sB, int p,
                                              int to) {
    B.x0[to] = A.x0[p]; B.y0[to] = A.y0[p]; B.x1[to] = A.x1[p]; B.y1[to] = A.y1[p];
    B.kn[to] = A.kn[p]; B.leaf[to] = A.leaf[p];
    sB[to] = ~0u;
    const int lcap = T.t.lcap;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) cB[qq * lcap + to] = 0;
    T.best[to] = 0;
}

__device__ __forceinline__ unsigned long long qt2_rep(int to) {
    const unsigned long long v = (unsigned)to & 0xffffu;
    return v | (v << 16) | (v << 32) | (v << 48);
}

// Regular pass (src:823-918) over the list A[0..nlist), wave 0.  Every non-leaf node is divided; its
// children were counted in cA by the last key phase.
__device__ void qt2_regular(QT2& T, const QGen& A, QGen& B, const int32_t* cA, int32_t* cB, uint32_t* sB, int nlist,
                            int N, int lane, int& new_size, int& nsplit, bool& fin, bool& ovf) {
    QTree& t = T.t;
    const int lcap = t.lcap;
    int total_children = 0, total_surv = 0;
    for (int b = 0; b < nlist; b += 64) {
        const int i = b + lane;
        int nc = 0, sv = 0;
        if (i < nlist) {
            if (A.leaf[i]) sv = 1;
            else for (int q = 0; q < 4; ++q) nc += cA[q * lcap + i] > 0;
        }
        total_children += wave_sum(nc);
        total_surv += wave_sum(sv);
    }
    total_children = uniform(total_children);
    total_surv = uniform(total_surv);
    new_size = total_children + total_surv;
    if (new_size > lcap) { ovf = true; return; }
    fin = new_size >= N || new_size == nlist;  // src:912-918
    int carry_c = 0, carry_s = 0, carry_p = 0;
    for (int b = 0; b < nlist; b += 64) {
        const int i = b + lane;
        int nc = 0, sv = 0, ns = 0, c[4] = {0, 0, 0, 0};
        if (i < nlist) {
            if (A.leaf[i]) sv = 1;
            else {
#pragma unroll
                for (int q = 0; q < 4; ++q) { c[q] = cA[q * lcap + i]; nc += c[q] > 0; ns += c[q] > 1; }
            }
        }
        const int ic = wave_incl_scan(nc, lane), is = wave_incl_scan(sv, lane), ip = wave_incl_scan(ns, lane);
        if (i < nlist) {
            unsigned long long cm = ~0ull;
            if (sv) {
                const int to = total_children + carry_s + is - 1;
                qt2_copy_node(T, A, B, cB, sB, i, to);
                cm = qt2_rep(to);
            } else {
                int r = 0, r2 = 0;
                const int stackpos = carry_c + ic - nc, splitpos = carry_p + ip - ns;
                for (int q = 0; q < 4; ++q) {
                    if (c[q] == 0) continue;
                    const int to = total_children - 1 - (stackpos + r);  // pushed to the front, src:846-897
                    qt2_write_child(T, A, B, cB, sB, i, q, c[q], to, !fin && c[q] > 1);
                    cm = (cm & ~(0xffffull << (16 * q))) | ((unsigned long long)to << (16 * q));
                    if (c[q] > 1) t.split[splitpos + r2++] = (uint16_t)to;
                    r++;
                }
            }
            T.cmap[i] = cm;
        }
        carry_c += __builtin_amdgcn_readlane(ic, 63);
        carry_s += __builtin_amdgcn_readlane(is, 63);
        carry_p += __builtin_amdgcn_readlane(ip, 63);
    }
    nsplit = carry_p;
}

// Careful round (src:937-1015), wave 0: the splittable children of the last step (t.split[0..np),
// counted in cA) are std::sort-ed with compareNodes and divided from the back until the list holds N.
__device__ void qt2_careful(QT2& T, const QGen& A, QGen& B, const int32_t* cA, int32_t* cB, uint32_t* sB, int nlist,
                            int np, int N, int lane, int debug_flags, bool reg_sort, int& new_size, int& nsplit, bool& fin, bool& ovf,
                            unsigned long long* tm, unsigned long long& t_last) {
    QTree& t = T.t;
    const int lcap = t.lcap;
    qt2_sort_space(T, cB);  // cB and cmap are rewritten only after the sort (qt2_write_child / qt2_copy_node)
    for (int i = lane; i < np; i += 64) t.prev[i] = t.split[i];
    wave_sync();
    if (debug_flags & 2) {  // reference single-lane port (A/B check)
        if (lane == 0) {
            const int16_t* x0a = A.x0;
            const int32_t* kc = A.kn;
            orb_std_sort(t.prev, np, [&](uint16_t a, uint16_t b) {
                const int ca = kc[a], cb = kc[b];
                return ca < cb || (ca == cb && x0a[a] < x0a[b]);
            }, t.sort_ws);
        }
        wave_sync();
    } else if (!(reg_sort && np <= 64 && !(debug_flags & 16) && qt_sort_reg(t, A, np, lane))) {
        qt_sort(t, A, np, lane);  // > 64 candidates, depth-limit fallback, or forced (flag 16)
    }
    if (tm) { const unsigned long long now = __builtin_amdgcn_s_memtime(); tm[4] += now - t_last; t_last = now; }
    // division order o = 0.. is prev[np-1-o]; stop once the list reaches N (src:1006)
    int ndiv = np, carry = 0;
    for (int b = 0; b < np; b += 64) {
        const int o = b + lane;
        int d = 0;
        if (o < np) {
            const int p = t.prev[np - 1 - o];
            for (int q = 0; q < 4; ++q) d += cA[q * lcap + p] > 0;
            d -= 1;
        }
        const int inc = wave_incl_scan(d, lane);
        const unsigned long long hit = ballot(o < np && nlist + carry + inc >= N);
        if (hit) { ndiv = b + __ffsll((long long)hit); break; }
        carry += __builtin_amdgcn_readlane(inc, 63);
    }
    ndiv = uniform(ndiv);
    for (int i = lane; i < nlist; i += 64) t.divided[i] = 0;
    wave_sync();
    for (int o = lane; o < ndiv; o += 64) t.divided[t.prev[np - 1 - o]] = 1;
    wave_sync();
    int total_children = 0;
    for (int b = 0; b < ndiv; b += 64) {
        const int o = b + lane;
        int nc = 0;
        if (o < ndiv) {
            const int p = t.prev[np - 1 - o];
            for (int q = 0; q < 4; ++q) nc += cA[q * lcap + p] > 0;
        }
        total_children += wave_sum(nc);
    }
    total_children = uniform(total_children);
    int kept = 0;
    for (int b = 0; b < nlist; b += 64) kept += __popcll(ballot(b + lane < nlist && !t.divided[b + lane]));
    new_size = total_children + kept;
    if (new_size > lcap) { ovf = true; return; }
    fin = new_size >= N || new_size == nlist;  // src:1013-1014
    int carry_c = 0, carry_p = 0;
    for (int b = 0; b < ndiv; b += 64) {
        const int o = b + lane;
        int nc = 0, ns = 0, c[4] = {0, 0, 0, 0}, p = 0;
        if (o < ndiv) {
            p = t.prev[np - 1 - o];
#pragma unroll
            for (int q = 0; q < 4; ++q) { c[q] = cA[q * lcap + p]; nc += c[q] > 0; ns += c[q] > 1; }
        }
        const int ic = wave_incl_scan(nc, lane), ip = wave_incl_scan(ns, lane);
        if (o < ndiv) {
            int r = 0, r2 = 0;
            const int stackpos = carry_c + ic - nc, splitpos = carry_p + ip - ns;
            unsigned long long cm = ~0ull;
            for (int q = 0; q < 4; ++q) {
                if (c[q] == 0) continue;
                const int to = total_children - 1 - (stackpos + r);
                qt2_write_child(T, A, B, cB, sB, p, q, c[q], to, !fin && c[q] > 1);
                cm = (cm & ~(0xffffull << (16 * q))) | ((unsigned long long)to << (16 * q));
                if (c[q] > 1) t.split[splitpos + r2++] = (uint16_t)to;
                r++;
            }
            T.cmap[p] = cm;
        }
        carry_c += __builtin_amdgcn_readlane(ic, 63);
        carry_p += __builtin_amdgcn_readlane(ip, 63);
    }
    nsplit = carry_p;
    int carry_k = 0;
    for (int b = 0; b < nlist; b += 64) {
        const int i = b + lane;
        const bool keep = i < nlist && !t.divided[i];
        const unsigned long long m = ballot(keep);
        if (keep) {
            const int to = total_children + carry_k + rank_in(m);
            qt2_copy_node(T, A, B, cB, sB, i, to);
            T.cmap[i] = qt2_rep(to);
        }
        carry_k += __popcll(m);
    }
}

// Adds one to cnt[q * lcap + p] for every active lane.  A wave's keys are neighbours in gather (cell)
// order, so most share a node: up to two leader rounds add a node's four counts from one lane (ballot
// counts, no same-address atomics); the remaining lanes use per-lane LDS atomics.
__device__ __forceinline__ void qt2_add_counts(int32_t* cnt, int lcap, int p, int q, bool active, int lane) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const unsigned long long am = ballot(active);
        if (!am) return;
        const int first = __ffsll((long long)am) - 1;
        const int leader = __builtin_amdgcn_readlane(p, first);
        const bool mine = active && p == leader;
        const int c0 = __popcll(ballot(mine && q == 0)), c1 = __popcll(ballot(mine && q == 1));
        const int c2 = __popcll(ballot(mine && q == 2)), c3 = __popcll(ballot(mine && q == 3));
        if (lane == first) {
            if (c0) atomicAdd(&cnt[leader], c0);
            if (c1) atomicAdd(&cnt[lcap + leader], c1);
            if (c2) atomicAdd(&cnt[2 * lcap + leader], c2);
            if (c3) atomicAdd(&cnt[3 * lcap + leader], c3);
        }
        active = active && !mine;
    }
    if (active) atomicAdd(&cnt[q * lcap + p], 1);
}

template <bool kKeysInLds>
__device__ void qt2_run(QT2& T, uint32_t* keys, uint16_t* node, int K, int N, int nroots, float root_w, int span_y,
                        const uint32_t* __restrict__ cand_level, const CellDesc* __restrict__ cells, int cell_begin,
                        int cell_count, const int32_t* __restrict__ ccount, int n_first, int slot_first,
                        uint32_t* __restrict__ sel_out, int sel_cap, int* n_sel, int* status, int debug_flags,
                        unsigned long long* stamps, const QPlace& place) {
    QTree& t = T.t;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lcap = t.lcap;
    int* ctrl = T.ctrl;
    // phase timers of thread 0 (debug_flags & 4): gather, roots, regular node, regular key, sort,
    // careful node, careful key, final, -, #regular passes, #careful rounds, K
    // (accumulated in the stamps record itself, by thread 0 only: no register state in normal runs)
    unsigned long long* tm = ((debug_flags & 4) && stamps && tid == 0) ? stamps : nullptr;
    if (tm)
        for (int i = 0; i < kQtStamps; ++i) tm[i] = 0;
    unsigned long long t_last = tm ? __builtin_amdgcn_s_memtime() : 0;
    auto stamp = [&](int i) {
        if (tm) { const unsigned long long now = __builtin_amdgcn_s_memtime(); tm[i] += now - t_last; t_last = now; }
    };
    // ---- gather (src:756-764): cells in chunks of 256, wave w owns 64 of them; a wave scan of the
    // counts gives each cell's start, the wave's keys are spread over its lanes, each finding its
    // key's cell by a binary search over the lanes' starts (8 x 64 loads in flight per round trip)
    int rcount[kMaxRoots];
#pragma unroll
    for (int r = 0; r < kMaxRoots; ++r) rcount[r] = 0;
    {
        constexpr int kGB = 8;
        int carry = 0;
        for (int cb = 0; cb < cell_count; cb += kQtThreads) {
            const int c = cb + tid;
            int n = 0, slot = 0;
            if (cb == 0) { n = n_first; slot = slot_first; }
            else if (c < cell_count) { n = ccount[c]; slot = cells[cell_begin + c].slot; }
            const int incl = wave_incl_scan(n, lane);
            const int start = incl - n;
            const int Tw = uniform(__builtin_amdgcn_readlane(incl, 63));
            if (lane == 0) ctrl[24 + wave] = Tw;
            __syncthreads();
            int base = carry, tot = 0;
#pragma unroll
            for (int w = 0; w < kQtWaves; ++w) {
                const int v = ctrl[24 + w];
                base += w < wave ? v : 0;
                tot += v;
            }
            __syncthreads();
            for (int j0 = 0; j0 < Tw; j0 += 64 * kGB) {
                uint32_t kk[kGB];
#pragma unroll
                for (int gi = 0; gi < kGB; ++gi) {
                    const int i = j0 + 64 * gi + lane;
                    int cl = 0;
#pragma unroll
                    for (int s = 32; s > 0; s >>= 1)
                        if (__shfl(start, cl + s, 64) <= i) cl += s;
                    const int sl = __shfl(slot, cl, 64), s0 = __shfl(start, cl, 64);
                    kk[gi] = i < Tw ? cand_level[sl + (i - s0)] : 0u;
                }
#pragma unroll
                for (int gi = 0; gi < kGB; ++gi) {
                    const int i = j0 + 64 * gi + lane;
                    if (i < Tw) {
                        int root = 0;
                        if (nroots > 1) {
                            root = (int)((float)key_x(kk[gi]) / root_w);  // vpIniNodes[kp.pt.x/hX], src:763
#pragma unroll
                            for (int r = 0; r < kMaxRoots; ++r) rcount[r] += root == r;
                        }
                        keys[base + i] = kk[gi];
                        node[base + i] = (uint16_t)root;
                    }
                }
            }
            carry += tot;
        }
    }
    if (tid < kMaxRoots) ctrl[16 + tid] = 0;
    __syncthreads();
    if (nroots > 1) {
#pragma unroll
        for (int r = 0; r < kMaxRoots; ++r) {
            if (r >= nroots) break;
            const int s = wave_sum(rcount[r]);
            if (lane == 0 && s) atomicAdd(&ctrl[16 + r], s);
        }
    } else if (tid == 0) {
        ctrl[16] = K;
    }
    __syncthreads();
    stamp(0);
    // ---- roots (src:733-786): empty roots erased, single-key roots are leaves
    QGen A = t.g0, B = t.g1;
    int32_t* cA = T.cnt[0];
    int32_t* cB = T.cnt[1];
    uint32_t* sA = T.sxy[0];
    uint32_t* sB = T.sxy[1];
    int nlist = 0;
    if (tid == 0) {
        for (int r = 0; r < nroots; ++r) {
            const int n = ctrl[16 + r];
            if (n > 0) {
                const int x0 = (int)(root_w * (float)r), x1 = (int)(root_w * (float)(r + 1));
                A.x0[nlist] = (int16_t)x0; A.x1[nlist] = (int16_t)x1;
                A.y0[nlist] = 0; A.y1[nlist] = (int16_t)span_y;
                A.kn[nlist] = n; A.leaf[nlist] = n == 1;
                sA[nlist] = n > 1 ? qt2_split_word(x0, 0, x1, span_y) : ~0u;
#pragma unroll
                for (int q = 0; q < 4; ++q) cA[q * lcap + nlist] = 0;
                ctrl[8 + r] = nlist;
                nlist++;
            }
        }
        ctrl[2] = nlist;
    }
    __syncthreads();
    nlist = ctrl[2];
    for (int kb = wave * 64; kb < K; kb += kQtThreads) {
        const int k = kb + lane;
        int p = 0, q = 0;
        bool counted = false;
        if (k < K) {
            if (nroots > 1) {
                p = ctrl[8 + node[k]];
                node[k] = (uint16_t)p;
            }
            const uint32_t s = sA[p];
            counted = s != ~0u;
            q = qt2_quadrant(keys[k], s);
        }
        if (counted) atomicAdd(&cA[q * lcap + p], 1);
    }
    __syncthreads();
    stamp(1);
    // ---- steps
    bool careful = false, fin = false, ovf = false;
    int nsplit = 0;
    while (true) {
        if (wave == 0) {
            int new_size = 0;
            if (!careful) {
                qt2_regular(T, A, B, cA, cB, sB, nlist, N, lane, new_size, nsplit, fin, ovf);
                // src:932: the next regular pass would overshoot N -> careful rounds
                if (!fin && !ovf && new_size + nsplit * 3 > N) careful = true;
                stamp(2);
                if (tm) tm[9]++;
            } else {
                if (tm) tm[8] += (unsigned long long)nsplit << (16 * min((int)tm[10], 3));  // candidates per round (debug)
                qt2_careful(T, A, B, cA, cB, sB, nlist, nsplit, N, lane, debug_flags, K < (1 << 20), new_size, nsplit, fin, ovf, tm,
                            t_last);
                stamp(5);
                if (tm) tm[10]++;
            }
            nlist = new_size;
            if (lane == 0) { ctrl[0] = fin; ctrl[1] = ovf; }
        }
        __syncthreads();
        fin = ctrl[0] != 0;
        ovf = ctrl[1] != 0;
        if (ovf) break;
        // key phase: move to the child's position; count for the next step, or take part in the best key
        // two keys per lane per round: both dependent LDS chains (node -> split/cmap -> next split) in flight
        for (int kb = wave * 128; kb < K; kb += 2 * kQtThreads) {
            const int k0 = kb + lane, k1 = kb + 64 + lane;
            const bool v0 = k0 < K, v1 = k1 < K;
            const int p0 = v0 ? node[k0] : 0, p1 = v1 ? node[k1] : 0;
            const uint32_t key0 = v0 ? keys[k0] : 0u, key1 = v1 ? keys[k1] : 0u;
            const uint32_t s0 = sA[p0], s1 = sA[p1];
            const unsigned long long m0 = T.cmap[p0], m1 = T.cmap[p1];
            const int n0 = (int)((m0 >> (16 * qt2_quadrant(key0, s0))) & 0xffff);
            const int n1 = (int)((m1 >> (16 * qt2_quadrant(key1, s1))) & 0xffff);
            if (v0) node[k0] = (uint16_t)n0;
            if (v1) node[k1] = (uint16_t)n1;
            if (fin) {
                if (v0) atomicMax(&T.best[n0], ((uint32_t)key_score(key0) << 24) | (0xffffffu - (uint32_t)k0));
                if (v1) atomicMax(&T.best[n1], ((uint32_t)key_score(key1) << 24) | (0xffffffu - (uint32_t)k1));
            } else {
                const uint32_t t0 = v0 ? sB[n0] : ~0u, t1 = v1 ? sB[n1] : ~0u;
                if (t0 != ~0u) atomicAdd(&cB[qt2_quadrant(key0, t0) * lcap + n0], 1);
                if (t1 != ~0u) atomicAdd(&cB[qt2_quadrant(key1, t1) * lcap + n1], 1);
            }
        }
        __syncthreads();
        stamp(careful && !fin ? 6 : 3);
        { const QGen g = A; A = B; B = g; }
        { int32_t* c = cA; cA = cB; cB = c; }
        { uint32_t* s = sA; sA = sB; sB = s; }
        if (fin) break;
    }
    if (wave != 0) return;
    if (ovf || nlist > sel_cap) {
        if (lane == 0) { *n_sel = 0; atomicMax(status, 1); }
        return;
    }
    // ---- the first max-response key of every node, in list order (src:1028-1053), ranked within its
    // vLappingArea class (src:1656-1676) as in qt_run
    int carry_lap = 0, carry_mono = 0;
    for (int b = 0; b < nlist; b += 64) {
        const int i = b + lane;
        bool lap = false;
        if (i < nlist) {
            const uint32_t bw = T.best[i];
            const uint32_t best = keys[0xffffffu - (bw & 0xffffffu)];
            sel_out[i] = best;
            float x = (float)(key_x(best) + place.minB);
            if (place.level != 0) x = x * place.scale;
            lap = x >= (float)place.lap0 && x <= (float)place.lap1;
        }
        const unsigned long long ml = ballot(i < nlist && lap), mm = ballot(i < nlist && !lap);
        if (i < nlist) place.rank_out[i] = lap ? -(1 + carry_lap + rank_in(ml)) : carry_mono + rank_in(mm);
        carry_lap += __popcll(ml);
        carry_mono += __popcll(mm);
    }
    if (lane == 0) { *n_sel = nlist; *place.n_lap = carry_lap; }
    stamp(7);
    if (tm) tm[11] = (unsigned long long)K;
}

__global__ __launch_bounds__(kQtThreads) void k_quadtree_kp(
    const KernelGeom* __restrict__ gp, const CellDesc* __restrict__ cells, const uint32_t* __restrict__ cand,
    const int32_t* __restrict__ cell_count, uint32_t* __restrict__ key_scratch, uint32_t* __restrict__ sel,
    int32_t* __restrict__ sel_count, int lds_bytes, int* __restrict__ status, unsigned long long* __restrict__ stamps,
    int lap0, int lap1, int32_t* __restrict__ rank_out, int32_t* __restrict__ lap_count, int level0) {
    const KernelGeom& g = *gp;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int level = level0 + blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const LevelGeom& L = g.lv[level];
    const int32_t* cc = cell_count + (size_t)f * g.ncells + L.cell_begin;
    int32_t* n_sel = sel_count + (size_t)f * g.nlevels + level;
    const int lcap = L.sel_cap + 64;
    const size_t meta = (qt2_meta_bytes(lcap) + 15) & ~(size_t)15;
    if (meta > (size_t)lds_bytes) {
        if (tid == 0) { *n_sel = 0; atomicMax(status, 2); }
        return;
    }
    QT2 T;
    qt2_carve(T, smem, lcap);
    // K (the first chunk's cell counts and slots stay in registers for the gather)
    int n_first = 0, slot_first = 0, Kp = 0;
    for (int c = tid; c < L.cell_count; c += kQtThreads) {
        const int v = cc[c];
        if (c == tid) { n_first = v; slot_first = cells[L.cell_begin + c].slot; }
        Kp += v;
    }
    Kp = wave_sum(Kp);
    if (lane == 0) T.ctrl[24 + kQtWaves + wave] = Kp;
    __syncthreads();
    int K = 0;
#pragma unroll
    for (int w = 0; w < kQtWaves; ++w) K += T.ctrl[24 + kQtWaves + w];
    uint32_t* sel_out = sel + (size_t)f * g.sel_frame_cap + L.sel_off;
    const uint32_t* cand_level = cand + (size_t)f * g.cand_frame_cap + L.cand_off;
    QPlace place{level, L.minB, lap0, lap1, L.scale, rank_out + (size_t)f * g.sel_frame_cap + L.sel_off,
                 lap_count + (size_t)f * g.nlevels + level};
    unsigned long long* st = stamps ? stamps + ((size_t)f * g.nlevels + level) * kQtStamps : nullptr;
    if (!(g.debug_flags & 8) && meta + (size_t)K * 6 <= (size_t)lds_bytes) {  // flag 8: force the scratch path (tests)
        uint32_t* keys = (uint32_t*)(smem + meta);
        uint16_t* node = (uint16_t*)(keys + K);
        qt2_run<true>(T, keys, node, K, L.nfeat, L.n_roots, L.root_w, L.maxBY - L.minB, cand_level, cells,
                      L.cell_begin, L.cell_count, cc, n_first, slot_first, sel_out, L.sel_cap, n_sel, status,
                      g.debug_flags, st, place);
    } else {  // keys and node ids in this level's scratch slots (2 x cand_cap words)
        uint32_t* keys = key_scratch + ((size_t)f * g.cand_frame_cap + L.cand_off) * 2;
        uint16_t* node = (uint16_t*)(keys + L.cand_cap);
        qt2_run<false>(T, keys, node, K, L.nfeat, L.n_roots, L.root_w, L.maxBY - L.minB, cand_level, cells,
                       L.cell_begin, L.cell_count, cc, n_first, slot_first, sel_out, L.sel_cap, n_sel, status,
                       g.debug_flags, st, place);
    }
}

// Debug: compareNodes sort of n (count, UL.x) records by the quad-tree's sort emulations, one wave
// (mode 0: the register version when n <= 64, else qt_sort; mode 1: qt_sort).  *used_reg = 1 if the
// register version produced the order.
__global__ __launch_bounds__(64) void k_debug_node_sort(const int* __restrict__ counts, const int* __restrict__ ulx,
                                                        int n, int mode, int* __restrict__ order, int* __restrict__ used_reg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    QT2 T;
    qt2_carve(T, smem, n + 64);
    QTree& t = T.t;
    QGen& A = t.g0;
    const int lane = threadIdx.x;
    for (int i = lane; i < n; i += 64) { A.kn[i] = counts[i]; A.x0[i] = (int16_t)ulx[i]; t.prev[i] = (uint16_t)i; }
    wave_sync();
    const bool reg = mode == 0 && n <= 64 && qt_sort_reg(t, A, n, lane);
    if (!reg) qt_sort(t, A, n, lane);
    for (int i = lane; i < n; i += 64) order[i] = t.prev[i];
    if (lane == 0) *used_reg = reg;
}

// ================================================================================================
// 5. IC_Angle + steered rBRIEF, src:91-138, 150-203, 1534-1547, 1656-1676
// ================================================================================================
// The exception keys live in registers (kExcPerLane per lane, loaded at kernel entry), so the lookup
// is a compare + half-wave ballot; only a hit (rare) reads the table again.
constexpr int kExcPerLane = (kNumSincosExc + 31) / 32;
// kLds: the (cos, sin) bits of the exceptions are in LDS (lds_cs), else read from the constant table.
template <bool kLds = false>
__device__ __forceinline__ void steer_sincos(float ang, const uint32_t (&exc)[kExcPerLane], int half, int hl,
                                             float* s, float* c, const uint2* lds_cs = nullptr) {
    orb_det_sincosf(ang, s, c);
    const uint32_t bits = __float_as_uint(ang);
    int idx = -1;
#pragma unroll
    for (int e = 0; e < kExcPerLane; ++e)
        if (32 * e + hl < kNumSincosExc && exc[e] == bits) idx = 32 * e + hl;
    const uint32_t hm = (uint32_t)(ballot(idx >= 0) >> (32 * (half & 1)));
    if (hm) {
        const int hit = __shfl(idx, 32 * (half & 1) + __builtin_ctz(hm), 64);
        if constexpr (kLds) {
            *c = __uint_as_float(lds_cs[hit].x);
            *s = __uint_as_float(lds_cs[hit].y);
        } else {
            *c = __uint_as_float(c_sincos_exc[hit][1]);
            *s = __uint_as_float(c_sincos_exc[hit][2]);
        }
    }
}

// One keypoint per 32-lane half-wave, 8 per block.  The keypoint's 43x43 level patch is staged in LDS
// with one round of dwordx4 loads (rBRIEF samples reach round(13*sqrt(2)) = 18 px, the 7x7 Gaussian
// 3 more; IC_Angle's 31-px disc lies inside), so the dependent memory phases are: key -> patch ->
// stores.  The blurred level is never materialised: the reference blurs a clone of every level
// (src:1629-1637) but reads it only at the 512 samples, so the kernel runs the same separable
// fixed-point GaussianBlur restricted to them -- the horizontal 7-tap pass over the 43 rows x 37
// columns the samples can touch (exact u16 sums, stored over the patch as row-pair u16x2 words), then
// the vertical 7-tap pass per sample (4 v_dot2_u32_u16).  Integer sums throughout, so the value is the
// reference's bit for bit.
constexpr int kDescKpPerBlock = 8;
constexpr int kPR = 43, kPRW = 12;   // patch rows, dwords per row (43 bytes + up to 3 alignment bytes)
constexpr int kHP = 22, kHPW = 40;   // horizontal-sum row pairs (rows 2j, 2j+1), words per pair (37 used)
constexpr int kDescWords = kHP * kHPW;  // 3520 bytes per keypoint: the sums, and before them the patch
static_assert(kDescWords >= (kPR + 1) * kPRW + 1, "patch + the last pair's odd row and over-read word fit the region");

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr f32x2 kRound2 = {12582912.0f, 12582912.0f};  // 1.5 * 2^23: v + it has ulp 1 (|v| < 2^22)
constexpr int kRoundBits = 0x4B400000;                 // its bit pattern

// Vertical 7-tap pass at one sample (r, c), |r|, |c| <= 18 from the keypoint: blurred row i = r + 18
// reads sum rows i .. i+6, i.e. the 4 row pairs from i >> 1 (odd i: the first pair's high half).
__device__ __forceinline__ int blur_sample(const uint32_t* __restrict__ H, int r, int c) {
    // (the masks are no-ops for |r|, |c| <= 18; they bound the range so the offsets stay 24-bit
    // multiplies and the four reads fold into two ds_read2_b32)
    const unsigned i = (unsigned)(r + 18) & 63u, cc = (unsigned)(c + 18) & 63u;
    const uint32_t* p = H + __umul24(i >> 1, (unsigned)kHPW) + cc;
    const bool odd = (i & 1) != 0;
    uint32_t acc = 1u << 15;
    acc = __builtin_amdgcn_udot2(as_u16x2(p[0]), odd ? w16(0, 18) : w16(18, 34), acc, false);
    acc = __builtin_amdgcn_udot2(as_u16x2(p[kHPW]), odd ? w16(34, 48) : w16(48, 56), acc, false);
    acc = __builtin_amdgcn_udot2(as_u16x2(p[2 * kHPW]), odd ? w16(56, 48) : w16(48, 34), acc, false);
    acc = __builtin_amdgcn_udot2(as_u16x2(p[3 * kHPW]), odd ? w16(34, 18) : w16(18, 0), acc, false);
    return (int)(acc >> 16);  // <= 255 exactly
}

__global__ __launch_bounds__(256) void k_describe(const KernelGeom* __restrict__ gp, const uint8_t* __restrict__ pyr,
                                                  const uint32_t* __restrict__ sel,
                                                  const int32_t* __restrict__ sel_count,
                                                  const int32_t* __restrict__ rank_in_class, const int32_t* __restrict__ lap_count,
                                                  int cap, orb_keypoint_t* __restrict__ kps, uint8_t* __restrict__ desc,
                                                  int32_t* __restrict__ counts, int chunks, int nblocks, int share,
                                                  int stage_levels, int stage_mode, orb_keypoint_t* __restrict__ st_kp,
                                                  uint8_t* __restrict__ st_desc) {
    const KernelGeom& g = *gp;
    __shared__ __attribute__((aligned(16))) uint32_t patch[kDescKpPerBlock][kDescWords];
    const int half = threadIdx.x >> 5, hl = threadIdx.x & 31;
    // blockIdx.x -> (level, chunk): level l owns ceil(sel_cap_l / 8) blocks, so the grid holds no block
    // beyond a level's capacity (scalar walk over the levels)
    // XCD-chunked block order (xcd_tile): each XCD walks a contiguous run of (frame, chunk) blocks,
    // so the patches of one frame's keypoints are fetched into one L2
    const int tb = xcd_tile(blockIdx.x, share);
    if (tb >= nblocks) return;
    const int f = tb / chunks, chunk0 = tb - f * chunks;
    int level = 0, chunk = chunk0;
#pragma unroll
    for (int l = 0; l + 1 < kMaxLevels; ++l) {
        const int c = (g.lv[l].sel_cap + kDescKpPerBlock - 1) / kDescKpPerBlock;
        if (l + 1 < g.nlevels && level == l && chunk >= c) { chunk -= c; level = l + 1; }
    }
    const int slot = chunk * kDescKpPerBlock + half;
    const LevelGeom& L = g.lv[level];
    // Every load that does not depend on the key is issued here, in one round trip with the key itself:
    // the key and its rank are read speculatively at a clamped (in-bounds) slot, and the rBRIEF pattern
    // and sincos exception keys go to registers.
    const size_t sbase = (size_t)f * g.sel_frame_cap + L.sel_off + (slot < L.sel_cap ? slot : L.sel_cap - 1);
    const uint32_t key_spec = L.sel_cap > 0 ? sel[sbase] : 0u;
    const int rk_spec = L.sel_cap > 0 ? rank_in_class[sbase] : 0;
    // per-frame totals over the levels (src:1586-1591) and this level's class bases (src:1613-1676)
    const int li = hl & 15;
    const int cnt_l = li < g.nlevels ? sel_count[(size_t)f * g.nlevels + li] : 0;
    const int lap_l = li < g.nlevels ? lap_count[(size_t)f * g.nlevels + li] : 0;
    uint32_t pat[8], exc[kExcPerLane], disc[16];
#pragma unroll
    for (int m = 0; m < 8; ++m) pat[m] = c_pattern_packed.w[32 * m + hl];
#pragma unroll
    for (int m = 0; m < 16; ++m) disc[m] = c_disc.w[hl][m];
#pragma unroll
    for (int e = 0; e < kExcPerLane; ++e) exc[e] = 32 * e + hl < kNumSincosExc ? c_sincos_exc[32 * e + hl][0] : 0u;
    int total = cnt_l, lap_before = li < level ? lap_l : 0, mono_before = li < level ? cnt_l - lap_l : 0;
    // sums within each 16-lane row, in every lane of it: DPP (xor 1, xor 2, row_ror 4, 8) instead of
    // four dependent ds_bpermute round trips per value
    total = row16_isum(total);
    lap_before = row16_isum(lap_before);
    mono_before = row16_isum(mono_before);
    // Split mode (levels [0, stage_levels) described early, on the side stream, before the later
    // levels' quad-tree exists): stage_mode 1 computes them into per-slot staging records (the output
    // slot needs every level's count); the final launch (stage_mode 2) moves them to their slots.
    const int n = __shfl(cnt_l, (threadIdx.x & ~15) + level, 64);
    const size_t st_idx = sbase;  // staging record of this half-wave's slot (valid when slot < n)
    if (stage_mode != 1 && chunk0 == 0 && threadIdx.x == 0) {
        int mono = 0;
        for (int l = 0; l < g.nlevels; ++l)
            mono += sel_count[(size_t)f * g.nlevels + l] - lap_count[(size_t)f * g.nlevels + l];
        counts[2 * f] = total;
        counts[2 * f + 1] = total > cap ? ORB_ERR_CAPACITY : mono;
    }
    if (chunk * kDescKpPerBlock >= n) return;                // whole block idle
    const bool active = slot < n && (stage_mode == 1 || total <= cap);  // frame within the caller's capacity
    if (stage_mode == 2 && level < stage_levels) {  // staged record -> output slot (block-uniform branch)
        if (!active) return;
        const int rk = rk_spec;
        const int dst = rk < 0 ? total - 1 - (lap_before + (-rk - 1)) : mono_before + rk;
        if (hl < 8)
            reinterpret_cast<uint32_t*>(desc + ((size_t)f * cap + dst) * 32)[hl] =
                reinterpret_cast<const uint32_t*>(st_desc + st_idx * 32)[hl];
        else if (hl == 8)
            kps[(size_t)f * cap + dst] = st_kp[st_idx];
        return;
    }
    const uint32_t key = active ? key_spec : 0;
    const int x = key_x(key) + L.minB, y = key_y(key) + L.minB;
    // ---- stage the patch: rows y-21 .. y+21, columns from x-21 rounded down to a dword.  Lane
    // (r, q) of a half-wave loads 16 bytes (quarter q of 3) of row r of a 10-row group; load k reads
    // rows 10k .. 10k+9 (raw buffer loads, plane base in the resource, the row step in soffset).  The
    // over-read rows (43 .. 49) and columns stay inside the padded plane and are not stored.
    constexpr int kGroups = (kPR + 9) / 10;
    const int pr = hl / 3, pq = hl - 3 * pr;
    const uint8_t* up = pyr + (size_t)f * g.pyr_frame_bytes + L.plane_off;
    const int po = (y + kEdge - 21) * L.pitch + (x + kEdge - 21);
    const int sh = po & 3;  // plane base and pitch are 128-B aligned
    const uint32_t vo = (uint32_t)(po - sh + pr * L.pitch + 16 * pq);
    const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(up), (short)0, 0x7fffffff, kBufDword3);
    uint32_t* P = patch[half];
    if (active && hl < 30) {
        v4u32 v[kGroups];
#pragma unroll
        for (int k = 0; k < kGroups; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(ru, vo, 10 * k * L.pitch, 0);
#pragma unroll
        for (int k = 0; k < kGroups; ++k)
            if (10 * k + pr < kPR) *reinterpret_cast<v4u32*>(P + (10 * k + pr) * kPRW + 4 * pq) = v[k];
    }
    wave_sync();
    // ---- IC_Angle on the level (src:91-138): lane = disc row v (lanes 0..30), its 32 bytes u = -15 ..
    // 16 as 8 dwords (aligned reads + v_alignbyte).  Row sum S = sum mask*I and W = sum (u+16)*mask*I
    // by v_dot4_u32_u8 against the lane's table row (loaded at entry), so m01 += v*S, m10 += W - 16 S.
    int m10 = 0, m01 = 0;
    {
        const int rb = sh + (hl + 6) * (kPRW * 4) + 6;  // byte of (v = hl - 15, u = -15)
        const uint32_t* rw = P + (rb >> 2);
        const int ra = rb & 3;
        uint32_t d[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) d[k] = rw[k];  // rows 6..37 of the patch region (lane 31: unused)
        uint32_t S = 0, W = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t x = __builtin_amdgcn_alignbyte(d[k + 1], d[k], ra);
            S = __builtin_amdgcn_udot4(x, disc[k], S, false);
            W = __builtin_amdgcn_udot4(x, disc[8 + k], W, false);
        }
        if (active && hl < 31) {
            m01 = (hl - 15) * (int)S;
            m10 = (int)W - 16 * (int)S;
        }
    }
    m10 = half_wave_sum(m10);
    m01 = half_wave_sum(m01);
    const float angle = orb_fast_atan2((float)m01, (float)m10);
    // ---- horizontal 7-tap pass (GaussianBlur 7x7 sigma 2, exact in 16 bits): item (pair j, quad qq)
    // = sum columns 4qq .. 4qq+3 of rows 2j, 2j+1 (v_alignbyte + v_dot4_u32_u8 on the patch bytes
    // shifted by sh), written over the patch in place.  Rounds run from the last pairs down: pair j's
    // words start at patch row 40j/12, above every row (<= 2j - 1, + 16 over-read bytes) a later,
    // lower round reads, and within a round the reads precede the writes (one wave, LDS in order).
    constexpr int kItems = kHP * 10, kIt = (kItems + 31) / 32;
#pragma unroll
    for (int it = kIt - 1; it >= 0; --it) {
        const int i = hl + 32 * it, ic = min(i, kItems - 1), j = ic / 10, qq = ic - 10 * j;
        uint32_t o[2][4];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const uint32_t* w = P + (2 * j + rr) * kPRW + qq;  // patch bytes 4qq .. 4qq+15 (2 x ds_read2)
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
            const uint32_t a0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
            const uint32_t a1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
            const uint32_t a2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
            // column k = bytes k .. k+6 of (a0, a1, a2): the kernel shifted by k bytes against the
            // aligned words (10 v_dot4 instead of 8 v_dot4 + 8 v_alignbyte)
            o[rr][0] = __builtin_amdgcn_udot4(a1, kBlurK1, __builtin_amdgcn_udot4(a0, kBlurK0, 0u, false), false);
            o[rr][1] = __builtin_amdgcn_udot4(a1, kBlurS1[1], __builtin_amdgcn_udot4(a0, kBlurS0[1], 0u, false), false);
            o[rr][2] = __builtin_amdgcn_udot4(a2, kBlurS2[2], __builtin_amdgcn_udot4(a1, kBlurS1[2],
                                              __builtin_amdgcn_udot4(a0, kBlurS0[2], 0u, false), false), false);
            o[rr][3] = __builtin_amdgcn_udot4(a2, kBlurS2[3], __builtin_amdgcn_udot4(a1, kBlurS1[3],
                                              __builtin_amdgcn_udot4(a0, kBlurS0[3], 0u, false), false), false);
        }
        if (i < kItems)
            *reinterpret_cast<uint4*>(P + j * kHPW + 4 * qq) =
                make_uint4(o[0][0] | o[1][0] << 16, o[0][1] | o[1][1] << 16, o[0][2] | o[1][2] << 16, o[0][3] | o[1][3] << 16);
    }
    wave_sync();
    // ---- steered BRIEF on the blurred samples (src:150-203)
    const float ang = angle * (float)(3.14159265358979323846 / 180.f);
    float a, b;
    steer_sincos(ang, exc, half, hl, &b, &a);  // a = cos, b = sin
    int t0[8], t1[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        // test j = 32 m + hl -> byte j/8, bit j%8 (src:173-199)
        const int pw4 = (int)pat[m];
        const float px0 = (float)((pw4 << 24) >> 24), py0 = (float)((pw4 << 16) >> 24);
        const float px1 = (float)((pw4 << 8) >> 24), py1 = (float)(pw4 >> 24);
        // (r, c) = (fma(x, b, y*a), fma(x, a, -(y*b))) as one packed multiply and one packed FMA
        // (y*(-b) == -(y*b) exactly), rounded to nearest-even by adding 1.5 * 2^23 and reading the
        // integer out of the mantissa (|r|, |c| <= 18)
        const f32x2 rc0 = __builtin_elementwise_fma(f32x2{px0, px0}, f32x2{b, a}, f32x2{py0, py0} * f32x2{a, -b}) + kRound2;
        const f32x2 rc1 = __builtin_elementwise_fma(f32x2{px1, px1}, f32x2{b, a}, f32x2{py1, py1} * f32x2{a, -b}) + kRound2;
        t0[m] = blur_sample(P, __float_as_int(rc0.x) - kRoundBits, __float_as_int(rc0.y) - kRoundBits);
        t1[m] = blur_sample(P, __float_as_int(rc1.x) - kRoundBits, __float_as_int(rc1.y) - kRoundBits);
    }
    uint32_t words[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) words[m] = (uint32_t)(ballot(t0[m] < t1[m]) >> (32 * (half & 1)));
    if (!active) return;
    const int rk = rk_spec;
    const int dst = rk < 0 ? total - 1 - (lap_before + (-rk - 1)) : mono_before + rk;
    uint8_t* drow = stage_mode == 1 ? st_desc + st_idx * 32 : desc + ((size_t)f * cap + dst) * 32;
    orb_keypoint_t* kdst = stage_mode == 1 ? st_kp + st_idx : kps + (size_t)f * cap + dst;
    if (hl < 8) {
        uint32_t w = words[0];
#pragma unroll
        for (int m = 1; m < 8; ++m) if (hl == m) w = words[m];
        reinterpret_cast<uint32_t*>(drow)[hl] = w;
    } else if (hl == 8) {
        orb_keypoint_t k;
        float fx = (float)x, fy = (float)y;
        if (level != 0) { fx = fx * L.scale; fy = fy * L.scale; }
        k.x = fx; k.y = fy;
        k.size = (float)L.patch_size;
        k.angle = angle;
        k.response = (float)key_score(key);
        k.octave = level;
        k.class_id = -1;
        *kdst = k;
    }
}

}  // namespace

// ================================================================================================
// host side
// ================================================================================================
namespace orbgpu {

enum { kLaunchPyramid = 0, kLaunchFast = 1, kLaunchQuadtree = 2, kLaunchDescribe = 3 };  // profile 3 tags

struct Extractor {
    Params P;
    int max_w = 0, max_h = 0, max_batch = 0;
    int cur_w = -1, cur_h = -1;
    Geometry geo;
    bool geo_ok = false;
    // device buffers
    orbgpu::KernelGeom* d_geom = nullptr;  // kernel geometry in device memory (read by every kernel)
    CellDesc* d_cells = nullptr; size_t cells_cap = 0;
    int2* d_xtab = nullptr; size_t xtab_cap = 0;
    int4* d_tiletab = nullptr; size_t tiletab_cap = 0;  // pyramid tile records (tile_tables)
    int4* d_pairtab = nullptr; size_t pairtab_cap = 0;  // their two-level records (pair_tables)
    bool pair_ok = false;                               // the geometry fits k_pyramid_pair's boxes
    int pyr_pair = 0;                                   // ORBGPU_PYR_PAIR=1: two levels per pyramid pass, 2: only
                                                        // levels 0 + 1 (level passes by default)
    int tile_off[orbgpu::kMaxLevels] = {};
    int4* d_ytab = nullptr; size_t ytab_cap = 0;
    uint8_t* d_pyr = nullptr; size_t pyr_cap = 0;
    uint32_t* d_cand = nullptr; size_t cand_cap = 0;
    uint32_t* d_scratch = nullptr; size_t scratch_cap = 0;
    int32_t* d_cell_count = nullptr; size_t cell_count_cap = 0;
    uint8_t* d_cell_thr = nullptr; size_t cell_thr_cap = 0;
    uint32_t* d_sel = nullptr; size_t sel_cap = 0;
    int32_t* d_dst = nullptr; size_t dst_cap = 0;
    int32_t* d_sel_count = nullptr; size_t selcount_cap = 0;
    int32_t* d_lap_count = nullptr; size_t lapcount_cap = 0;
    int* d_status = nullptr;      // the handle's status word: d_status_own, or inside d_out once orb_extract
    int* d_status_own = nullptr;  // has allocated it (so the one download carries it)
    bool clear_status_l0 = false;  // this batch's level-0 launch clears d_status (see launch_batch)
    // synchronous path (orb_extract): the image, and one output block (keypoints | descriptors |
    // counts | status) downloaded in one copy into pinned staging
    uint8_t* d_img = nullptr; size_t img_cap = 0;
    uint8_t* d_out = nullptr; uint8_t* h_out = nullptr;
    orb_keypoint_t* d_kps = nullptr; uint8_t* d_desc = nullptr; int32_t* d_counts = nullptr; size_t out_cap = 0;
    // its launch sequence and download captured as one graph, replayed while g1_key (sizes, buffers) holds
    hipGraph_t g1_graph = nullptr;
    hipGraphExec_t g1_exec = nullptr;
    std::vector<uintptr_t> g1_key;
    hipStream_t stream = nullptr;
    int last_n = 0;
    int qt_lds = 0;
    // optional per-stage timing: HIP events recorded on the launch stream between the stages
    // sub-batching over internal streams
    static constexpr int kMaxStreams = 4;
    int chunk = 1 << 30, nstreams = 1;  // off by default: measured slower (streams did not overlap)
    bool fast_stamps = false, pyr_stamps = false;  // debug phase clocks (ORBGPU_FAST_STAMPS / _PYR_STAMPS)
    int fast_split = 3;                 // FAST on levels [0, fast_split) overlaps the small pyramid levels
    int fast_split_cfg = 3;             // the configured split (orb_extractor_set_overlap(h, 0) sets fast_split 0)
    int chain_fast_split = 1;           // one-chain FAST launches (see launch_chunk; ORBGPU_CHAIN_FAST)
    int qt_key_room = 4;                // KB of quad-tree LDS for keys beyond the node tables (ORBGPU_QT_KEYROOM)
    int pyr_affine = 1;                 // pyramid tiles of a frame on one XCD (ORBGPU_PYR_AFFINE=0: spread, for the A/B)
    int ablate = 0;                     // timing study only (ORBGPU_ABLATE): skip stage launches, outputs stale --
                                        // 1 pyramid levels > 0, 2 level 0, 4 FAST, 8 quad-tree, 16 describe,
                                        // 32 levels >= 4, 64 levels 1-3
    int fast_per_level = 0;             // 1: FAST of each later level right after its pyramid level (side2); measured slower
    int desc_split = 1;                 // 1: quad-tree + descriptors of levels [0, fast_split) on the side stream (ORBGPU_DESC_SPLIT)
    orb_keypoint_t* d_st_kp = nullptr; size_t st_kp_cap = 0;   // their staging records (desc_split)
    uint8_t* d_st_desc = nullptr; size_t st_desc_cap = 0;
    int qt_split = 0;                   // 1: quad-tree of levels [0, fast_split) on the side stream (ORBGPU_QT_SPLIT)
    hipStream_t side = nullptr, side2 = nullptr;
    hipEvent_t split_ev[3] = {};
    hipEvent_t lvl_ev[orbgpu::kMaxLevels] = {};
    hipStream_t sub[kMaxStreams] = {};
    hipEvent_t fork_ev = nullptr, join_ev[kMaxStreams] = {};
    long long batches = 0;
    int profile = 0;  // 0 off, 1 every stage boundary, 2 only the pyramid stage (marks 0 and 1),
                      // 3 an event pair around every pyramid level launch (k_pyramid_level durations)
    std::vector<hipEvent_t> pyr_events;  // profile 3: an event pair around every recorded pyramid launch
    size_t pyr_ev_used = 0;              // events recorded since profiling was enabled (2 per launch)
    std::vector<int> pyr_ev_kernel;      // profile 3: the kernel of each recorded pair (kLaunch*)
    std::vector<hipEvent_t> events;   // kStages + 1 per profiled sub-batch launch
    int ev_used = 0;                  // launches recorded since the last read
    long long frames_profiled = 0;
    unsigned long long* d_stamps = nullptr;  // quad-tree phase timers (ORBGPU_DEBUG_FLAGS & 4)
    size_t stamps_cap = 0;
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

// Tile records of every pyramid level, one int4 per tile of a frame (row-major):
//   x: X0 | Y0 << 16 (padded-plane origin)
//   y: bx0 | bw << 16, z: by0 | bh << 16 (level > 0): the previous-level view box the tile reads --
//      the view range its (clamped) columns and rows cover under REFLECT_101, mapped through
//      cv::resize's source index (the kernel's double expressions), plus the second bilinear tap
// Tiles cover the written region [kEdge - kBorder, kEdge + len + kBorder) of each axis.
int pyr_tiles_x(const orbgpu::LevelGeom& L) { return (L.w + 2 * kBorder + kTileW - 1) / kTileW; }
int pyr_tiles_y(const orbgpu::LevelGeom& L) { return (L.h + 2 * kBorder + kTileH - 1) / kTileH; }
void tile_tables(const orbgpu::KernelGeom& k, std::vector<int4>& tab, int* off) {
    auto refl = [](int a, int b, int len, int& lo, int& hi) {
        lo = 1 << 30; hi = -1;
        if (a < 0) { const int e2 = std::min(b, -1); lo = std::min(lo, -e2); hi = std::max(hi, -a); }
        if (b >= 0 && a < len) { lo = std::min(lo, std::max(a, 0)); hi = std::max(hi, std::min(b, len - 1)); }
        if (b >= len) { const int s0 = std::max(a, len); lo = std::min(lo, 2 * len - 2 - b); hi = std::max(hi, 2 * len - 2 - s0); }
    };
    auto src = [](int d, double scale, int slen) {
        const float f = (float)((d + 0.5) * scale - 0.5);
        int s2 = (int)f;
        s2 -= (s2 > f);
        return std::min(std::max(s2, 0), slen - 1);
    };
    tab.clear();
    for (int l = 0; l < k.nlevels; ++l) {
        const orbgpu::LevelGeom& L = k.lv[l];
        off[l] = (int)tab.size();
        for (int ty = 0; ty < pyr_tiles_y(L); ++ty)
            for (int tx = 0; tx < pyr_tiles_x(L); ++tx) {
                const int X0 = kEdge - kBorder + tx * kTileW, Y0 = kEdge - kBorder + ty * kTileH;
                int4 r = make_int4(X0 | Y0 << 16, 0, 0, 0);
                if (l > 0) {
                    const orbgpu::LevelGeom& P = k.lv[l - 1];
                    const double scx = 1. / ((double)L.w / P.w), scy = 1. / ((double)L.h / P.h);
                    int a, b;
                    refl(X0 - kEdge, std::min(X0 + kTileW - 1 - kEdge, L.w + kBorder - 1), L.w, a, b);
                    const int bx0 = src(a, scx, P.w), bw = std::min(src(b, scx, P.w) + 1, P.w - 1) - bx0 + 1;
                    refl(Y0 - kEdge, std::min(Y0 + kTileH - 1 - kEdge, L.h + kBorder - 1), L.h, a, b);
                    const int by0 = src(a, scy, P.h), bh = std::min(src(b, scy, P.h) + 1, P.h - 1) - by0 + 1;
                    r.y = bx0 | bw << 16;
                    r.z = by0 | bh << 16;
                }
                tab.push_back(r);
            }
    }
}

// Two-level records (k_pyramid_pair), two int4 per tile of each level n = l + 1 with l even, at twice the
// tile's index in the tile table (other entries unused):
//   {ux0 | uw << 16, uy0 | uh << 16, cx0 | cw << 16, cy0 | ch << 16}: U, the level-l view box the workgroup
//     computes, and C, the level-(l-1) view box U's taps read (l > 0; the kernel's double expressions, as
//     tile_tables);
//   {ox0 | ox1 << 16, oy0 | oy1 << 16} (16-bit signed): the level-l range it writes, border included.
// The tile columns cut level l's written columns at their first source column (tile_tables' bx0), the
// tile rows its rows likewise.  U is the hull of the tile's own box and the owned range's REFLECT_101
// sources.  Returns false if a box exceeds the kernel's LDS boxes (the level-by-level path runs then).
bool pair_tables(const orbgpu::KernelGeom& k, const std::vector<int4>& tiles, const int* off, std::vector<int4>& tab) {
    auto src = [](int d, double scale, int slen) {
        const float f = (float)((d + 0.5) * scale - 0.5);
        int s2 = (int)f;
        s2 -= (s2 > f);
        return std::min(std::max(s2, 0), slen - 1);
    };
    auto refl = [](int p, int len) { p = p < 0 ? -p : p; return p >= len ? 2 * len - 2 - p : p; };
    tab.assign(2 * tiles.size(), make_int4(0, 0, 0, 0));
    for (int nl = 1; nl < k.nlevels; nl += 2) {
        const orbgpu::LevelGeom &N = k.lv[nl], &L = k.lv[nl - 1];
        const int ntx = pyr_tiles_x(N), nty = pyr_tiles_y(N);
        std::vector<int> cx(ntx + 1), cy(nty + 1);
        cx[0] = -kBorder; cx[ntx] = L.w + kBorder;
        cy[0] = -kBorder; cy[nty] = L.h + kBorder;
        for (int i = 1; i < ntx; ++i) cx[i] = tiles[off[nl] + i].y & 0xffff;
        for (int j = 1; j < nty; ++j) cy[j] = tiles[off[nl] + j * ntx].z & 0xffff;
        for (int i = 0; i < ntx; ++i) if (cx[i] >= cx[i + 1]) return false;
        for (int j = 0; j < nty; ++j) if (cy[j] >= cy[j + 1]) return false;
        for (int ty = 0; ty < nty; ++ty)
            for (int tx = 0; tx < ntx; ++tx) {
                const int idx = off[nl] + ty * ntx + tx;
                const int4 T = tiles[idx];
                int ux0 = T.y & 0xffff, ux1 = ux0 + (T.y >> 16), uy0 = T.z & 0xffff, uy1 = uy0 + (T.z >> 16);
                const int ox0 = cx[tx], ox1 = cx[tx + 1], oy0 = cy[ty], oy1 = cy[ty + 1];
                for (int x = ox0; x < ox1; ++x) { const int v = refl(x, L.w); ux0 = std::min(ux0, v); ux1 = std::max(ux1, v + 1); }
                for (int y = oy0; y < oy1; ++y) { const int v = refl(y, L.h); uy0 = std::min(uy0, v); uy1 = std::max(uy1, v + 1); }
                const int uw = ux1 - ux0, uh = uy1 - uy0;
                const int nch = ((ox1 + kEdge - 1) >> 3) - ((ox0 + kEdge) >> 3) + 1;  // 8-byte chunks of a row
                if (uw + 8 > kPairUP || uw > 128 + 32 || uh > kPairUH || nch > 21 || ox0 < -32768 || ox1 > 32767) return false;
                int cx0 = 0, cw = 0, cy0 = 0, chh = 0;
                if (nl > 1) {
                    const orbgpu::LevelGeom& Pv = k.lv[nl - 2];
                    const double scx = 1. / ((double)L.w / Pv.w), scy = 1. / ((double)L.h / Pv.h);
                    cx0 = src(ux0, scx, Pv.w);
                    cw = std::min(src(ux1 - 1, scx, Pv.w) + 1, Pv.w - 1) - cx0 + 1;
                    cy0 = src(uy0, scy, Pv.h);
                    chh = std::min(src(uy1 - 1, scy, Pv.h) + 1, Pv.h - 1) - cy0 + 1;
                    if (cw + 3 + 8 > kPairCW || chh > kPairCH) return false;
                }
                tab[2 * idx] = make_int4(ux0 | uw << 16, uy0 | uh << 16, cx0 | cw << 16, cy0 | chh << 16);
                tab[2 * idx + 1] = make_int4((ox0 & 0xffff) | ox1 << 16, (oy0 & 0xffff) | oy1 << 16, 0, 0);
            }
    }
    return true;
}

int prepare(Extractor* e, int w, int h, int n) {
    if (w != e->cur_w || h != e->cur_h) {
        // the tables below are read by in-flight launches of the previous frame size
        if (e->cur_w >= 0 && hipDeviceSynchronize() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "sync failed");
        orbgpu::Geometry g;
        if (!orbgpu::build_geometry(e->P, w, h, g)) return orbgpu_fail(ORB_ERR_ARG, "image too small for the pyramid/cell grid");
        for (int v = 0; v < 16; ++v)  // k_describe's compile-time disc table (c_disc) assumes these
            if (g.k.umax[v] != kDiscUmax[v]) return orbgpu_fail(ORB_ERR_INTERNAL, "umax differs from the IC_Angle disc table");
        e->geo = g;
        e->cur_w = w;
        e->cur_h = h;
        int rc;
        if ((rc = grow(e->d_cells, e->cells_cap, g.cells.size())) != ORB_OK) return rc;
        if ((rc = grow(e->d_xtab, e->xtab_cap, std::max<size_t>(1, g.xtab.size() / 2))) != ORB_OK) return rc;
        if ((rc = grow(e->d_ytab, e->ytab_cap, std::max<size_t>(1, g.ytab.size() / 4))) != ORB_OK) return rc;
        if (!e->d_geom && hipMalloc(&e->d_geom, sizeof(orbgpu::KernelGeom)) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
        if (hipMemcpy(e->d_geom, &g.k, sizeof(orbgpu::KernelGeom), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(e->d_cells, g.cells.data(), g.cells.size() * sizeof(orbgpu::CellDesc), hipMemcpyHostToDevice) != hipSuccess ||
            (!g.xtab.empty() && hipMemcpy(e->d_xtab, g.xtab.data(), g.xtab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
            (!g.ytab.empty() && hipMemcpy(e->d_ytab, g.ytab.data(), g.ytab.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
            return orbgpu_fail(ORB_ERR_DEVICE, "table upload failed");
        std::vector<int4> tt;
        tile_tables(g.k, tt, e->tile_off);
        // every tile's source box must fit the LDS box of the k_pyramid_level instance its level
        // launches (launch_chunk: the small box for level ratios <= 1.25, else the wide one, sized for
        // ratios up to 2; the alignment shift takes up to 3 more bytes)
        for (int l = 1; l < g.k.nlevels; ++l) {
            const bool small = 4 * g.k.lv[l - 1].w <= 5 * g.k.lv[l].w && 4 * g.k.lv[l - 1].h <= 5 * g.k.lv[l].h;
            const int bwmax = (small ? kSmallBoxW : kBoxW) - 3, bhmax = small ? kSmallBoxH : kBoxH;
            const int t1 = l + 1 < g.k.nlevels ? e->tile_off[l + 1] : (int)tt.size();
            for (int t = e->tile_off[l]; t < t1; ++t)
                if ((tt[t].y >> 16) > bwmax || (tt[t].z >> 16) > bhmax) {
                    e->cur_w = e->cur_h = -1;  // the next call rebuilds (and rejects) the geometry
                    e->geo_ok = false;
                    return orbgpu_fail(ORB_ERR_ARG, "pyramid level ratio above 2 (scale factor too large)");
                }
        }
        if ((rc = grow(e->d_tiletab, e->tiletab_cap, tt.size())) != ORB_OK) return rc;
        if (hipMemcpy(e->d_tiletab, tt.data(), tt.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "table upload failed");
        std::vector<int4> pt;
        e->pair_ok = pair_tables(g.k, tt, e->tile_off, pt);
        if (e->pair_ok) {
            if ((rc = grow(e->d_pairtab, e->pairtab_cap, pt.size())) != ORB_OK) return rc;
            if (hipMemcpy(e->d_pairtab, pt.data(), pt.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess)
                return orbgpu_fail(ORB_ERR_DEVICE, "table upload failed");
        }
        e->geo_ok = true;
        // quad-tree LDS: node metadata of the largest level (larger feature budgets, e.g. the 5x
        // monocular-init extractor, need more) + key room
        size_t meta = 0;
        for (int l = 0; l < g.k.nlevels; ++l) {
            const int lcap = g.k.lv[l].sel_cap + 64;
            meta = std::max(meta, (qt2_meta_bytes(lcap) + 15) & ~(size_t)15);
        }
        // node tables + room for the keys of a small level (6 B per key); levels with more keys use
        // the global scratch.  Kept small: the quad-tree blocks are long-lived and latency-bound, and
        // the LDS they do not hold lets another batch's FAST / pyramid / describe blocks share the CU
        // (round 4, 3 batches in flight: 32 KB 313-315k, 12 KB 318-320k, 4 KB 322-326k features/ms).
        const size_t want = meta + (size_t)e->qt_key_room * 1024;
        if (meta > 160 * 1024) return orbgpu_fail(ORB_ERR_ARG, "nfeatures too large for the quad-tree LDS budget");
        e->qt_lds = (int)std::min<size_t>(want, 160 * 1024);
        // the attribute is per function (shared by every handle): allow the whole LDS, each launch
        // requests its handle's qt_lds
        if (hipFuncSetAttribute((const void*)k_quadtree_kp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "cannot raise the quad-tree LDS limit");
    }
    const orbgpu::KernelGeom& k = e->geo.k;
    int rc;
    if ((rc = grow(e->d_pyr, e->pyr_cap, (size_t)k.pyr_frame_bytes * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_cand, e->cand_cap, (size_t)k.cand_frame_cap * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_scratch, e->scratch_cap, (size_t)k.cand_frame_cap * n * 2)) != ORB_OK) return rc;
    if ((rc = grow(e->d_cell_count, e->cell_count_cap, (size_t)k.ncells * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_cell_thr, e->cell_thr_cap, (size_t)k.ncells * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_sel, e->sel_cap, (size_t)k.sel_frame_cap * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_dst, e->dst_cap, (size_t)k.sel_frame_cap * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_sel_count, e->selcount_cap, (size_t)k.nlevels * n)) != ORB_OK) return rc;
    if ((rc = grow(e->d_lap_count, e->lapcount_cap, (size_t)k.nlevels * n)) != ORB_OK) return rc;
    if (e->desc_split) {
        if ((rc = grow(e->d_st_kp, e->st_kp_cap, (size_t)k.sel_frame_cap * n)) != ORB_OK) return rc;
        if ((rc = grow(e->d_st_desc, e->st_desc_cap, (size_t)k.sel_frame_cap * n * 32)) != ORB_OK) return rc;
    }
    if ((k.debug_flags & 4) && (rc = grow(e->d_stamps, e->stamps_cap, (size_t)k.nlevels * n * kQtStamps)) != ORB_OK) return rc;
    return ORB_OK;
}

// Enqueue the five stages for frames [f0, f0 + n) of the handle's buffers on stream st.
int launch_chunk(Extractor* e, int f0, const uint8_t* d_images, int n, int stride, size_t frame_stride, int lap0,
                 int lap1, orb_keypoint_t* d_kps, uint8_t* d_desc, int cap, int32_t* d_counts, hipStream_t st) {
    const orbgpu::Geometry& G = e->geo;
    const orbgpu::KernelGeom& k = G.k;
    hipEvent_t* ev = nullptr;
    if (e->profile == 1 || e->profile == 2) {
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
    auto mark = [&](int i) {  // profile 3 (per-launch event pairs) records no stage events
        if (ev && (e->profile == 1 || (e->profile == 2 && i <= 1))) hipEventRecord(ev[i], st);
    };
    uint8_t* pyr = e->d_pyr + (size_t)f0 * k.pyr_frame_bytes;
    uint32_t* cand = e->d_cand + (size_t)f0 * k.cand_frame_cap;
    uint32_t* scratch = e->d_scratch + (size_t)f0 * k.cand_frame_cap * 2;
    int32_t* ccount = e->d_cell_count + (size_t)f0 * k.ncells;
    uint8_t* cthr = e->d_cell_thr + (size_t)f0 * k.ncells;
    uint32_t* sel = e->d_sel + (size_t)f0 * k.sel_frame_cap;
    int32_t* dst = e->d_dst + (size_t)f0 * k.sel_frame_cap;
    int32_t* scount = e->d_sel_count + (size_t)f0 * k.nlevels;
    int32_t* lapc = e->d_lap_count + (size_t)f0 * k.nlevels;
    const uint8_t* imgs = d_images + (size_t)f0 * frame_stride;
    orb_keypoint_t* kps = d_kps + (size_t)f0 * cap;
    uint8_t* desc = d_desc + (size_t)f0 * cap * 32;
    int32_t* counts = d_counts + 2 * (size_t)f0;
    mark(0);
    // FAST on the first `split` levels runs on a side stream as soon as those pyramid levels exist,
    // overlapping the latency-bound launches of the small levels (k.lv[split..] ) on `st`.
    // (a single frame runs as one chain: too few blocks per level for the overlap to pay)
    const int split = (n > 1 && e->fast_split > 0 && e->fast_split < k.nlevels) ? e->fast_split : 0;
    const bool fast_stamps = e->fast_stamps;
    // profile 3: the next free event pair, tagged with its kernel (nullptr when not profiling)
    auto launch_events = [&](int kernel) -> hipEvent_t* {
        if (e->profile != 3 || e->pyr_ev_used + 2 > e->pyr_events.size()) return nullptr;
        hipEvent_t* pe = &e->pyr_events[e->pyr_ev_used];
        e->pyr_ev_kernel[e->pyr_ev_used / 2] = kernel;
        e->pyr_ev_used += 2;
        return pe;
    };
    auto launch_fast = [&](int l0, int l1, hipStream_t s2) {
        if (e->ablate & 4) return;
        const int c0 = k.lv[l0].cell_begin, c1 = k.lv[l1 - 1].cell_begin + k.lv[l1 - 1].cell_count;
        if (c1 <= c0) return;
        unsigned long long* stamps = nullptr;
        const size_t ns = (size_t)(c1 - c0) * n * 12;
        if (fast_stamps && hipMalloc(&stamps, ns * 8) == hipSuccess) (void)hipMemsetAsync(stamps, 0, ns * 8, s2);
        // LDS per wave sized by the largest window of the launched levels: the early levels' smaller
        // windows allow more resident waves than the level-7 window would
        int mw = 0, md = 0, ms = 0;
        for (int l = l0; l < l1; ++l) {
            mw = std::max(mw, G.max_win_lv[l]);
            md = std::max(md, G.max_det_lv[l]);
            ms = std::max(ms, G.max_sc_lv[l]);
        }
        const int win_cap = (mw + 15) & ~15, sc_cap = (ms + 15) & ~15;
        // per wave: window | score map | candidate list (u16, at most one entry per detectable pixel)
        const int wave_lds = win_cap + sc_cap + ((2 * md + 15) & ~15);
        const int groups = (c1 - c0 + 3) / 4, nblocks = groups * n, share = (nblocks + 7) / 8;
        if (hipEvent_t* pe = launch_events(kLaunchFast))
            hipExtLaunchKernelGGL(k_fast_cells, dim3(8 * share), dim3(256), 4 * wave_lds, s2, pe[0], pe[1], 0, e->d_geom,
                                  e->d_cells, win_cap, sc_cap, wave_lds, pyr, cand, ccount, cthr, c0, c1, stamps, groups, nblocks,
                                  share);
        else
            hipLaunchKernelGGL(k_fast_cells, dim3(8 * share), dim3(256), 4 * wave_lds, s2, e->d_geom, e->d_cells, win_cap,
                               sc_cap, wave_lds, pyr, cand, ccount, cthr, c0, c1, stamps, groups, nblocks, share);
        if (stamps) {  // debug: mean phase clocks over the launch's cells
            std::vector<unsigned long long> h(ns);
            (void)hipStreamSynchronize(s2);
            (void)hipMemcpy(h.data(), stamps, ns * 8, hipMemcpyDeviceToHost);
            (void)hipFree(stamps);
            double ph[6] = {0}, life = 0, sv = 0, cn = 0;
            unsigned long long t0 = ~0ull, t1 = 0;
            size_t cnt = 0;
            for (size_t i = 0; i < ns; i += 12) {
                if (!h[i + 7]) continue;
                ++cnt;
                for (int q = 1; q <= 6; ++q) ph[q - 1] += (double)(h[i + q] - h[i + q - 1]);
                life += (double)(h[i + 8] - h[i + 7]);
                sv += (double)h[i + 9];
                cn += (double)h[i + 10];
                t0 = std::min(t0, h[i + 7]);
                t1 = std::max(t1, h[i + 8]);
            }
            fprintf(stderr, "fast-stamps L%d-%d cells %zu span %.1f us life %.2f us conc %.0f | stage %.0f compass %.0f full %.0f score %.0f thr %.0f emit %.0f cyc | surv %.1f corners %.1f\n",
                    l0, l1 - 1, cnt, (t1 - t0) * 0.01, life / cnt * 0.01, life / (double)(t1 - t0), ph[0] / cnt, ph[1] / cnt,
                    ph[2] / cnt, ph[3] / cnt, ph[4] / cnt, ph[5] / cnt, sv / cnt, cn / cnt);
        }
    };
    // quad-tree of levels [l0, l1): one wave per (level, frame)
    auto launch_qt = [&](int l0, int l1, hipStream_t s2) {
        if (l1 <= l0 || (e->ablate & 8)) return;
        unsigned long long* qst = e->d_stamps ? e->d_stamps + (size_t)f0 * k.nlevels * kQtStamps : nullptr;
        if (hipEvent_t* pe = launch_events(kLaunchQuadtree))
            hipExtLaunchKernelGGL(k_quadtree_kp, dim3(l1 - l0, n), dim3(kQtThreads), e->qt_lds, s2, pe[0], pe[1], 0,
                                  e->d_geom, e->d_cells, cand, ccount, scratch, sel, scount, e->qt_lds, e->d_status, qst,
                                  lap0, lap1, dst, lapc, l0);
        else
            hipLaunchKernelGGL(k_quadtree_kp, dim3(l1 - l0, n), dim3(kQtThreads), e->qt_lds, s2, e->d_geom, e->d_cells, cand,
                               ccount, scratch, sel, scount, e->qt_lds, e->d_status, qst, lap0, lap1, dst, lapc, l0);
    };
    // descriptors of levels [0, lim) (stage_mode 1: into the staging records; 2: all levels, the first
    // `split` from their staging records; 0: all levels computed here)
    bool desc_split = false;  // set once the pyramid path is known (below)
    auto launch_desc = [&](int mode, int lim, hipStream_t s2) {
        if (e->ablate & 16) return;
        int chunks = 0;  // blocks per frame: ceil(sel_cap_l / 8) per level (see k_describe)
        for (int l = 0; l < lim; ++l) chunks += (k.lv[l].sel_cap + kDescKpPerBlock - 1) / kDescKpPerBlock;
        const int total = chunks * n, share = (total + 7) / 8;
        orb_keypoint_t* skp = e->d_st_kp ? e->d_st_kp + (size_t)f0 * k.sel_frame_cap : nullptr;
        uint8_t* sdesc = e->d_st_desc ? e->d_st_desc + (size_t)f0 * k.sel_frame_cap * 32 : nullptr;
        if (hipEvent_t* pe = launch_events(kLaunchDescribe))
            hipExtLaunchKernelGGL(k_describe, dim3(8 * share), dim3(256), 0, s2, pe[0], pe[1], 0, e->d_geom, pyr, sel, scount,
                                  dst, lapc, cap, kps, desc, counts, chunks, total, share, split, mode, skp, sdesc);
        else
            hipLaunchKernelGGL(k_describe, dim3(8 * share), dim3(256), 0, s2, e->d_geom, pyr, sel, scount, dst, lapc, cap,
                               kps, desc, counts, chunks, total, share, split, mode, skp, sdesc);
    };
    // One chain (no side-stream split): FAST of levels [0, chain_s) and [chain_s, n) as two launches, each
    // sizing its LDS for its own windows (the tall level-6/7 windows would otherwise set the level-0
    // occupancy); chain_lds_split 1: both after the pyramid, 2: the first right after level chain_s - 1
    const int chain_s = std::min(std::max(e->fast_split_cfg, 1), k.nlevels);
    const int chain_lds_split = (n > 1 && chain_s < k.nlevels) ? e->chain_fast_split : 0;
    // the early levels' FAST (and with desc_split their quad-tree + descriptors) go to the side stream
    desc_split = e->desc_split && split > 0 && !e->fast_per_level && e->d_st_kp;
    const bool qts = (e->qt_split || desc_split) && split > 0 && !e->fast_per_level;
    const bool pyr_stamps = e->pyr_stamps;
    // what follows pyramid level l on the streams (FAST of the early levels once they exist)
    auto level_done = [&](int l) {
        if (!split && chain_lds_split == 2 && l == chain_s - 1) {
            launch_fast(0, chain_s, st);  // one chain: the early levels' FAST right after their pyramid levels
        } else if (split && l == split - 1) {
            hipEventRecord(e->split_ev[0], st);
            hipStreamWaitEvent(e->side, e->split_ev[0], 0);
            launch_fast(0, split, e->side);
            if (qts) launch_qt(0, split, e->side);
            if (desc_split) launch_desc(1, split, e->side);
            hipEventRecord(e->split_ev[1], e->side);
        } else if (split && l >= split && e->fast_per_level) {
            // later (small) levels: FAST as soon as the level exists, on a second side stream
            hipEventRecord(e->lvl_ev[l], st);
            hipStreamWaitEvent(e->side2, e->lvl_ev[l], 0);
            launch_fast(l, l + 1, e->side2);
        }
    };
    // two levels per pass (k_pyramid_pair) when the geometry fits its boxes; the phase-clock debug
    // mode (ORBGPU_PYR_STAMPS) times the level kernel
    const bool pairs = e->pyr_pair && e->pair_ok && !pyr_stamps;
    for (int l = 0; l < k.nlevels; ++l) {
        if (pairs && (l & 1) == 0 && l + 1 < k.nlevels && (e->pyr_pair == 1 || l == 0)) {
            const orbgpu::LevelGeom &Ll = k.lv[l], &Ln = k.lv[l + 1];
            PairArgs A{};
            A.frame_bytes = k.pyr_frame_bytes;
            A.plane_l = Ll.plane_off;
            A.plane_n = Ln.plane_off;
            if (l > 0) {
                const orbgpu::LevelGeom& P = k.lv[l - 1];
                A.src_off = P.plane_off + (long long)kEdge * P.pitch + kEdge;
                A.spitch = P.pitch;
            }
            A.wl = Ll.w; A.hl = Ll.h; A.pitch_l = Ll.pitch; A.xtab_l = Ll.xtab_off; A.ytab_l = Ll.ytab_off; A.simd_l = Ll.simd_end;
            A.wn = Ln.w; A.hn = Ln.h; A.pitch_n = Ln.pitch; A.xtab_n = Ln.xtab_off; A.ytab_n = Ln.ytab_off; A.simd_n = Ln.simd_end;
            A.tab_off = e->tile_off[l + 1];
            A.tiles_per_frame = pyr_tiles_x(Ln) * pyr_tiles_y(Ln);
            A.share = (A.tiles_per_frame + 7) / 8;
            A.frame_affine = e->pyr_affine && n % 8 == 0;
            const dim3 grid(8 * A.share, n);
            hipEvent_t* pe = launch_events(kLaunchPyramid);
            auto go = [&](auto kern, auto... args) {
                if (e->ablate & (l == 0 ? 3 : 1)) return;
                if (pe) hipExtLaunchKernelGGL(kern, grid, dim3(256), 0, st, pe[0], pe[1], 0, args...);
                else hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, args...);
            };
            if (l == 0)
                go(k_pyramid_pair<true>, A, imgs, (long long)frame_stride, stride, pyr, (const int2*)e->d_xtab,
                   (const int4*)e->d_ytab, (const int4*)e->d_tiletab, (const int4*)e->d_pairtab,
                   e->clear_status_l0 && f0 == 0 ? e->d_status : (int*)nullptr);
            else
                go(k_pyramid_pair<false>, A, (const uint8_t*)nullptr, 0LL, 0, pyr, (const int2*)e->d_xtab,
                   (const int4*)e->d_ytab, (const int4*)e->d_tiletab, (const int4*)e->d_pairtab, (int*)nullptr);
            level_done(l);
            level_done(l + 1);
            ++l;
            continue;
        }
        const orbgpu::LevelGeom& L = k.lv[l];
        PyrArgs A{};
        A.frame_bytes = k.pyr_frame_bytes;
        A.plane_off = L.plane_off;
        A.w = L.w; A.h = L.h; A.pw = L.pw; A.ph = L.ph; A.pitch = L.pitch;
        A.xtab_off = L.xtab_off; A.ytab_off = L.ytab_off; A.simd_end = L.simd_end;
        if (l > 0) {
            const orbgpu::LevelGeom& P = k.lv[l - 1];
            A.src_off = P.plane_off + (long long)kEdge * P.pitch + kEdge;
            A.sw = P.w; A.sh = P.h; A.spitch = P.pitch;
        }
        A.tab_off = e->tile_off[l];
        A.tiles_per_frame = pyr_tiles_x(L) * pyr_tiles_y(L);
        A.share = (A.tiles_per_frame + 7) / 8;  // tiles of a frame per XCD (xcd_tile)
        A.frame_affine = e->pyr_affine && n % 8 == 0;
        const dim3 grid(8 * A.share, n);
        unsigned long long* stamps = nullptr;
        const size_t nblk = (size_t)grid.x * grid.y;
        if (pyr_stamps && hipMalloc(&stamps, sizeof(unsigned long long) * 8 * nblk) == hipSuccess)
            (void)hipMemsetAsync(stamps, 0, sizeof(unsigned long long) * 8 * nblk, st);
        // profile 3: the launch carries an event pair (hipExtLaunchKernel) that takes the dispatch's own
        // begin / end timestamps -- the interval rocprofv3's kernel trace reports for it
        hipEvent_t* pe = launch_events(kLaunchPyramid);
        auto go = [&](auto kern, auto... args) {
            if (e->ablate & (l == 0 ? 2 : 1)) return;
            if ((e->ablate & 32) && l >= 4) return;
            if ((e->ablate & 64) && l >= 1 && l < 4) return;
            if (pe) hipExtLaunchKernelGGL(kern, grid, dim3(256), 0, st, pe[0], pe[1], 0, args...);
            else hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, args...);
        };
        const int2* xt = e->d_xtab;
        const int4* yt = e->d_ytab;
        const int4* tt = e->d_tiletab;
        if (l == 0)
            go(k_pyramid_level<true>, A, imgs, (long long)frame_stride, stride, pyr, xt, yt, tt, stamps,
               e->clear_status_l0 && f0 == 0 ? e->d_status : (int*)nullptr);
        else if (4 * k.lv[l - 1].w <= 5 * L.w && 4 * k.lv[l - 1].h <= 5 * L.h)  // level ratio <= 1.25
            go(k_pyramid_level<false, kSmallBoxH, kSmallBoxW>, A, (const uint8_t*)nullptr, 0LL, 0, pyr, xt, yt, tt, stamps,
               (int*)nullptr);
        else
            go(k_pyramid_level<false, kBoxH, kBoxW>, A, (const uint8_t*)nullptr, 0LL, 0, pyr, xt, yt, tt, stamps,
               (int*)nullptr);
        if (stamps && pyr_stamps) {  // debug: phase clocks of this level's blocks
            std::vector<unsigned long long> hst((size_t)8 * nblk);
            (void)hipStreamSynchronize(st);
            (void)hipMemcpy(hst.data(), stamps, hst.size() * 8, hipMemcpyDeviceToHost);
            (void)hipFree(stamps);
            double ph[4] = {0}, life = 0;
            unsigned long long t0 = ~0ull, t1 = 0;
            int cnt = 0;
            for (size_t b = 0; b < nblk; ++b) {
                const unsigned long long* q = &hst[(size_t)8 * b];
                if (!q[6]) continue;
                ++cnt;
                for (int i = 1; i < 4; ++i) ph[i] += (double)(q[i] - q[i - 1]);
                life += (double)(q[7] - q[6]);
                t0 = std::min(t0, q[6]);
                t1 = std::max(t1, q[7]);
            }
            fprintf(stderr, "pyr-stamps L%d blocks %d span %.1f us  mean life %.2f us  concurrency %.0f  phases(cyc) box %.0f resize %.0f store %.0f\n",
                    l, cnt, (t1 - t0) * 0.01, life / cnt * 0.01, life / (double)(t1 - t0), ph[1] / cnt, ph[2] / cnt,
                    ph[3] / cnt);
        }
        level_done(l);
    }
    mark(1);
    if (split && e->fast_per_level) {
        hipEventRecord(e->split_ev[2], e->side2);
        hipStreamWaitEvent(st, e->split_ev[2], 0);
    } else if (!split && chain_lds_split == 1) {
        launch_fast(0, chain_s, st);
        launch_fast(chain_s, k.nlevels, st);
    } else if (!split && chain_lds_split == 2) {
        launch_fast(chain_s, k.nlevels, st);
    } else {
        launch_fast(split, k.nlevels, st);
    }
    // qt_split: the quad-tree of the early levels runs on the side stream right after their FAST
    // (desc_split: and their descriptors, into the staging records)
    if (!qts && split) hipStreamWaitEvent(st, e->split_ev[1], 0);
    mark(2);
    launch_qt(qts ? split : 0, k.nlevels, st);
    if (qts) hipStreamWaitEvent(st, e->split_ev[1], 0);
    mark(3);
    mark(4);
    launch_desc(desc_split ? 2 : 0, k.nlevels, st);
    mark(5);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "kernel launch failed");
    return ORB_OK;
}

// A batch is split into sub-batches of e->chunk frames on the handle's internal streams (fork/join
// with events against the caller's stream), so the latency-bound stages of one sub-batch (quad-tree,
// descriptors) overlap the compute-bound stages (pyramid, FAST) of another.
int launch_batch(Extractor* e, const uint8_t* d_images, int n, int w, int h, int stride, size_t frame_stride,
                 int lap0, int lap1, orb_keypoint_t* d_kps, uint8_t* d_desc, int cap, int32_t* d_counts,
                 hipStream_t st) {
    (void)w; (void)h;
    {   // timing study only: re-read per call, so a handle warmed with every stage can then skip some
        const char* c = getenv("ORBGPU_ABLATE");
        e->ablate = c ? atoi(c) : 0;
    }
    // the level-0 pyramid launch of the first (sub-)batch clears the status; sub-batches on several
    // streams need it cleared before the fork
    e->clear_status_l0 = !(e->nstreams > 1 && (n + e->chunk - 1) / e->chunk > 1);
    if (!e->clear_status_l0) hipMemsetAsync(e->d_status, 0, sizeof(int), st);
    const int nchunks = (n + e->chunk - 1) / e->chunk;
    if (nchunks <= 1 || e->nstreams <= 1) {
        const int rc = launch_chunk(e, 0, d_images, n, stride, frame_stride, lap0, lap1, d_kps, d_desc, cap, d_counts, st);
        if (rc != ORB_OK) return rc;
    } else {
        hipEventRecord(e->fork_ev, st);
        for (int s = 0; s < e->nstreams; ++s) hipStreamWaitEvent(e->sub[s], e->fork_ev, 0);
        for (int c = 0; c < nchunks; ++c) {
            const int f0 = c * e->chunk, m = std::min(e->chunk, n - f0);
            const int rc = launch_chunk(e, f0, d_images, m, stride, frame_stride, lap0, lap1, d_kps, d_desc, cap, d_counts,
                                        e->sub[c % e->nstreams]);
            if (rc != ORB_OK) return rc;
        }
        for (int s = 0; s < e->nstreams; ++s) {
            hipEventRecord(e->join_ev[s], e->sub[s]);
            hipStreamWaitEvent(st, e->join_ev[s], 0);
        }
    }
    e->batches++;
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
    e->qt_lds = 64 * 1024;  // set per frame size in prepare()
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&e->d_status_own, sizeof(int)) != hipSuccess) {
        delete e;
        return orbgpu_fail(ORB_ERR_DEVICE, "stream/status allocation failed");
    }
    e->d_status = e->d_status_own;
    hipFuncSetAttribute((const void*)k_quadtree_kp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (const char* c = getenv("ORBGPU_CHUNK")) e->chunk = std::max(1, atoi(c));
    if (const char* c = getenv("ORBGPU_STREAMS")) e->nstreams = std::min(Extractor::kMaxStreams, std::max(1, atoi(c)));
    if (const char* c = getenv("ORBGPU_FAST_SPLIT")) e->fast_split = atoi(c);
    e->fast_split_cfg = e->fast_split;
    if (const char* c = getenv("ORBGPU_CHAIN_FAST")) e->chain_fast_split = atoi(c);
    if (const char* c = getenv("ORBGPU_QT_KEYROOM")) e->qt_key_room = std::max(0, atoi(c));
    if (const char* c = getenv("ORBGPU_PYR_AFFINE")) e->pyr_affine = atoi(c);
    if (const char* c = getenv("ORBGPU_PYR_PAIR")) e->pyr_pair = atoi(c);
    bool ok = hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming) == hipSuccess &&
              hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&e->side2, hipStreamNonBlocking) == hipSuccess;
    for (int k2 = 0; k2 < 3 && ok; ++k2) ok = hipEventCreateWithFlags(&e->split_ev[k2], hipEventDisableTiming) == hipSuccess;
    for (int k2 = 0; k2 < orbgpu::kMaxLevels && ok; ++k2)
        ok = hipEventCreateWithFlags(&e->lvl_ev[k2], hipEventDisableTiming) == hipSuccess;
    if (const char* c = getenv("ORBGPU_FAST_PER_LEVEL")) e->fast_per_level = atoi(c);
    if (const char* c = getenv("ORBGPU_QT_SPLIT")) e->qt_split = atoi(c);
    if (const char* c = getenv("ORBGPU_DESC_SPLIT")) e->desc_split = atoi(c);
    e->fast_stamps = getenv("ORBGPU_FAST_STAMPS") != nullptr;
    e->pyr_stamps = getenv("ORBGPU_PYR_STAMPS") != nullptr;
    for (int s = 0; s < Extractor::kMaxStreams && ok; ++s)
        ok = hipStreamCreateWithFlags(&e->sub[s], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&e->join_ev[s], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        orb_extractor_destroy(reinterpret_cast<orb_extractor_t>(e));
        return orbgpu_fail(ORB_ERR_DEVICE, "stream/event creation failed");
    }
    *out = reinterpret_cast<orb_extractor_t>(e);
    return ORB_OK;
}

int orbgpu_extractor_pyramid(orb_extractor_t h, OrbPyramidView* out) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !out) return orbgpu_fail(ORB_ERR_ARG, "null handle");
    if (!e->geo_ok || e->last_n <= 0) return orbgpu_fail(ORB_ERR_ARG, "the extractor has not run yet");
    const orbgpu::KernelGeom& k = e->geo.k;
    *out = OrbPyramidView{};
    out->base = e->d_pyr;
    out->frame_bytes = k.pyr_frame_bytes;
    out->nframes = e->last_n;
    out->nlevels = k.nlevels;
    for (int l = 0; l < k.nlevels; ++l) {
        out->plane_off[l] = k.lv[l].plane_off;
        out->pitch[l] = k.lv[l].pitch;
        out->w[l] = k.lv[l].w;
        out->h[l] = k.lv[l].h;
        out->scale[l] = e->P.scale[l];
        out->inv_scale[l] = e->P.inv_scale[l];
    }
    out->stream = e->stream;
    return ORB_OK;
}

int orb_extractor_destroy(orb_extractor_t h) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e) return ORB_ERR_ARG;
    if (e->stream) hipStreamSynchronize(e->stream);
    void* bufs[] = {e->d_st_kp, e->d_st_desc, e->d_stamps, e->d_geom, e->d_cells, e->d_xtab, e->d_tiletab, e->d_pairtab, e->d_ytab, e->d_pyr, e->d_cand, e->d_scratch,
                    e->d_cell_count, e->d_cell_thr, e->d_sel, e->d_dst, e->d_sel_count, e->d_lap_count, e->d_status_own,
                    e->d_img, e->d_out};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->g1_exec) (void)hipGraphExecDestroy(e->g1_exec);
    if (e->g1_graph) (void)hipGraphDestroy(e->g1_graph);
    for (hipEvent_t x : e->events) (void)hipEventDestroy(x);
    for (hipEvent_t x : e->pyr_events) (void)hipEventDestroy(x);
    if (e->side) { hipStreamSynchronize(e->side); hipStreamDestroy(e->side); }
    if (e->side2) { hipStreamSynchronize(e->side2); hipStreamDestroy(e->side2); }
    for (int k2 = 0; k2 < 3; ++k2)
        if (e->split_ev[k2]) hipEventDestroy(e->split_ev[k2]);
    for (int k2 = 0; k2 < orbgpu::kMaxLevels; ++k2)
        if (e->lvl_ev[k2]) hipEventDestroy(e->lvl_ev[k2]);
    for (int s = 0; s < Extractor::kMaxStreams; ++s) {
        if (e->sub[s]) { hipStreamSynchronize(e->sub[s]); hipStreamDestroy(e->sub[s]); }
        if (e->join_ev[s]) hipEventDestroy(e->join_ev[s]);
    }
    if (e->fork_ev) hipEventDestroy(e->fork_ev);
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

int orb_extractor_set_overlap(orb_extractor_t h, int mode) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || (mode != 0 && mode != 1)) return orbgpu_fail(ORB_ERR_ARG, "bad handle or overlap mode");
    e->fast_split = mode ? e->fast_split_cfg : 0;
    return ORB_OK;
}

int orb_extract(orb_extractor_t h, const uint8_t* image, int width, int height, int stride, int lap_x0, int lap_x1,
                orb_keypoint_t* kps, uint8_t* desc, int cap, int* n_kps) {
    orbgpu::StageTimer timer("ORB Extraction");  // mTimeORB_Ext (src/Frame.cc:132-146)
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
    const size_t desc_off = (sizeof(orb_keypoint_t) * dcap + 255) & ~(size_t)255;
    const size_t cnt_off = desc_off + ((32 * (size_t)dcap + 255) & ~(size_t)255), st_off = cnt_off + 8, blk = st_off + 8;
    if (e->out_cap < (size_t)dcap || !e->d_out) {
        (void)hipStreamSynchronize(e->stream);
        if (e->d_out) (void)hipFree(e->d_out);
        if (e->h_out) (void)hipHostFree(e->h_out);
        e->d_out = e->h_out = nullptr;
        e->out_cap = 0;
        e->d_status = e->d_status_own;
        if (hipMalloc(&e->d_out, blk) != hipSuccess || hipHostMalloc(&e->h_out, blk, 0) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "output allocation failed");
        e->out_cap = dcap;
        e->d_status = reinterpret_cast<int*>(e->d_out + st_off);  // downloaded with the outputs
    }
    e->d_kps = reinterpret_cast<orb_keypoint_t*>(e->d_out);
    e->d_desc = e->d_out + desc_off;
    e->d_counts = reinterpret_cast<int32_t*>(e->d_out + cnt_off);
    if (hipMemcpy2DAsync(e->d_img, width, image, stride, width, height, hipMemcpyHostToDevice, e->stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "upload failed");
    // the launches and one download of the whole output block (keypoints, descriptors, counts) plus
    // the status word
    auto enqueue = [&]() -> int {
        const int r = launch_batch(e, e->d_img, 1, width, height, width, (size_t)width * height, lap_x0, lap_x1, e->d_kps,
                                   e->d_desc, cap, e->d_counts, e->stream);
        if (r != ORB_OK) return r;
        if (hipMemcpyAsync(e->h_out, e->d_out, st_off + 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "download failed");
        return ORB_OK;
    };
    // Tracking calls this once per frame with the same sizes: the ~20 launches and their event
    // hand-offs are replayed as one graph (host enqueue gaps between the device's launches otherwise
    // dominate a single frame).  Timing / debug modes launch directly.
    static const bool graph_off = getenv("ORBGPU_FAST_STAMPS") || getenv("ORBGPU_PYR_STAMPS");
    bool use_graph = !graph_off && e->profile == 0 && !(e->geo.k.debug_flags & 4);
    if (use_graph) {
        const std::vector<uintptr_t> key = {
            (uintptr_t)width, (uintptr_t)height, (uintptr_t)lap_x0, (uintptr_t)lap_x1, (uintptr_t)cap,
            (uintptr_t)e->d_img, (uintptr_t)e->d_out, (uintptr_t)e->h_out, (uintptr_t)e->d_pyr, (uintptr_t)e->d_cand,
            (uintptr_t)e->d_scratch, (uintptr_t)e->d_cell_count, (uintptr_t)e->d_cell_thr, (uintptr_t)e->d_sel,
            (uintptr_t)e->d_dst, (uintptr_t)e->d_sel_count, (uintptr_t)e->d_lap_count, (uintptr_t)e->d_st_kp,
            (uintptr_t)e->d_st_desc, (uintptr_t)e->d_geom, (uintptr_t)e->d_cells, (uintptr_t)e->d_xtab,
            (uintptr_t)e->d_ytab, (uintptr_t)e->d_tiletab, (uintptr_t)e->d_pairtab, (uintptr_t)(e->pyr_pair && e->pair_ok),
            (uintptr_t)e->qt_lds, (uintptr_t)e->d_stamps};
        if (!e->g1_exec || key != e->g1_key) {
            if (e->g1_exec) { (void)hipGraphExecDestroy(e->g1_exec); e->g1_exec = nullptr; }
            if (e->g1_graph) { (void)hipGraphDestroy(e->g1_graph); e->g1_graph = nullptr; }
            bool ok = hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
            if (ok) {
                const int r = enqueue();
                ok = hipStreamEndCapture(e->stream, &e->g1_graph) == hipSuccess && r == ORB_OK && e->g1_graph &&
                     hipGraphInstantiate(&e->g1_exec, e->g1_graph, nullptr, nullptr, 0) == hipSuccess;
            }
            if (!ok) {  // launch directly
                (void)hipGetLastError();
                if (e->g1_graph) { (void)hipGraphDestroy(e->g1_graph); e->g1_graph = nullptr; }
                e->g1_exec = nullptr;
                use_graph = false;
            } else {
                e->g1_key = key;
            }
        }
    }
    if (use_graph) {
        if (hipGraphLaunch(e->g1_exec, e->stream) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "graph launch failed");
        e->batches++;
        e->last_n = 1;
    } else if ((rc = enqueue()) != ORB_OK) {
        return rc;
    }
    if (hipStreamSynchronize(e->stream) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "download failed");
    int32_t cnt[2];
    int status;
    memcpy(cnt, e->h_out + cnt_off, 8);
    memcpy(&status, e->h_out + st_off, 4);
    if (status != 0) return orbgpu_fail(ORB_ERR_INTERNAL, "quad-tree capacity guard tripped");
    if (n_kps) *n_kps = cnt[0];
    if (cnt[1] < 0) return orbgpu_fail(ORB_ERR_CAPACITY, "output capacity too small");
    if (cnt[0] > 0) {
        memcpy(kps, e->h_out, sizeof(orb_keypoint_t) * cnt[0]);
        memcpy(desc, e->h_out + desc_off, 32 * (size_t)cnt[0]);
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
    // the ring beyond the device's 3-pixel border: cv::borderInterpolate(p, len, BORDER_REFLECT_101)
    auto reflect101 = [](int p, int len) {
        if (len == 1) return 0;
        while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - 2 - p;
        return p;
    };
    const int E = orbgpu::kEdge, w = L.w, hh = L.h;
    for (int y = 0; y < hh; ++y) {
        uint8_t* row = host_padded + (size_t)(y + E) * L.pw + E;
        for (int x = -E; x < 0; ++x) row[x] = row[reflect101(x, w)];
        for (int x = w; x < w + E; ++x) row[x] = row[reflect101(x, w)];
    }
    for (int y = -E; y < hh + E; ++y)
        if (y < 0 || y >= hh)
            memcpy(host_padded + (size_t)(y + E) * L.pw, host_padded + (size_t)(reflect101(y, hh) + E) * L.pw, (size_t)L.pw);
    return ORB_OK;
}

// ---- debug: the quad-tree's compareNodes sort on given records (returns 1 if the register version ran,
// 0 if qt_sort did, < 0 on error); order[i] = index of the i-th record in sorted order
int orb_debug_node_sort(const int* counts, const int* ulx, int n, int mode, int* order) {
    if (n < 0 || n > 1024 || (n && (!counts || !ulx || !order))) return orbgpu_fail(ORB_ERR_ARG, "bad node sort args");
    for (int i = 0; i < n; ++i)
        if (counts[i] < 0 || counts[i] >= (1 << 20) || ulx[i] < 0 || ulx[i] >= 4096)
            return orbgpu_fail(ORB_ERR_ARG, "node record out of range");
    int* d = nullptr;
    const size_t words = 3 * (size_t)n + 1;
    if (hipMalloc(&d, 4 * words) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
    int used = -1;
    const int lds = (int)((qt2_meta_bytes(n + 64) + 15) & ~(size_t)15);
    bool ok = hipFuncSetAttribute((const void*)k_debug_node_sort, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess &&
              (n == 0 || (hipMemcpy(d, counts, 4 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess &&
                          hipMemcpy(d + n, ulx, 4 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess));
    if (ok) {
        hipLaunchKernelGGL(k_debug_node_sort, dim3(1), dim3(64), lds, 0, d, d + n, n, mode, d + 2 * n, d + 3 * n);
        ok = hipDeviceSynchronize() == hipSuccess &&
             (n == 0 || hipMemcpy(order, d + 2 * n, 4 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess) &&
             hipMemcpy(&used, d + 3 * n, 4, hipMemcpyDeviceToHost) == hipSuccess;
    }
    (void)hipFree(d);
    if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "node sort failed");
    return used;
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
    const uint8_t* view = e->d_pyr + (size_t)frame * e->geo.k.pyr_frame_bytes + L.plane_off +
                          (size_t)orbgpu::kEdge * L.pitch + orbgpu::kEdge;
    uint8_t* d = nullptr;
    if (hipDeviceSynchronize() != hipSuccess || hipMalloc(&d, (size_t)L.w * L.h) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "debug blur allocation failed");
    hipLaunchKernelGGL(k_debug_blur, dim3((L.w + 255) / 256, L.h), dim3(256), 0, 0, view, L.pitch, L.w, L.h, d);
    const bool ok = hipMemcpy(host_view, d, (size_t)L.w * L.h, hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d);
    return ok ? ORB_OK : orbgpu_fail(ORB_ERR_DEVICE, "download failed");
}

// Per-stage timing (HIP events on the launch stream).  enable != 0 starts recording (and clears
// what was recorded); orb_extractor_stage_ms waits for the recorded launches and returns the summed
// milliseconds of [pyramid, fast, quadtree, place, describe] and the number of launches / frames.
int orb_extractor_profile(orb_extractor_t h, int enable) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e) return ORB_ERR_ARG;
    e->profile = (enable == 2 || enable == 3) ? enable : (enable != 0 ? 1 : 0);
    e->ev_used = 0;
    e->pyr_ev_used = 0;
    if (enable == 3) {  // event pairs for 256 batches of every launch, created before the timed region
        const size_t want = (size_t)2 * (orbgpu::kMaxLevels + 8) * 256;
        while (e->pyr_events.size() < want) {
            hipEvent_t x;
            if (hipEventCreate(&x) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipEventCreate failed");
            e->pyr_events.push_back(x);
        }
        e->pyr_ev_kernel.assign(want / 2, -1);
    }
    e->frames_profiled = 0;
    e->batches = 0;
    return ORB_OK;
}

int orb_extractor_stage_ms(orb_extractor_t h, float* ms, int* launches, long long* frames) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !ms) return ORB_ERR_ARG;
    for (int s = 0; s < orbgpu::kStages; ++s) ms[s] = 0.f;
    for (int i = 0; i < e->ev_used; ++i) {
        hipEvent_t* ev = &e->events[(size_t)i * (orbgpu::kStages + 1)];
        const int last = e->profile == 2 ? 1 : orbgpu::kStages;
        if (hipEventSynchronize(ev[last]) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "event sync");
        for (int s = 0; s < last; ++s) {
            float t = 0.f;
            hipEventElapsedTime(&t, ev[s], ev[s + 1]);
            ms[s] += t;
        }
    }
    if (launches) *launches = (int)e->batches;  // batch calls (each may be several sub-batch launches)
    if (frames) *frames = e->frames_profiled;
    return ORB_OK;
}

// Profile mode 3: summed milliseconds of the recorded pyramid level launches (event pair around each
// k_pyramid_level launch) and their number
int orb_extractor_pyramid_launch_ms(orb_extractor_t h, float* ms, int* launches) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !ms) return ORB_ERR_ARG;
    *ms = 0.f;
    if (launches) *launches = 0;
    double tot = 0;
    int cnt = 0;
    for (size_t i = 0; i + 1 < e->pyr_ev_used; i += 2) {
        if (e->pyr_ev_kernel[i / 2] != kLaunchPyramid) continue;
        float t = 0.f;
        if (hipEventSynchronize(e->pyr_events[i + 1]) != hipSuccess ||
            hipEventElapsedTime(&t, e->pyr_events[i], e->pyr_events[i + 1]) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "pyramid launch events failed");
        tot += t;
        ++cnt;
    }
    *ms = (float)tot;
    if (launches) *launches = cnt;
    return ORB_OK;
}

// Profile mode 3: each recorded launch of one stage kernel (0 k_pyramid_level, 1 k_fast_cells,
// 2 k_quadtree_kp, 3 k_describe), in launch order: its duration from the dispatch's own event pair
// (hipExtLaunchKernel: the dispatch's begin / end timestamps, as rocprofv3's kernel trace).
int orb_extractor_launch_durations(orb_extractor_t h, int kernel, float* ms, int cap, int* n) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !n || (cap > 0 && !ms)) return ORB_ERR_ARG;
    int cnt = 0;
    for (size_t i = 0; i + 1 < e->pyr_ev_used; i += 2) {
        if (e->pyr_ev_kernel[i / 2] != kernel) continue;
        float t = 0.f;
        if (hipEventSynchronize(e->pyr_events[i + 1]) != hipSuccess ||
            hipEventElapsedTime(&t, e->pyr_events[i], e->pyr_events[i + 1]) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "launch events failed");
        if (cnt < cap) ms[cnt] = t;
        ++cnt;
    }
    *n = cnt;
    return ORB_OK;
}

int orb_debug_qt_stamps(orb_extractor_t h, unsigned long long* out, int n) {
    Extractor* e = reinterpret_cast<Extractor*>(h);
    if (!e || !e->d_stamps) return ORB_ERR_ARG;
    hipDeviceSynchronize();
    const int m = std::min<int>(n, (int)e->stamps_cap);
    hipMemcpy(out, e->d_stamps, sizeof(unsigned long long) * m, hipMemcpyDeviceToHost);
    return m;
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
