// Host-side geometry of one ORB extraction problem (frame size + ORBextractor parameters):
// scale tables, pyramid level sizes and plane offsets in HBM, the FAST cell grid, the INTER_LINEAR
// coefficient tables and the quad-tree roots.  Everything here is derived exactly as the reference
// derives it (file:line cited per item) so the kernels only have to index tables.
#pragma once
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <vector>

namespace orbgpu {

constexpr int kMaxLevels = 12;
constexpr int kEdge = 19;       // EDGE_THRESHOLD, src/ORBextractor.cc:78
constexpr int kHalfPatch = 15;  // HALF_PATCH_SIZE, src/ORBextractor.cc:77
constexpr int kPatchSize = 31;  // PATCH_SIZE, src/ORBextractor.cc:76
constexpr int kCellW = 35;      // W, src/ORBextractor.cc:1069
constexpr int kMaxRoots = 8;
constexpr int kStages = 5;      // timed stages of one extraction launch

// per level, passed to kernels by value (inside KernelGeom)
struct LevelGeom {
    int w, h;             // level image (the reference's mvImagePyramid[l] view)
    int pw, ph, pitch;    // padded plane ((w+38) x (h+38)) and its row pitch in bytes
    long long plane_off;  // byte offset of the padded plane inside one frame's pyramid block
    int minB, maxBX, maxBY;          // FAST/quad-tree bounds: 16, w-16, h-16 (src:1076-1079)
    int cell_begin, cell_count;      // this level's cells in the cell table
    int cand_off, cand_cap;          // candidate slots of this level inside one frame's block
    int nfeat;                       // mnFeaturesPerLevel[l]
    int sel_off, sel_cap;            // selected keypoints of this level inside one frame's block
    int n_roots;                     // DistributeOctTree nIni (src:718)
    float root_w;                    // hX (src:721)
    float scale;                     // mvScaleFactor[l]
    int patch_size;                  // (int)(PATCH_SIZE * scale) (src:1184)
    int xtab_off, ytab_off;          // INTER_LINEAR tables (level >= 1)
    int simd_end;                    // columns handled by the 128-bit vertical path (see resize)
};

struct KernelGeom {
    int nlevels;
    int ini_th, min_th;
    int ncells;
    long long pyr_frame_bytes;   // one frame's padded pyramid (also the blurred pyramid's layout)
    int cand_frame_cap;          // candidate slots per frame
    int sel_frame_cap;           // selected-keypoint slots per frame
    int umax[kHalfPatch + 1];
    int debug_flags;             // timing experiments only (ORBGPU_DEBUG_FLAGS); 0 in production
    LevelGeom lv[kMaxLevels];
};

struct CellDesc {      // one FAST cell window (src:1098-1129), row-major within its level
    int16_t level, ini_x, ini_y, win_w, win_h;  // window in level coordinates and its size
    int16_t off_x, off_y;                        // j*wCell, i*hCell: candidate offset (src:1159-1160)
    int16_t pad;
    int32_t slot, cap;                           // candidate slot offset / capacity inside the level
};
static_assert(sizeof(CellDesc) == 24, "CellDesc layout");

struct Params {
    int nfeatures = 0, nlevels = 0, ini_th = 0, min_th = 0;
    double scale_factor = 0;  // double member set from a float (include/ORBextractor.h:96)
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> per_level, umax;
};

inline int round_half_even(float v) { return (int)std::lrintf(v); }  // cvRound
inline int floor_f(float v) { int i = (int)v; return i - (i > v); }  // cvFloor
inline int ceil_f(float v) { int i = (int)v; return i + (i < v); }   // cvCeil

// ORBextractor::ORBextractor, src/ORBextractor.cc:474-570
inline Params make_params(int nfeatures, float scale_factor, int nlevels, int ini_th, int min_th) {
    Params p;
    p.nfeatures = nfeatures; p.nlevels = nlevels; p.ini_th = ini_th; p.min_th = min_th;
    p.scale_factor = scale_factor;
    p.scale.assign(nlevels, 1.0f);
    p.sigma2.assign(nlevels, 1.0f);
    for (int i = 1; i < nlevels; ++i) {
        p.scale[i] = (float)(p.scale[i - 1] * p.scale_factor);
        p.sigma2[i] = p.scale[i] * p.scale[i];
    }
    p.inv_scale.resize(nlevels);
    p.inv_sigma2.resize(nlevels);
    for (int i = 0; i < nlevels; ++i) {
        p.inv_scale[i] = 1.0f / p.scale[i];
        p.inv_sigma2[i] = 1.0f / p.sigma2[i];
    }
    const float factor = (float)(1.0f / p.scale_factor);
    float per_scale = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    p.per_level.assign(nlevels, 0);
    for (int l = 0; l < nlevels - 1; ++l) {
        p.per_level[l] = round_half_even(per_scale);
        sum += p.per_level[l];
        per_scale *= factor;
    }
    p.per_level[nlevels - 1] = std::max(nfeatures - sum, 0);
    p.umax.assign(kHalfPatch + 1, 0);
    const int vmax = floor_f(kHalfPatch * std::sqrt(2.f) / 2 + 1);
    const int vmin = ceil_f(kHalfPatch * std::sqrt(2.f) / 2);
    const double r2 = kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) p.umax[v] = (int)std::lrint(std::sqrt(r2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {  // keep the disc symmetric
        while (p.umax[v0] == p.umax[v0 + 1]) ++v0;
        p.umax[v] = v0;
        ++v0;
    }
    return p;
}

struct Geometry {
    KernelGeom k{};
    std::vector<CellDesc> cells;
    std::vector<int32_t> xtab;  // per level >= 1, per column: sx, (a0 | a1 << 16)
    std::vector<int32_t> ytab;  // per level >= 1, per row: r0, r1, b0, b1
    int max_win = 0;            // largest FAST window (bytes)
    int max_win_lv[kMaxLevels] = {};  // the same per level (a launch's LDS is sized for its levels)
    int max_det_lv[kMaxLevels] = {};  // largest detectable region of a window per level (candidate list entries)
    int max_sc_lv[kMaxLevels] = {};   // largest FAST score map per level (bytes, k_fast_cells' layout)
    int max_level_cands = 0;    // largest per-level candidate capacity
    int max_sel = 0;            // largest per-level selected capacity
};

inline int sat16(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }

// cv::resize INTER_LINEAR coefficient tables for src (sw x sh) -> dst (dw x dh), OpenCV 4.x resize.cpp
inline void resize_tables(int sw, int sh, int dw, int dh, std::vector<int32_t>& xt, std::vector<int32_t>& yt) {
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = floor_f(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        const int a0 = sat16(round_half_even((1.f - fx) * 2048));
        const int a1 = sat16(round_half_even(fx * 2048));
        xt.push_back(sx);
        xt.push_back((a0 & 0xffff) | (a1 << 16));
    }
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = floor_f(fy);
        fy -= sy;
        const int b0 = sat16(round_half_even((1.f - fy) * 2048));
        const int b1 = sat16(round_half_even(fy * 2048));
        const int r0 = std::min(std::max(sy, 0), sh - 1), r1 = std::min(std::max(sy + 1, 0), sh - 1);
        yt.push_back(r0); yt.push_back(r1); yt.push_back(b0); yt.push_back(b1);
    }
}

inline int align_up(long long v, int a) { return (int)((v + a - 1) / a * a); }

// Returns false if the frame is too small for the reference's cell grid (nCols or nRows == 0).
inline bool build_geometry(const Params& P, int width, int height, Geometry& g) {
    g = Geometry();
    KernelGeom& k = g.k;
    k.nlevels = P.nlevels;
    k.ini_th = std::min(std::max(P.ini_th, 0), 255);
    k.min_th = std::min(std::max(P.min_th, 0), 255);
    k.debug_flags = 0;
    if (const char* d = getenv("ORBGPU_DEBUG_FLAGS")) k.debug_flags = atoi(d);
    for (int v = 0; v <= kHalfPatch; ++v) k.umax[v] = P.umax[v];
    long long plane_off = 0;
    int cand_off = 0, sel_off = 0;
    int prev_w = width, prev_h = height;
    for (int l = 0; l < P.nlevels; ++l) {
        LevelGeom& L = k.lv[l];
        L.w = round_half_even((float)width * P.inv_scale[l]);   // src:1692
        L.h = round_half_even((float)height * P.inv_scale[l]);
        if (L.w < 2 * kEdge || L.h < 2 * kEdge) return false;
        L.pw = L.w + 2 * kEdge;
        L.ph = L.h + 2 * kEdge;
        L.pitch = align_up(L.pw, 128);
        L.plane_off = plane_off;
        plane_off += (long long)L.pitch * L.ph;
        plane_off = (plane_off + 255) / 256 * 256;
        L.scale = P.scale[l];
        L.patch_size = (int)(kPatchSize * P.scale[l]);
        L.nfeat = P.per_level[l];
        // FAST cell grid, src:1076-1129
        L.minB = kEdge - 3;
        L.maxBX = L.w - kEdge + 3;
        L.maxBY = L.h - kEdge + 3;
        const float wid = (float)(L.maxBX - L.minB), hei = (float)(L.maxBY - L.minB);
        const int ncols = (int)(wid / kCellW), nrows = (int)(hei / kCellW);
        if (ncols <= 0 || nrows <= 0) return false;
        const int wcell = (int)std::ceil(wid / ncols), hcell = (int)std::ceil(hei / nrows);
        L.cell_begin = (int)g.cells.size();
        L.cand_off = cand_off;
        int level_cap = 0;
        for (int i = 0; i < nrows; ++i) {
            const float ini_y = (float)(L.minB + i * hcell);
            float max_y = ini_y + hcell + 6;
            if (ini_y >= L.maxBY - 3) continue;
            if (max_y > L.maxBY) max_y = (float)L.maxBY;
            for (int j = 0; j < ncols; ++j) {
                const float ini_x = (float)(L.minB + j * wcell);
                float max_x = ini_x + wcell + 6;
                if (ini_x >= L.maxBX - 6) continue;
                if (max_x > L.maxBX) max_x = (float)L.maxBX;
                CellDesc c{};
                c.level = (int16_t)l;
                c.ini_x = (int16_t)ini_x;
                c.ini_y = (int16_t)ini_y;
                c.win_w = (int16_t)((int)max_x - (int)ini_x);
                c.win_h = (int16_t)((int)max_y - (int)ini_y);
                c.off_x = (int16_t)(j * wcell);
                c.off_y = (int16_t)(i * hcell);
                // strict 3x3 maxima are pairwise non-adjacent: at most ceil(w/2)*ceil(h/2)
                const int dw = std::max(0, c.win_w - 6), dh = std::max(0, c.win_h - 6);
                c.cap = ((dw + 1) / 2) * ((dh + 1) / 2);
                c.slot = level_cap;
                level_cap += c.cap;
                // dword-aligned rows; at least 52 bytes (k_fast_cells uses a fixed 52-byte stride when the window fits)
                const int wbytes = std::max((int)c.win_w + 6, 52) * c.win_h;  // k_fast_cells row stride
                g.max_win = std::max(g.max_win, wbytes);
                g.max_win_lv[l] = std::max(g.max_win_lv[l], wbytes);
                g.max_det_lv[l] = std::max(g.max_det_lv[l], dw * dh);
                if (c.win_w >= 128 || c.win_h >= 512) return false;  // k_fast_cells' (row << 7 | column) entries
                // score map: rows 2 .. win_h-3, columns 2 .. win_w-3, row stride 40 (win_w <= 44) or
                // 48 (the fixed-stride kernel path), else win_w - 4 rounded up to a dword
                const int ss = c.win_w <= 44 ? 40 : std::max(48, (c.win_w - 4 + 3) & ~3);
                g.max_sc_lv[l] = std::max(g.max_sc_lv[l], std::max(0, c.win_h - 4) * ss);
                g.cells.push_back(c);
            }
        }
        L.cell_count = (int)g.cells.size() - L.cell_begin;
        L.cand_cap = level_cap;
        cand_off += level_cap;
        g.max_level_cands = std::max(g.max_level_cands, level_cap);
        // quad-tree roots, src:718-721
        const int spanx = L.maxBX - L.minB, spany = L.maxBY - L.minB;
        L.n_roots = (int)std::round((float)spanx / spany);
        if (L.n_roots <= 0 || L.n_roots > kMaxRoots) return false;
        L.root_w = (float)spanx / L.n_roots;
        // at most max(N + 2, 4 * nIni) nodes survive DistributeOctTree
        L.sel_cap = std::max(L.nfeat + 2, 4 * L.n_roots) + 2;
        L.sel_off = sel_off;
        sel_off += L.sel_cap;
        g.max_sel = std::max(g.max_sel, L.sel_cap);
        // INTER_LINEAR tables from the previous level view, src:1702-1707
        if (l > 0) {
            L.xtab_off = (int)g.xtab.size() / 2;
            L.ytab_off = (int)g.ytab.size() / 4;
            resize_tables(prev_w, prev_h, L.w, L.h, g.xtab, g.ytab);
            int x = 0;
            for (; x <= L.w - 16; x += 16) {}
            for (; x < L.w - 8; x += 8) {}
            L.simd_end = x;
        }
        prev_w = L.w;
        prev_h = L.h;
    }
    k.ncells = (int)g.cells.size();
    k.pyr_frame_bytes = plane_off;
    k.cand_frame_cap = cand_off;
    k.sel_frame_cap = sel_off;
    return true;
}

}  // namespace orbgpu
