// MI355X Hamming matching kernels (ORBmatcher, reference src/ORBmatcher.cc).
//
// DescriptorDistance (src:2384-2404) is popcount(a ^ b) over 256 bits; on gfx950 that is 8 v_xor +
// 8 v_bcnt_u32 (popcount-accumulate) per descriptor pair.  No MFMA: this is bit-count work.
//
// Best / second-best search (the kernel of every ORBmatcher scan and of BFMatcher::knnMatch(k = 2)):
// scanning the train set in index order, a strictly smaller distance replaces the best (ties keep the
// first index, src:1160-1175) and otherwise a smaller one replaces the second.  The result is
//   best = min, idx = the first index attaining it, second = the second smallest of the multiset
// so partial results over consecutive train ranges merge exactly:
//   best = min(b1, b2), idx = b1 <= b2 ? i1 : i2 (range 1 first), second = min(max(b1, b2), s1, s2).
// A train set that fits one block's LDS (<= 1024 descriptors, a frame) is one launch that writes the
// results directly (k_hamming_knn2_frame: 16 queries per block, the train set cut into 64 parts merged
// in order in LDS): a frame-sized call is latency bound, so a second (merge) launch and its partial
// buffer cost more than they buy.  Larger train sets: 64-query tiles (one query per lane) x train
// chunks (enough blocks to fill the chip); the waves of a block scan consecutive parts of the chunk
// (staged in LDS, read as broadcasts) and merge in wave order, and the chunks' partials merge in chunk
// order in a second kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kKnnWaves = 4, kKnnThreads = 64 * kKnnWaves;  // chunked launch
constexpr int kKnnMaxChunk = 1024;  // train descriptors per block (32 KiB of LDS)
constexpr int kKnnMinChunk = 64;
constexpr int kKnnTargetBlocks = 1024;

struct Knn {
    int best, second, idx;
};

__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    int d = __popc(a0.x ^ b0.x);
    d += __popc(a0.y ^ b0.y);
    d += __popc(a0.z ^ b0.z);
    d += __popc(a0.w ^ b0.w);
    d += __popc(a1.x ^ b1.x);
    d += __popc(a1.y ^ b1.y);
    d += __popc(a1.z ^ b1.z);
    d += __popc(a1.w ^ b1.w);
    return d;
}

// a: the earlier train range, b: the later one
__device__ __forceinline__ Knn knn_merge(const Knn& a, const Knn& b) {
    Knn r;
    r.best = min(a.best, b.best);
    r.idx = a.best <= b.best ? a.idx : b.idx;
    r.second = min(max(a.best, b.best), min(a.second, b.second));
    return r;
}

// grid (query tiles, chunks).  nchunk == 1: the block writes the final result; otherwise its partial
// goes to part[(chunk * nq + query)].
template <int kW>
__global__ __launch_bounds__(64 * kW) void k_hamming_knn2(const uint8_t* __restrict__ q, int nq,
                                                              const uint8_t* __restrict__ t, int nt, int chunk,
                                                              Knn* __restrict__ part, int32_t* __restrict__ best_idx,
                                                              int32_t* __restrict__ best_dist,
                                                              int32_t* __restrict__ second_dist) {
    __shared__ uint4 tile[kKnnMaxChunk * 2];
    __shared__ Knn wpart[kW - 1][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qi = blockIdx.x * 64 + lane;
    const int c0 = blockIdx.y * chunk, n = min(chunk, nt - c0);
    for (int i = threadIdx.x; i < 2 * n; i += 64 * kW) tile[i] = reinterpret_cast<const uint4*>(t)[2 * (size_t)c0 + i];
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < nq) {
        a0 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi];
        a1 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi + 1];
    }
    __syncthreads();
    const int sub = (n + kW - 1) / kW, j0 = w * sub, j1 = min(n, j0 + sub);
    Knn r{257, 257, -1};
    for (int j = j0; j < j1; ++j) {
        const int d = hamming256(a0, a1, tile[2 * j], tile[2 * j + 1]);
        if (d < r.best) { r.second = r.best; r.best = d; r.idx = c0 + j; }
        else if (d < r.second) r.second = d;
    }
    if (w > 0) wpart[w - 1][lane] = r;
    __syncthreads();
    if (w != 0 || qi >= nq) return;
#pragma unroll
    for (int k = 0; k < kW - 1; ++k) r = knn_merge(r, wpart[k][lane]);
    if (part) {
        part[(size_t)blockIdx.y * nq + qi] = r;
    } else {
        best_idx[qi] = r.idx;
        best_dist[qi] = r.best;
        second_dist[qi] = r.second;
    }
}

// Frame-sized train sets (<= kKnnMaxChunk): 16 queries per 1024-thread block and the train set cut
// into 64 consecutive parts, so each lane scans ~16 rows instead of a whole chunk.  Lane l of wave w
// takes query 16 blockIdx.x + (l & 15) and part 4 w + (l >> 4).  The 64 partials of a query merge in
// part order by an adjacent-pair tree in LDS (knn_merge is associative over consecutive ranges).
constexpr int kKnnQ = 16, kKnnParts = 64;
__global__ __launch_bounds__(1024) void k_hamming_knn2_frame(const uint8_t* __restrict__ q, int nq,
                                                             const uint8_t* __restrict__ t, int nt,
                                                             int32_t* __restrict__ best_idx,
                                                             int32_t* __restrict__ best_dist,
                                                             int32_t* __restrict__ second_dist) {
    __shared__ uint4 tile[kKnnMaxChunk * 2];
    __shared__ Knn red[kKnnParts][kKnnQ];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ql = lane & (kKnnQ - 1), part = 4 * w + (lane >> 4);
    const int qi = blockIdx.x * kKnnQ + ql;
    for (int i = threadIdx.x; i < 2 * nt; i += 1024) tile[i] = reinterpret_cast<const uint4*>(t)[i];
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < nq) {
        a0 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi];
        a1 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi + 1];
    }
    __syncthreads();
    const int sub = (nt + kKnnParts - 1) / kKnnParts, j0 = part * sub, j1 = min(nt, j0 + sub);
    Knn r{257, 257, -1};
    for (int j = j0; j < j1; ++j) {
        const int d = hamming256(a0, a1, tile[2 * j], tile[2 * j + 1]);
        if (d < r.best) { r.second = r.best; r.best = d; r.idx = j; }
        else if (d < r.second) r.second = d;
    }
    red[part][ql] = r;
    __syncthreads();
#pragma unroll
    for (int s = 1; s < kKnnParts; s <<= 1) {
        if ((int)threadIdx.x < (kKnnParts / (2 * s)) * kKnnQ) {
            const int p = (threadIdx.x / kKnnQ) * 2 * s, qq = threadIdx.x & (kKnnQ - 1);
            red[p][qq] = knn_merge(red[p][qq], red[p + s][qq]);
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < kKnnQ) {
        const int qo = blockIdx.x * kKnnQ + threadIdx.x;
        if (qo < nq) {
            const Knn f = red[0][threadIdx.x];
            best_idx[qo] = f.idx;
            best_dist[qo] = f.best;
            second_dist[qo] = f.second;
        }
    }
}

__global__ __launch_bounds__(256) void k_hamming_knn2_merge(int nq, int nchunk, const Knn* __restrict__ part,
                                                            int32_t* __restrict__ best_idx, int32_t* __restrict__ best_dist,
                                                            int32_t* __restrict__ second_dist) {
    const int qi = blockIdx.x * 256 + threadIdx.x;
    if (qi >= nq) return;
    Knn r = part[qi];
    for (int c = 1; c < nchunk; ++c) r = knn_merge(r, part[(size_t)c * nq + qi]);
    best_idx[qi] = r.idx;
    best_dist[qi] = r.best;
    second_dist[qi] = r.second;
}

// Many (query frame, train frame) pairs of one batch of feature blocks in one launch (cross-frame
// matching after the C4 all-gather): block (x, p) takes queries 16x .. 16x + 15 of pair p's query
// frame against the whole train frame staged in LDS (up to `cap` descriptors, dynamic shared
// memory), the same 64-part scan and in-order merge as k_hamming_knn2_frame.  Frame sizes come from
// the device counts (no host round trip); rows at or beyond the query frame's count get (-1, 257, 257).
__global__ __launch_bounds__(1024) void k_hamming_knn2_frames(const uint8_t* __restrict__ desc,
                                                              const int32_t* __restrict__ counts, int cstride, int cap,
                                                              const int32_t* __restrict__ pairs,
                                                              int32_t* __restrict__ best_idx,
                                                              int32_t* __restrict__ best_dist,
                                                              int32_t* __restrict__ second_dist) {
    extern __shared__ uint4 ftile[];
    __shared__ Knn red[kKnnParts][kKnnQ];
    const int p = blockIdx.y;
    const int qf = pairs[2 * p], tf = pairs[2 * p + 1];
    const int nq = min(max(counts[(size_t)qf * cstride], 0), cap), nt = min(max(counts[(size_t)tf * cstride], 0), cap);
    const size_t o = (size_t)p * cap;
    const int q0 = blockIdx.x * kKnnQ;
    if (q0 >= nq) {  // (block-uniform) nothing to match here: the rows get "no match"
        const int qo = q0 + (int)threadIdx.x;
        if ((int)threadIdx.x < kKnnQ && qo < cap) {
            best_idx[o + qo] = -1;
            best_dist[o + qo] = 257;
            second_dist[o + qo] = 257;
        }
        return;
    }
    const uint4* t = reinterpret_cast<const uint4*>(desc + (size_t)tf * cap * 32);
    const uint4* q = reinterpret_cast<const uint4*>(desc + (size_t)qf * cap * 32);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ql = lane & (kKnnQ - 1), part = 4 * w + (lane >> 4);
    const int qi = q0 + ql;
    for (int i = threadIdx.x; i < 2 * nt; i += 1024) ftile[i] = t[i];
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < nq) {
        a0 = q[2 * (size_t)qi];
        a1 = q[2 * (size_t)qi + 1];
    }
    __syncthreads();
    const int sub = (nt + kKnnParts - 1) / kKnnParts, j0 = part * sub, j1 = min(nt, j0 + sub);
    Knn r{257, 257, -1};
    for (int j = j0; j < j1; ++j) {
        const int d = hamming256(a0, a1, ftile[2 * j], ftile[2 * j + 1]);
        if (d < r.best) { r.second = r.best; r.best = d; r.idx = j; }
        else if (d < r.second) r.second = d;
    }
    red[part][ql] = r;
    __syncthreads();
#pragma unroll
    for (int s = 1; s < kKnnParts; s <<= 1) {
        if ((int)threadIdx.x < (kKnnParts / (2 * s)) * kKnnQ) {
            const int pp = (threadIdx.x / kKnnQ) * 2 * s, qq = threadIdx.x & (kKnnQ - 1);
            red[pp][qq] = knn_merge(red[pp][qq], red[pp + s][qq]);
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < kKnnQ) {
        const int qo = q0 + threadIdx.x;
        if (qo < cap) {
            const Knn f = qo < nq ? red[0][threadIdx.x] : Knn{257, 257, -1};
            best_idx[o + qo] = f.idx;
            best_dist[o + qo] = f.best;
            second_dist[o + qo] = f.second;
        }
    }
}

constexpr int kKnnFramesMaxCap = 2048;  // 64 KiB of train descriptors in LDS

}  // namespace

extern "C" int orb_hamming_knn2_device(const uint8_t* d_query, int n_query, const uint8_t* d_train, int n_train,
                                       int32_t* d_best_idx, int32_t* d_best_dist, int32_t* d_second_dist,
                                       void* stream) {
    if (n_query < 0 || n_train < 0 || (n_query > 0 && (!d_query || !d_best_idx || !d_best_dist || !d_second_dist)) ||
        (n_train > 0 && !d_train))
        return orbgpu_fail(ORB_ERR_ARG, "bad matcher arguments");
    if (n_query == 0) return ORB_OK;
    if ((reinterpret_cast<uintptr_t>(d_query) | reinterpret_cast<uintptr_t>(d_train)) & 15)
        return orbgpu_fail(ORB_ERR_ARG, "descriptor arrays must be 16-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    const int qtiles = (n_query + 63) / 64;
    if (n_train <= kKnnMaxChunk) {  // one chunk: a single launch, results written by the blocks
        hipLaunchKernelGGL(k_hamming_knn2_frame, dim3((n_query + kKnnQ - 1) / kKnnQ), dim3(1024), 0, s, d_query, n_query,
                           d_train, n_train, d_best_idx, d_best_dist, d_second_dist);
        if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hamming launch failed");
        return ORB_OK;
    }
    // chunks: enough blocks to fill the chip, at least kKnnMinChunk descriptors per block, at most
    // what one block stages in LDS
    int nchunk = std::max(1, std::min((kKnnTargetBlocks + qtiles - 1) / qtiles, (n_train + kKnnMinChunk - 1) / kKnnMinChunk));
    int chunk = n_train > 0 ? (n_train + nchunk - 1) / nchunk : 1;
    if (chunk > kKnnMaxChunk) {
        chunk = kKnnMaxChunk;
        nchunk = (n_train + chunk - 1) / chunk;
    }
    nchunk = n_train > 0 ? (n_train + chunk - 1) / chunk : 1;
    if (nchunk > 65535) return orbgpu_fail(ORB_ERR_ARG, "train set too large (more than 65535 x 1024 descriptors)");
    Knn* part = nullptr;
    if (nchunk > 1 &&
        hipMallocAsync(reinterpret_cast<void**>(&part), sizeof(Knn) * (size_t)nchunk * n_query, s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "knn2 partial buffer");
    hipLaunchKernelGGL(k_hamming_knn2<kKnnWaves>, dim3(qtiles, nchunk), dim3(kKnnThreads), 0, s, d_query, n_query, d_train, n_train,
                       chunk, part, d_best_idx, d_best_dist, d_second_dist);
    if (part) {
        hipLaunchKernelGGL(k_hamming_knn2_merge, dim3((n_query + 255) / 256), dim3(256), 0, s, n_query, nchunk, part,
                           d_best_idx, d_best_dist, d_second_dist);
        if (hipFreeAsync(part, s) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "knn2 partial buffer free");
    }
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hamming launch failed");
    return ORB_OK;
}

extern "C" int orb_hamming_knn2_frames_device(const uint8_t* d_desc, const int32_t* d_counts, int count_stride,
                                              int cap, const int32_t* d_pairs, int n_pairs, int32_t* d_best_idx,
                                              int32_t* d_best_dist, int32_t* d_second_dist, void* stream) {
    if (n_pairs < 0 || cap < 1 || cap > kKnnFramesMaxCap || count_stride < 1 ||
        (n_pairs > 0 && (!d_desc || !d_counts || !d_pairs || !d_best_idx || !d_best_dist || !d_second_dist)))
        return orbgpu_fail(ORB_ERR_ARG, "bad frame-pair matcher arguments");
    if (n_pairs == 0) return ORB_OK;
    if (n_pairs > 65535) return orbgpu_fail(ORB_ERR_ARG, "more than 65535 frame pairs in one call");
    if (reinterpret_cast<uintptr_t>(d_desc) & 15) return orbgpu_fail(ORB_ERR_ARG, "descriptor blocks must be 16-byte aligned");
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_hamming_knn2_frames, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kKnnFramesMaxCap * 32);
        (void)hipGetLastError();
        attr = true;
    }
    hipLaunchKernelGGL(k_hamming_knn2_frames, dim3((cap + kKnnQ - 1) / kKnnQ, n_pairs), dim3(1024), (size_t)cap * 32,
                       (hipStream_t)stream, d_desc, d_counts, count_stride, cap, d_pairs, d_best_idx, d_best_dist,
                       d_second_dist);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "frame-pair hamming launch failed");
    return ORB_OK;
}

// ---- MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:438-529), batched over map points ----
// Per point, N descriptors (its observations' rows).  The reference builds the N x N distance matrix
// (DescriptorDistance, diagonal 0), takes for every row i the element at index floor(0.5 (N - 1)) of
// the sorted row -- the median, self distance included -- and keeps the first row with the smallest
// median.  One wave per point: lane i computes row i's distances on the fly into a lane-private
// 257-bin u16 histogram in LDS (hist[bin][lane]), then walks the histogram to the
// median; the wave reduces (median, i) lexicographically (first index on ties).  Rows beyond 64 are
// taken 64 at a time.  That kernel serves only points of more than 64 observations: the usual point
// (a few to a few dozen observations) goes to k_distinctive_wave, which needs no LDS at all.
namespace {
constexpr int kDdBins = 257;
constexpr int kDdWaveMax = 64;  // k_distinctive_wave: observations per point

// Points of at most 64 observations.  Lane j holds descriptor j.  For each row i, in order, row i's
// descriptor is broadcast (v_readlane), every lane computes d_ij, and the row's k-th smallest distance
// is found by a 9-step radix select over wave ballots (d <= 256): at each bit, the candidates with a 0
// there number nz; k < nz keeps them, otherwise k -= nz and the prefix takes a 1.  The first row with
// the smallest median wins (strict <, rows in order), as src/MapPoint.cc:509-517 does.
__global__ __launch_bounds__(64) void k_distinctive_wave(const uint4* __restrict__ desc, const int32_t* __restrict__ off,
                                                         int n_points, int32_t* __restrict__ best,
                                                         uint4* __restrict__ out) {
    const int p = blockIdx.x, lane = threadIdx.x;
    const int o = off[p], N = off[p + 1] - o;
    if (N <= 0) {
        if (lane == 0) best[p] = -1;
        return;
    }
    if (N > kDdWaveMax) return;  // k_distinctive
    const int k = (int)(0.5 * (double)(N - 1));  // vDists[0.5*(N-1)]: the size_t index truncates
    const bool act = lane < N;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (act) {
        a0 = desc[2 * (size_t)(o + lane)];
        a1 = desc[2 * (size_t)(o + lane) + 1];
    }
    const unsigned long long live = __ballot(act);
    int bmed = 1 << 30, bi = 0;
    for (int i = 0; i < N; ++i) {
        const auto rl = [i](unsigned v) { return (unsigned)__builtin_amdgcn_readlane((int)v, i); };
        const uint4 r0 = make_uint4(rl(a0.x), rl(a0.y), rl(a0.z), rl(a0.w));
        const uint4 r1 = make_uint4(rl(a1.x), rl(a1.y), rl(a1.z), rl(a1.w));
        const int d = hamming256(a0, a1, r0, r1);
        int kk = k, med = 0;
        unsigned long long cand = live;
#pragma unroll
        for (int bit = 8; bit >= 0; --bit) {
            const unsigned long long zeros = cand & __ballot(((d >> bit) & 1) == 0);
            const int nz = __popcll(zeros);
            if (kk < nz) {
                cand = zeros;
            } else {
                kk -= nz;
                cand &= ~zeros;
                med |= 1 << bit;
            }
        }
        if (med < bmed) {
            bmed = med;
            bi = i;
        }
    }
    if (lane == 0) best[p] = bi;
    if (lane < 2) out[2 * (size_t)p + lane] = desc[2 * (size_t)(o + bi) + lane];
}

__global__ __launch_bounds__(64) void k_distinctive(const uint4* __restrict__ desc, const int32_t* __restrict__ off,
                                                    int n_points, int32_t* __restrict__ best,
                                                    uint4* __restrict__ out) {
    __shared__ uint16_t hist[kDdBins * 64];
    const int lane = threadIdx.x;
    // grid-stride over the points (a bounded grid: most points have <= 64 rows and are skipped here)
    for (int p = blockIdx.x; p < n_points; p += gridDim.x) {
    const int o = off[p], N = off[p + 1] - o;
    if (N <= kDdWaveMax) continue;  // k_distinctive_wave (empty points included)
    const int k = (int)(0.5 * (double)(N - 1));  // vDists[0.5*(N-1)]: the size_t index truncates
    unsigned long long bestkey = ~0ull;
    for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        for (int b = 0; b < kDdBins; ++b) hist[b * 64 + lane] = 0;
        if (i < N) {
            const uint4 a0 = desc[2 * (size_t)(o + i)], a1 = desc[2 * (size_t)(o + i) + 1];
            for (int j = 0; j < N; ++j) {  // descriptor j: the same address in every lane (one fetch)
                const int d = hamming256(a0, a1, desc[2 * (size_t)(o + j)], desc[2 * (size_t)(o + j) + 1]);
                hist[d * 64 + lane] = (uint16_t)(hist[d * 64 + lane] + 1);
            }
            int acc = 0, med = 0;
            for (int b = 0; b < kDdBins; ++b) {  // the k-th smallest (0-based) of the row
                acc += (int)hist[b * 64 + lane];
                if (acc > k) { med = b; break; }
            }
            const unsigned long long key = ((unsigned long long)med << 32) | (unsigned)i;
            bestkey = key < bestkey ? key : bestkey;
        }
    }
    for (int s = 32; s > 0; s >>= 1) {
        const unsigned long long v = __shfl_xor(bestkey, s, 64);
        bestkey = v < bestkey ? v : bestkey;
    }
    const int bi = (int)(bestkey & 0xffffffffu);
    if (lane == 0) best[p] = bi;
    if (lane < 2) out[2 * (size_t)p + lane] = desc[2 * (size_t)(o + bi) + lane];
    __syncthreads();  // hist is reused by the next point
    }
}
constexpr int kDdBigGrid = 512;  // k_distinctive blocks (grid-stride over the points)
}  // namespace

// Defined in orb_triangulation.hip: the matcher handle's staging buffers.
int orbgpu_matcher_reserve(orb_matcher_t m, size_t bytes, char** d_buf, char** h_buf, hipStream_t* stream,
                           int* check_ori);

extern "C" int orb_compute_distinctive_descriptors_device(const uint8_t* d_desc, const int32_t* d_offsets, int n_points,
                                                          int32_t* d_best, uint8_t* d_out, void* stream) {
    if (n_points < 0 || (n_points > 0 && (!d_desc || !d_offsets || !d_best || !d_out)))
        return orbgpu_fail(ORB_ERR_ARG, "bad ComputeDistinctiveDescriptors arguments");
    if (n_points == 0) return ORB_OK;
    if ((reinterpret_cast<uintptr_t>(d_desc) | reinterpret_cast<uintptr_t>(d_out)) & 15)
        return orbgpu_fail(ORB_ERR_ARG, "descriptor arrays must be 16-byte aligned");
    hipLaunchKernelGGL(k_distinctive_wave, dim3(n_points), dim3(64), 0, (hipStream_t)stream, (const uint4*)d_desc,
                       d_offsets, n_points, d_best, (uint4*)d_out);
    // (points of more than 64 rows; the caller keeps every point below 65536 rows, the u16 histogram's range)
    hipLaunchKernelGGL(k_distinctive, dim3(std::min(n_points, kDdBigGrid)), dim3(64), 0, (hipStream_t)stream,
                       (const uint4*)d_desc, d_offsets, n_points, d_best, (uint4*)d_out);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "distinctive descriptors launch failed");
    return ORB_OK;
}

extern "C" int orb_compute_distinctive_descriptors(orb_matcher_t m, const uint8_t* desc, const int32_t* offsets,
                                                   int n_points, int32_t* best, uint8_t* out) {
    if (!m || n_points < 0 || (n_points > 0 && (!offsets || !best || !out)))
        return orbgpu_fail(ORB_ERR_ARG, "bad ComputeDistinctiveDescriptors arguments");
    if (n_points == 0) return ORB_OK;
    if (offsets[0] != 0) return orbgpu_fail(ORB_ERR_ARG, "offsets[0] must be 0");
    for (int p = 0; p < n_points; ++p) {
        if (offsets[p + 1] < offsets[p]) return orbgpu_fail(ORB_ERR_ARG, "offsets must be non-decreasing");
        if (offsets[p + 1] - offsets[p] >= 65536) return orbgpu_fail(ORB_ERR_ARG, "a point has 65536 or more descriptors");
    }
    const size_t nd = (size_t)offsets[n_points];
    if (nd && !desc) return orbgpu_fail(ORB_ERR_ARG, "null descriptors");
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_d = 0, o_off = al(nd * 32), o_best = o_off + al((size_t)(n_points + 1) * 4),
                 o_out = o_best + al((size_t)n_points * 4), total = o_out + al((size_t)n_points * 32);
    char *d = nullptr, *h = nullptr;
    hipStream_t s = nullptr;
    int check_ori = 0;
    if (int rc = orbgpu_matcher_reserve(m, total, &d, &h, &s, &check_ori)) return rc;
    if (nd) memcpy(h + o_d, desc, nd * 32);
    memcpy(h + o_off, offsets, (size_t)(n_points + 1) * 4);
    bool ok = hipMemcpyAsync(d, h, o_best, hipMemcpyHostToDevice, s) == hipSuccess;
    int max_n = 0;
    for (int p = 0; p < n_points; ++p) max_n = std::max(max_n, offsets[p + 1] - offsets[p]);
    if (ok) hipLaunchKernelGGL(k_distinctive_wave, dim3(n_points), dim3(64), 0, s, (const uint4*)(d + o_d),
                               (const int32_t*)(d + o_off), n_points, (int32_t*)(d + o_best), (uint4*)(d + o_out));
    if (ok && max_n > kDdWaveMax)  // points of more than 64 observations
        hipLaunchKernelGGL(k_distinctive, dim3(std::min(n_points, kDdBigGrid)), dim3(64), 0, s, (const uint4*)(d + o_d),
                           (const int32_t*)(d + o_off), n_points, (int32_t*)(d + o_best), (uint4*)(d + o_out));
    ok = ok && hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(h + o_best, d + o_best, total - o_best, hipMemcpyDeviceToHost, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "ComputeDistinctiveDescriptors failed");
    memcpy(best, h + o_best, (size_t)n_points * 4);
    for (int p = 0; p < n_points; ++p)  // an empty point keeps its descriptor (the reference returns early)
        if (best[p] >= 0) memcpy(out + 32 * (size_t)p, h + o_out + 32 * (size_t)p, 32);
    return ORB_OK;
}
