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
// The launch is cut two ways so that one frame (~1000 queries) fills the chip: 64-query tiles (one
// query per lane) x train chunks; the four waves of a block scan quarters of the block's chunk (staged
// in LDS, read as broadcasts) and merge in wave order; chunks merge in chunk order in a second kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kKnnWaves = 4, kKnnThreads = 64 * kKnnWaves;
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
__global__ __launch_bounds__(kKnnThreads) void k_hamming_knn2(const uint8_t* __restrict__ q, int nq,
                                                              const uint8_t* __restrict__ t, int nt, int chunk,
                                                              Knn* __restrict__ part, int32_t* __restrict__ best_idx,
                                                              int32_t* __restrict__ best_dist,
                                                              int32_t* __restrict__ second_dist) {
    __shared__ uint4 tile[kKnnMaxChunk * 2];
    __shared__ Knn wpart[kKnnWaves - 1][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int qi = blockIdx.x * 64 + lane;
    const int c0 = blockIdx.y * chunk, n = min(chunk, nt - c0);
    for (int i = threadIdx.x; i < 2 * n; i += kKnnThreads) tile[i] = reinterpret_cast<const uint4*>(t)[2 * (size_t)c0 + i];
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < nq) {
        a0 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi];
        a1 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi + 1];
    }
    __syncthreads();
    const int sub = (n + kKnnWaves - 1) / kKnnWaves, j0 = w * sub, j1 = min(n, j0 + sub);
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
    for (int k = 0; k < kKnnWaves - 1; ++k) r = knn_merge(r, wpart[k][lane]);
    if (part) {
        part[(size_t)blockIdx.y * nq + qi] = r;
    } else {
        best_idx[qi] = r.idx;
        best_dist[qi] = r.best;
        second_dist[qi] = r.second;
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
    hipLaunchKernelGGL(k_hamming_knn2, dim3(qtiles, nchunk), dim3(kKnnThreads), 0, s, d_query, n_query, d_train, n_train,
                       chunk, part, d_best_idx, d_best_dist, d_second_dist);
    if (part) {
        hipLaunchKernelGGL(k_hamming_knn2_merge, dim3((n_query + 255) / 256), dim3(256), 0, s, n_query, nchunk, part,
                           d_best_idx, d_best_dist, d_second_dist);
        if (hipFreeAsync(part, s) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "knn2 partial buffer free");
    }
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hamming launch failed");
    return ORB_OK;
}
