// MI355X Hamming matching kernels (ORBmatcher, reference src/ORBmatcher.cc).
//
// DescriptorDistance (src:2384-2404) is popcount(a ^ b) over 256 bits; on gfx950 that is 8 v_xor +
// 8 v_bcnt_u32 (popcount-accumulate) per descriptor pair.  No MFMA: this is bit-count work.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kQueryPerBlock = 256;
constexpr int kTrainTile = 256;

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

// One thread per query; train descriptors stream through LDS in tiles of 256 (8 KiB), read as
// wave-uniform broadcasts.  Best / second-best follow the reference's scan order: a strictly
// smaller distance replaces the best (ties keep the first index), src:1160-1175.
__global__ __launch_bounds__(kQueryPerBlock) void k_hamming_knn2(const uint8_t* __restrict__ q, int nq,
                                                                 const uint8_t* __restrict__ t, int nt,
                                                                 int32_t* __restrict__ best_idx,
                                                                 int32_t* __restrict__ best_dist,
                                                                 int32_t* __restrict__ second_dist) {
    __shared__ uint4 tile[kTrainTile * 2];
    const int qi = blockIdx.x * kQueryPerBlock + threadIdx.x;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < nq) {
        a0 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi];
        a1 = reinterpret_cast<const uint4*>(q)[2 * (size_t)qi + 1];
    }
    int best = 257, second = 257, bidx = -1;
    for (int base = 0; base < nt; base += kTrainTile) {
        const int n = min(kTrainTile, nt - base);
        __syncthreads();
        for (int i = threadIdx.x; i < 2 * n; i += kQueryPerBlock)
            tile[i] = reinterpret_cast<const uint4*>(t)[2 * (size_t)base + i];
        __syncthreads();
        for (int j = 0; j < n; ++j) {
            const int d = hamming256(a0, a1, tile[2 * j], tile[2 * j + 1]);
            if (d < best) { second = best; best = d; bidx = base + j; }
            else if (d < second) second = d;
        }
    }
    if (qi < nq) {
        best_idx[qi] = bidx;
        best_dist[qi] = best;
        second_dist[qi] = second;
    }
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
    hipLaunchKernelGGL(k_hamming_knn2, dim3((n_query + kQueryPerBlock - 1) / kQueryPerBlock), dim3(kQueryPerBlock), 0,
                       (hipStream_t)stream, d_query, n_query, d_train, n_train, d_best_idx, d_best_dist, d_second_dist);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hamming launch failed");
    return ORB_OK;
}
