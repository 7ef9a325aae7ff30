// MI355X DBoW2 TemplatedVocabulary::transform (reference Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h
// :1125-1260), the BoW step of KeyFrame::ComputeBoW / Frame::ComputeBoW, batched over frames.
//
//   k_bow_descend    one thread per descriptor: walk the vocabulary tree from the root, at every
//                    level the first child of minimal FORB distance (popcount of XOR), record the
//                    node of level L - levelsup and the leaf's word and weight
//   k_bow_aggregate  one workgroup per frame: the BowVector and FeatureVector are std::maps in
//                    DBoW2, so both are (id, feature) keys bitonic-sorted in LDS; each word's weights
//                    are summed in feature order (addWeight's order), the L1 / L2 norm is summed in
//                    ascending word order (the map's iteration order) by one lane, so every double
//                    comes out bit-identical to the CPU's
// Integer / popcount work; no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

struct orb_vocabulary_s {
    int k = 0, L = 0, weighting = 0, scoring = 0, n_nodes = 0;
    int32_t* d_child_begin = nullptr;
    int32_t* d_child_idx = nullptr;
    int32_t* d_word = nullptr;
    uint8_t* d_desc = nullptr;
    double* d_weight = nullptr;
    // staging of the synchronous single-frame path
    uint8_t* d_stage = nullptr;
    size_t stage_cap = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
};

namespace {

constexpr int kMaxFrameFeatures = 8192;  // 13-bit feature index in the sort keys
constexpr int kAggThreads = 1024;

__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__global__ __launch_bounds__(256) void k_bow_descend(const int32_t* __restrict__ child_begin,
                                                     const int32_t* __restrict__ child_idx,
                                                     const uint8_t* __restrict__ vdesc,
                                                     const int32_t* __restrict__ word_id,
                                                     const double* __restrict__ weight, int L,
                                                     const uint8_t* __restrict__ feat, int n, int levelsup,
                                                     int32_t* __restrict__ word, double* __restrict__ w,
                                                     int32_t* __restrict__ nid, const int32_t* __restrict__ kp_counts,
                                                     int cap) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (kp_counts) {  // frames at stride cap: past the count, or a frame the extractor could not place
        const int fr = i / cap, c = kp_counts[2 * fr];
        if (kp_counts[2 * fr + 1] == ORB_ERR_CAPACITY || c < 0 || c > cap || i % cap >= c) return;
    }
    const uint4* fp = reinterpret_cast<const uint4*>(feat + 32 * (size_t)i);
    const uint4 a0 = fp[0], a1 = fp[1];
    const uint4* D = reinterpret_cast<const uint4*>(vdesc);
    const int nid_level = L - levelsup;
    int node_at = nid_level <= 0 ? 0 : -1;
    int final_id = 0, level = 0;
    // Children are visited in groups of kGroup: the group's child ids are loaded together, then their
    // descriptors together, so a level costs two dependent round trips per group instead of two per
    // child.  Within a group the comparisons still run in child order (first minimum kept).
    constexpr int kGroup = 8;
    int cb = child_begin[0], ce = child_begin[1];
    while (ce > cb && level < 64) {
        ++level;
        int best_d = 1 << 30, best_id = -1;
        for (int g = cb; g < ce; g += kGroup) {
            int ids[kGroup];
#pragma unroll
            for (int u = 0; u < kGroup; ++u) ids[u] = g + u < ce ? child_idx[g + u] : -1;
            uint4 b0[kGroup], b1[kGroup];
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                const size_t o = 2 * (size_t)(ids[u] < 0 ? 0 : ids[u]);
                b0[u] = D[o];
                b1[u] = D[o + 1];
            }
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                const int d = hamming256(a0, a1, b0[u], b1[u]);
                if (ids[u] >= 0 && d < best_d) {  // first minimum (the reference compares doubles of these ints)
                    best_d = d;
                    best_id = ids[u];
                }
            }
        }
        final_id = best_id;
        if (level == nid_level) node_at = final_id;
        cb = child_begin[final_id];
        ce = child_begin[final_id + 1];
    }
    word[i] = word_id[final_id];
    w[i] = weight[final_id];
    nid[i] = node_at < 0 ? final_id : node_at;  // leaf above level L - levelsup: the leaf (see oracle)
}

__device__ void bitonic_sort(unsigned long long* keys, int P) {
    if (P <= kAggThreads) {
        // One key per thread (position tid).  The stages with partner distance j < 64 stay inside a
        // wave: the pair is exchanged by a lane shuffle and each side keeps its element of the
        // compare-swap (the lower position the minimum when ascending), with no LDS round trip or
        // barrier; only the stages with j >= 64 go through LDS.  Same network, same result.
        const int i = threadIdx.x;
        unsigned long long key = i < P ? keys[i] : 0ull;
        for (int k = 2; k <= P; k <<= 1) {
            int j = k >> 1;
            if (j >= 64) {
                if (i < P) keys[i] = key;
                __syncthreads();
                for (; j >= 64; j >>= 1) {
                    if (i < P) {
                        const int ixj = i ^ j;
                        if (ixj > i) {
                            const unsigned long long a = keys[i], b = keys[ixj];
                            if ((a > b) == ((i & k) == 0)) {
                                keys[i] = b;
                                keys[ixj] = a;
                            }
                        }
                    }
                    __syncthreads();
                }
                if (i < P) key = keys[i];
            }
            const bool up = (i & k) == 0;
            for (; j > 0; j >>= 1) {
                const unsigned long long other = __shfl_xor(key, j, 64);
                const bool lower = (i & j) == 0;
                const unsigned long long lo = key < other ? key : other, hi = key < other ? other : key;
                key = (lower == up) ? lo : hi;
            }
        }
        __syncthreads();  // every read of the LDS stage is done before the write-back
        if (i < P) keys[i] = key;
        __syncthreads();
        return;
    }
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += kAggThreads) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long a = keys[i], b = keys[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        keys[i] = b;
                        keys[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// exclusive scan of one int per thread over the workgroup; returns the total
__device__ int block_exclusive_scan(int v, int& excl, int* scan) {
    scan[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kAggThreads; o <<= 1) {
        const int t = threadIdx.x >= o ? scan[threadIdx.x - o] : 0;
        __syncthreads();
        scan[threadIdx.x] += t;
        __syncthreads();
    }
    excl = scan[threadIdx.x] - v;
    const int total = scan[kAggThreads - 1];
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(kAggThreads) void k_bow_aggregate(
    const int32_t* __restrict__ frame_begin, const int32_t* __restrict__ word, const double* __restrict__ w,
    const int32_t* __restrict__ nid, int weighting, int scoring, int32_t* __restrict__ bow_word,
    double* __restrict__ bow_value, int32_t* __restrict__ fv_node, int32_t* __restrict__ fv_begin,
    int32_t* __restrict__ fv_feat, int32_t* __restrict__ counts, const int32_t* __restrict__ kp_counts, int cap) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];
    __shared__ int scan[kAggThreads];
    __shared__ double s_norm;
    const int f = blockIdx.x, tid = threadIdx.x;
    // contiguous frames (frame_begin) or the extractor's layout (frame f at f * cap, kp_counts[2 f] features)
    const int base = kp_counts ? f * cap : frame_begin[f];
    const int n = kp_counts ? kp_counts[2 * f] : frame_begin[f + 1] - base;
    double* vals = reinterpret_cast<double*>(keys + kMaxFrameFeatures);
    // A frame over the extractor's capacity has no features in its slice (orb_extract_batch_device flags
    // it with ORB_ERR_CAPACITY and still reports the needed count): it fails here too, and the
    // triangulation skips it by its negative n_nodes.
    const bool failed = kp_counts && (kp_counts[2 * f + 1] == ORB_ERR_CAPACITY || n < 0 || n > cap);
    if (failed || n > kMaxFrameFeatures) {
        if (tid == 0) counts[2 * f] = counts[2 * f + 1] = ORB_ERR_CAPACITY;
        return;
    }
    int P = 2;
    while (P < n) P <<= 1;
    const bool tf = weighting == 0 || weighting == 1;
    const bool must = scoring != 5, l1 = scoring != 1;
    constexpr unsigned long long kNone = ~0ull;
    // ---- BowVector: (word, feature) keys of the non-stop words
    for (int i = tid; i < P; i += kAggThreads)
        keys[i] = (i < n && w[base + i] > 0) ? ((unsigned long long)(unsigned)word[base + i] << 13) | (unsigned)i : kNone;
    __syncthreads();
    bitonic_sort(keys, P);
    // segments of equal word: thread t owns positions [t*c, (t+1)*c)
    const int chunk = (P + kAggThreads - 1) / kAggThreads;
    const int p0 = tid * chunk, p1 = min(p0 + chunk, P);
    auto seg_start = [&](int p, int shift) {
        const unsigned long long k = keys[p];
        return k != kNone && (p == 0 || (keys[p - 1] >> shift) != (k >> shift));
    };
    int mine = 0;
    for (int p = p0; p < p1; ++p) mine += seg_start(p, 13);
    int excl;
    const int n_words = block_exclusive_scan(mine, excl, scan);
    for (int p = p0, s = excl; p < p1; ++p) {
        if (!seg_start(p, 13)) continue;
        const unsigned long long k = keys[p];
        double v = w[base + (int)(k & 8191)];
        if (tf)  // addWeight: += in feature order
            for (int q = p + 1; q < P && keys[q] != kNone && (keys[q] >> 13) == (k >> 13); ++q)
                v += w[base + (int)(keys[q] & 8191)];
        vals[s] = v;  // addIfNotExist (IDF, BINARY): the first feature's weight
        bow_word[base + s] = (int)(k >> 13);
        ++s;
    }
    __syncthreads();
    if (tid == 0) {
        double norm = 0.0;
        if (tf && n_words > 0 && !must) norm = (double)n_words;  // v[i] /= v.size()
        if (must) {
            if (l1) {
                for (int s = 0; s < n_words; ++s) norm += fabs(vals[s]);
            } else {
                for (int s = 0; s < n_words; ++s) norm += vals[s] * vals[s];
                norm = sqrt(norm);
            }
        }
        s_norm = norm;
    }
    __syncthreads();
    const double norm = s_norm;
    for (int s = tid; s < n_words; s += kAggThreads) bow_value[base + s] = norm > 0.0 ? vals[s] / norm : vals[s];
    __syncthreads();
    // ---- FeatureVector: (node, feature) keys of the same features
    for (int i = tid; i < P; i += kAggThreads)
        keys[i] = (i < n && w[base + i] > 0) ? ((unsigned long long)(unsigned)nid[base + i] << 13) | (unsigned)i : kNone;
    __syncthreads();
    bitonic_sort(keys, P);
    mine = 0;
    int valid = 0;
    for (int p = p0; p < p1; ++p) {
        mine += seg_start(p, 13);
        valid += keys[p] != kNone;
    }
    const int n_nodes = block_exclusive_scan(mine, excl, scan);
    int vexcl;
    const int n_valid = block_exclusive_scan(valid, vexcl, scan);
    int32_t* fb = fv_begin + base + f;
    for (int p = p0, s = excl; p < p1; ++p) {
        const unsigned long long k = keys[p];
        if (k == kNone) continue;
        fv_feat[base + p] = (int)(k & 8191);
        if (seg_start(p, 13)) {
            fv_node[base + s] = (int)(k >> 13);
            fb[s] = p;
            ++s;
        }
    }
    if (tid == 0) {
        fb[n_nodes] = n_valid;
        counts[2 * f] = n_words;
        counts[2 * f + 1] = n_nodes;
    }
}

int launch(orb_vocabulary_t v, const uint8_t* d_desc, const int32_t* d_frame_begin, int n_frames, int n_total,
           int levelsup, int32_t* d_word_tmp, double* d_w_tmp, int32_t* d_nid_tmp, int32_t* d_bow_word,
           double* d_bow_value, int32_t* d_fv_node, int32_t* d_fv_begin, int32_t* d_fv_feat, int32_t* d_counts,
           hipStream_t st, const int32_t* d_kp_counts = nullptr, int cap = 0) {
    if (n_total > 0)
        hipLaunchKernelGGL(k_bow_descend, dim3((n_total + 255) / 256), dim3(256), 0, st, v->d_child_begin, v->d_child_idx,
                           v->d_desc, v->d_word, v->d_weight, v->L, d_desc, n_total, levelsup, d_word_tmp, d_w_tmp,
                           d_nid_tmp, d_kp_counts, cap);
    const size_t lds = (size_t)kMaxFrameFeatures * 16;
    static bool attr = hipFuncSetAttribute((const void*)k_bow_aggregate, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds) == hipSuccess;
    if (!attr) return orbgpu_fail(ORB_ERR_DEVICE, "cannot raise the BoW aggregation LDS limit");
    hipLaunchKernelGGL(k_bow_aggregate, dim3(n_frames), dim3(kAggThreads), lds, st, d_frame_begin, d_word_tmp, d_w_tmp,
                       d_nid_tmp, v->weighting, v->scoring, d_bow_word, d_bow_value, d_fv_node, d_fv_begin, d_fv_feat,
                       d_counts, d_kp_counts, cap);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "BoW kernel launch failed");
    return ORB_OK;
}


}  // namespace

extern "C" {

int orb_vocabulary_create(const orb_vocabulary_view_t* view, orb_vocabulary_t* out) {
    if (!view || !out || view->n_nodes < 1 || !view->child_begin || (view->n_nodes > 1 && (!view->child_idx || !view->desc)) ||
        !view->word_id || !view->weight || view->L < 0)
        return orbgpu_fail(ORB_ERR_ARG, "invalid vocabulary");
    const int nn = view->n_nodes, nc = view->child_begin[nn];
    for (int i = 0; i < nn; ++i)
        if (view->child_begin[i] > view->child_begin[i + 1] || view->child_begin[i] < 0) return orbgpu_fail(ORB_ERR_ARG, "bad child ranges");
    for (int c = 0; c < nc; ++c)
        if (view->child_idx[c] <= 0 || view->child_idx[c] >= nn) return orbgpu_fail(ORB_ERR_ARG, "bad child index");
    if (orb_device_count() <= 0) return orbgpu_fail(ORB_ERR_DEVICE, "no HIP device visible");
    orb_vocabulary_t v = new orb_vocabulary_s();
    v->k = view->k; v->L = view->L; v->weighting = view->weighting; v->scoring = view->scoring; v->n_nodes = nn;
    bool ok = hipMalloc(&v->d_child_begin, 4 * (size_t)(nn + 1)) == hipSuccess &&
              hipMalloc(&v->d_child_idx, 4 * (size_t)std::max(nc, 1)) == hipSuccess &&
              hipMalloc(&v->d_word, 4 * (size_t)nn) == hipSuccess && hipMalloc(&v->d_desc, 32 * (size_t)nn) == hipSuccess &&
              hipMalloc(&v->d_weight, 8 * (size_t)nn) == hipSuccess &&
              hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMemcpy(v->d_child_begin, view->child_begin, 4 * (size_t)(nn + 1), hipMemcpyHostToDevice) == hipSuccess &&
         (nc == 0 || hipMemcpy(v->d_child_idx, view->child_idx, 4 * (size_t)nc, hipMemcpyHostToDevice) == hipSuccess) &&
         hipMemcpy(v->d_word, view->word_id, 4 * (size_t)nn, hipMemcpyHostToDevice) == hipSuccess &&
         (!view->desc || hipMemcpy(v->d_desc, view->desc, 32 * (size_t)nn, hipMemcpyHostToDevice) == hipSuccess) &&
         hipMemcpy(v->d_weight, view->weight, 8 * (size_t)nn, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
        orb_vocabulary_destroy(v);
        return orbgpu_fail(ORB_ERR_DEVICE, "vocabulary upload failed");
    }
    *out = v;
    return ORB_OK;
}

int orb_vocabulary_destroy(orb_vocabulary_t v) {
    if (!v) return ORB_ERR_ARG;
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    void* bufs[] = {v->d_child_begin, v->d_child_idx, v->d_word, v->d_desc, v->d_weight, v->d_stage};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
    return ORB_OK;
}

int orb_bow_transform_batch_device(orb_vocabulary_t v, const uint8_t* d_desc, const int32_t* d_frame_begin,
                                   int n_frames, int n_total, int levelsup, int32_t* d_bow_word,
                                   double* d_bow_value, int32_t* d_fv_node, int32_t* d_fv_begin, int32_t* d_fv_feat,
                                   int32_t* d_counts, void* stream) {
    if (!v || n_frames < 0 || n_total < 0 || (n_total && !d_desc) || !d_frame_begin || !d_bow_word || !d_bow_value ||
        !d_fv_node || !d_fv_begin || !d_fv_feat || !d_counts)
        return orbgpu_fail(ORB_ERR_ARG, "invalid BoW arguments");
    if (n_frames == 0) return ORB_OK;
    if (v->n_nodes <= 1) return orbgpu_fail(ORB_ERR_ARG, "empty vocabulary");
    // per-descriptor word / weight / node scratch, stream-ordered (allocated and freed on the call's
    // stream), so calls on different streams may run concurrently
    const size_t m = std::max(n_total, 1);
    uint8_t* tmp = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&tmp), m * 16, (hipStream_t)stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    int rc = launch(v, d_desc, d_frame_begin, n_frames, n_total, levelsup, reinterpret_cast<int32_t*>(tmp + 8 * m),
                    reinterpret_cast<double*>(tmp), reinterpret_cast<int32_t*>(tmp + 12 * m), d_bow_word, d_bow_value,
                    d_fv_node, d_fv_begin, d_fv_feat, d_counts, (hipStream_t)stream);
    if (hipFreeAsync(tmp, (hipStream_t)stream) != hipSuccess && rc == ORB_OK) rc = orbgpu_fail(ORB_ERR_DEVICE, "hipFreeAsync failed");
    return rc;
}

int orb_bow_transform_frames_device(orb_vocabulary_t v, const uint8_t* d_desc, const int32_t* d_kp_counts, int n_frames,
                                    int cap, int levelsup, int32_t* d_bow_word, double* d_bow_value, int32_t* d_fv_node,
                                    int32_t* d_fv_begin, int32_t* d_fv_feat, int32_t* d_counts, void* stream) {
    if (!v || n_frames < 0 || cap <= 0 || (n_frames && (!d_desc || !d_kp_counts)) || !d_bow_word || !d_bow_value ||
        !d_fv_node || !d_fv_begin || !d_fv_feat || !d_counts)
        return orbgpu_fail(ORB_ERR_ARG, "invalid BoW arguments");
    if (n_frames == 0) return ORB_OK;
    if (v->n_nodes <= 1) return orbgpu_fail(ORB_ERR_ARG, "empty vocabulary");
    const size_t total = (size_t)n_frames * (size_t)cap;
    if (total >= (size_t)INT32_MAX / 32) return orbgpu_fail(ORB_ERR_ARG, "BoW batch too large");
    uint8_t* tmp = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&tmp), total * 16, (hipStream_t)stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    int rc = launch(v, d_desc, nullptr, n_frames, (int)total, levelsup, reinterpret_cast<int32_t*>(tmp + 8 * total),
                    reinterpret_cast<double*>(tmp), reinterpret_cast<int32_t*>(tmp + 12 * total), d_bow_word,
                    d_bow_value, d_fv_node, d_fv_begin, d_fv_feat, d_counts, (hipStream_t)stream, d_kp_counts, cap);
    if (hipFreeAsync(tmp, (hipStream_t)stream) != hipSuccess && rc == ORB_OK) rc = orbgpu_fail(ORB_ERR_DEVICE, "hipFreeAsync failed");
    return rc;
}

int orb_bow_transform(orb_vocabulary_t v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                      double* bow_value, int32_t* n_words, int32_t* fv_node, int32_t* fv_begin, int32_t* fv_feat,
                      int32_t* n_nodes) {
    if (!v || n < 0 || n > kMaxFrameFeatures || (n && (!desc || !bow_word || !bow_value || !fv_node || !fv_feat)) ||
        !fv_begin || !n_words || !n_nodes)
        return orbgpu_fail(ORB_ERR_ARG, "invalid BoW arguments");
    *n_words = *n_nodes = 0;
    fv_begin[0] = 0;
    if (n == 0 || v->n_nodes <= 1) return ORB_OK;  // empty(): nothing
    std::lock_guard<std::mutex> lk(v->mu);
    // staging: frame_begin (2) | desc | word | w | nid | bow_word | bow_value | fv_node | fv_begin | fv_feat | counts
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_fb = 0, o_d = 256, o_w = o_d + al(32 * (size_t)n), o_wt = o_w + al(4 * (size_t)n);
    const size_t o_n = o_wt + al(8 * (size_t)n), o_bw = o_n + al(4 * (size_t)n), o_bv = o_bw + al(4 * (size_t)n);
    const size_t o_fn = o_bv + al(8 * (size_t)n), o_fbg = o_fn + al(4 * (size_t)n), o_ff = o_fbg + al(4 * (size_t)(n + 1));
    const size_t o_c = o_ff + al(4 * (size_t)n), total = o_c + 256;
    if (total > v->stage_cap) {
        if (v->d_stage) (void)hipFree(v->d_stage);
        v->d_stage = nullptr;
        v->stage_cap = 0;
        if (hipMalloc(&v->d_stage, total) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
        v->stage_cap = total;
    }
    uint8_t* d = v->d_stage;
    const int32_t fb[2] = {0, n};
    hipStream_t st = v->stream;
    if (hipMemcpyAsync(d + o_fb, fb, sizeof(fb), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d + o_d, desc, 32 * (size_t)n, hipMemcpyHostToDevice, st) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "BoW upload failed");
    int rc = launch(v, d + o_d, reinterpret_cast<int32_t*>(d + o_fb), 1, n, levelsup, reinterpret_cast<int32_t*>(d + o_w),
                    reinterpret_cast<double*>(d + o_wt), reinterpret_cast<int32_t*>(d + o_n),
                    reinterpret_cast<int32_t*>(d + o_bw), reinterpret_cast<double*>(d + o_bv),
                    reinterpret_cast<int32_t*>(d + o_fn), reinterpret_cast<int32_t*>(d + o_fbg),
                    reinterpret_cast<int32_t*>(d + o_ff), reinterpret_cast<int32_t*>(d + o_c), st);
    if (rc != ORB_OK) return rc;
    int32_t cnt[2];
    if (hipMemcpyAsync(cnt, d + o_c, 8, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "BoW download failed");
    if (cnt[0] < 0) return orbgpu_fail(ORB_ERR_CAPACITY, "too many features in one frame");
    if (hipMemcpyAsync(bow_word, d + o_bw, 4 * (size_t)cnt[0], hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(bow_value, d + o_bv, 8 * (size_t)cnt[0], hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(fv_node, d + o_fn, 4 * (size_t)cnt[1], hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(fv_begin, d + o_fbg, 4 * (size_t)(cnt[1] + 1), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(fv_feat, d + o_ff, 4 * (size_t)n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "BoW download failed");
    *n_words = cnt[0];
    *n_nodes = cnt[1];
    return ORB_OK;
}

}  // extern "C"
