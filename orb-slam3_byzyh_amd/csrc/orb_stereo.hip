// MI355X Frame::ComputeStereoMatches (reference src/Frame.cc:1102-1358): sparse stereo matching of a
// rectified pair on the extractors' device pyramids, batched over B frames.
//
//   k_stereo_match  one wave per left keypoint:
//                   (1) row-band Hamming search: the 64 lanes scan the right keypoints; a right
//                       keypoint is a candidate iff the left row lies in its band
//                       [floor(y - 2 s), ceil(y + 2 s)] (the reference's vRowIndices table,
//                       :1134-1152), its octave is within +-1 and uR in [uL - bf/b, uL]; the
//                       reference's "first strict minimum in ascending iR" is the lexicographic
//                       minimum of (distance, iR), a wave min-reduction
//                   (2) SAD refinement: 11 offsets x 11 rows = 121 row-SADs spread over the lanes
//                       (aligned dword loads of the padded planes), summed per offset in LDS;
//                       first strict minimum = min of (SAD, offset)
//                   (3) parabola fit, disparity test, depth (lane 0, reference float order)
//   k_stereo_cull   one block per frame: the median SAD of the kept matches by a two-pass radix
//                   select (8 + 7 bits: SAD <= 121 * 255 < 2^15), then SAD >= 1.5f*1.4f*median
//                   is dropped -- the reference's sorted-suffix loop (:1340-1352) removes exactly
//                   those
// Integer / popcount work plus a few float ops per keypoint; no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kThHigh = 100, kThLow = 50;          // ORBmatcher::TH_HIGH / TH_LOW (src/ORBmatcher.cc:36-37)
constexpr int kWavesPerBlock = 4;
constexpr int kEdge = 19;                          // EDGE_THRESHOLD: view origin in the padded plane
constexpr int kMaxLevels = 12;

struct StereoGeom {
    long long frame_bytes;
    long long plane_off[kMaxLevels];
    int pitch[kMaxLevels], w[kMaxLevels], h[kMaxLevels];
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    int nlevels;
};

__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 64));
    return v;
}

// 11 bytes starting at p (any alignment) from 4 aligned dwords; byte k = (v[k>>2] >> 8(k&3)) after
// the shift, returned as 16 bytes in q[0..3] aligned so that q byte 0 = p[0]
__device__ __forceinline__ void load11(const uint8_t* p, uint32_t (&q)[4]) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    const unsigned sh = (unsigned)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint32_t w0 = a[0], w1 = a[1], w2 = a[2], w3 = a[3];
    q[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
    q[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
    q[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
    q[3] = 0;
}

__device__ __forceinline__ int sad11(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < 11; ++k) {
        const int x = (a[k >> 2] >> (8 * (k & 3))) & 0xff, y = (b[k >> 2] >> (8 * (k & 3))) & 0xff;
        s += abs(x - y);
    }
    return s;
}

__global__ __launch_bounds__(64 * kWavesPerBlock) void k_stereo_match(
    const orb_keypoint_t* __restrict__ kps_l, const int32_t* __restrict__ counts_l, const uint8_t* __restrict__ desc_l,
    int cap_l, const orb_keypoint_t* __restrict__ kps_r, const int32_t* __restrict__ counts_r,
    const uint8_t* __restrict__ desc_r, int cap_r, const uint8_t* __restrict__ pyr_l, const uint8_t* __restrict__ pyr_r,
    StereoGeom G, float bf, float b, float* __restrict__ u_right, float* __restrict__ depth, int32_t* __restrict__ sad_out) {
    __shared__ int row_sad[kWavesPerBlock][128];
    __shared__ int off_sad[kWavesPerBlock][16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, f = blockIdx.y;
    const int iL = blockIdx.x * kWavesPerBlock + wv;
    const int n_l = counts_l[2 * f], n_r = counts_r[2 * f];
    if (iL >= n_l) return;
    const size_t oL = (size_t)f * cap_l + iL;
    const orb_keypoint_t kpL = kps_l[oL];
    float out_u = -1.0f, out_d = -1.0f;
    int out_sad = -1;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;                     // vRowIndices[vL]: size_t conversion (vL >= 0)
    const float minZ = b, minD = 0, maxD = bf / minZ;  // :1160-1163
    const float minU = uL - maxD, maxU = uL - minD;
    if (maxU >= 0 && row < G.h[0]) {
        // (1) row-band Hamming search, :1176-1226
        const uint4* dl = reinterpret_cast<const uint4*>(desc_l + 32 * oL);
        const uint4 a0 = dl[0], a1 = dl[1];
        unsigned best = 0xffffffffu;
        const orb_keypoint_t* KR = kps_r + (size_t)f * cap_r;
        const uint4* DR = reinterpret_cast<const uint4*>(desc_r + 32 * (size_t)f * cap_r);
        for (int c = 0; c < n_r; c += 64) {
            const int j = c + lane;
            if (j < n_r) {
                const orb_keypoint_t kpR = KR[j];
                const float r = 2.0f * G.scale[kpR.octave];
                const int maxr = (int)ceilf(kpR.y + r), minr = (int)floorf(kpR.y - r);
                if (row >= minr && row <= maxr && kpR.octave >= levelL - 1 && kpR.octave <= levelL + 1 &&
                    kpR.x >= minU && kpR.x <= maxU) {
                    const int dist = hamming256(a0, a1, DR[2 * j], DR[2 * j + 1]);
                    best = min(best, ((unsigned)dist << 16) | (unsigned)j);
                }
            }
        }
        best = wave_min_u32(best);
        const int bestDist = best == 0xffffffffu ? kThHigh : (int)(best >> 16);
        if (bestDist < kThHigh && bestDist < (kThHigh + kThLow) / 2) {
            // (2) SAD refinement at the keypoint's level, :1228-1280
            const int bestIdxR = (int)(best & 0xffff);
            const float uR0 = KR[bestIdxR].x;
            const float scaleFactor = G.inv_scale[levelL];
            const float scaleduL = roundf(kpL.x * scaleFactor);
            const float scaledvL = roundf(kpL.y * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            constexpr int w = 5, L = 5;
            const int cuL = (int)scaleduL, cvL = (int)scaledvL, cuR = (int)scaleduR0;
            const int lw = G.w[levelL], lh = G.h[levelL];
            const float iniu = scaleduR0 + L - w, endu = scaleduR0 + L + w + 1;
            // the reference's bound (:1262-1265) + the view bounds its cv::Mat ranges assert
            const bool inside = !(iniu < 0 || endu >= lw) && cuR - L - w >= 0 && cvL - w >= 0 && cvL + w < lh &&
                                cuL - w >= 0 && cuL + w < lw;
            if (inside) {
                const int pitch = G.pitch[levelL];
                const uint8_t* IL = pyr_l + (size_t)f * G.frame_bytes + G.plane_off[levelL] + (size_t)kEdge * pitch + kEdge;
                const uint8_t* IR = pyr_r + (size_t)f * G.frame_bytes + G.plane_off[levelL] + (size_t)kEdge * pitch + kEdge;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int p = lane + 64 * k;  // (offset, row) pair
                    if (p < 121) {
                        const int inc = p / 11 - L, y = p % 11 - w;
                        uint32_t ql[4], qr[4];
                        load11(IL + (size_t)(cvL + y) * pitch + cuL - w, ql);
                        load11(IR + (size_t)(cvL + y) * pitch + cuR + inc - w, qr);
                        row_sad[wv][p] = sad11(ql, qr);
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                unsigned key = 0xffffffffu;
                if (lane < 2 * L + 1) {
                    int s = 0;
#pragma unroll
                    for (int y = 0; y < 11; ++y) s += row_sad[wv][lane * 11 + y];
                    off_sad[wv][lane] = s;
                    key = ((unsigned)s << 4) | (unsigned)lane;  // first strict minimum over incR order
                }
                key = wave_min_u32(key);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int bestincR = (int)(key & 15) - L;
                if (bestincR != -L && bestincR != L) {
                    // (3) parabola + disparity, :1286-1328 (float, the reference's operation order)
                    const float dist1 = (float)off_sad[wv][L + bestincR - 1];
                    const float dist2 = (float)off_sad[wv][L + bestincR];
                    const float dist3 = (float)off_sad[wv][L + bestincR + 1];
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = G.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
                        float disparity = (uL - bestuR);
                        if (disparity >= minD && disparity < maxD) {
                            if (disparity <= 0) {
                                disparity = 0.01;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            out_d = bf / disparity;
                            out_u = bestuR;
                            out_sad = (int)(key >> 4);
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) {
        u_right[oL] = out_u;
        depth[oL] = out_d;
        sad_out[oL] = out_sad;
    }
}

// One block per frame: median of the kept SADs (the (M/2)-th smallest), then the cull.
__global__ __launch_bounds__(256) void k_stereo_cull(const int32_t* __restrict__ counts_l, int cap_l,
                                                     const int32_t* __restrict__ sad, float* __restrict__ u_right,
                                                     float* __restrict__ depth, int32_t* __restrict__ kept) {
    __shared__ int hist[256];
    __shared__ int sel_bin, sel_rank, total;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = counts_l[2 * f];
    const int32_t* S = sad + (size_t)f * cap_l;
    hist[tid] = 0;
    if (tid == 0) total = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256)
        if (S[i] >= 0) { atomicAdd(&hist[S[i] >> 7], 1); atomicAdd(&total, 1); }
    __syncthreads();
    const int M = total;
    if (M == 0) {  // the reference reads vDistIdx[0] of an empty vector here; nothing to cull
        if (tid == 0) kept[f] = 0;
        return;
    }
    const int k = M / 2;
    if (tid == 0) {
        int acc = 0, bin = 0;
        while (acc + hist[bin] <= k) acc += hist[bin++];
        sel_bin = bin;
        sel_rank = k - acc;
    }
    __syncthreads();
    const int bin = sel_bin;
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256)
        if (S[i] >= 0 && (S[i] >> 7) == bin) atomicAdd(&hist[S[i] & 127], 1);
    __syncthreads();
    if (tid == 0) {
        int acc = 0, lo = 0;
        while (acc + hist[lo] <= sel_rank) acc += hist[lo++];
        sel_bin = (bin << 7) | lo;  // the median SAD
        total = 0;
    }
    __syncthreads();
    const float median = (float)sel_bin;
    const float thDist = 1.5f * 1.4f * median;
    int mine = 0;
    for (int i = tid; i < n; i += 256) {
        if (S[i] < 0) continue;
        if ((float)S[i] < thDist) { ++mine; continue; }
        u_right[(size_t)f * cap_l + i] = -1.0f;
        depth[(size_t)f * cap_l + i] = -1.0f;
    }
    atomicAdd(&total, mine);
    __syncthreads();
    if (tid == 0) kept[f] = total;
}

// Workspace of the synchronous single-frame path (one per thread: calls on different handles may
// run concurrently).
struct HostStage {
    void* buf = nullptr;
    size_t cap = 0;
    ~HostStage() { if (buf) (void)hipFree(buf); }
};

int make_geom(orb_extractor_t left, orb_extractor_t right, int n, StereoGeom& G, OrbPyramidView& vl, OrbPyramidView& vr) {
    int rc;
    if ((rc = orbgpu_extractor_pyramid(left, &vl)) != ORB_OK) return rc;
    if ((rc = orbgpu_extractor_pyramid(right, &vr)) != ORB_OK) return rc;
    if (vl.nlevels != vr.nlevels || vl.frame_bytes != vr.frame_bytes || n > vl.nframes || n > vr.nframes)
        return orbgpu_fail(ORB_ERR_ARG, "left / right pyramids differ or hold fewer frames");
    G = StereoGeom{};
    G.frame_bytes = vl.frame_bytes;
    G.nlevels = vl.nlevels;
    for (int l = 0; l < vl.nlevels; ++l) {
        if (vl.w[l] != vr.w[l] || vl.h[l] != vr.h[l] || vl.pitch[l] != vr.pitch[l] || vl.plane_off[l] != vr.plane_off[l] ||
            vl.scale[l] != vr.scale[l])
            return orbgpu_fail(ORB_ERR_ARG, "left / right extractors differ in frame size or parameters");
        G.plane_off[l] = vl.plane_off[l];
        G.pitch[l] = vl.pitch[l];
        G.w[l] = vl.w[l];
        G.h[l] = vl.h[l];
        G.scale[l] = vl.scale[l];
        G.inv_scale[l] = vl.inv_scale[l];
    }
    return ORB_OK;
}

int launch(const StereoGeom& G, const OrbPyramidView& vl, const OrbPyramidView& vr, int n, const orb_keypoint_t* kps_l,
           const int32_t* counts_l, const uint8_t* desc_l, int cap_l, const orb_keypoint_t* kps_r,
           const int32_t* counts_r, const uint8_t* desc_r, int cap_r, float bf, float b, float* u_right,
           float* depth, int32_t* sad, int32_t* kept, hipStream_t st) {
    if (cap_l > 0) {
        hipLaunchKernelGGL(k_stereo_match, dim3((cap_l + kWavesPerBlock - 1) / kWavesPerBlock, n), dim3(64 * kWavesPerBlock),
                           0, st, kps_l, counts_l, desc_l, cap_l, kps_r, counts_r, desc_r, cap_r, vl.base, vr.base, G, bf, b,
                           u_right, depth, sad);
    }
    hipLaunchKernelGGL(k_stereo_cull, dim3(n), dim3(256), 0, st, counts_l, cap_l, sad, u_right, depth, kept);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "stereo kernel launch failed");
    return ORB_OK;
}

}  // namespace

extern "C" {

int orb_compute_stereo_matches_batch_device(orb_extractor_t left, orb_extractor_t right, int n,
                                            const orb_keypoint_t* d_kps_l, const int32_t* d_counts_l,
                                            const uint8_t* d_desc_l, int cap_l, const orb_keypoint_t* d_kps_r,
                                            const int32_t* d_counts_r, const uint8_t* d_desc_r, int cap_r,
                                            float bf, float b, float* d_u_right, float* d_depth, int32_t* d_kept,
                                            void* stream) {
    if (!left || !right || n <= 0 || cap_l < 0 || cap_r < 0 || cap_r > 65536 || !d_kps_l || !d_counts_l || !d_desc_l ||
        !d_kps_r || !d_counts_r || !d_desc_r || !d_u_right || !d_depth || !d_kept || !(b > 0.0f))
        return orbgpu_fail(ORB_ERR_ARG, "invalid stereo matching arguments");
    StereoGeom G;
    OrbPyramidView vl, vr;
    int rc = make_geom(left, right, n, G, vl, vr);
    if (rc != ORB_OK) return rc;
    // the per-keypoint SAD scratch is stream-ordered (allocated and freed on the call's stream), so
    // calls on different handles and streams may run concurrently
    const size_t need = (size_t)n * std::max(cap_l, 1);
    int32_t* sad = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&sad), need * sizeof(int32_t), (hipStream_t)stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    rc = launch(G, vl, vr, n, d_kps_l, d_counts_l, d_desc_l, cap_l, d_kps_r, d_counts_r, d_desc_r, cap_r, bf, b,
                d_u_right, d_depth, sad, d_kept, (hipStream_t)stream);
    if (hipFreeAsync(sad, (hipStream_t)stream) != hipSuccess && rc == ORB_OK)
        rc = orbgpu_fail(ORB_ERR_DEVICE, "hipFreeAsync failed");
    return rc;
}

int orb_compute_stereo_matches(orb_extractor_t left, orb_extractor_t right, const orb_keypoint_t* kps_l, int n_l,
                               const uint8_t* desc_l, const orb_keypoint_t* kps_r, int n_r, const uint8_t* desc_r,
                               float bf, float b, float* u_right, float* depth) {
    orbgpu::StageTimer timer("Stereo Matching");  // src/Frame.cc:158-170
    if (!left || !right || n_l < 0 || n_r < 0 || n_r > 65536 || (n_l && (!kps_l || !desc_l || !u_right || !depth)) ||
        (n_r && (!kps_r || !desc_r)) || !(b > 0.0f))
        return orbgpu_fail(ORB_ERR_ARG, "invalid stereo matching arguments");
    if (n_l == 0) return 0;
    StereoGeom G;
    OrbPyramidView vl, vr;
    int rc = make_geom(left, right, 1, G, vl, vr);
    if (rc != ORB_OK) return rc;
    // one staging block: counts (4 ints) | kps_l | kps_r | desc_l | desc_r | u | depth | sad | kept
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_cnt = 0, o_kl = 256, o_kr = o_kl + al(28 * (size_t)n_l), o_dl = o_kr + al(28 * (size_t)std::max(n_r, 1));
    const size_t o_dr = o_dl + al(32 * (size_t)n_l), o_u = o_dr + al(32 * (size_t)std::max(n_r, 1));
    const size_t o_d = o_u + al(4 * (size_t)n_l), o_s = o_d + al(4 * (size_t)n_l), o_k = o_s + al(4 * (size_t)n_l);
    const size_t total = o_k + 256;
    thread_local HostStage stage;
    if (total > stage.cap) {
        if (stage.buf) (void)hipFree(stage.buf);
        stage.buf = nullptr;
        stage.cap = 0;
        if (hipMalloc(&stage.buf, total) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
        stage.cap = total;
    }
    std::vector<uint8_t> h(o_u);
    const int32_t cnt[4] = {n_l, 0, n_r, 0};
    memcpy(h.data() + o_cnt, cnt, sizeof(cnt));
    memcpy(h.data() + o_kl, kps_l, 28 * (size_t)n_l);
    if (n_r) memcpy(h.data() + o_kr, kps_r, 28 * (size_t)n_r);
    memcpy(h.data() + o_dl, desc_l, 32 * (size_t)n_l);
    if (n_r) memcpy(h.data() + o_dr, desc_r, 32 * (size_t)n_r);
    uint8_t* d = static_cast<uint8_t*>(stage.buf);
    hipStream_t st = (hipStream_t)vl.stream;
    if (hipMemcpyAsync(d, h.data(), o_u, hipMemcpyHostToDevice, st) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "stereo upload failed");
    const int32_t* dc = reinterpret_cast<const int32_t*>(d + o_cnt);
    rc = launch(G, vl, vr, 1, reinterpret_cast<const orb_keypoint_t*>(d + o_kl), dc, d + o_dl, n_l,
                reinterpret_cast<const orb_keypoint_t*>(d + o_kr), dc + 2, d + o_dr, std::max(n_r, 1), bf, b,
                reinterpret_cast<float*>(d + o_u), reinterpret_cast<float*>(d + o_d), reinterpret_cast<int32_t*>(d + o_s),
                reinterpret_cast<int32_t*>(d + o_k), st);
    if (rc != ORB_OK) return rc;
    int32_t kept = 0;
    if (hipMemcpyAsync(u_right, d + o_u, 4 * (size_t)n_l, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(depth, d + o_d, 4 * (size_t)n_l, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&kept, d + o_k, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "stereo download failed");
    return kept;
}

}  // extern "C"
