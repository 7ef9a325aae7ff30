// ORBmatcher::SearchForTriangulation on MI355X (reference src/ORBmatcher.cc:1046-1324).
//
// The reference walks the two keyframes' DBoW2 FeatureVectors (std::map node -> feature indices)
// in step and, inside every shared node, scans node-2 features for each node-1 feature: Hamming
// distance <= TH_LOW and <= the best so far (ties go to the LATER candidate), the epipole check
// for mono-mono pairs, and Pinhole::epipolarConstrain (src/CameraModels/Pinhole.cpp:186-216).
// Matches of different node-1 features are independent, so the device form is:
//
//   k_tri_match   one wave per (neighbour keyframe, node of KF1): binary-search the node in KF2's
//                 sorted node ids, one lane per KF1 feature of the node, sequential scan over the
//                 node-2 list (uniform across the wave -> broadcast loads), same order and the same
//                 tie rule as the reference.
//   k_tri_finish  one block per neighbour: match count, and the rotation-histogram filter with
//                 ComputeThreeMaxima (src:1270-1297, 2336-2378) when the matcher checks orientation.
//
// Float arithmetic follows the reference build (g++ -O3 -march=native contracts a*b + c*d into
// fma(a, b, c*d)); this file is compiled with -ffp-contract=off and every contraction is explicit.
// F12 is computed once per pair on the host (the reference recomputes the same value per call).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kThLow = 50;        // src/ORBmatcher.cc:37
constexpr int kHistoLength = 30;  // src/ORBmatcher.cc:38
constexpr int kMaxLevels = 12;
constexpr int kWaves = 4;

// One keypoint as the matcher reads it (16 B): pt, angle, octave | has-MapPoint << 8 | stereo << 9.
struct KpRec {
    float x, y, angle;
    int32_t meta;
};

struct KfDev {
    int32_t n, n_nodes;
    int32_t kp_off;    // into the KpRec / descriptor arrays
    int32_t node_off;  // into the node-id array
    int32_t csr_off;   // into the CSR offset array (n_nodes + 1 entries)
    int32_t pad[3];
};

struct PairDev {
    float F[9];                 // F12 row-major
    float ep[2];                // epipole of KF1's centre in KF2
    float pad;
    float scale100[kMaxLevels]; // 100 * mvScaleFactors of KF2 (float product, src:1193)
    double thr[kMaxLevels];     // 3.84 * mvLevelSigma2 of KF2 (double, Pinhole.cpp:215)
};

__device__ __forceinline__ int hamming(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Keyframes packed host-side into one upload (orb_search_for_triangulation).
struct PackedSrc {
    const KfDev* kfs;
    const KpRec* kps;
    const uint4* desc;
    const uint32_t* nodes;
    const int32_t* csr;
    const int32_t* fidx;
    __device__ int n(int k) const { return kfs[k].n; }
    __device__ int n_nodes(int k) const { return kfs[k].n_nodes; }
    __device__ bool failed(int) const { return false; }  // validated on the host
    __device__ uint32_t node(int k, int i) const { return nodes[kfs[k].node_off + i]; }
    __device__ int node_begin(int k, int i) const { return csr[kfs[k].csr_off + i]; }
    __device__ int feat(int k, int j) const { return fidx[j]; }
    __device__ KpRec kp(int k, int idx) const { return kps[kfs[k].kp_off + idx]; }
    __device__ float angle(int k, int idx) const { return kps[kfs[k].kp_off + idx].angle; }
    __device__ void descriptor(int k, int idx, uint4& a, uint4& b) const {
        const size_t o = 2 * (size_t)(kfs[k].kp_off + idx);
        a = desc[o];
        b = desc[o + 1];
    }
};

// Keyframes left on the device by the extraction / stereo / BoW kernels (orb_search_for_triangulation_device).
struct KfPtrs {
    const orb_keypoint_t* kps;
    const uint4* desc;
    const int32_t* n;
    const float* u_right;
    const uint8_t* has_mp;
    const int32_t* fv_node;
    const int32_t* fv_begin;
    const int32_t* fv_feat;
    const int32_t* n_nodes;
    int32_t cap, pad;
};
struct DirectSrc {
    const KfPtrs* kfs;
    // The counts are the producers' device outputs: clamped to the keyframe's capacity, and a keyframe
    // the extractor or the BoW transform flagged (count above cap, negative FeatureVector size) fails.
    __device__ bool failed(int k) const {
        const int c = *kfs[k].n, nn = *kfs[k].n_nodes;
        return c < 0 || c > kfs[k].cap || nn < 0 || nn > kfs[k].cap;
    }
    __device__ int n(int k) const { return min(max(*kfs[k].n, 0), kfs[k].cap); }
    __device__ int n_nodes(int k) const { return min(max(*kfs[k].n_nodes, 0), kfs[k].cap); }
    __device__ uint32_t node(int k, int i) const { return (uint32_t)kfs[k].fv_node[i]; }
    __device__ int node_begin(int k, int i) const { return kfs[k].fv_begin[i]; }
    __device__ int feat(int k, int j) const { return kfs[k].fv_feat[j]; }
    __device__ KpRec kp(int k, int idx) const {
        const KfPtrs& K = kfs[k];
        const float* f = reinterpret_cast<const float*>(K.kps + idx);  // x, y, size, angle, response, octave
        const float2 xy = *reinterpret_cast<const float2*>(f);
        const int oct = reinterpret_cast<const int32_t*>(f)[5];
        const bool mp = K.has_mp && K.has_mp[idx];
        const bool st = K.u_right && K.u_right[idx] >= 0;  // bStereo = mvuRight[i] >= 0 (src:1135)
        return KpRec{xy.x, xy.y, f[3], oct | (mp ? 0x100 : 0) | (st ? 0x200 : 0)};
    }
    __device__ float angle(int k, int idx) const { return kfs[k].kps[idx].angle; }
    __device__ void descriptor(int k, int idx, uint4& a, uint4& b) const {
        a = kfs[k].desc[2 * (size_t)idx];
        b = kfs[k].desc[2 * (size_t)idx + 1];
    }
};

// matches12 row p starts at p * mstride (KF1's N for the packed form, its capacity for the device form)
// Keyframe indices of pair p: KF1 = k1of[p] (0 without the table), KF2 = k2base + p.
template <class Src>
__global__ __launch_bounds__(64 * kWaves) void k_tri_match(Src src, const PairDev* __restrict__ pairs,
                                                         const int32_t* __restrict__ k1of, int k2base, int only_stereo,
                                                         int coarse, int mstride, int32_t* __restrict__ matches) {
    const int lane = threadIdx.x & 63;
    const int node1 = blockIdx.x * kWaves + (threadIdx.x >> 6);
    const int p = blockIdx.y;
    const int K1 = k1of ? k1of[p] : 0, K2 = k2base + p;
    if (node1 >= src.n_nodes(K1) || src.failed(K1) || src.failed(K2)) return;
    const int nn2 = src.n_nodes(K2);
    // the shared-node walk of src:1112-1287 visits exactly the node ids present in both maps
    const uint32_t id = src.node(K1, node1);
    int lo = 0, hi = nn2;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (src.node(K2, mid) < id) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= nn2 || src.node(K2, lo) != id) return;
    const int b1 = src.node_begin(K1, node1), e1 = src.node_begin(K1, node1 + 1);
    const int b2 = src.node_begin(K2, lo), e2 = src.node_begin(K2, lo + 1);
    const PairDev& pd = pairs[p];
    const float F00 = pd.F[0], F01 = pd.F[1], F02 = pd.F[2], F10 = pd.F[3], F11 = pd.F[4], F12 = pd.F[5],
                F20 = pd.F[6], F21 = pd.F[7], F22 = pd.F[8];
    for (int i1 = b1 + lane; i1 < e1; i1 += 64) {
        const int idx1 = src.feat(K1, i1);
        const KpRec r1 = src.kp(K1, idx1);
        if (r1.meta & 0x100) continue;  // pMP1 != NULL (src:1127-1132)
        const bool stereo1 = (r1.meta & 0x200) != 0;
        if (only_stereo && !stereo1) continue;
        uint4 d10, d11;
        src.descriptor(K1, idx1, d10, d11);
        // epipolar line of kp1 (Pinhole.cpp:200-202), fma(x, F0j, y*F1j) + F2j as compiled upstream
        const float la = __fmaf_rn(r1.x, F00, r1.y * F10) + F20;
        const float lb = __fmaf_rn(r1.x, F01, r1.y * F11) + F21;
        const float lc = __fmaf_rn(r1.x, F02, r1.y * F12) + F22;
        int best = kThLow, bi = -1;
        for (int i2 = b2; i2 < e2; ++i2) {
            const int idx2 = src.feat(K2, i2);
            const KpRec r2 = src.kp(K2, idx2);
            if (r2.meta & 0x100) continue;  // vbMatched2[idx2] is never set (src:1158); pMP2 != NULL
            const bool stereo2 = (r2.meta & 0x200) != 0;
            if (only_stereo && !stereo2) continue;
            uint4 d20, d21;
            src.descriptor(K2, idx2, d20, d21);
            const int dist = hamming(d10, d11, d20, d21);
            if (dist > kThLow || dist > best) continue;  // src:1178
            const int oct2 = r2.meta & 0xFF;
            if (!stereo1 && !stereo2) {  // too close to the epipole (src:1190-1202)
                const float ex = pd.ep[0] - r2.x, ey = pd.ep[1] - r2.y;
                if (__fmaf_rn(ex, ex, ey * ey) < pd.scale100[oct2]) continue;
            }
            bool ok = coarse != 0;
            if (!ok) {  // Pinhole::epipolarConstrain
                const float num = __fmaf_rn(la, r2.x, lb * r2.y) + lc;
                const float den = __fmaf_rn(la, la, lb * lb);
                if (den != 0.f) {
                    const float dsqr = num * num / den;
                    ok = (double)dsqr < pd.thr[oct2];
                }
            }
            if (ok) {
                bi = idx2;
                best = dist;
            }
        }
        matches[(size_t)p * mstride + idx1] = bi;
    }
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {
    float rot = a1 - a2;  // src:1262-1266
    if ((double)rot < 0.0) rot += 360.0f;
    const float factor = 1.0f / kHistoLength;  // the reference's factor (src:1099), kept as is
    int bin = (int)roundf(rot * factor);
    if (bin == kHistoLength) bin = 0;
    return bin;
}

template <class Src>
__global__ __launch_bounds__(256) void k_tri_finish(Src src, const int32_t* __restrict__ k1of, int k2base, int check_ori,
                                                    int mstride, int32_t* __restrict__ matches,
                                                    int32_t* __restrict__ counts) {
    __shared__ int hist[kHistoLength];
    __shared__ int keep[3];
    __shared__ int total;
    const int p = blockIdx.x;
    const int K1 = k1of ? k1of[p] : 0, K2 = k2base + p;
    if (src.failed(K1) || src.failed(K2)) {  // no matches (the rows stay -1), the pair reports the failure
        if (threadIdx.x == 0) counts[p] = ORB_ERR_CAPACITY;
        return;
    }
    const int n1 = src.n(K1);
    int32_t* m = matches + (size_t)p * mstride;
    if (threadIdx.x < kHistoLength) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) total = 0;
    __syncthreads();
    int cnt = 0;
    for (int i = threadIdx.x; i < n1; i += blockDim.x) {
        const int j = m[i];
        if (j < 0) continue;
        ++cnt;
        if (check_ori) {
            const int bin = rot_bin(src.angle(K1, i), src.angle(K2, j));
            if (bin >= 0 && bin < kHistoLength) atomicAdd(&hist[bin], 1);
        }
    }
    if (check_ori) {
        __syncthreads();
        if (threadIdx.x == 0) {  // ComputeThreeMaxima (src:2336-2378)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kHistoLength; ++i) {
                const int s = hist[i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    ind3 = ind2; ind2 = ind1; ind1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    ind3 = ind2; ind2 = i;
                } else if (s > max3) {
                    max3 = s; ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) ind3 = -1;
            keep[0] = ind1; keep[1] = ind2; keep[2] = ind3;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < n1; i += blockDim.x) {
            const int j = m[i];
            if (j < 0) continue;
            const int bin = rot_bin(src.angle(K1, i), src.angle(K2, j));
            if (bin != keep[0] && bin != keep[1] && bin != keep[2]) {
                m[i] = -1;
                --cnt;
            }
        }
    }
    atomicAdd(&total, cnt);
    __syncthreads();
    if (threadIdx.x == 0) counts[p] = total;
}

// ---- host-side float geometry -------------------------------------------------------------------

// Eigen's closed-form 3x3 inverse (Eigen/src/LU/InverseImpl.h, compute_inverse<.., 3>): signed
// cofactors by cyclic indices, det from the first column, inv(i, j) = cofactor(j, i) / det.
void inverse3(const float m[9], float out[9]) {
    auto at = [&](int r, int c) { return m[3 * r + c]; };
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return std::fma(at(i1, j1), at(i2, j2), -(at(i1, j2) * at(i2, j1)));
    };
    const float c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const float det = std::fma(c2, at(2, 0), std::fma(c0, at(0, 0), c1 * at(1, 0)));
    const float invdet = 1.0f / det;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out[3 * i + j] = cof(j, i) * invdet;
}

// 3x3 float product; each coefficient is the unrolled 3-term redux as g++ contracts it.
void matmul3(const float a[9], const float b[9], float out[9]) {
    float t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            t[3 * i + j] = std::fma(a[3 * i + 2], b[6 + j], std::fma(a[3 * i], b[j], a[3 * i + 1] * b[3 + j]));
    memcpy(out, t, sizeof(t));
}

// F12 = K1^-T * [t12]x * R12 * K2^-1 (Pinhole.cpp:191-194); k = fx, fy, cx, cy.
void fundamental(const float k1[4], const float k2[4], const orb_kf_pair_geom_t& g, float F[9]) {
    const float K1t[9] = {k1[0], 0.f, 0.f, 0.f, k1[1], 0.f, k1[2], k1[3], 1.f};
    const float K2[9] = {k2[0], 0.f, k2[2], 0.f, k2[1], k2[3], 0.f, 0.f, 1.f};
    const float* t = g.t12;
    const float tx[9] = {0.f, -t[2], t[1], t[2], 0.f, -t[0], -t[1], t[0], 0.f};  // Sophus::SO3f::hat
    float K1ti[9], K2i[9];
    inverse3(K1t, K1ti);
    inverse3(K2, K2i);
    matmul3(K1ti, tx, F);
    matmul3(F, g.R12, F);
    matmul3(F, K2i, F);
}

bool check_view(const orb_kf_view_t* v, bool first) {
    if (!v || v->n < 0 || v->n_nodes < 0 || v->nlevels <= 0 || v->nlevels > kMaxLevels) return false;
    if (v->n > 0 && (!v->kps_un || !v->desc)) return false;
    if (v->n_nodes > 0 && (!v->fv_node || !v->fv_offset || !v->fv_index)) return false;
    if (!v->scale_factors || !v->level_sigma2) return false;
    if (v->n_nodes > 0 && v->fv_offset[0] != 0) return false;
    for (int i = 0; i < v->n_nodes; ++i) {
        if (v->fv_offset[i + 1] < v->fv_offset[i]) return false;
        if (i > 0 && v->fv_node[i] <= v->fv_node[i - 1]) return false;
    }
    const int nidx = v->n_nodes > 0 ? v->fv_offset[v->n_nodes] : 0;
    std::vector<uint8_t> seen(first ? v->n : 0, 0);
    for (int i = 0; i < nidx; ++i) {
        const int j = v->fv_index[i];
        if (j < 0 || j >= v->n) return false;
        if (first) {  // a DBoW2 FeatureVector lists each feature once
            if (seen[j]) return false;
            seen[j] = 1;
        }
    }
    for (int i = 0; i < v->n; ++i)
        if (v->kps_un[i].octave < 0 || v->kps_un[i].octave >= v->nlevels) return false;
    return true;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// The per-pair constants of k_tri_match: F12, the epipole, 100 * scale (src:1193), 3.84 sigma2 (Pinhole.cpp:215).
PairDev make_pair(const float k1[4], const float k2[4], int nlevels2, const float* scale2, const float* sigma2_2,
                  const orb_kf_pair_geom_t& g) {
    PairDev d{};
    fundamental(k1, k2, g, d.F);
    d.ep[0] = g.ep[0];
    d.ep[1] = g.ep[1];
    for (int l = 0; l < kMaxLevels; ++l) {
        d.scale100[l] = l < nlevels2 ? 100 * scale2[l] : 0.f;
        d.thr[l] = l < nlevels2 ? 3.84 * (double)sigma2_2[l] : 0.0;
    }
    return d;
}

}  // namespace

struct orb_matcher_s {
    float nnratio = 0.6f;
    int check_ori = 1;
    hipStream_t stream = nullptr;
    // pinned upload slot of the device-resident entry points; `dev_ev` marks the end of its last copy
    char* h_dev = nullptr;
    size_t h_dev_cap = 0;
    hipEvent_t dev_ev = nullptr;
    char* d_buf = nullptr;
    size_t d_cap = 0;
    char* h_buf = nullptr;
    size_t h_cap = 0;

    int reserve(size_t bytes) {
        if (bytes > d_cap) {
            if (d_buf) hipFree(d_buf);
            d_buf = nullptr;
            d_cap = 0;
            if (hipMalloc(&d_buf, bytes) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "matcher device alloc");
            d_cap = bytes;
        }
        if (bytes > h_cap) {
            if (h_buf) hipHostFree(h_buf);
            h_buf = nullptr;
            h_cap = 0;
            if (hipHostMalloc(&h_buf, bytes, hipHostMallocDefault) != hipSuccess)
                return orbgpu_fail(ORB_ERR_DEVICE, "matcher pinned alloc");
            h_cap = bytes;
        }
        return ORB_OK;
    }
};

// Staging buffers of a matcher handle for the other matcher entry points (orb_projection.hip).
int orbgpu_matcher_reserve(orb_matcher_t m, size_t bytes, char** d_buf, char** h_buf, hipStream_t* stream,
                           int* check_ori) {
    if (int rc = m->reserve(bytes)) return rc;
    *d_buf = m->d_buf;
    *h_buf = m->h_buf;
    *stream = m->stream;
    *check_ori = m->check_ori;
    return ORB_OK;
}

float orbgpu_matcher_nnratio(orb_matcher_t m) { return m->nnratio; }
int orbgpu_matcher_check_ori(orb_matcher_t m) { return m->check_ori; }

extern "C" {

int orb_matcher_create(float nnratio, int check_orientation, orb_matcher_t* out) {
    if (!out) return orbgpu_fail(ORB_ERR_ARG, "null handle pointer");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return orbgpu_fail(ORB_ERR_DEVICE, "no HIP device");
    }
    auto* m = new orb_matcher_s();
    m->nnratio = nnratio;
    m->check_ori = check_orientation ? 1 : 0;
    if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) {
        delete m;
        return orbgpu_fail(ORB_ERR_DEVICE, "stream create");
    }
    *out = m;
    return ORB_OK;
}

int orb_matcher_destroy(orb_matcher_t m) {
    if (!m) return ORB_OK;
    if (m->stream) hipStreamSynchronize(m->stream);
    if (m->dev_ev) {
        hipEventSynchronize(m->dev_ev);
        hipEventDestroy(m->dev_ev);
    }
    if (m->h_dev) hipHostFree(m->h_dev);
    if (m->d_buf) hipFree(m->d_buf);
    if (m->h_buf) hipHostFree(m->h_buf);
    if (m->stream) hipStreamDestroy(m->stream);
    delete m;
    return ORB_OK;
}

// T12 = T1w * T2w^-1, C2 = T2w * Cw1 with Cw1 = -R1w^T t1w, ep = project(C2) (Pinhole.cpp:61-68).
int orb_kf_pair_geometry(const float T1w[12], const float T2w[12], float fx2, float fy2, float cx2, float cy2,
                         orb_kf_pair_geom_t* out) {
    if (!T1w || !T2w || !out) return orbgpu_fail(ORB_ERR_ARG, "null pose");
    auto R1 = [&](int r, int c) { return T1w[4 * r + c]; };
    auto R2 = [&](int r, int c) { return T2w[4 * r + c]; };
    float tw2[3];  // Tw2 translation = -R2^T t2
    for (int i = 0; i < 3; ++i) tw2[i] = -(R2(0, i) * T2w[3] + R2(1, i) * T2w[7] + R2(2, i) * T2w[11]);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) out->R12[3 * i + j] = R1(i, 0) * R2(j, 0) + R1(i, 1) * R2(j, 1) + R1(i, 2) * R2(j, 2);
        out->t12[i] = R1(i, 0) * tw2[0] + R1(i, 1) * tw2[1] + R1(i, 2) * tw2[2] + T1w[4 * i + 3];
    }
    float cw[3], c2[3];
    for (int i = 0; i < 3; ++i) cw[i] = -(R1(0, i) * T1w[3] + R1(1, i) * T1w[7] + R1(2, i) * T1w[11]);
    for (int i = 0; i < 3; ++i) c2[i] = R2(i, 0) * cw[0] + R2(i, 1) * cw[1] + R2(i, 2) * cw[2] + T2w[4 * i + 3];
    out->ep[0] = fx2 * c2[0] / c2[2] + cx2;
    out->ep[1] = fy2 * c2[1] / c2[2] + cy2;
    return ORB_OK;
}

int orb_search_for_triangulation(orb_matcher_t m, const orb_kf_view_t* kf1, const orb_kf_view_t* kf2s,
                                 const orb_kf_pair_geom_t* geoms, int n_pairs, int only_stereo, int coarse,
                                 int32_t* matches12, int32_t* n_matches) {
    if (!m || !kf1 || n_pairs < 0 || (n_pairs > 0 && (!kf2s || !geoms || !n_matches)))
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchForTriangulation arguments");
    if (n_pairs == 0) return ORB_OK;
    if (kf1->n > 0 && !matches12) return orbgpu_fail(ORB_ERR_ARG, "null matches12");
    if (!check_view(kf1, true)) return orbgpu_fail(ORB_ERR_ARG, "invalid keyframe 1 view");
    for (int p = 0; p < n_pairs; ++p)
        if (!check_view(&kf2s[p], false)) return orbgpu_fail(ORB_ERR_ARG, "invalid keyframe 2 view");

    const int nkf = n_pairs + 1;
    auto view = [&](int k) -> const orb_kf_view_t& { return k == 0 ? *kf1 : kf2s[k - 1]; };
    std::vector<KfDev> kd(nkf);
    size_t nkp = 0, nnode = 0, ncsr = 0, nidx = 0;
    for (int k = 0; k < nkf; ++k) {
        const orb_kf_view_t& v = view(k);
        kd[k] = KfDev{v.n, v.n_nodes, (int32_t)nkp, (int32_t)nnode, (int32_t)ncsr, {0, 0, 0}};
        nkp += v.n;
        nnode += v.n_nodes;
        ncsr += v.n_nodes + 1;
        nidx += v.n_nodes ? v.fv_offset[v.n_nodes] : 0;
    }
    if (nkp >= (size_t)INT32_MAX / 2 || nidx >= (size_t)INT32_MAX) return orbgpu_fail(ORB_ERR_ARG, "problem too large");
    // packed layout (one H2D copy): kfs | pairs | kps | desc | nodes | csr | idx | matches | counts
    size_t off = 0;
    const size_t o_kf = off; off = align256(off + nkf * sizeof(KfDev));
    const size_t o_pair = off; off = align256(off + n_pairs * sizeof(PairDev));
    const size_t o_kp = off; off = align256(off + nkp * sizeof(KpRec));
    const size_t o_desc = off; off = align256(off + nkp * 32);
    const size_t o_node = off; off = align256(off + nnode * 4);
    const size_t o_csr = off; off = align256(off + ncsr * 4);
    const size_t o_idx = off; off = align256(off + nidx * 4);
    const size_t o_match = off; off = align256(off + (size_t)n_pairs * kf1->n * 4);  // -1 from the host, uploaded
    const size_t in_bytes = off;
    const size_t o_cnt = off; off = align256(off + (size_t)n_pairs * 4);
    if (int rc = m->reserve(off)) return rc;

    char* h = m->h_buf;
    memcpy(h + o_kf, kd.data(), nkf * sizeof(KfDev));
    auto* pd = reinterpret_cast<PairDev*>(h + o_pair);
    const float K1[4] = {kf1->fx, kf1->fy, kf1->cx, kf1->cy};
    for (int p = 0; p < n_pairs; ++p) {
        const orb_kf_view_t& v2 = kf2s[p];
        const float K2[4] = {v2.fx, v2.fy, v2.cx, v2.cy};
        pd[p] = make_pair(K1, K2, v2.nlevels, v2.scale_factors, v2.level_sigma2, geoms[p]);
    }
    auto* kp = reinterpret_cast<KpRec*>(h + o_kp);
    auto* nodes = reinterpret_cast<uint32_t*>(h + o_node);
    auto* csr = reinterpret_cast<int32_t*>(h + o_csr);
    auto* idx = reinterpret_cast<int32_t*>(h + o_idx);
    size_t ik = 0, in = 0, ic = 0, ii = 0;
    for (int k = 0; k < nkf; ++k) {
        const orb_kf_view_t& v = view(k);
        for (int i = 0; i < v.n; ++i) {
            const orb_keypoint_t& s = v.kps_un[i];
            const bool mp = v.has_mappoint && v.has_mappoint[i];
            const bool st = v.u_right && v.u_right[i] >= 0;  // bStereo = mvuRight[i] >= 0 (src:1135)
            kp[ik + i] = KpRec{s.x, s.y, s.angle, s.octave | (mp ? 0x100 : 0) | (st ? 0x200 : 0)};
        }
        if (v.n) memcpy(h + o_desc + ik * 32, v.desc, (size_t)v.n * 32);
        if (v.n_nodes) {
            memcpy(nodes + in, v.fv_node, v.n_nodes * 4);
            for (int i = 0; i <= v.n_nodes; ++i) csr[ic + i] = (int32_t)ii + v.fv_offset[i];
            memcpy(idx + ii, v.fv_index, (size_t)v.fv_offset[v.n_nodes] * 4);
            ii += v.fv_offset[v.n_nodes];
        }
        ik += v.n;
        in += v.n_nodes;
        ic += v.n_nodes + 1;
    }

    char* d = m->d_buf;
    hipStream_t s = m->stream;
    memset(h + o_match, 0xFF, (size_t)n_pairs * kf1->n * 4);
    bool ok = hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s) == hipSuccess;
    const PackedSrc src{(const KfDev*)(d + o_kf), (const KpRec*)(d + o_kp), (const uint4*)(d + o_desc),
                        (const uint32_t*)(d + o_node), (const int32_t*)(d + o_csr), (const int32_t*)(d + o_idx)};
    if (ok && kf1->n_nodes > 0) {
        hipLaunchKernelGGL(k_tri_match<PackedSrc>, dim3((kf1->n_nodes + kWaves - 1) / kWaves, n_pairs), dim3(64 * kWaves),
                           0, s, src, (const PairDev*)(d + o_pair), (const int32_t*)nullptr, 1, only_stereo ? 1 : 0,
                           coarse ? 1 : 0, kf1->n, (int32_t*)(d + o_match));
        ok = hipGetLastError() == hipSuccess;
    }
    if (ok) {
        hipLaunchKernelGGL(k_tri_finish<PackedSrc>, dim3(n_pairs), dim3(256), 0, s, src, (const int32_t*)nullptr, 1,
                           m->check_ori, kf1->n, (int32_t*)(d + o_match), (int32_t*)(d + o_cnt));
        ok = hipGetLastError() == hipSuccess;
    }
    ok = ok && hipMemcpyAsync(h + o_match, d + o_match, o_cnt + (size_t)n_pairs * 4 - o_match, hipMemcpyDeviceToHost,
                              s) == hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "SearchForTriangulation device error");
    if (kf1->n) memcpy(matches12, h + o_match, (size_t)n_pairs * kf1->n * 4);
    memcpy(n_matches, h + o_cnt, (size_t)n_pairs * 4);
    return ORB_OK;
}

int orb_search_for_triangulation_device(orb_matcher_t m, const orb_kf_device_t* kf1s, int n_kf1,
                                        const orb_kf_device_t* kf2s, const int32_t* pair_kf1,
                                        const orb_kf_pair_geom_t* geoms, int n_pairs, int only_stereo, int coarse,
                                        int32_t* d_matches12, int32_t* d_n_matches, void* stream) {
    if (!m || !kf1s || n_kf1 <= 0 || n_pairs < 0 || (n_pairs > 0 && (!kf2s || !geoms || !d_matches12 || !d_n_matches)))
        return orbgpu_fail(ORB_ERR_ARG, "bad SearchForTriangulation arguments");
    if (n_pairs == 0) return ORB_OK;
    auto bad = [](const orb_kf_device_t& k) {
        return k.cap <= 0 || !k.kps || !k.desc || !k.n || !k.fv_node || !k.fv_begin || !k.fv_feat || !k.n_nodes ||
               k.nlevels <= 0 || k.nlevels > kMaxLevels || !k.scale_factors || !k.level_sigma2 ||
               (reinterpret_cast<uintptr_t>(k.desc) & 15) != 0;
    };
    int C = 0;
    for (int k = 0; k < n_kf1; ++k) {
        if (bad(kf1s[k])) return orbgpu_fail(ORB_ERR_ARG, "invalid keyframe 1 device view");
        C = std::max(C, kf1s[k].cap);
    }
    for (int p = 0; p < n_pairs; ++p) {
        if (bad(kf2s[p])) return orbgpu_fail(ORB_ERR_ARG, "invalid keyframe 2 device view");
        if (pair_kf1 && (pair_kf1[p] < 0 || pair_kf1[p] >= n_kf1)) return orbgpu_fail(ORB_ERR_ARG, "bad pair_kf1");
    }
    hipStream_t s = (hipStream_t)stream;
    const int nkf = n_kf1 + n_pairs;
    // upload: KfPtrs [n_kf1 first keyframes | n_pairs neighbours] | PairDev [n_pairs] | kf1 index per pair
    const size_t o_pair = align256(nkf * sizeof(KfPtrs)), o_k1 = o_pair + align256(n_pairs * sizeof(PairDev));
    const size_t bytes = o_k1 + align256(4 * (size_t)n_pairs);
    // the pinned slot: wait until the previous call's upload has left it
    if (!m->dev_ev && hipEventCreateWithFlags(&m->dev_ev, hipEventDisableTiming) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "event create");
    if (hipEventSynchronize(m->dev_ev) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "device error");
    if (bytes > m->h_dev_cap) {
        if (m->h_dev) hipHostFree(m->h_dev);
        m->h_dev = nullptr;
        m->h_dev_cap = 0;
        if (hipHostMalloc(&m->h_dev, bytes, hipHostMallocDefault) != hipSuccess)
            return orbgpu_fail(ORB_ERR_DEVICE, "matcher pinned alloc");
        m->h_dev_cap = bytes;
    }
    auto* kp = reinterpret_cast<KfPtrs*>(m->h_dev);
    auto* pd = reinterpret_cast<PairDev*>(m->h_dev + o_pair);
    auto* k1 = reinterpret_cast<int32_t*>(m->h_dev + o_k1);
    for (int k = 0; k < nkf; ++k) {
        const orb_kf_device_t& v = k < n_kf1 ? kf1s[k] : kf2s[k - n_kf1];
        kp[k] = KfPtrs{v.kps, reinterpret_cast<const uint4*>(v.desc), v.n, v.u_right, v.has_mappoint, v.fv_node,
                       v.fv_begin, v.fv_feat, v.n_nodes, v.cap, 0};
    }
    for (int p = 0; p < n_pairs; ++p) {
        const orb_kf_device_t& v1 = kf1s[pair_kf1 ? pair_kf1[p] : 0];
        const orb_kf_device_t& v2 = kf2s[p];
        const float K1[4] = {v1.fx, v1.fy, v1.cx, v1.cy}, K2[4] = {v2.fx, v2.fy, v2.cx, v2.cy};
        pd[p] = make_pair(K1, K2, v2.nlevels, v2.scale_factors, v2.level_sigma2, geoms[p]);
        k1[p] = pair_kf1 ? pair_kf1[p] : 0;
    }
    // device copy, stream-ordered (calls on different streams do not share it)
    char* d = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&d), bytes, s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    bool ok = hipMemcpyAsync(d, m->h_dev, bytes, hipMemcpyHostToDevice, s) == hipSuccess &&
              hipEventRecord(m->dev_ev, s) == hipSuccess &&
              hipMemsetAsync(d_matches12, 0xFF, (size_t)n_pairs * C * 4, s) == hipSuccess;
    const DirectSrc src{reinterpret_cast<const KfPtrs*>(d)};
    const int32_t* k1of = reinterpret_cast<const int32_t*>(d + o_k1);
    if (ok) {  // node1 < *n_nodes <= cap: the grid covers the capacity, waves past the count return
        hipLaunchKernelGGL(k_tri_match<DirectSrc>, dim3((C + kWaves - 1) / kWaves, n_pairs), dim3(64 * kWaves), 0, s, src,
                           reinterpret_cast<const PairDev*>(d + o_pair), k1of, n_kf1, only_stereo ? 1 : 0,
                           coarse ? 1 : 0, C, d_matches12);
        hipLaunchKernelGGL(k_tri_finish<DirectSrc>, dim3(n_pairs), dim3(256), 0, s, src, k1of, n_kf1, m->check_ori, C,
                           d_matches12, d_n_matches);
        ok = hipGetLastError() == hipSuccess;
    }
    if (hipFreeAsync(d, s) != hipSuccess) ok = false;
    return ok ? ORB_OK : orbgpu_fail(ORB_ERR_DEVICE, "SearchForTriangulation device error");
}

}  // extern "C"
