// The glue of the device-resident tracking chain (Tracking::TrackWithMotionModel -> TrackLocalMap,
// reference src/Tracking.cc:4112-4217, 4234-4300, 4742-4825): the steps between the matchers and
// PoseOptimization that the reference runs on its Frame object, restated for device arrays so that a
// tracked frame makes no host round trip between
//   SearchByProjection(F, LastFrame)  -> PoseOptimization -> discard outliers -> isInFrustum
//   -> SearchByProjection(F, local map points) -> PoseOptimization.
//   k_track_pose_edges    Optimizer::PoseOptimization's graph (src/Optimizer.cc:93-180): one unary edge
//                         per keypoint i < N that holds a map point, in keypoint order (a stable
//                         compaction), mono when mvuRight[i] < 0, information mvInvLevelSigma2[octave];
//                         the start pose is the frame's (host) or the previous optimisation's (device).
//   k_track_discard       TrackWithMotionModel's outlier discard (src/Tracking.cc:4180-4203): a keypoint
//                         whose edge came back an outlier loses its map point; counts nmatchesMap.
//   k_track_gate_*        TrackWithMotionModel's decisions (src/Tracking.cc:4149-4217) on the device: the
//                         2 th retry of the search, and the frame's failure (< 20 matches after it, or
//                         nmatchesMap < 10 after PoseOptimization).  They write per-frame gated counts --
//                         the frame's keypoint count, or 0 -- that the later stages read in place of the
//                         frame's own count: a stage on a 0-keypoint frame builds no grid, finds no
//                         match and no edge, so a failed frame's remaining launches do no work and
//                         write the "not run" outputs, with no host round trip and no change to the
//                         stage kernels.
// Map points are referenced by index into a device table of world positions (float xyz, as
// MapPoint::GetWorldPos returns them); a keypoint's map point comes from the second match array when it
// has one there (SearchByProjection(F, local points) overwrites, src/ORBmatcher.cc:156), else the first.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>
#include <unordered_map>
#include <mutex>

#include <cstdint>
#include <cstring>

#include "orbgpu.h"
#include "orb_pose_frame.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kThreads = 1024, kMaxLevels = 12;

struct EdgeParams {
    float inv_sigma2[kMaxLevels];
    int nlevels, cap, has_pose_dev, has_b;
    int edge_begin;  // the frame record's edge_begin (a batch's frame b: b cap into the batch's edge array)
    double pose[7];
    orb_ba_camera_t cam;
};

__device__ __forceinline__ void k_track_pose_edges_body(EdgeParams P, const orb_keypoint_t* __restrict__ kps,
                                                                const float* __restrict__ u_right,
                                                                const int32_t* __restrict__ n_ptr,
                                                                const int32_t* __restrict__ match_a,
                                                                const float* __restrict__ xyz_a,
                                                                const int32_t* __restrict__ match_b,
                                                                const float* __restrict__ xyz_b,
                                                                const double* __restrict__ pose_dev,
                                                                orb_pose_frame_t* __restrict__ frame,
                                                                orb_pose_edge_t* __restrict__ edges,
                                                                int32_t* __restrict__ edge_kp) {
    __shared__ int part[kThreads];
    const int tid = threadIdx.x;
    const int n = min(max(*n_ptr, 0), P.cap);
    const int per = (n + kThreads - 1) / kThreads;  // each thread a contiguous run of keypoints (order kept)
    const int b0 = min(tid * per, n), b1 = min(b0 + per, n);
    auto point_of = [&](int i, const float*& xyz) {
        const int mb = P.has_b ? match_b[i] : -1;
        if (mb >= 0) { xyz = xyz_b; return mb; }
        xyz = xyz_a;
        return match_a[i];
    };
    int cnt = 0;
    for (int i = b0; i < b1; ++i) {
        const float* t;
        cnt += point_of(i, t) >= 0;
    }
    part[tid] = cnt;
    __syncthreads();
    for (int o = 1; o < kThreads; o <<= 1) {
        const int v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int e = part[tid] - cnt;
    for (int i = b0; i < b1; ++i) {
        const float* xyz;
        const int p = point_of(i, xyz);
        if (p < 0) continue;
        const orb_keypoint_t kp = kps[i];
        orb_pose_edge_t E;
        E.xw[0] = (double)xyz[3 * (size_t)p];
        E.xw[1] = (double)xyz[3 * (size_t)p + 1];
        E.xw[2] = (double)xyz[3 * (size_t)p + 2];
        const float ur = u_right ? u_right[i] : -1.0f;
        E.stereo = ur >= 0 ? 1 : 0;  // src/Optimizer.cc:103 (mono), :140 (stereo)
        E.obs[0] = kp.x;
        E.obs[1] = kp.y;
        E.obs[2] = E.stereo ? (double)ur : 0.0;
        const int oct = min(max(kp.octave, 0), P.nlevels - 1);
        E.inv_sigma2 = P.inv_sigma2[oct];
        edges[e] = E;
        edge_kp[e] = i;
        ++e;
    }
    if (tid == kThreads - 1) {
        orb_pose_frame_t F;
        if (P.has_pose_dev) {  // the previous optimisation's pose as the Frame kept it (float, Sophus)
            double p[7];
            for (int k = 0; k < 7; ++k) p[k] = pose_dev[k];
            orb_pose7_float_roundtrip(p, F.pose);
        } else {
            for (int k = 0; k < 7; ++k) F.pose[k] = P.pose[k];
        }
        F.cam = P.cam;
        F.edge_begin = P.edge_begin;
        F.n_edges = part[kThreads - 1];
        *frame = F;
    }
}
__global__ __launch_bounds__(kThreads) void k_track_pose_edges(EdgeParams P, const orb_keypoint_t* __restrict__ kps,
                                                                const float* __restrict__ u_right,
                                                                const int32_t* __restrict__ n_ptr,
                                                                const int32_t* __restrict__ match_a,
                                                                const float* __restrict__ xyz_a,
                                                                const int32_t* __restrict__ match_b,
                                                                const float* __restrict__ xyz_b,
                                                                const double* __restrict__ pose_dev,
                                                                orb_pose_frame_t* __restrict__ frame,
                                                                orb_pose_edge_t* __restrict__ edges,
                                                                int32_t* __restrict__ edge_kp) {
    k_track_pose_edges_body(P, kps, u_right, n_ptr, match_a, xyz_a, match_b, xyz_b, pose_dev, frame, edges, edge_kp);
}
struct k_track_pose_edges_args {
    EdgeParams P;
    const orb_keypoint_t* kps;
    const float* u_right;
    const int32_t* n_ptr;
    const int32_t* match_a;
    const float* xyz_a;
    const int32_t* match_b;
    const float* xyz_b;
    const double* pose_dev;
    orb_pose_frame_t* frame;
    orb_pose_edge_t* edges;
    int32_t* edge_kp;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(kThreads) void k_track_pose_edges_b(const k_track_pose_edges_args* __restrict__ a) {
    const k_track_pose_edges_args& A = a[blockIdx.y];
    k_track_pose_edges_body(A.P, A.kps, A.u_right, A.n_ptr, A.match_a, A.xyz_a, A.match_b, A.xyz_b, A.pose_dev, A.frame,
                            A.edges, A.edge_kp);
}

// outliers lose their map point; n_out[0] = the edges kept, n_out[1] = those whose map point has
// observations (nmatchesMap, src/Tracking.cc:4198-4200)
__device__ __forceinline__ void k_track_discard_body(const orb_pose_frame_t* __restrict__ frame,
                                                       const int32_t* __restrict__ edge_kp,
                                                       const uint8_t* __restrict__ outlier, int32_t* __restrict__ match_a,
                                                       const uint8_t* __restrict__ observed_a, int32_t* __restrict__ match_b,
                                                       const uint8_t* __restrict__ observed_b, int32_t* __restrict__ n_out,
                                                       int cap, uint8_t* __restrict__ taken) {
    __shared__ int keep, obs;
    if (threadIdx.x == 0) keep = obs = 0;
    __syncthreads();
    const int ne = frame->n_edges;
    int k = 0, o = 0;
    for (int e = threadIdx.x; e < ne; e += kThreads) {
        const int i = edge_kp[e];
        const int mb = match_b ? match_b[i] : -1;
        if (outlier[e]) {
            match_a[i] = -1;
            if (match_b) match_b[i] = -1;
            continue;
        }
        ++k;
        o += mb >= 0 ? (observed_b ? observed_b[mb] != 0 : 1) : (observed_a ? observed_a[match_a[i]] != 0 : 1);
    }
    for (int off = 32; off > 0; off >>= 1) {  // wave sums, then one LDS atomic per wave
        k += __shfl_xor(k, off, 64);
        o += __shfl_xor(o, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&keep, k);
        atomicAdd(&obs, o);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        n_out[0] = keep;
        n_out[1] = obs;
    }
    if (!taken) return;
    // SearchLocalPoints' skip set for the local-map search (src/ORBmatcher.cc:103-105): the keypoints
    // that now hold a map point with observations
    __threadfence_block();
    __syncthreads();
    for (int i = threadIdx.x; i < cap; i += kThreads) {
        const int mb = match_b ? match_b[i] : -1, ma = match_a[i];
        uint8_t t = 0;
        if (mb >= 0) t = observed_b ? observed_b[mb] != 0 : 1;
        else if (ma >= 0) t = observed_a ? observed_a[ma] != 0 : 1;
        taken[i] = t;
    }
}
__global__ __launch_bounds__(kThreads) void k_track_discard(const orb_pose_frame_t* __restrict__ frame,
                                                       const int32_t* __restrict__ edge_kp,
                                                       const uint8_t* __restrict__ outlier, int32_t* __restrict__ match_a,
                                                       const uint8_t* __restrict__ observed_a, int32_t* __restrict__ match_b,
                                                       const uint8_t* __restrict__ observed_b, int32_t* __restrict__ n_out,
                                                       int cap, uint8_t* __restrict__ taken) {
    k_track_discard_body(frame, edge_kp, outlier, match_a, observed_a, match_b, observed_b, n_out, cap, taken);
}
struct k_track_discard_args {
    const orb_pose_frame_t* frame;
    const int32_t* edge_kp;
    const uint8_t* outlier;
    int32_t* match_a;
    const uint8_t* observed_a;
    int32_t* match_b;
    const uint8_t* observed_b;
    int32_t* n_out;
    int cap;
    uint8_t* taken;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(kThreads) void k_track_discard_b(const k_track_discard_args* __restrict__ a) {
    const k_track_discard_args& A = a[blockIdx.y];
    k_track_discard_body(A.frame, A.edge_kp, A.outlier, A.match_a, A.observed_a, A.match_b, A.observed_b, A.n_out,
                         A.cap, A.taken);
}

// SearchLocalPoints' first loop (src/Tracking.cc:4250-4266): a local map point the frame already holds
// (mnLastFrameSeen == mCurrentFrame.mnId) is not tested against the frustum.  With the local map as its own
// table, local point j is the last frame's row last_row[j] (-1: a point the last frame does not track);
// the rows the frame still holds after the discard go into an LDS bitmap.
constexpr int kSeenBits = 16384;

__device__ __forceinline__ void k_track_local_seen_body(const int32_t* __restrict__ match_a, int cap, int last_cap,
                                                                const int32_t* __restrict__ last_row, int n_local,
                                                                uint8_t* __restrict__ in_view) {
    __shared__ uint32_t bits[kSeenBits / 32];
    for (int w = threadIdx.x; w < kSeenBits / 32; w += kThreads) bits[w] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < cap; i += kThreads) {
        const int k = match_a[i];
        if (k >= 0 && k < last_cap) atomicOr(&bits[k >> 5], 1u << (k & 31));
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n_local; j += kThreads) {
        const int r = last_row[j];
        if (r >= 0 && r < last_cap && ((bits[r >> 5] >> (r & 31)) & 1u)) in_view[j] = 0;
    }
}
__global__ __launch_bounds__(kThreads) void k_track_local_seen(const int32_t* __restrict__ match_a, int cap, int last_cap,
                                                                const int32_t* __restrict__ last_row, int n_local,
                                                                uint8_t* __restrict__ in_view) {
    k_track_local_seen_body(match_a, cap, last_cap, last_row, n_local, in_view);
}
struct k_track_local_seen_args {
    const int32_t* match_a;
    int cap;
    int last_cap;
    const int32_t* last_row;
    int n_local;
    uint8_t* in_view;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(kThreads) void k_track_local_seen_b(const k_track_local_seen_args* __restrict__ a) {
    const k_track_local_seen_args& A = a[blockIdx.y];
    k_track_local_seen_body(A.match_a, A.cap, A.last_cap, A.last_row, A.n_local, A.in_view);
}

// ---- TrackWithMotionModel's decisions (src/Tracking.cc:4149-4217)
constexpr int kMinMotionMatches = 20;  // nmatches < 20: the 2 th search, then failure (:4153, :4163)
constexpr int kMinMapMatches = 10;     // return nmatchesMap >= 10 (:4216)

// Per frame: the counts the gated stages read as their frame's (or last frame's) keypoint count, the
// 2 th search's count, and its matches at m1w (cap entries) in the scratch.
struct ChainGate {
    int32_t n_wide;    // the 2 th search's current-frame count: N when it runs, else 0
    int32_t nl_wide;   // its last-frame count
    int32_t n_alive1;  // PoseOptimization's graph / the discard: N unless the search failed
    int32_t n_alive2;  // the local-map stages: N unless TrackWithMotionModel failed
    int32_t n1w;       // the 2 th search's match count
    int32_t status;    // ORB_TRACK_* bits (copied to the caller's status word)
    int32_t pad[2];
};
static_assert(sizeof(ChainGate) == 32, "gate record");

struct GateArgs {
    ChainGate* g;
    const int32_t* cur_n;     // the frame's keypoint count (device)
    const int32_t* last_n;    // the last frame's
    int32_t* n1;              // SearchByProjection(LastFrame)'s count (n_match[0])
    int32_t* m1;              // its matches (cap)
    const int32_t* m1w;       // the 2 th search's matches (cap)
    const orb_pose_frame_t* frame1;
    const int32_t* edge_kp1;
    const uint8_t* outlier1;
    const uint8_t* observed;  // the last frame's map points' Observations() > 0 (NULL: all)
    int32_t* status;          // the caller's status word, or NULL
    int cap;
};

// after the first search: < 20 matches -> the 2 th search runs (its counts are the frame's)
__device__ __forceinline__ void k_track_gate_retry_body(const GateArgs& a) {
    if (threadIdx.x) return;
    const bool retry = *a.n1 < kMinMotionMatches;
    a.g->n_wide = retry ? *a.cur_n : 0;
    a.g->nl_wide = retry ? *a.last_n : 0;
    a.g->status = retry ? ORB_TRACK_RETRIED : 0;
}
__global__ __launch_bounds__(64) void k_track_gate_retry(GateArgs a) { k_track_gate_retry_body(a); }
__global__ __launch_bounds__(64) void k_track_gate_retry_b(const GateArgs* __restrict__ a) {
    k_track_gate_retry_body(a[blockIdx.y]);
}

// after the 2 th search: its matches replace the first ones (Tracking.cc:4156-4158 clears and searches
// again); still < 20 -> TrackWithMotionModel returns false (:4161-4168): no graph, no local-map stages
__device__ __forceinline__ void k_track_gate_search_body(const GateArgs& a) {
    const int st = a.g->status;
    if (st & ORB_TRACK_RETRIED)
        for (int i = threadIdx.x; i < a.cap; i += kThreads) a.m1[i] = a.m1w[i];
    __syncthreads();
    if (threadIdx.x) return;
    int n = *a.n1;
    if (st & ORB_TRACK_RETRIED) *a.n1 = n = a.g->n1w;
    const bool ok = n >= kMinMotionMatches;
    a.g->n_alive1 = a.g->n_alive2 = ok ? *a.cur_n : 0;
    a.g->status = ok ? st : (st | ORB_TRACK_FAIL_SEARCH);
    if (a.status) *a.status = a.g->status;
}
__global__ __launch_bounds__(kThreads) void k_track_gate_search(GateArgs a) { k_track_gate_search_body(a); }
__global__ __launch_bounds__(kThreads) void k_track_gate_search_b(const GateArgs* __restrict__ a) {
    k_track_gate_search_body(a[blockIdx.y]);
}

// after the first PoseOptimization: nmatchesMap (the kept edges whose map point has observations,
// :4176-4203, as the discard counts it) < 10 -> TrackWithMotionModel returns false (:4216)
__device__ __forceinline__ void k_track_gate_map_body(const GateArgs& a) {
    __shared__ int obs;
    const int st = a.g->status;
    if (st & ORB_TRACK_FAIL_SEARCH) return;  // (uniform: the whole block leaves)
    if (threadIdx.x == 0) obs = 0;
    __syncthreads();
    const int ne = a.frame1->n_edges;
    int o = 0;
    for (int e = threadIdx.x; e < ne; e += kThreads)
        if (!a.outlier1[e]) o += a.observed ? a.observed[a.m1[a.edge_kp1[e]]] != 0 : 1;
    for (int off = 32; off > 0; off >>= 1) o += __shfl_xor(o, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&obs, o);
    __syncthreads();
    if (threadIdx.x) return;
    if (obs < kMinMapMatches) {
        a.g->n_alive2 = 0;
        a.g->status = st | ORB_TRACK_FAIL_MAP;
    }
    if (a.status) *a.status = a.g->status;
}
__global__ __launch_bounds__(kThreads) void k_track_gate_map(GateArgs a) { k_track_gate_map_body(a); }
__global__ __launch_bounds__(kThreads) void k_track_gate_map_b(const GateArgs* __restrict__ a) {
    k_track_gate_map_body(a[blockIdx.y]);
}

// A frame view whose keypoint count is read from `n` (a gate word) instead of the frame's own
__host__ orb_frame_device_t gated(const orb_frame_device_t* F, const int32_t* n) {
    orb_frame_device_t G = *F;
    G.n = n;
    return G;
}
__host__ orb_last_points_device_t gated(const orb_last_points_device_t* L, const int32_t* n) {
    orb_last_points_device_t G = *L;
    G.n = n;
    return G;
}

// Tracking-chain scratch: the stages' region, then the gate record and the 2 th search's matches
size_t stage_bytes(int cap, int last_cap, int n_local) {
    return (std::max({orbgpu_sbp_frame_scratch_bytes(cap, last_cap), orbgpu_sbp_local_scratch_bytes(cap, n_local),
                      (size_t)cap * sizeof(double)}) + 255) & ~(size_t)255;
}

// the batch's argument areas: one per stage, each room for B frames' largest argument blocks (the
// SearchByProjection stages pack five kernels' blocks, 256-B aligned); 7: the gates, 8: the 2 th search
constexpr int kBatchArgStages = 9;
size_t batch_args_bytes(int B) { return ((size_t)B * 4096 + 8 * 256 + 255) & ~(size_t)255; }

// The pinned host side of a batch's argument areas, per batch scratch (the caller's batch object): a
// ring of two, taken by the calls in turn, each with an event after its call's last copy -- a call
// rewrites an area only once the copies of the call two back have read it (stream-ordered copies read
// pinned memory when they run), so in steady state the host does not wait on the call just queued
// (round 6: with one area every call blocked the host thread on the previous call's event).  An event
// after each call's last launch is what release waits for.
constexpr int kStagingRing = 2;
struct BatchStaging {
    void* host[kStagingRing] = {};         // the calls take the areas in turn
    size_t bytes = 0;
    hipEvent_t copied[kStagingRing] = {};  // after that area's call's last argument copy
    hipEvent_t done = nullptr;             // after the last call's last launch
    int next = 0;
};
std::mutex g_staging_mu;
std::unordered_map<const void*, BatchStaging> g_staging;

}  // namespace

extern "C" {

int orb_tracking_local_seen_device(const int32_t* d_match_a, int cap, int last_cap, const int32_t* d_last_row,
                                   int n_local, uint8_t* d_in_view, void* stream) {
    if (!d_match_a || cap <= 0 || last_cap < 0 || last_cap > kSeenBits || n_local < 0 ||
        (n_local > 0 && (!d_last_row || !d_in_view)))
        return orbgpu_fail(ORB_ERR_ARG, "bad tracking local-seen arguments");
    hipLaunchKernelGGL(k_track_local_seen, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, d_match_a, cap, last_cap,
                       d_last_row, n_local, d_in_view);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "tracking local-seen launch failed");
    return ORB_OK;
}

int orb_tracking_pose_edges_device(const orb_frame_device_t* F, const int32_t* d_match_a, const float* d_xyz_a,
                                   const int32_t* d_match_b, const float* d_xyz_b, const float* inv_level_sigma2,
                                   const double* d_pose, const double pose[7], orb_pose_frame_t* d_frame,
                                   orb_pose_edge_t* d_edges, int32_t* d_edge_kp, void* stream) {
    if (!F || !F->kps_un || !F->n || F->cap <= 0 || F->nlevels <= 0 || F->nlevels > kMaxLevels || !d_match_a ||
        !d_xyz_a || (d_match_b && !d_xyz_b) || !inv_level_sigma2 || (!d_pose && !pose) || !d_frame || !d_edges ||
        !d_edge_kp)
        return orbgpu_fail(ORB_ERR_ARG, "bad tracking pose-edge arguments");
    EdgeParams P{};
    for (int l = 0; l < F->nlevels; ++l) P.inv_sigma2[l] = inv_level_sigma2[l];
    P.nlevels = F->nlevels;
    P.cap = F->cap;
    P.has_pose_dev = d_pose != nullptr;
    P.has_b = d_match_b != nullptr;
    if (!d_pose) memcpy(P.pose, pose, sizeof(P.pose));
    P.cam = orb_ba_camera_t{F->fx, F->fy, F->cx, F->cy, F->bf};
    hipLaunchKernelGGL(k_track_pose_edges, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, P, F->kps_un, F->u_right, F->n,
                       d_match_a, d_xyz_a, d_match_b, d_xyz_b, d_pose, d_frame, d_edges, d_edge_kp);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "tracking pose-edge launch failed");
    return ORB_OK;
}

int orb_tracking_discard_outliers_device(const orb_pose_frame_t* d_frame, const int32_t* d_edge_kp,
                                         const uint8_t* d_outlier, int32_t* d_match_a, const uint8_t* d_observed_a,
                                         int32_t* d_match_b, const uint8_t* d_observed_b, int32_t* d_n_out, int cap,
                                         uint8_t* d_taken, void* stream) {
    if (!d_frame || !d_edge_kp || !d_outlier || !d_match_a || !d_n_out || (d_taken && cap <= 0))
        return orbgpu_fail(ORB_ERR_ARG, "bad tracking discard arguments");
    hipLaunchKernelGGL(k_track_discard, dim3(1), dim3(kThreads), 0, (hipStream_t)stream, d_frame, d_edge_kp, d_outlier, d_match_a,
                       d_observed_a, d_match_b, d_observed_b, d_n_out, cap, d_taken);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "tracking discard launch failed");
    return ORB_OK;
}

size_t orb_tracking_chain_scratch_bytes(int cap, int last_cap, int n_local) {
    if (cap <= 0 || last_cap < 0 || n_local < 0) return 0;
    return stage_bytes(cap, last_cap, n_local) + 256 + (((size_t)cap * sizeof(int32_t) + 255) & ~(size_t)255);
}

int orb_tracking_chain_device(orb_matcher_t m_motion, orb_matcher_t m_local, const orb_frame_device_t* F,
                              const orb_last_points_device_t* last, const orb_local_points_device_t* local,
                              const float* d_pos, const float* d_normal, const float* d_min_dist,
                              const float* d_max_dist, const int32_t* d_last_row, const orb_frustum_frame_t* frustum,
                              const float* inv_level_sigma2, const double pose7[7],
                              const orb_tracking_chain_params_t* P, const orb_tracking_chain_buffers_t* B,
                              void* stream) {
    if (!m_motion || !m_local || !F || !last || !local || !frustum || !inv_level_sigma2 || !pose7 || !P || !B ||
        !B->m1 || !B->m2 || !B->n_match || !B->frames || !B->edges1 || !B->edges2 || !B->edge_kp1 || !B->edge_kp2 ||
        !B->outlier1 || !B->outlier2 || !B->poses || !B->inliers || !B->n_out || !B->taken || !B->scratch ||
        F->cap <= 0 || last->cap < 0 || last->cap > kSeenBits || local->n < 0 || !last->n ||
        (local->n > 0 && (!d_pos || !d_normal || !d_min_dist || !d_max_dist)))
        return orbgpu_fail(ORB_ERR_ARG, "bad tracking chain arguments");
    hipStream_t s = (hipStream_t)stream;
    int rc;
    void* const z = B->scratch;  // stream order: each stage's scratch is free again when the next one runs
    char* const tail = static_cast<char*>(z) + stage_bytes(F->cap, last->cap, local->n);
    ChainGate* const g = reinterpret_cast<ChainGate*>(tail);
    int32_t* const m1w = reinterpret_cast<int32_t*>(tail + 256);
    const bool gate = P->motion_gate != 0;
    GateArgs ga{g, F->n, last->n, B->n_match, B->m1, m1w, B->frames, B->edge_kp1, B->outlier1, last->observed,
                B->status, F->cap};
    // the stages after a gate read the gated counts (the frame's own count when gating is off)
    const orb_frame_device_t F1 = gate ? gated(F, &g->n_alive1) : *F, F2 = gate ? gated(F, &g->n_alive2) : *F;
    if ((rc = orbgpu_sbp_frame_device_scratch(m_motion, F, last, P->th_motion, P->mono, B->m1, B->n_match, stream, z)))
        return rc;
    if (gate) {  // TrackWithMotionModel's retry (src/Tracking.cc:4153-4160)
        hipLaunchKernelGGL(k_track_gate_retry, dim3(1), dim3(64), 0, s, ga);
        const orb_frame_device_t Fw = gated(F, &g->n_wide);
        const orb_last_points_device_t Lw = gated(last, &g->nl_wide);
        if ((rc = orbgpu_sbp_frame_device_scratch(m_motion, &Fw, &Lw, 2 * P->th_motion, P->mono, m1w, &g->n1w, stream, z)))
            return rc;
        hipLaunchKernelGGL(k_track_gate_search, dim3(1), dim3(kThreads), 0, s, ga);
    } else if (B->status && hipMemsetAsync(B->status, 0, sizeof(int32_t), s) != hipSuccess) {
        return orbgpu_fail(ORB_ERR_DEVICE, "tracking chain status reset failed");
    }
    if ((rc = orb_tracking_pose_edges_device(&F1, B->m1, last->xyz, nullptr, nullptr, inv_level_sigma2, nullptr, pose7,
                                             B->frames, B->edges1, B->edge_kp1, stream)))
        return rc;
    if ((rc = orbgpu_pose_optimization_device_scratch(1, B->frames, F->cap, B->edges1, B->poses, B->outlier1, B->inliers,
                                                      stream, static_cast<double*>(z))))
        return rc;
    if (gate) hipLaunchKernelGGL(k_track_gate_map, dim3(1), dim3(kThreads), 0, s, ga);  // (:4216)
    // isInFrustum at the first pose and the seen skip read the first search's assignments, which the
    // discard does not change (the reference marks its discarded outliers seen too, Tracking.cc:4195)
    if (local->n > 0) {
        if ((rc = orb_is_in_frustum_pose_device(frustum, B->poses, local->n, d_pos, d_normal, d_min_dist, d_max_dist,
                                                P->viewing_cos_limit, const_cast<uint8_t*>(local->track_in_view),
                                                const_cast<float*>(local->track_proj), const_cast<float*>(local->track_depth),
                                                const_cast<int32_t*>(local->track_level),
                                                const_cast<float*>(local->track_view_cos), stream)))
            return rc;
        if (d_last_row &&
            (rc = orb_tracking_local_seen_device(B->m1, F->cap, last->cap, d_last_row, local->n,
                                                 const_cast<uint8_t*>(local->track_in_view), stream)))
            return rc;
    }
    if ((rc = orb_tracking_discard_outliers_device(B->frames, B->edge_kp1, B->outlier1, B->m1, last->observed, nullptr,
                                                   nullptr, B->n_out, F->cap, B->taken, stream)))
        return rc;
    if ((rc = orbgpu_sbp_local_device_scratch(m_local, &F2, B->taken, local, P->th_local, P->far_points, P->th_far_points,
                                              B->m2, B->n_match + 1, stream, z)))
        return rc;
    const bool has_local = local->n > 0;  // an empty local map: the second search assigned nothing
    if ((rc = orb_tracking_pose_edges_device(&F2, B->m1, last->xyz, has_local ? B->m2 : nullptr, has_local ? d_pos : nullptr,
                                             inv_level_sigma2, B->poses, nullptr, B->frames + 1, B->edges2, B->edge_kp2,
                                             stream)))
        return rc;
    return orbgpu_pose_optimization_device_scratch(1, B->frames + 1, F->cap, B->edges2, B->poses + 7, B->outlier2,
                                                   B->inliers + 1, stream, static_cast<double*>(z));
}

size_t orb_tracking_chain_batch_scratch_bytes(int n_frames, int cap, int last_cap, int n_local) {
    if (n_frames <= 0 || cap <= 0 || last_cap < 0 || n_local < 0) return 0;
    const size_t stride = (std::max(orbgpu_sbp_frame_scratch_bytes(cap, last_cap),
                                    orbgpu_sbp_local_scratch_bytes(cap, n_local)) + 255) & ~(size_t)255;
    const size_t args = (size_t)kBatchArgStages * batch_args_bytes(n_frames);
    const size_t chi = ((size_t)n_frames * cap * sizeof(double) + 255) & ~(size_t)255;
    const size_t gates = ((size_t)n_frames * sizeof(ChainGate) + 255) & ~(size_t)255;
    return args + (size_t)n_frames * stride + chi + gates + (size_t)n_frames * cap * sizeof(int32_t) + 256;
}

int orb_tracking_chain_batch_release(void* scratch) {
    std::lock_guard<std::mutex> lock(g_staging_mu);
    auto it = g_staging.find(scratch);
    if (it == g_staging.end()) return ORB_OK;
    BatchStaging& stg = it->second;
    if (stg.done) {  // the last call's every kernel (its outputs and the scratch are free afterwards)
        (void)hipEventSynchronize(stg.done);
        (void)hipEventDestroy(stg.done);
    }
    for (int r = 0; r < kStagingRing; ++r) {
        if (stg.copied[r]) {
            (void)hipEventSynchronize(stg.copied[r]);
            (void)hipEventDestroy(stg.copied[r]);
        }
        if (stg.host[r]) (void)hipHostFree(stg.host[r]);
    }
    g_staging.erase(it);
    return ORB_OK;
}

int orb_tracking_chain_batch_device(orb_matcher_t m_motion, orb_matcher_t m_local, int B,
                                    const orb_tracking_chain_frame_t* fr, const orb_tracking_chain_params_t* P,
                                    const orb_tracking_chain_batch_buffers_t* Bf, void* stream) {
    if (!m_motion || !m_local || B <= 0 || B > 65535 /* one grid row per frame */ || !fr || !P || !Bf || !Bf->m1 || !Bf->m2 || !Bf->n_match || !Bf->frames ||
        !Bf->edges1 || !Bf->edges2 || !Bf->edge_kp1 || !Bf->edge_kp2 || !Bf->outlier1 || !Bf->outlier2 || !Bf->poses ||
        !Bf->inliers || !Bf->n_out || !Bf->taken || !Bf->scratch)
        return orbgpu_fail(ORB_ERR_ARG, "bad tracking chain batch arguments");
    // every per-frame check before the first copy or launch: a refused call enqueues nothing
    int C = 0, NL = 0, NP = 0;
    for (int b = 0; b < B; ++b) {
        const orb_tracking_chain_frame_t& f = fr[b];
        if (!f.frame || !f.last || !f.local || !f.frustum || !f.inv_level_sigma2 || f.frame->cap <= 0 ||
            (b && f.frame->cap != C) || f.frame->nlevels <= 0 || f.frame->nlevels > kMaxLevels || !f.frame->n ||
            !f.frame->kps_un || !f.last->n || f.last->cap < 0 || f.last->cap > kSeenBits || f.local->n < 0 ||
            f.frustum->n_levels <= 0 ||
            (f.local->n > 0 && (!f.pos || !f.normal || !f.min_dist || !f.max_dist || !f.local->track_in_view ||
                                !f.local->track_proj || !f.local->track_depth || !f.local->track_level ||
                                !f.local->track_view_cos || !f.local->is_bad || !f.local->observed || !f.local->desc ||
                                (reinterpret_cast<uintptr_t>(f.local->desc) & 15))))
            return orbgpu_fail(ORB_ERR_ARG, "bad tracking chain batch frame (every frame the same cap)");
        C = f.frame->cap;
        NL = std::max(NL, f.last->cap);
        NP = std::max(NP, f.local->n);
    }
    hipStream_t s = (hipStream_t)stream;
    const bool gate = P->motion_gate != 0;
    // scratch: argument areas (one per stage) | the frames' SearchByProjection scratch | PoseOptimization chi2 |
    // gate records | the 2 th search's matches
    const size_t abytes = batch_args_bytes(B);
    char* base = static_cast<char*>(Bf->scratch);
    auto args = [&](int stage) { return static_cast<void*>(base + (size_t)stage * abytes); };
    const size_t stride = (std::max(orbgpu_sbp_frame_scratch_bytes(C, NL), orbgpu_sbp_local_scratch_bytes(C, NP)) + 255) &
                          ~(size_t)255;
    char* sbp = base + (size_t)kBatchArgStages * abytes;
    double* chi = reinterpret_cast<double*>(sbp + (size_t)B * stride);
    ChainGate* gates = reinterpret_cast<ChainGate*>(reinterpret_cast<char*>(chi) +
                                                    (((size_t)B * C * sizeof(double) + 255) & ~(size_t)255));
    int32_t* m1w = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(gates) +
                                              (((size_t)B * sizeof(ChainGate) + 255) & ~(size_t)255));
    std::lock_guard<std::mutex> lock(g_staging_mu);
    BatchStaging& stg = g_staging[Bf->scratch];
    const int ring = stg.next;
    if (stg.copied[ring] && hipEventSynchronize(stg.copied[ring]) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "batch staging wait failed");
    if (stg.bytes < (size_t)kBatchArgStages * abytes) {  // (re)size every area: the others' calls are done
        for (int r = 0; r < kStagingRing; ++r) {
            if (stg.copied[r] && hipEventSynchronize(stg.copied[r]) != hipSuccess)
                return orbgpu_fail(ORB_ERR_DEVICE, "batch staging wait failed");
            if (stg.host[r]) (void)hipHostFree(stg.host[r]);
            stg.host[r] = nullptr;
        }
        stg.bytes = 0;
        for (int r = 0; r < kStagingRing; ++r)
            if (hipHostMalloc(&stg.host[r], (size_t)kBatchArgStages * abytes, hipHostMallocDefault) != hipSuccess)
                return orbgpu_fail(ORB_ERR_DEVICE, "hipHostMalloc failed");
        stg.bytes = (size_t)kBatchArgStages * abytes;
    }
    if ((!stg.copied[ring] && hipEventCreateWithFlags(&stg.copied[ring], hipEventDisableTiming) != hipSuccess) ||
        (!stg.done && hipEventCreateWithFlags(&stg.done, hipEventDisableTiming) != hipSuccess))
        return orbgpu_fail(ORB_ERR_DEVICE, "hipEventCreate failed");
    stg.next = (ring + 1) % kStagingRing;
    // from here on every exit marks the staging's copies (the next call waits for them before it
    // rewrites the staging) and the call's end (release waits for it)
    struct Marks {
        BatchStaging& stg;
        int ring;
        hipStream_t s;
        bool copied = false;
        void Copied() {
            copied = hipEventRecord(stg.copied[ring], s) == hipSuccess;
        }
        ~Marks() {
            if (!copied) (void)hipEventRecord(stg.copied[ring], s);
            (void)hipEventRecord(stg.done, s);
        }
    } marks{stg, ring, s};
    auto hargs = [&](int stage) { return static_cast<void*>(static_cast<char*>(stg.host[ring]) + (size_t)stage * abytes); };
    std::vector<const orb_frame_device_t*> cur(B), cur1(B), cur2(B), curw(B);
    std::vector<const orb_last_points_device_t*> last(B), lastw(B);
    std::vector<orb_frame_device_t> g1(B), g2(B), gw(B);
    std::vector<orb_last_points_device_t> glw(B);
    std::vector<const orb_local_points_device_t*> loc(B);
    std::vector<int32_t*> m1(B), m2(B), n1(B), n2(B), mw(B), nw(B);
    std::vector<const uint8_t*> taken(B);
    std::vector<GateArgs> ga(B);
    for (int b = 0; b < B; ++b) {
        cur[b] = fr[b].frame;
        last[b] = fr[b].last;
        loc[b] = fr[b].local;
        m1[b] = Bf->m1 + (size_t)b * C;
        m2[b] = Bf->m2 + (size_t)b * C;
        n1[b] = Bf->n_match + 2 * (size_t)b;
        n2[b] = n1[b] + 1;
        mw[b] = m1w + (size_t)b * C;
        nw[b] = &gates[b].n1w;
        taken[b] = Bf->taken + (size_t)b * C;
        g1[b] = gate ? gated(cur[b], &gates[b].n_alive1) : *cur[b];
        g2[b] = gate ? gated(cur[b], &gates[b].n_alive2) : *cur[b];
        gw[b] = gated(cur[b], &gates[b].n_wide);
        glw[b] = gated(last[b], &gates[b].nl_wide);
        cur1[b] = &g1[b];
        cur2[b] = &g2[b];
        curw[b] = &gw[b];
        lastw[b] = &glw[b];
        ga[b] = GateArgs{&gates[b], cur[b]->n, last[b]->n, n1[b], m1[b], mw[b], Bf->frames + b, Bf->edge_kp1 + (size_t)b * C,
                         Bf->outlier1 + (size_t)b * C, last[b]->observed, Bf->status ? Bf->status + b : nullptr, C};
    }
    orb_pose_frame_t* fr1 = Bf->frames;
    orb_pose_frame_t* fr2 = Bf->frames + B;
    double* pose1 = Bf->poses;
    double* pose2 = Bf->poses + 7 * (size_t)B;
    auto upload = [&](int stage, const void* h, size_t n) {
        if (n > abytes) return false;
        memcpy(hargs(stage), h, n);
        return hipMemcpyAsync(args(stage), hargs(stage), n, hipMemcpyHostToDevice, s) == hipSuccess;
    };
    int rc;
    if ((rc = orbgpu_sbp_frame_batch(m_motion, B, cur.data(), last.data(), P->th_motion, P->mono, m1.data(), n1.data(),
                                     sbp, stride, args(0), hargs(0), abytes, s)))
        return rc;
    if (gate) {  // TrackWithMotionModel's retry and failure (src/Tracking.cc:4153-4168)
        if (!upload(7, ga.data(), B * sizeof(ga[0]))) return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
        const GateArgs* dga = static_cast<const GateArgs*>(args(7));
        hipLaunchKernelGGL(k_track_gate_retry_b, dim3(1, B), dim3(64), 0, s, dga);
        if ((rc = orbgpu_sbp_frame_batch(m_motion, B, curw.data(), lastw.data(), 2 * P->th_motion, P->mono, mw.data(),
                                         nw.data(), sbp, stride, args(8), hargs(8), abytes, s)))
            return rc;
        hipLaunchKernelGGL(k_track_gate_search_b, dim3(1, B), dim3(kThreads), 0, s, dga);
    } else if (Bf->status && hipMemsetAsync(Bf->status, 0, sizeof(int32_t) * B, s) != hipSuccess) {
        return orbgpu_fail(ORB_ERR_DEVICE, "tracking chain status reset failed");
    }
    // the first graphs: the last frame's points, the motion model's pose
    auto edges_args = [&](int b, bool second) {
        const orb_tracking_chain_frame_t& f = fr[b];
        const orb_frame_device_t* F = second ? cur2[b] : cur1[b];
        EdgeParams E{};
        for (int l = 0; l < F->nlevels; ++l) E.inv_sigma2[l] = f.inv_level_sigma2[l];
        E.nlevels = F->nlevels;
        E.cap = C;
        E.has_pose_dev = second;
        E.has_b = second && f.local->n > 0;
        E.edge_begin = b * C;
        if (!second) memcpy(E.pose, f.pose7, sizeof(E.pose));
        E.cam = orb_ba_camera_t{F->fx, F->fy, F->cx, F->cy, F->bf};
        const size_t o = (size_t)b * C;
        return k_track_pose_edges_args{E, F->kps_un, F->u_right, F->n, m1[b], f.last->xyz, E.has_b ? m2[b] : nullptr,
                                       E.has_b ? f.pos : nullptr, second ? pose1 + 7 * (size_t)b : nullptr,
                                       second ? fr2 + b : fr1 + b, (second ? Bf->edges2 : Bf->edges1) + o,
                                       (second ? Bf->edge_kp2 : Bf->edge_kp1) + o};
    };
    std::vector<k_track_pose_edges_args> ea(B);
    for (int b = 0; b < B; ++b) ea[b] = edges_args(b, false);
    if (!upload(1, ea.data(), B * sizeof(ea[0]))) return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
    hipLaunchKernelGGL(k_track_pose_edges_b, dim3(1, B), dim3(kThreads), 0, s, (const k_track_pose_edges_args*)args(1));
    if ((rc = orbgpu_pose_optimization_device_scratch(B, fr1, B * C, Bf->edges1, pose1, Bf->outlier1, Bf->inliers, stream, chi)))
        return rc;
    if (gate)  // nmatchesMap < 10: TrackWithMotionModel false (:4216); the gate blocks uploaded for the retry
        hipLaunchKernelGGL(k_track_gate_map_b, dim3(1, B), dim3(kThreads), 0, s, static_cast<const GateArgs*>(args(7)));
    // isInFrustum at the first poses, the seen skip, the discard
    if ((rc = orbgpu_frustum_chain_batch(B, fr, pose1, P->viewing_cos_limit, args(2), hargs(2), abytes, stream))) return rc;
    std::vector<k_track_local_seen_args> sa(B);
    bool any_seen = false;
    for (int b = 0; b < B; ++b) {
        const bool on = fr[b].last_row && fr[b].local->n > 0;
        any_seen |= on;
        sa[b] = k_track_local_seen_args{m1[b], C, fr[b].last->cap, fr[b].last_row, on ? fr[b].local->n : 0,
                                        const_cast<uint8_t*>(fr[b].local->track_in_view)};
    }
    if (any_seen) {
        if (!upload(3, sa.data(), B * sizeof(sa[0]))) return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
        hipLaunchKernelGGL(k_track_local_seen_b, dim3(1, B), dim3(kThreads), 0, s, (const k_track_local_seen_args*)args(3));
    }
    std::vector<k_track_discard_args> da(B);
    for (int b = 0; b < B; ++b)
        da[b] = k_track_discard_args{fr1 + b, Bf->edge_kp1 + (size_t)b * C, Bf->outlier1 + (size_t)b * C, m1[b],
                                     fr[b].last->observed, nullptr, nullptr, Bf->n_out + 2 * (size_t)b, C,
                                     Bf->taken + (size_t)b * C};
    if (!upload(4, da.data(), B * sizeof(da[0]))) return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
    hipLaunchKernelGGL(k_track_discard_b, dim3(1, B), dim3(kThreads), 0, s, (const k_track_discard_args*)args(4));
    if ((rc = orbgpu_sbp_local_batch(m_local, B, cur2.data(), taken.data(), loc.data(), P->th_local, P->far_points,
                                     P->th_far_points, m2.data(), n2.data(), sbp, stride, args(5), hargs(5), abytes, s)))
        return rc;
    // the second graphs: both searches, the first poses
    for (int b = 0; b < B; ++b) ea[b] = edges_args(b, true);
    if (!upload(6, ea.data(), B * sizeof(ea[0]))) return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
    marks.Copied();  // the call's last copy from the staging
    hipLaunchKernelGGL(k_track_pose_edges_b, dim3(1, B), dim3(kThreads), 0, s, (const k_track_pose_edges_args*)args(6));
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "tracking chain batch launch failed");
    return orbgpu_pose_optimization_device_scratch(B, fr2, B * C, Bf->edges2, pose2, Bf->outlier2, Bf->inliers + B, stream,
                                                   chi);
}

}  // extern "C"
