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
// Map points are referenced by index into a device table of world positions (float xyz, as
// MapPoint::GetWorldPos returns them); a keypoint's map point comes from the second match array when it
// has one there (SearchByProjection(F, local points) overwrites, src/ORBmatcher.cc:156), else the first.
#include <hip/hip_runtime.h>

#include <algorithm>

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
    double pose[7];
    orb_ba_camera_t cam;
};

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
        F.edge_begin = 0;
        F.n_edges = part[kThreads - 1];
        *frame = F;
    }
}

// outliers lose their map point; n_out[0] = the edges kept, n_out[1] = those whose map point has
// observations (nmatchesMap, src/Tracking.cc:4198-4200)
__global__ __launch_bounds__(kThreads) void k_track_discard(const orb_pose_frame_t* __restrict__ frame,
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

// SearchLocalPoints' first loop (src/Tracking.cc:4250-4266): a local map point the frame already holds
// (mnLastFrameSeen == mCurrentFrame.mnId) is not tested against the frustum.  With the local map as its own
// table, local point j is the last frame's row last_row[j] (-1: a point the last frame does not track);
// the rows the frame still holds after the discard go into an LDS bitmap.
constexpr int kSeenBits = 16384;

__global__ __launch_bounds__(kThreads) void k_track_local_seen(const int32_t* __restrict__ match_a, int cap, int last_cap,
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
    return std::max({orbgpu_sbp_frame_scratch_bytes(cap, last_cap), orbgpu_sbp_local_scratch_bytes(cap, n_local),
                     (size_t)cap * sizeof(double)});
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
        !B->outlier1 || !B->outlier2 || !B->poses || !B->inliers || !B->n_out || !B->taken ||
        (local->n > 0 && (!d_pos || !d_normal || !d_min_dist || !d_max_dist)))
        return orbgpu_fail(ORB_ERR_ARG, "bad tracking chain arguments");
    int rc;
    void* const z = B->scratch;  // stream order: each stage's scratch is free again when the next one runs
    if ((rc = orbgpu_sbp_frame_device_scratch(m_motion, F, last, P->th_motion, P->mono, B->m1, B->n_match, stream, z)))
        return rc;
    if ((rc = orb_tracking_pose_edges_device(F, B->m1, last->xyz, nullptr, nullptr, inv_level_sigma2, nullptr, pose7,
                                             B->frames, B->edges1, B->edge_kp1, stream)))
        return rc;
    if ((rc = orbgpu_pose_optimization_device_scratch(1, B->frames, F->cap, B->edges1, B->poses, B->outlier1, B->inliers,
                                                      stream, static_cast<double*>(z))))
        return rc;
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
    if ((rc = orbgpu_sbp_local_device_scratch(m_local, F, B->taken, local, P->th_local, P->far_points, P->th_far_points,
                                              B->m2, B->n_match + 1, stream, z)))
        return rc;
    const bool has_local = local->n > 0;  // an empty local map: the second search assigned nothing
    if ((rc = orb_tracking_pose_edges_device(F, B->m1, last->xyz, has_local ? B->m2 : nullptr, has_local ? d_pos : nullptr,
                                             inv_level_sigma2, B->poses, nullptr, B->frames + 1, B->edges2, B->edge_kp2,
                                             stream)))
        return rc;
    return orbgpu_pose_optimization_device_scratch(1, B->frames + 1, F->cap, B->edges2, B->poses + 7, B->outlier2,
                                                   B->inliers + 1, stream, static_cast<double*>(z));
}

}  // extern "C"
