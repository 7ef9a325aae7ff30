// MI355X Frame::isInFrustum (reference src/Frame.cc:667-773, pinhole, Nleft == -1) with
// MapPoint::PredictScale (src/MapPoint.cc:715-731): the per-map-point tracking fields that
// SearchByProjection(Frame, local MapPoints) reads (orb_search_by_projection_local), one thread per
// point.  Float operations are written out explicitly with the contractions g++ -O3 -march=native
// applies to the reference (the oracle, oracle/orb_frustum_oracle.cpp, uses the same ones); the
// library is built with -ffp-contract=off, so nothing else is fused.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "orb_pose_frame.h"
#include "orb_predict_scale.h"
#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

// PredictScale's thresholds for (log scale factor, levels), memoised per thread: a binary search of
// ~31 logf per level, which a batch of frames with one camera would otherwise repeat per frame (the
// tracking-chain batch's host enqueue, round 6)
bool scale_thresholds(float lsf, int n_levels, float* T) {
    thread_local float m_lsf = -1.0f;
    thread_local int m_n = -1;
    thread_local float m_T[orbgpu::kPredictMaxLevels];
    if (n_levels != m_n || std::memcmp(&lsf, &m_lsf, sizeof(float)) != 0) {
        if (!orbgpu::predict_scale_thresholds(lsf, n_levels, m_T)) return false;
        m_lsf = lsf;
        m_n = n_levels;
    }
    std::memcpy(T, m_T, sizeof(float) * (n_levels > 1 ? n_levels - 1 : 0));
    return true;
}


struct ScaleSteps {  // MapPoint::PredictScale level thresholds (orb_predict_scale.h)
    float t[orbgpu::kPredictMaxLevels];
};

__device__ __forceinline__ float dot3(const float a[3], const float b[3]) {
    return fmaf(a[2], b[2], fmaf(a[0], b[0], a[1] * b[1]));
}

__device__ __forceinline__ void k_is_in_frustum_body(orb_frustum_frame_t F, const double* __restrict__ pose7, int n,
                                                       const float* __restrict__ pos,
                                                       const float* __restrict__ normal,
                                                       const float* __restrict__ min_dist,
                                                       const float* __restrict__ max_dist, float viewingCosLimit,
                                                       ScaleSteps steps, uint8_t* __restrict__ in_view, float* __restrict__ proj,
                                                       float* __restrict__ depth, int32_t* __restrict__ level,
                                                       float* __restrict__ view_cos) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (pose7) {  // the frame's pose is the device result of PoseOptimization (Frame::SetPose)
        double p[7];
        for (int k = 0; k < 7; ++k) p[k] = pose7[k];
        orb_pose7_to_frame(p, F.Tcw, F.Ow);
    }
    uint8_t in = 0;
    float px = -1, py = -1, pxr = 0, dep = 0, vc = 0;
    int lev = 0;
    const float P[3] = {pos[3 * (size_t)i], pos[3 * (size_t)i + 1], pos[3 * (size_t)i + 2]};
    float Pc[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
        Pc[r] = fmaf(F.Tcw[4 * r + 2], P[2], fmaf(F.Tcw[4 * r], P[0], F.Tcw[4 * r + 1] * P[1])) + F.Tcw[4 * r + 3];
    const float Pc_dist = sqrtf(dot3(Pc, Pc));
    const float PcZ = Pc[2];
    const float invz = 1.0f / PcZ;
    do {
        if (PcZ < 0.0f) break;
        const float u = F.fx * Pc[0] / Pc[2] + F.cx;  // Pinhole::project(Eigen::Vector3f)
        const float v = F.fy * Pc[1] / Pc[2] + F.cy;
        if (u < F.min_x || u > F.max_x) break;
        if (v < F.min_y || v > F.max_y) break;
        px = u;
        py = v;
        const float maxDistance = 1.2f * max_dist[i], minDistance = 0.8f * min_dist[i];
        const float PO[3] = {P[0] - F.Ow[0], P[1] - F.Ow[1], P[2] - F.Ow[2]};
        const float dist = sqrtf(dot3(PO, PO));
        if (dist < minDistance || dist > maxDistance) break;
        const float Pn[3] = {normal[3 * (size_t)i], normal[3 * (size_t)i + 1], normal[3 * (size_t)i + 2]};
        const float viewCos = dot3(PO, Pn) / dist;
        if (viewCos < viewingCosLimit) break;
        // PredictScale: ceilf(logf(ratio) / mfLogScaleFactor) clamped, through glibc-exact steps
        const float ratio = max_dist[i] / dist;
        const int nScale = orbgpu::predict_scale_level(ratio, steps.t, F.n_levels);
        in = 1;
        pxr = fmaf(-F.bf, invz, u);
        dep = Pc_dist;
        lev = nScale;
        vc = viewCos;
    } while (false);
    in_view[i] = in;
    proj[3 * (size_t)i] = px;
    proj[3 * (size_t)i + 1] = py;
    proj[3 * (size_t)i + 2] = pxr;
    depth[i] = dep;
    level[i] = lev;
    view_cos[i] = vc;
}
__global__ __launch_bounds__(256) void k_is_in_frustum(orb_frustum_frame_t F, const double* __restrict__ pose7, int n,
                                                       const float* __restrict__ pos,
                                                       const float* __restrict__ normal,
                                                       const float* __restrict__ min_dist,
                                                       const float* __restrict__ max_dist, float viewingCosLimit,
                                                       ScaleSteps steps, uint8_t* __restrict__ in_view, float* __restrict__ proj,
                                                       float* __restrict__ depth, int32_t* __restrict__ level,
                                                       float* __restrict__ view_cos) {
    k_is_in_frustum_body(F, pose7, n, pos, normal, min_dist, max_dist, viewingCosLimit, steps, in_view, proj, depth,
                         level, view_cos);
}
struct k_is_in_frustum_args {
    orb_frustum_frame_t F;
    const double* pose7;
    int n;
    const float* pos;
    const float* normal;
    const float* min_dist;
    const float* max_dist;
    float viewingCosLimit;
    ScaleSteps steps;
    uint8_t* in_view;
    float* proj;
    float* depth;
    int32_t* level;
    float* view_cos;
};
// the same on frame blockIdx.y of a batch (one argument block per frame)
__global__ __launch_bounds__(256) void k_is_in_frustum_b(const k_is_in_frustum_args* __restrict__ a) {
    const k_is_in_frustum_args& A = a[blockIdx.y];
    k_is_in_frustum_body(A.F, A.pose7, A.n, A.pos, A.normal, A.min_dist, A.max_dist, A.viewingCosLimit, A.steps,
                         A.in_view, A.proj, A.depth, A.level, A.view_cos);
}

}  // namespace

extern "C" {

int orb_is_in_frustum_pose_device(const orb_frustum_frame_t* frame, const double* d_pose7, int n, const float* d_pos,
                                  const float* d_normal, const float* d_min_dist, const float* d_max_dist,
                                  float viewing_cos_limit, uint8_t* d_in_view, float* d_proj, float* d_depth,
                                  int32_t* d_level, float* d_view_cos, void* stream) {
    if (!frame || n < 0 || (n && (!d_pos || !d_normal || !d_min_dist || !d_max_dist || !d_in_view || !d_proj ||
                                  !d_depth || !d_level || !d_view_cos)) || frame->n_levels <= 0)
        return orbgpu_fail(ORB_ERR_ARG, "invalid frustum arguments");
    ScaleSteps steps{};
    if (!scale_thresholds(frame->log_scale_factor, frame->n_levels, steps.t))
        return orbgpu_fail(ORB_ERR_ARG, "log_scale_factor must be > 0 and n_levels <= 32");
    if (n == 0) return ORB_OK;
    hipLaunchKernelGGL(k_is_in_frustum, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, *frame, d_pose7, n, d_pos,
                       d_normal, d_min_dist, d_max_dist, viewing_cos_limit, steps, d_in_view, d_proj, d_depth, d_level,
                       d_view_cos);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "frustum kernel launch failed");
    return ORB_OK;
}

}  // extern "C"

// The tracking chain's batch: frame b's local map tested at its optimised pose d_poses[7 b], one grid row
// per frame (argument blocks copied into d_args).
int orbgpu_frustum_chain_batch(int B, const orb_tracking_chain_frame_t* fr, const double* d_poses, float viewing_cos_limit,
                               void* d_args, void* h_args, size_t args_cap, void* stream) {
    if (B <= 0 || !fr || !d_poses || !d_args || !h_args) return orbgpu_fail(ORB_ERR_ARG, "invalid frustum batch arguments");
    std::vector<k_is_in_frustum_args> a(B);
    int maxn = 0;
    for (int b = 0; b < B; ++b) {
        const orb_frustum_frame_t* F = fr[b].frustum;
        const orb_local_points_device_t* L = fr[b].local;
        if (!F || !L || L->n < 0 || F->n_levels <= 0 ||
            (L->n && (!fr[b].pos || !fr[b].normal || !fr[b].min_dist || !fr[b].max_dist || !L->track_in_view ||
                      !L->track_proj || !L->track_depth || !L->track_level || !L->track_view_cos)))
            return orbgpu_fail(ORB_ERR_ARG, "invalid frustum batch frame");
        ScaleSteps steps{};
        if (!scale_thresholds(F->log_scale_factor, F->n_levels, steps.t))
            return orbgpu_fail(ORB_ERR_ARG, "log_scale_factor must be > 0 and n_levels <= 32");
        a[b] = k_is_in_frustum_args{*F, d_poses + 7 * (size_t)b, L->n, fr[b].pos, fr[b].normal, fr[b].min_dist,
                                    fr[b].max_dist, viewing_cos_limit, steps, const_cast<uint8_t*>(L->track_in_view),
                                    const_cast<float*>(L->track_proj), const_cast<float*>(L->track_depth),
                                    const_cast<int32_t*>(L->track_level), const_cast<float*>(L->track_view_cos)};
        maxn = std::max(maxn, L->n);
    }
    if (maxn == 0) return ORB_OK;
    if (a.size() * sizeof(k_is_in_frustum_args) > args_cap)
        return orbgpu_fail(ORB_ERR_ARG, "frustum batch: argument area too small");
    hipStream_t s = (hipStream_t)stream;
    memcpy(h_args, a.data(), a.size() * sizeof(k_is_in_frustum_args));  // pinned staging
    if (hipMemcpyAsync(d_args, h_args, a.size() * sizeof(k_is_in_frustum_args), hipMemcpyHostToDevice, s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "batch argument upload failed");
    hipLaunchKernelGGL(k_is_in_frustum_b, dim3((maxn + 255) / 256, B), dim3(256), 0, s,
                       (const k_is_in_frustum_args*)d_args);
    return hipGetLastError() == hipSuccess ? ORB_OK : orbgpu_fail(ORB_ERR_DEVICE, "frustum batch launch failed");
}

extern "C" {

int orb_is_in_frustum_device(const orb_frustum_frame_t* frame, int n, const float* d_pos, const float* d_normal,
                             const float* d_min_dist, const float* d_max_dist, float viewing_cos_limit,
                             uint8_t* d_in_view, float* d_proj, float* d_depth, int32_t* d_level, float* d_view_cos,
                             void* stream) {
    return orb_is_in_frustum_pose_device(frame, nullptr, n, d_pos, d_normal, d_min_dist, d_max_dist, viewing_cos_limit,
                                         d_in_view, d_proj, d_depth, d_level, d_view_cos, stream);
}

int orb_is_in_frustum(const orb_frustum_frame_t* frame, int n, const float* pos, const float* normal,
                      const float* min_dist, const float* max_dist, float viewing_cos_limit, uint8_t* in_view,
                      float* proj, float* depth, int32_t* level, float* view_cos) {
    if (!frame || n < 0 || (n && (!pos || !normal || !min_dist || !max_dist || !in_view || !proj || !depth || !level ||
                                  !view_cos)) || frame->n_levels <= 0)
        return orbgpu_fail(ORB_ERR_ARG, "invalid frustum arguments");
    if (n == 0) return 0;
    if (orb_device_count() <= 0) return orbgpu_fail(ORB_ERR_DEVICE, "no HIP device visible");
    // inputs: pos 12 n | normal 12 n | min 4 n | max 4 n; outputs: in 1 n | proj 12 n | depth 4 n | level 4 n | cos 4 n
    const size_t N = (size_t)n, in_bytes = 32 * N, out_bytes = 25 * N;
    uint8_t* d = nullptr;
    if (hipMalloc(&d, in_bytes + out_bytes + 64) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
    float* dp = reinterpret_cast<float*>(d);
    float* dn = dp + 3 * N;
    float* dmin = dn + 3 * N;
    float* dmax = dmin + N;
    float* dproj = dmax + N;
    float* ddep = dproj + 3 * N;
    int32_t* dlev = reinterpret_cast<int32_t*>(ddep + N);
    float* dcos = reinterpret_cast<float*>(dlev + N);
    uint8_t* din = reinterpret_cast<uint8_t*>(dcos + N);
    int rc = ORB_OK;
    if (hipMemcpy(dp, pos, 12 * N, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dn, normal, 12 * N, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dmin, min_dist, 4 * N, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dmax, max_dist, 4 * N, hipMemcpyHostToDevice) != hipSuccess)
        rc = orbgpu_fail(ORB_ERR_DEVICE, "frustum upload failed");
    if (rc == ORB_OK)
        rc = orb_is_in_frustum_device(frame, n, dp, dn, dmin, dmax, viewing_cos_limit, din, dproj, ddep, dlev, dcos,
                                      nullptr);
    if (rc == ORB_OK &&
        (hipMemcpy(in_view, din, N, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(proj, dproj, 12 * N, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(depth, ddep, 4 * N, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(level, dlev, 4 * N, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(view_cos, dcos, 4 * N, hipMemcpyDeviceToHost) != hipSuccess))
        rc = orbgpu_fail(ORB_ERR_DEVICE, "frustum download failed");
    (void)hipFree(d);
    if (rc != ORB_OK) return rc;
    int cnt = 0;
    for (int i = 0; i < n; ++i) cnt += in_view[i];
    return cnt;
}

}  // extern "C"
