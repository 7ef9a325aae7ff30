// MI355X Frame::UndistortKeyPoints (reference src/Frame.cc:1003-1051): mvKeysUn from mvKeys by
// cv::undistortPoints(mat, mat, K, mDistCoef, cv::Mat(), mK) -- OpenCV 4.x's cvUndistortPointsInternal
// for R empty, P = K and the default TermCriteria(COUNT, 5, 0.01): five fixed-point iterations of the
// inverse radial/tangential model in double, then the projection by K, rounded to float.  One thread
// per keypoint, on the extractor's device layout (frame f's keypoints at f * cap, its count at
// d_counts[2 f]), so the device chains (stereo / BoW / SearchForTriangulation / SearchByProjection)
// read undistorted coordinates without a host hop.  The library builds with -ffp-contract=off, and the
// operations follow the OpenCV source's order, as the oracle (oracle/orb_undistort_oracle.cpp) does;
// parity with a real OpenCV build is unpinned (no OpenCV in this image).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

struct UndistortParams {
    double fx, fy, cx, cy;
    double k[5];  // k1, k2, p1, p2, k3 (doubles of mDistCoef's floats; k3 = 0 for a 4-entry vector)
    int copy;     // mDistCoef[0] == 0: mvKeysUn = mvKeys
};

__global__ __launch_bounds__(256) void k_undistort(const orb_keypoint_t* __restrict__ kps,
                                                   const int32_t* __restrict__ counts, int n_frames, int cap,
                                                   UndistortParams P, orb_keypoint_t* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_frames * cap) return;
    const int f = t / cap, i = t - f * cap;
    const int c = counts[2 * f];
    // a frame the extractor flagged (ORB_ERR_CAPACITY, or a count outside [0, cap]) has no keypoints here
    if (counts[2 * f + 1] == ORB_ERR_CAPACITY || c < 0 || c > cap || i >= c) return;
    orb_keypoint_t kp = kps[t];
    if (!P.copy) {
        const double u = kp.x, v = kp.y;
        const double ifx = 1. / P.fx, ify = 1. / P.fy;
        double x = (u - P.cx) * ifx;
        double y = (v - P.cy) * ify;
        // the tilt compensation with the identity matrix (k[12] = k[13] = 0), as OpenCV evaluates it
        const double ux = 1.0 * x + 0.0 * y + 0.0 * 1.0, uy = 0.0 * x + 1.0 * y + 0.0 * 1.0;
        const double uz = 0.0 * x + 0.0 * y + 1.0 * 1.0;
        const double invProj = uz != 0.0 ? 1. / uz : 1;
        const double x0 = x = invProj * ux;
        const double y0 = y = invProj * uy;
        const double k5 = 0, k6 = 0, k7 = 0, k8 = 0, k9 = 0, k10 = 0, k11 = 0;
        for (int j = 0; j < 5; ++j) {
            const double r2 = x * x + y * y;
            const double icdist =
                (1 + ((k7 * r2 + k6) * r2 + k5) * r2) / (1 + ((P.k[4] * r2 + P.k[1]) * r2 + P.k[0]) * r2);
            if (icdist < 0) {  // OpenCV's guard (undistortPoints.regression_14583)
                x = (u - P.cx) * ifx;
                y = (v - P.cy) * ify;
                break;
            }
            const double deltaX = 2 * P.k[2] * x * y + P.k[3] * (r2 + 2 * x * x) + k8 * r2 + k9 * r2 * r2;
            const double deltaY = P.k[2] * (r2 + 2 * y * y) + 2 * P.k[3] * x * y + k10 * r2 + k11 * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        const double xx = P.fx * x + 0.0 * y + P.cx;  // RR = P R = K
        const double yy = 0.0 * x + P.fy * y + P.cy;
        const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
        kp.x = (float)(xx * ww);
        kp.y = (float)(yy * ww);
    }
    out[t] = kp;
}

}  // namespace

extern "C" {

int orb_undistort_keypoints_device(const orb_keypoint_t* d_kps, const int32_t* d_counts, int n_frames, int cap,
                                   const float K[4], const float* dist, int n_dist, orb_keypoint_t* d_kps_un,
                                   void* stream) {
    if (n_frames < 0 || cap <= 0 || !K || !dist || n_dist < 4 || n_dist > 5 ||
        (n_frames > 0 && (!d_kps || !d_counts || !d_kps_un)))
        return orbgpu_fail(ORB_ERR_ARG, "bad UndistortKeyPoints arguments");
    if (n_frames == 0) return ORB_OK;
    if ((long long)n_frames * cap > (1ll << 30)) return orbgpu_fail(ORB_ERR_ARG, "too many keypoints");
    UndistortParams P{};
    P.fx = K[0];
    P.fy = K[1];
    P.cx = K[2];
    P.cy = K[3];
    for (int i = 0; i < n_dist; ++i) P.k[i] = (double)dist[i];
    P.copy = dist[0] == 0.0f;  // src/Frame.cc:1007
    const int n = n_frames * cap;
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_kps, d_counts, n_frames,
                       cap, P, d_kps_un);
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "UndistortKeyPoints launch failed");
    return ORB_OK;
}

}  // extern "C"
