// ORACLE (test infrastructure only): Frame::UndistortKeyPoints (src/Frame.cc:1003-1051), which calls
//   cv::undistortPoints(mat, mat, K, mDistCoef, cv::Mat(), mK)
// for the N keypoints' pt.  OpenCV is absent from this image, so the OpenCV 4.x algorithm is restated
// here (modules/calib3d/src/undistort.dispatch.cpp, cvUndistortPointsInternal; the reference's
// CMakeLists.txt:35 asks for OpenCV 4.x), for the case the reference uses: R empty, P = K, the default
// TermCriteria(COUNT, 5, 0.01) of the overload without criteria, so exactly five fixed-point iterations
// and no reprojection-error test.  PARITY UNPINNED against a real OpenCV: the reference ships no
// undistorted keypoints, and OpenCV's build (its FMA use in this baseline-ISA function) cannot be
// observed here; the restatement evaluates in double without contraction, as OpenCV's portable C++
// does without -mfma.
//
// Per point (u, v), with the distortion vector k[0..4] = (k1, k2, p1, p2, k3) as doubles of the float
// mDistCoef entries (k[5..13] = 0, so the tilt matrices are the identity and the rational numerator 1):
//   x = (u - cx) / fx ... as (u - cx) * (1 / fx); x0 = x, y0 = y
//   5 times:  r2 = x x + y y
//             icdist = 1 / (1 + ((k3 r2 + k2) r2 + k1) r2)        (numerator (1 + ((0 r2 + 0) r2 + 0) r2) = 1)
//             if icdist < 0: x, y = the undistorted-free normalised point, stop
//             dx = 2 p1 x y + p2 (r2 + 2 x x) + 0 r2 + 0 r2 r2, dy = p1 (r2 + 2 y y) + 2 p2 x y + ...
//             x = (x0 - dx) icdist, y = (y0 - dy) icdist
//   then the P = K projection with R = I: x' = (fx x + 0 y + cx) * (1 / (0 x + 0 y + 1)), as float.
// If mDistCoef[0] == 0 the reference copies mvKeys unchanged (src/Frame.cc:1007-1011).
#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

struct Kp {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

// One point; the operations in the order the OpenCV source writes them (no contraction).
void undistort_point(double u, double v, double fx, double fy, double cx, double cy, const double k[5], float* ox,
                     float* oy) {
    const double ifx = 1. / fx, ify = 1. / fy;
    double x = (u - cx) * ifx;
    double y = (v - cy) * ify;
    // tilt compensation with the identity matrix: (1 x + 0 y + 0 1, 0 x + 1 y + 0 1, 0 x + 0 y + 1 1)
    const double ux = 1.0 * x + 0.0 * y + 0.0 * 1.0, uy = 0.0 * x + 1.0 * y + 0.0 * 1.0, uz = 0.0 * x + 0.0 * y + 1.0 * 1.0;
    const double invProj = uz ? 1. / uz : 1;
    const double x0 = x = invProj * ux;
    const double y0 = y = invProj * uy;
    const double k5 = 0, k6 = 0, k7 = 0, k8 = 0, k9 = 0, k10 = 0, k11 = 0;
    for (int j = 0; j < 5; ++j) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k7 * r2 + k6) * r2 + k5) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k8 * r2 + k9 * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k10 * r2 + k11 * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P R = K (3x3): xx = RR00 x + RR01 y + RR02, yy = RR10 x + RR11 y + RR12, ww = 1 / (RR20 x + RR21 y + RR22)
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *ox = (float)(xx * ww);
    *oy = (float)(yy * ww);
}

}  // namespace

extern "C" {

// kps / kps_un: n cv::KeyPoint records; K = (fx, fy, cx, cy) as the float camera matrix holds them;
// dist: n_dist (4 or 5) floats, mDistCoef.
void oracle_undistort_keypoints(const void* kps, int n, const float* K, const float* dist, int n_dist, void* kps_un) {
    const Kp* in = static_cast<const Kp*>(kps);
    Kp* out = static_cast<Kp*>(kps_un);
    if (n <= 0) return;
    memmove(out, in, sizeof(Kp) * (size_t)n);
    if (dist[0] == 0.0f) return;  // mvKeysUn = mvKeys
    double k[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < n_dist && i < 5; ++i) k[i] = (double)dist[i];
    for (int i = 0; i < n; ++i)
        undistort_point((double)in[i].x, (double)in[i].y, (double)K[0], (double)K[1], (double)K[2], (double)K[3], k,
                        &out[i].x, &out[i].y);
}

}  // extern "C"
