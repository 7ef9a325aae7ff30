// ORACLE -- TEST INFRASTRUCTURE ONLY.  CPU restatement of Frame::isInFrustum for pinhole frames
// (reference src/Frame.cc:667-773, Nleft == -1), MapPoint::GetMin/MaxDistanceInvariance
// (src/MapPoint.cc:658-671) and MapPoint::PredictScale(const float&, Frame*) (src/MapPoint.cc:715-731).
//
// Float arithmetic follows what g++ -O3 -march=native makes of the reference (as in
// orb_projection_oracle.cpp): Eigen's 3-term row sums and squared norms are contracted as
// fma(a2, b2, fma(a0, b0, a1 * b1)), `u - bf * invz` as fma(-bf, invz, u); the pose is applied as a
// 3x4 matrix (the reference's mRcw / mtcw).  PredictScale's unqualified `log(ratio)` and `ceil`
// resolve to the float overloads: Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:36 has a global
// `using namespace std` that MapPoint.cc includes (MapPoint.h -> Frame.h -> ORBVocabulary.h), so the
// level is ceilf(logf(ratio) / mfLogScaleFactor) in float with glibc's logf.  Parity with the real
// reference: unpinned at the ulp level (Eigen's exact evaluation order is not observable without Eigen).
#include <cmath>
#include <cstdint>

#include "../include/orbgpu.h"

namespace {
inline float dot3(const float a[3], const float b[3]) { return std::fma(a[2], b[2], std::fma(a[0], b[0], a[1] * b[1])); }
}  // namespace

extern "C" int oracle_is_in_frustum(const orb_frustum_frame_t* F, int n, const float* pos, const float* normal,
                                    const float* min_dist, const float* max_dist, float viewingCosLimit,
                                    uint8_t* in_view, float* proj, float* depth, int32_t* level, float* view_cos) {
    int n_in = 0;
    for (int i = 0; i < n; ++i) {
        in_view[i] = 0;
        proj[3 * i] = -1;  // mTrackProjX = -1, mTrackProjY = -1
        proj[3 * i + 1] = -1;
        proj[3 * i + 2] = 0;
        depth[i] = 0;
        level[i] = 0;
        view_cos[i] = 0;
        const float* P = pos + 3 * i;
        float Pc[3];
        for (int r = 0; r < 3; ++r)
            Pc[r] = std::fma(F->Tcw[4 * r + 2], P[2], std::fma(F->Tcw[4 * r], P[0], F->Tcw[4 * r + 1] * P[1])) + F->Tcw[4 * r + 3];
        const float Pc_dist = std::sqrt(dot3(Pc, Pc));
        const float PcZ = Pc[2];
        const float invz = 1.0f / PcZ;
        if (PcZ < 0.0f) continue;
        const float u = F->fx * Pc[0] / Pc[2] + F->cx;  // Pinhole::project(Eigen::Vector3f)
        const float v = F->fy * Pc[1] / Pc[2] + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        proj[3 * i] = u;
        proj[3 * i + 1] = v;
        const float maxDistance = 1.2f * max_dist[i];
        const float minDistance = 0.8f * min_dist[i];
        const float PO[3] = {P[0] - F->Ow[0], P[1] - F->Ow[1], P[2] - F->Ow[2]};
        const float dist = std::sqrt(dot3(PO, PO));
        if (dist < minDistance || dist > maxDistance) continue;
        const float viewCos = dot3(PO, normal + 3 * i) / dist;
        if (viewCos < viewingCosLimit) continue;
        const float ratio = max_dist[i] / dist;  // PredictScale, src/MapPoint.cc:715-731
        int nScale = (int)std::ceil(std::log(ratio) / F->log_scale_factor);  // logf, float division, ceilf
        if (nScale < 0) nScale = 0;
        else if (nScale >= F->n_levels) nScale = F->n_levels - 1;
        in_view[i] = 1;
        proj[3 * i + 2] = std::fma(-F->bf, invz, u);
        depth[i] = Pc_dist;
        level[i] = nScale;
        view_cos[i] = viewCos;
        ++n_in;
    }
    return n_in;
}
