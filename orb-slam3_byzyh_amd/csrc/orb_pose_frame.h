// Frame::SetPose after PoseOptimization (src/Optimizer.cc:390-395 -> src/Frame.cc:533-599): the g2o
// SE3Quat estimate (tx ty tz qx qy qz qw, double) cast to float, Sophus::SE3<float> (its SO3 constructor
// normalises the quaternion, Thirdparty/Sophus/sophus/so3.hpp:480-487), then UpdatePoseMatrices:
// mRcw = rotationMatrix() (Eigen's Quaternion::toRotationMatrix), mtcw = translation(), mOw =
// Twc.translation() with Twc = Tcw.inverse(): SO3::inverse() builds a NEW SO3 from the conjugate, which
// normalises again (so3.hpp:229-231), then SO3 * (t * -1) (so3.hpp:358-367, se3.hpp:208-211).
// Eigen's norm() of the float[4] coefficients is one SSE packet reduced by predux<Packet4f>:
// (x^2 + z^2) + (y^2 + w^2).  Float arithmetic in the written order, no contraction; used by the device
// tracking chain (csrc/orb_frustum.hip, csrc/orb_tracking.hip).  The oracle restates the same reference
// lines on its own (oracle/orb_tracking_oracle.cpp); tests/native/pose_frame_check.cpp compares the two
// bit for bit.  Parity with a real Eigen / Sophus build is unpinned beyond that operation order.
#pragma once

#ifdef __HIPCC__
#define ORB_PF_HD __host__ __device__
#else
#define ORB_PF_HD
#endif

#include <cmath>

// Eigen QuaternionBase::norm() on x86: sqrt of one SSE packet's predux (lanes 0+2, 1+3, then the sum)
ORB_PF_HD inline float orb_quat_norm_f(float x, float y, float z, float w) {
    return sqrtf((x * x + z * z) + (y * y + w * w));
}

ORB_PF_HD inline void orb_pose7_to_frame(const double p[7], float Tcw[12], float Ow[3]) {
    float x = (float)p[3], y = (float)p[4], z = (float)p[5], w = (float)p[6];
    const float n = orb_quat_norm_f(x, y, z, w);  // SO3(Quaternion) -> normalize()
    x = x / n; y = y / n; z = z / n; w = w / n;
    const float tx = 2.0f * x, ty = 2.0f * y, tz = 2.0f * z;  // Quaternion::toRotationMatrix
    const float twx = tx * w, twy = ty * w, twz = tz * w;
    const float txx = tx * x, txy = ty * x, txz = tz * x;
    const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
    const float R[9] = {1.0f - (tyy + tzz), txy - twz, txz + twy,
                        txy + twz, 1.0f - (txx + tzz), tyz - twx,
                        txz - twy, tyz + twx, 1.0f - (txx + tyy)};
    const float t[3] = {(float)p[0], (float)p[1], (float)p[2]};
    for (int r = 0; r < 3; ++r) {
        Tcw[4 * r] = R[3 * r];
        Tcw[4 * r + 1] = R[3 * r + 1];
        Tcw[4 * r + 2] = R[3 * r + 2];
        Tcw[4 * r + 3] = t[r];
    }
    // Twc = Tcw.inverse(): invR = SO3(conj(q)) (normalised again), Ow = invR * (-t) = v + w uv + qv x uv,
    // uv = 2 (qv x v)
    const float ni = orb_quat_norm_f(-x, -y, -z, w);
    const float qv[3] = {-x / ni, -y / ni, -z / ni}, wi = w / ni;
    const float v[3] = {t[0] * -1.0f, t[1] * -1.0f, t[2] * -1.0f};
    float uv[3] = {qv[1] * v[2] - qv[2] * v[1], qv[2] * v[0] - qv[0] * v[2], qv[0] * v[1] - qv[1] * v[0]};
    for (int k = 0; k < 3; ++k) uv[k] = uv[k] + uv[k];
    const float c2[3] = {qv[1] * uv[2] - qv[2] * uv[1], qv[2] * uv[0] - qv[0] * uv[2], qv[0] * uv[1] - qv[1] * uv[0]};
    for (int k = 0; k < 3; ++k) Ow[k] = (v[k] + wi * uv[k]) + c2[k];
}

// The pose the next PoseOptimization starts from after Frame::SetPose (src/Optimizer.cc:76-80 reads
// pFrame->GetPose(): g2o::SE3Quat(Tcw.unit_quaternion().cast<double>(), Tcw.translation().cast<double>())):
// the float cast, the quaternion normalised as Sophus's SO3 constructor does, back to double.
ORB_PF_HD inline void orb_pose7_float_roundtrip(const double p[7], double out[7]) {
    float x = (float)p[3], y = (float)p[4], z = (float)p[5], w = (float)p[6];
    const float n = orb_quat_norm_f(x, y, z, w);
    x = x / n; y = y / n; z = z / n; w = w / n;
    out[0] = (double)(float)p[0];
    out[1] = (double)(float)p[1];
    out[2] = (double)(float)p[2];
    out[3] = (double)x;
    out[4] = (double)y;
    out[5] = (double)z;
    out[6] = (double)w;
}
