// Frame::SetPose after PoseOptimization (src/Optimizer.cc:390-395 -> src/Frame.cc:533-599): the g2o
// SE3Quat estimate (tx ty tz qx qy qz qw, double) cast to float, Sophus::SE3<float> (its SO3 constructor
// normalises the quaternion), then UpdatePoseMatrices: mRcw = rotationMatrix() (Eigen's
// Quaternion::toRotationMatrix), mtcw = translation(), mOw = Twc.translation() = q^-1 * (-t) (Eigen's
// _transformVector with the conjugate).  Float arithmetic in the written order, no contraction; shared by
// the device tracking chain (csrc/orb_frustum.hip) and the oracle (oracle/orb_tracking_oracle.cpp).
// Parity with a real Eigen / Sophus build is unpinned (its vectorised sums cannot be observed here).
#pragma once

#ifdef __HIPCC__
#define ORB_PF_HD __host__ __device__
#else
#define ORB_PF_HD
#endif

#include <cmath>

ORB_PF_HD inline void orb_pose7_to_frame(const double p[7], float Tcw[12], float Ow[3]) {
    float x = (float)p[3], y = (float)p[4], z = (float)p[5], w = (float)p[6];
    const float n = sqrtf(((x * x + y * y) + z * z) + w * w);  // SO3(Quaternion) -> normalize()
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
    // Twc = Tcw.inverse(): invR = conj(q), Ow = invR * (-t) = v + w uv + qv x uv, uv = 2 (qv x v)
    const float qv[3] = {-x, -y, -z}, v[3] = {t[0] * -1.0f, t[1] * -1.0f, t[2] * -1.0f};
    float uv[3] = {qv[1] * v[2] - qv[2] * v[1], qv[2] * v[0] - qv[0] * v[2], qv[0] * v[1] - qv[1] * v[0]};
    for (int k = 0; k < 3; ++k) uv[k] = uv[k] + uv[k];
    const float c2[3] = {qv[1] * uv[2] - qv[2] * uv[1], qv[2] * uv[0] - qv[0] * uv[2], qv[0] * uv[1] - qv[1] * uv[0]};
    for (int k = 0; k < 3; ++k) Ow[k] = (v[k] + w * uv[k]) + c2[k];
}

// The pose the next PoseOptimization starts from after Frame::SetPose (src/Optimizer.cc:76-80 reads
// pFrame->GetPose(): g2o::SE3Quat(Tcw.unit_quaternion().cast<double>(), Tcw.translation().cast<double>())):
// the float cast, the quaternion normalised as Sophus's SO3 constructor does, back to double.
ORB_PF_HD inline void orb_pose7_float_roundtrip(const double p[7], double out[7]) {
    float x = (float)p[3], y = (float)p[4], z = (float)p[5], w = (float)p[6];
    const float n = sqrtf(((x * x + y * y) + z * z) + w * w);
    x = x / n; y = y / n; z = z / n; w = w / n;
    out[0] = (double)(float)p[0];
    out[1] = (double)(float)p[1];
    out[2] = (double)(float)p[2];
    out[3] = (double)x;
    out[4] = (double)y;
    out[5] = (double)z;
    out[6] = (double)w;
}
