// ORACLE (test infrastructure only; never linked into or called by the product path).
//
// Frame::SetPose after PoseOptimization, restated from the reference and its vendored Sophus, on its own
// (it shares no code with the device chain; tests/native/pose_frame_check.cpp compares the two bit for
// bit):
//   src/Optimizer.cc:390-395   Sophus::SE3<float> pose(SE3quat.rotation().cast<float>(),
//                                                      SE3quat.translation().cast<float>());
//                              pFrame->SetPose(pose);
//   src/Frame.cc:533-540,591-599   SetPose -> UpdatePoseMatrices: Twc = mTcw.inverse(); mRwc, mOw =
//                              Twc.translation(); mRcw = mTcw.rotationMatrix(); mtcw = mTcw.translation()
//   Thirdparty/Sophus/sophus/se3.hpp:488-490   SE3(Quaternion, Point): so3_(quaternion) -> SO3 ctor
//   Thirdparty/Sophus/sophus/so3.hpp:480-487   SO3(QuaternionBase): unit_quaternion_(quat); normalize()
//   Thirdparty/Sophus/sophus/so3.hpp:297-303   normalize(): length = norm(); coeffs() /= length
//   Thirdparty/Sophus/sophus/so3.hpp:229-231   inverse(): SO3(unit_quaternion().conjugate()) -- the SO3
//                                              constructor normalises the conjugate AGAIN
//   Thirdparty/Sophus/sophus/se3.hpp:208-211   inverse(): invR = so3().inverse();
//                                              SE3(invR, invR * (translation() * Scalar(-1)))
//   Thirdparty/Sophus/sophus/so3.hpp:358-367   SO3 * p: uv = q.vec().cross(p); uv += uv;
//                                              return p + q.w() * uv + q.vec().cross(uv)
//   Thirdparty/Sophus/sophus/so3.hpp:310-312   matrix() = unit_quaternion().toRotationMatrix()
// External (Eigen 3.3/3.4, not in this image):
//   QuaternionBase::norm() = sqrt(coeffs().cwiseAbs2().sum()); for the 16-byte aligned float[4] coeffs
//   (x, y, z, w) the x86 build reduces one SSE packet with predux<Packet4f>: tmp = a + movehl(a, a),
//   result = tmp[0] + tmp[1], i.e. (x^2 + z^2) + (y^2 + w^2).  coeffs() /= s divides every coefficient.
//   Quaternion::toRotationMatrix (Eigen/src/Geometry/Quaternion.h): tx = 2x, ..., twx = tx*w, ...,
//   R = [[1-(tyy+tzz), txy-twz, txz+twy], [txy+twz, 1-(txx+tzz), tyz-twx], [txz-twy, tyz+twx, 1-(txx+tyy)]].
//   MatrixBase::cross for 3-vectors: (a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0).
// Float arithmetic in the written order, no contraction (oracle/Makefile: -ffp-contract=off).  Whether
// the reference build's g++ contracts any of these products is not observable here: parity with a real
// Eigen/Sophus build is unpinned beyond the operation order stated above.
#include <cmath>

namespace {

struct QuatF {  // Eigen::Quaternionf coefficient order
    float c[4];  // x, y, z, w
};

struct Vec3F {
    float v[3];
};

// Eigen: coeffs().cwiseAbs2().sum() on one SSE packet (predux<Packet4f>)
float eigen_coeffs_squared_norm(const QuatF& q) {
    const float a0 = q.c[0] * q.c[0], a1 = q.c[1] * q.c[1], a2 = q.c[2] * q.c[2], a3 = q.c[3] * q.c[3];
    const float lo = a0 + a2;  // _mm_add_ps(a, _mm_movehl_ps(a, a)) lanes 0, 1
    const float hi = a1 + a3;
    return lo + hi;            // _mm_add_ss(tmp, shuffle(tmp, 1))
}

// Sophus SO3 constructor: copy then normalize()
QuatF sophus_so3(const QuatF& q) {
    QuatF r = q;
    const float length = std::sqrt(eigen_coeffs_squared_norm(r));
    for (float& c : r.c) c /= length;
    return r;
}

QuatF conjugate(const QuatF& q) { return QuatF{{-q.c[0], -q.c[1], -q.c[2], q.c[3]}}; }

Vec3F cross(const float a[3], const float b[3]) {
    return Vec3F{{a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]}};
}

// Sophus SO3 * point
Vec3F so3_act(const QuatF& q, const Vec3F& p) {
    const float* qv = q.c;  // q.vec() = (x, y, z)
    Vec3F uv = cross(qv, p.v);
    for (float& u : uv.v) u += u;
    const Vec3F c2 = cross(qv, uv.v);
    Vec3F out;
    for (int k = 0; k < 3; ++k) out.v[k] = (p.v[k] + q.c[3] * uv.v[k]) + c2.v[k];
    return out;
}

// Eigen Quaternion::toRotationMatrix, row-major 3x3
void to_rotation_matrix(const QuatF& q, float R[9]) {
    const float x = q.c[0], y = q.c[1], z = q.c[2], w = q.c[3];
    const float tx = 2.0f * x, ty = 2.0f * y, tz = 2.0f * z;
    const float twx = tx * w, twy = ty * w, twz = tz * w;
    const float txx = tx * x, txy = ty * x, txz = tz * x;
    const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0f - (tyy + tzz); R[1] = txy - twz;          R[2] = txz + twy;
    R[3] = txy + twz;          R[4] = 1.0f - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;          R[7] = tyz + twx;          R[8] = 1.0f - (txx + tyy);
}

// g2o SE3Quat (tx ty tz qx qy qz qw, double) -> Sophus::SE3f as PoseOptimization builds it
void se3f_from_pose7(const double p[7], QuatF& q, Vec3F& t) {
    const QuatF qf{{(float)p[3], (float)p[4], (float)p[5], (float)p[6]}};  // Quaterniond::cast<float>()
    q = sophus_so3(qf);
    t = Vec3F{{(float)p[0], (float)p[1], (float)p[2]}};
}

}  // namespace

// Tcw as the 3x4 row-major [mRcw | mtcw] and mOw = Twc.translation()
extern "C" void oracle_pose7_to_frame(const double* pose7, float* Tcw, float* Ow) {
    QuatF q;
    Vec3F t;
    se3f_from_pose7(pose7, q, t);
    float R[9];
    to_rotation_matrix(q, R);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) Tcw[4 * r + c] = R[3 * r + c];
        Tcw[4 * r + 3] = t.v[r];
    }
    const QuatF inv = sophus_so3(conjugate(q));  // SO3::inverse(): a new SO3, normalised again
    Vec3F mt;
    for (int k = 0; k < 3; ++k) mt.v[k] = t.v[k] * -1.0f;  // translation() * Scalar(-1)
    const Vec3F o = so3_act(inv, mt);
    for (int k = 0; k < 3; ++k) Ow[k] = o.v[k];
}

// The pose the next PoseOptimization starts from (src/Optimizer.cc:76-80: g2o::SE3Quat(
// Tcw.unit_quaternion().cast<double>(), Tcw.translation().cast<double>()) of the Frame's mTcw)
extern "C" void oracle_pose7_float_roundtrip(const double* pose7, double* out) {
    QuatF q;
    Vec3F t;
    se3f_from_pose7(pose7, q, t);
    for (int k = 0; k < 3; ++k) out[k] = (double)t.v[k];
    for (int k = 0; k < 4; ++k) out[3 + k] = (double)q.c[k];
}
