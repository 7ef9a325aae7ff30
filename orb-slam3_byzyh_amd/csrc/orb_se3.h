// Device restatements of g2o's SE3Quat (types/se3quat.h), the Eigen quaternion formulas it uses and
// RobustKernelHuber (core/robust_kernel_impl.cpp:78-91), shared by the FP64 optimisers
// (orb_ba.hip: LocalBundleAdjustment, orb_pose.hip: PoseOptimization).
#pragma once
#include <hip/hip_runtime.h>

namespace {

// ---- SE3Quat / Eigen quaternion helpers (types/se3quat.h) ---------------------------------------

__device__ __forceinline__ void qrotate(const double q[4], const double v[3], double o[3]) {
    // Eigen _transformVector: uv = 2 q.vec x v; v + w uv + q.vec x uv
    double uv0 = 2 * (q[1] * v[2] - q[2] * v[1]);
    double uv1 = 2 * (q[2] * v[0] - q[0] * v[2]);
    double uv2 = 2 * (q[0] * v[1] - q[1] * v[0]);
    o[0] = v[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
    o[1] = v[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
    o[2] = v[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

__device__ __forceinline__ void qmatrix(const double q[4], double R[9]) {
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

__device__ __forceinline__ void qnormalize(double q[4]) {  // SE3Quat::normalizeRotation
    if (q[3] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (n > 0) for (int i = 0; i < 4; ++i) q[i] /= n;
}

__device__ void qfrom_matrix(const double m[9], double q[4]) {  // Eigen Quaternion(Matrix3)
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else if (m[4] <= m[0] && m[8] <= m[0]) {  // i = 0, j = 1, k = 2
        t = sqrt(m[0] - m[4] - m[8] + 1.0);
        q[0] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[7] - m[5]) * t;
        q[1] = (m[3] + m[1]) * t;
        q[2] = (m[6] + m[2]) * t;
    } else if (m[8] <= m[4]) {  // i = 1, j = 2, k = 0
        t = sqrt(m[4] - m[8] - m[0] + 1.0);
        q[1] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[2] - m[6]) * t;
        q[2] = (m[7] + m[5]) * t;
        q[0] = (m[1] + m[3]) * t;
    } else {  // i = 2, j = 0, k = 1
        t = sqrt(m[8] - m[0] - m[4] + 1.0);
        q[2] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3] - m[1]) * t;
        q[0] = (m[2] + m[6]) * t;
        q[1] = (m[5] + m[7]) * t;
    }
}

// pose <- exp(u) * pose (VertexSE3Expmap::oplusImpl, SE3Quat::exp then operator*)
__device__ void se3_oplus(double T[7], const double u[6]) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int k = 0; k < 9; ++k) R[k] = V[k] = (k % 4 == 0 ? 1.0 : 0.0) + O[k] + O2[k];
    } else {
        const double s = sin(theta), c = cos(theta);
        const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / (theta * theta * theta);
        for (int k = 0; k < 9; ++k) {
            const double I = (k % 4 == 0 ? 1.0 : 0.0);
            R[k] = I + a * O[k] + b * O2[k];
            V[k] = I + b * O[k] + d * O2[k];
        }
    }
    double eq[4], et[3];
    qfrom_matrix(R, eq);
    for (int i = 0; i < 3; ++i) et[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
    qnormalize(eq);  // SE3Quat(Quaterniond(R), V*upsilon)
    // (eq, et) * (q, t): t' = et + eq * t, q' = eq * q, normalised
    const double q[4] = {T[3], T[4], T[5], T[6]};
    double rt[3];
    qrotate(eq, T, rt);
    double nq[4] = {eq[3] * q[0] + eq[0] * q[3] + eq[1] * q[2] - eq[2] * q[1],
                    eq[3] * q[1] + eq[1] * q[3] + eq[2] * q[0] - eq[0] * q[2],
                    eq[3] * q[2] + eq[2] * q[3] + eq[0] * q[1] - eq[1] * q[0],
                    eq[3] * q[3] - eq[0] * q[0] - eq[1] * q[1] - eq[2] * q[2]};
    qnormalize(nq);
    T[0] = et[0] + rt[0];
    T[1] = et[1] + rt[1];
    T[2] = et[2] + rt[2];
    for (int i = 0; i < 4; ++i) T[3 + i] = nq[i];
}

// RobustKernelHuber with its float dsqr member (robust_kernel_impl.cpp:78-91)
__device__ __forceinline__ void huber(double e, double delta, float dsqr, double& rho0, double& rho1) {
    if (e <= (double)dsqr) {
        rho0 = e;
        rho1 = 1.0;
    } else {
        const double sqrte = sqrt(e);
        rho0 = 2 * sqrte * delta - (double)dsqr;
        rho1 = delta / sqrte;
    }
}

struct Huber2 {
    double delta_mono, delta_stereo;
    float dsqr_mono, dsqr_stereo;
};

}  // namespace
