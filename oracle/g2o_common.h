// ORACLE -- TEST INFRASTRUCTURE ONLY.  g2o / Eigen pieces shared by the optimiser restatements
// (orb_ba_oracle.cpp: LocalBundleAdjustment, orb_pose_oracle.cpp: PoseOptimization): SE3Quat
// (types/se3quat.h), Eigen quaternion formulas, RobustKernelHuber (core/robust_kernel_impl.cpp:65-91)
// and a dense LDL^T standing in for the Eigen factorisations (same solution up to rounding).
#pragma once
#include <cmath>
#include <vector>

namespace oracle_g2o {

struct Quat {
    double x, y, z, w;
};

inline Quat qmul(const Quat& a, const Quat& b) {  // Eigen Quaternion::operator*
    return Quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}

inline void qrotate(const Quat& q, const double v[3], double out[3]) {  // Eigen _transformVector
    double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    for (double& u : uv) u += u;
    const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
    for (int i = 0; i < 3; ++i) out[i] = v[i] + q.w * uv[i] + c[i];
}

inline void qmatrix(const Quat& q, double R[9]) {  // Eigen toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

inline Quat qfrom_matrix(const double m[9]) {  // Eigen quaternionbase_assign_impl<Matrix3>
    auto M = [&](int r, int c) { return m[3 * r + c]; };
    Quat q;
    double t = M(0, 0) + M(1, 1) + M(2, 2);
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (M(2, 1) - M(1, 2)) * t;
        q.y = (M(0, 2) - M(2, 0)) * t;
        q.z = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (M(k, j) - M(j, k)) * t;
        c[j] = (M(j, i) + M(i, j)) * t;
        c[k] = (M(k, i) + M(i, k)) * t;
        q.x = c[0]; q.y = c[1]; q.z = c[2];
    }
    return q;
}

inline void normalize_rotation(Quat& q) {  // SE3Quat::normalizeRotation
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    if (n > 0) { q.x /= n; q.y /= n; q.z /= n; q.w /= n; }
}

struct SE3 {
    Quat r;
    double t[3];
    void map(const double X[3], double out[3]) const {
        qrotate(r, X, out);
        for (int i = 0; i < 3; ++i) out[i] += t[i];
    }
};

inline SE3 se3_exp(const double u[6]) {  // SE3Quat::exp (omega first, then upsilon)
    const double w[3] = {u[0], u[1], u[2]};
    const double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double O2[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    double R[9], V[9];
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (theta < 0.00001) {
        for (int k = 0; k < 9; ++k) R[k] = V[k] = I[k] + O[k] + O2[k];
    } else {
        const double s = std::sin(theta), c = std::cos(theta);
        const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / std::pow(theta, 3);
        for (int k = 0; k < 9; ++k) {
            R[k] = I[k] + a * O[k] + b * O2[k];
            V[k] = I[k] + b * O[k] + d * O2[k];
        }
    }
    SE3 out;
    out.r = qfrom_matrix(R);
    for (int i = 0; i < 3; ++i) out.t[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
    normalize_rotation(out.r);
    return out;
}

inline SE3 se3_mul(const SE3& a, const SE3& b) {  // SE3Quat::operator*
    SE3 r = a;
    double rt[3];
    qrotate(a.r, b.t, rt);
    for (int i = 0; i < 3; ++i) r.t[i] += rt[i];
    r.r = qmul(a.r, b.r);
    normalize_rotation(r.r);
    return r;
}

struct Huber {  // RobustKernelHuber: `dsqr` is a float member (robust_kernel_impl.h:84)
    double delta;
    float dsqr;
    explicit Huber(float d) : delta(d), dsqr((float)((double)d * (double)d)) {}
    void robustify(double e, double rho[3]) const {
        if (e <= dsqr) {
            rho[0] = e; rho[1] = 1.; rho[2] = 0.;
        } else {
            const double sqrte = std::sqrt(e);
            rho[0] = 2 * sqrte * delta - dsqr;
            rho[1] = delta / sqrte;
            rho[2] = -0.5 * rho[1] / e;
        }
    }
};

// dense LDL^T of the n x n symmetric matrix (upper triangle given), solve in place
inline bool ldlt_solve(std::vector<double>& S, int n, const std::vector<double>& b, std::vector<double>& x) {
    std::vector<double> L(S.size(), 0.0), d(n);
    for (int j = 0; j < n; ++j) {
        double dj = S[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) dj -= L[(size_t)j * n + k] * L[(size_t)j * n + k] * d[k];
        if (dj == 0) return false;
        d[j] = dj;
        for (int i = j + 1; i < n; ++i) {
            double v = S[(size_t)j * n + i];  // upper triangle: (j, i) = (i, j)
            for (int k = 0; k < j; ++k) v -= L[(size_t)i * n + k] * L[(size_t)j * n + k] * d[k];
            L[(size_t)i * n + j] = v / dj;
        }
    }
    x = b;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < i; ++k) x[i] -= L[(size_t)i * n + k] * x[k];
    for (int i = 0; i < n; ++i) x[i] /= d[i];
    for (int i = n - 1; i >= 0; --i)
        for (int k = i + 1; k < n; ++k) x[i] -= L[(size_t)k * n + i] * x[k];
    return true;
}

}  // namespace oracle_g2o
