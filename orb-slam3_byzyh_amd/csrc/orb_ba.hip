// Optimizer::LocalBundleAdjustment on MI355X: g2o's Levenberg-Marquardt with the BlockSolver_6_3
// Schur complement, FP64 (reference src/Optimizer.cc:1740-2188 and the vendored g2o:
// core/optimization_algorithm_levenberg.cpp:61-194, core/block_solver.hpp:354-560,
// core/base_binary_edge.hpp:55-120, types/types_six_dof_expmap.*, types/se3quat.h,
// src/OptimizableTypes.cpp:175-197).
//
// Device data (per handle, grown on demand; all FP64 except the float inputs the reference has):
//   pose[7] (t, q) + backup, point[3] + backup, edges (40 B), per-edge scratch (error, robust
//   chi2, Hpl = B^T W A, the point and pose parts of the quadratic form), Hpp (6x6 per free pose),
//   Hll (3x3 per landmark), b, Dinv, Z = Hpl Dinv, S (dense n x n, n = 6 * free poses), x.
// Host-built structure (once per call, g2o's buildStructure): Hessian indices (free poses by id,
// then landmarks by id), landmark -> edges CSR (pose rows ascending), pose -> edges CSR, and the
// list of (edge, edge) products feeding each upper block of S, in landmark order.
//
// One LM iteration = k_ba_build (per edge: error, Huber weight, Jacobians, quadratic form parts)
// -> k_ba_reduce_land / k_ba_reduce_pose (fixed-order reductions) -> per trial:
// k_ba_schur_land (Dinv, Z, Hpl*db) -> k_ba_schur_blocks (S = Hpp + lambda I - sum Z Hpl^T, one
// wave per 6x6 block) -> k_ba_schur_rhs -> k_ba_chol (single-workgroup blocked Cholesky + both
// triangular solves) -> k_ba_backsub (x_l) -> k_ba_update (push + oplus) -> k_ba_error -> k_ba_sums
// (robust chi2 and g2o's computeScale).  The host reads two scalars per trial and runs g2o's
// accept / reject logic (rejection restores the backup, like g2o's pop()).
//
// Reductions run in a fixed order, so results are deterministic; they differ from g2o's serial
// sums by rounding only (parity bar: 1e-6 RMSE on poses).  S is factored with Cholesky; Eigen's
// SimplicialLDLT differs only by rounding on the SPD matrices LM produces (H PSD, lambda > 0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {

constexpr int kT = 256;
constexpr int kCholThreads = 1024;

struct EdgeDev {  // == orb_ba_edge_t
    int32_t point, pose, stereo;
    float inv_sigma2;
    double obs[3];
};
static_assert(sizeof(EdgeDev) == sizeof(orb_ba_edge_t), "edge layout");

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
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * t;
        c[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        c[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q[0] = c[0]; q[1] = c[1]; q[2] = c[2];
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

// ---- per-edge error / linearisation ------------------------------------------------------------

template <bool kBuild>
__global__ __launch_bounds__(kT) void k_ba_edges(int ne, const EdgeDev* __restrict__ edges,
                                                 const orb_ba_camera_t* __restrict__ cams,
                                                 const double* __restrict__ pose, const double* __restrict__ point,
                                                 const int32_t* __restrict__ pose_h, Huber2 hub,
                                                 double* __restrict__ err, double* __restrict__ rho0_out,
                                                 double* __restrict__ ecl, double* __restrict__ hpl,
                                                 double* __restrict__ ecp) {
    const int e = blockIdx.x * kT + threadIdx.x;
    if (e >= ne) return;
    const EdgeDev E = edges[e];
    const orb_ba_camera_t cam = cams[E.pose];
    double T[7], X[3], Xc[3];
    for (int i = 0; i < 7; ++i) T[i] = pose[7 * (size_t)E.pose + i];
    for (int i = 0; i < 3; ++i) X[i] = point[3 * (size_t)E.point + i];
    const double q[4] = {T[3], T[4], T[5], T[6]};
    qrotate(q, X, Xc);
    Xc[0] += T[0]; Xc[1] += T[1]; Xc[2] += T[2];
    double er[3];
    if (!E.stereo) {  // obs - Pinhole::project (src/CameraModels/Pinhole.cpp:47-54)
        er[0] = E.obs[0] - ((double)cam.fx * Xc[0] / Xc[2] + (double)cam.cx);
        er[1] = E.obs[1] - ((double)cam.fy * Xc[1] / Xc[2] + (double)cam.cy);
        er[2] = 0.0;
    } else {  // EdgeStereoSE3ProjectXYZ::cam_project: float invz and bf (types_six_dof_expmap.cpp:190-197)
        const float invz = (float)(1.0f / Xc[2]);
        const double u = Xc[0] * invz * (double)cam.fx + (double)cam.cx;
        const double v = Xc[1] * invz * (double)cam.fy + (double)cam.cy;
        er[0] = E.obs[0] - u;
        er[1] = E.obs[1] - v;
        er[2] = E.obs[2] - (u - (double)(cam.bf * invz));
    }
    const double info = (double)E.inv_sigma2;
    double chi2 = er[0] * info * er[0] + er[1] * info * er[1];
    if (E.stereo) chi2 += er[2] * info * er[2];
    double rho0, rho1;
    if (E.stereo) huber(chi2, hub.delta_stereo, hub.dsqr_stereo, rho0, rho1);
    else huber(chi2, hub.delta_mono, hub.dsqr_mono, rho0, rho1);
    err[3 * (size_t)e] = er[0];
    err[3 * (size_t)e + 1] = er[1];
    err[3 * (size_t)e + 2] = er[2];
    rho0_out[e] = rho0;
    if (!kBuild) return;

    // Jacobians: A = d e / d point (D x 3), B = d e / d pose (D x 6, rotation first)
    double R[9];
    qmatrix(q, R);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double fx = cam.fx, fy = cam.fy;
    const int D = E.stereo ? 3 : 2;
    double A[9], B[18];
    if (!E.stereo) {  // src/OptimizableTypes.cpp:175-197 with -Pinhole::projectJac
        const double j00 = -(fx / z), j02 = -(-fx * x / (z * z)), j11 = -(fy / z), j12 = -(-fy * y / (z * z));
        for (int c = 0; c < 3; ++c) {
            A[c] = j00 * R[c] + j02 * R[6 + c];
            A[3 + c] = j11 * R[3 + c] + j12 * R[6 + c];
        }
        // [j00 0 j02; 0 j11 j12] * [0 z -y 1 0 0; -z 0 x 0 1 0; y -x 0 0 0 1]
        B[0] = j02 * y;  B[1] = j00 * z - j02 * x; B[2] = -j00 * y; B[3] = j00; B[4] = 0;   B[5] = j02;
        B[6] = -j11 * z + j12 * y; B[7] = -j12 * x; B[8] = j11 * x;  B[9] = 0;  B[10] = j11; B[11] = j12;
        A[6] = A[7] = A[8] = 0;
        for (int k = 12; k < 18; ++k) B[k] = 0;
    } else {  // types_six_dof_expmap.cpp:228-274
        const double bf = cam.bf, z2 = z * z;
        for (int c = 0; c < 3; ++c) {
            A[c] = -fx * R[c] / z + fx * x * R[6 + c] / z2;
            A[3 + c] = -fy * R[3 + c] / z + fy * y * R[6 + c] / z2;
            A[6 + c] = A[c] - bf * R[6 + c] / z2;
        }
        B[0] = x * y / z2 * fx; B[1] = -(1 + (x * x / z2)) * fx; B[2] = y / z * fx;
        B[3] = -1. / z * fx; B[4] = 0; B[5] = x / z2 * fx;
        B[6] = (1 + y * y / z2) * fy; B[7] = -x * y / z2 * fy; B[8] = -x / z * fy;
        B[9] = 0; B[10] = -1. / z * fy; B[11] = y / z2 * fy;
        B[12] = B[0] - bf * y / z2; B[13] = B[1] + bf * x / z2; B[14] = B[2];
        B[15] = B[3]; B[16] = 0; B[17] = B[5] - bf / z2;
    }
    // BaseBinaryEdge::constructQuadraticForm, robust branch: W = rho1 * Omega, omega_r = -Omega e rho1
    const double w = rho1 * info;
    double omr[3];
    for (int r = 0; r < 3; ++r) omr[r] = -info * er[r] * rho1;
    double* pl = ecl + 12 * (size_t)e;  // Hll part (3x3) + b_l part (3)
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int r = 0; r < D; ++r) s += A[3 * r + i] * w * A[3 * r + j];
            pl[3 * i + j] = s;
        }
        double bs = 0;
        for (int r = 0; r < D; ++r) bs += A[3 * r + i] * omr[r];
        pl[9 + i] = bs;
    }
    if (pose_h[E.pose] < 0) return;
    double* hx = hpl + 18 * (size_t)e;  // B^T W A (6 x 3)
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int r = 0; r < D; ++r) s += B[6 * r + i] * w * A[3 * r + j];
            hx[3 * i + j] = s;
        }
    double* pp = ecp + 42 * (size_t)e;  // Hpp part (6x6) + b_p part (6)
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) {
            double s = 0;
            for (int r = 0; r < D; ++r) s += B[6 * r + i] * w * B[6 * r + j];
            pp[6 * i + j] = s;
        }
        double bs = 0;
        for (int r = 0; r < D; ++r) bs += B[6 * r + i] * omr[r];
        pp[36 + i] = bs;
    }
}

// Hll and b_l per landmark: sum of its edges in edge order (g2o accumulates in edge id order)
__global__ __launch_bounds__(kT) void k_ba_reduce_land(int nl, const int32_t* __restrict__ off,
                                                       const int32_t* __restrict__ eidx, const double* __restrict__ ecl,
                                                       double* __restrict__ hll, double* __restrict__ bl) {
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l >= nl) return;
    double s[12] = {0};
    for (int k = off[l]; k < off[l + 1]; ++k) {
        const double* p = ecl + 12 * (size_t)eidx[k];
        for (int i = 0; i < 12; ++i) s[i] += p[i];
    }
    for (int i = 0; i < 9; ++i) hll[9 * (size_t)l + i] = s[i];
    for (int i = 0; i < 3; ++i) bl[3 * (size_t)l + i] = s[9 + i];
}

// Hpp and b_p per free pose: one wave, lanes stride the pose's edges, fixed-order tree in LDS
__global__ __launch_bounds__(64) void k_ba_reduce_pose(const int32_t* __restrict__ off, const int32_t* __restrict__ eidx,
                                                       const double* __restrict__ ecp, double* __restrict__ hpp,
                                                       double* __restrict__ bp) {
    __shared__ double red[42][65];
    const int p = blockIdx.x, lane = threadIdx.x;
    double s[42];
    for (int i = 0; i < 42; ++i) s[i] = 0;
    for (int k = off[p] + lane; k < off[p + 1]; k += 64) {
        const double* q = ecp + 42 * (size_t)eidx[k];
        for (int i = 0; i < 42; ++i) s[i] += q[i];
    }
    for (int i = 0; i < 42; ++i) red[i][lane] = s[i];
    __syncthreads();
    for (int w = 32; w >= 1; w >>= 1) {
        if (lane < w)
            for (int i = 0; i < 42; ++i) red[i][lane] += red[i][lane + w];
        __syncthreads();
    }
    if (lane < 36) hpp[36 * (size_t)p + lane] = red[lane][0];
    else if (lane < 42) bp[6 * (size_t)p + lane - 36] = red[lane][0];
}

// max |diag| over the free vertices' Hessian blocks (computeLambdaInit)
__global__ __launch_bounds__(kT) void k_ba_maxdiag(int nf, int nl, const double* __restrict__ hpp,
                                                   const double* __restrict__ hll, double* __restrict__ out) {
    __shared__ double red[kT];
    double m = 0;
    for (int i = threadIdx.x; i < 6 * nf; i += kT) m = fmax(m, fabs(hpp[36 * (size_t)(i / 6) + 7 * (i % 6)]));
    for (int i = threadIdx.x; i < 3 * nl; i += kT) m = fmax(m, fabs(hll[9 * (size_t)(i / 3) + 4 * (i % 3)]));
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = kT / 2; w >= 1; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

__device__ __forceinline__ void inverse3(const double m[9], double o[9]) {  // Eigen closed form
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return m[3 * i1 + j1] * m[3 * i2 + j2] - m[3 * i1 + j2] * m[3 * i2 + j1];
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double invdet = 1.0 / (c0 * m[0] + c1 * m[3] + c2 * m[6]);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o[3 * i + j] = cof(j, i) * invdet;
}

// per landmark: Dinv = (Hll + lambda I)^-1, db = Dinv b_l, Z_e = Hpl_e Dinv, cb_e = Hpl_e db
__global__ __launch_bounds__(kT) void k_ba_schur_land(int nl, double lambda, const int32_t* __restrict__ off,
                                                      const int32_t* __restrict__ eidx, const double* __restrict__ hll,
                                                      const double* __restrict__ bl, const double* __restrict__ hpl,
                                                      double* __restrict__ dinv, double* __restrict__ z,
                                                      double* __restrict__ cb) {
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l >= nl) return;
    double D[9], Di[9];
    for (int i = 0; i < 9; ++i) D[i] = hll[9 * (size_t)l + i] + (i % 4 == 0 ? lambda : 0.0);
    inverse3(D, Di);
    for (int i = 0; i < 9; ++i) dinv[9 * (size_t)l + i] = Di[i];
    const double b0 = bl[3 * (size_t)l], b1 = bl[3 * (size_t)l + 1], b2 = bl[3 * (size_t)l + 2];
    double db[3];
    for (int r = 0; r < 3; ++r) db[r] = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
    for (int k = off[l]; k < off[l + 1]; ++k) {
        const int e = eidx[k];
        const double* H = hpl + 18 * (size_t)e;
        double* Z = z + 18 * (size_t)e;
        double* C = cb + 6 * (size_t)e;
        for (int r = 0; r < 6; ++r) {
            const double h0 = H[3 * r], h1 = H[3 * r + 1], h2 = H[3 * r + 2];
            for (int c = 0; c < 3; ++c) Z[3 * r + c] = h0 * Di[c] + h1 * Di[3 + c] + h2 * Di[6 + c];
            C[r] = h0 * db[0] + h1 * db[1] + h2 * db[2];
        }
    }
}

// S block (bi, bj), bi <= bj: one wave, lane = 6*r + c (36 lanes); S = [Hpp + lambda I] - sum Z_a Hpl_b^T
__global__ __launch_bounds__(256) void k_ba_schur_blocks(int nblk, int n, double lambda, const int32_t* __restrict__ bi,
                                                         const int32_t* __restrict__ bj, const int32_t* __restrict__ off,
                                                         const int32_t* __restrict__ pa, const int32_t* __restrict__ pb,
                                                         const double* __restrict__ z, const double* __restrict__ hpl,
                                                         const double* __restrict__ hpp, double* __restrict__ S) {
    const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (blk >= nblk || lane >= 36) return;
    const int r = lane / 6, c = lane % 6;
    const int i = bi[blk], j = bj[blk];
    double s = 0;
    if (i == j) s = hpp[36 * (size_t)i + 6 * r + c] + (r == c ? lambda : 0.0);
    double acc = 0;
    for (int k = off[blk]; k < off[blk + 1]; ++k) {
        const double* Z = z + 18 * (size_t)pa[k] + 3 * r;
        const double* H = hpl + 18 * (size_t)pb[k] + 3 * c;
        acc += Z[0] * H[0] + Z[1] * H[1] + Z[2] * H[2];
    }
    s -= acc;
    S[(size_t)(6 * i + r) * n + 6 * j + c] = s;
    S[(size_t)(6 * j + c) * n + 6 * i + r] = s;
}

// b_S = b_p - sum over the pose's edges of Hpl_e db (one wave per free pose)
__global__ __launch_bounds__(64) void k_ba_schur_rhs(const int32_t* __restrict__ off, const int32_t* __restrict__ eidx,
                                                     const double* __restrict__ cb, const double* __restrict__ bp,
                                                     double* __restrict__ bs) {
    __shared__ double red[6][65];
    const int p = blockIdx.x, lane = threadIdx.x;
    double s[6] = {0, 0, 0, 0, 0, 0};
    for (int k = off[p] + lane; k < off[p + 1]; k += 64) {
        const double* q = cb + 6 * (size_t)eidx[k];
        for (int i = 0; i < 6; ++i) s[i] += q[i];
    }
    for (int i = 0; i < 6; ++i) red[i][lane] = s[i];
    __syncthreads();
    for (int w = 32; w >= 1; w >>= 1) {
        if (lane < w)
            for (int i = 0; i < 6; ++i) red[i][lane] += red[i][lane + w];
        __syncthreads();
    }
    if (lane < 6) bs[6 * (size_t)p + lane] = bp[6 * (size_t)p + lane] - red[lane][0];
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// Dense Cholesky S = L L^T (lower, in place) and the solves L y = b, L^T x = y, one workgroup.
// Right-looking, panel width NB: wave 0 factors the NB x NB diagonal block in registers (lane r =
// row r, cross-lane reads through v_readlane), all threads solve the panel rows against it and
// apply the trailing update from the LDS-staged panel (4x4 register tiles).
template <int NB>
__global__ __launch_bounds__(kCholThreads) void k_ba_chol(int n, double* __restrict__ S, const double* __restrict__ b,
                                                          double* __restrict__ x, int32_t* __restrict__ status) {
    extern __shared__ double lds[];
    double* P = lds;                              // panel rows [m][NB + 1]
    double* y = lds + (size_t)n * (NB + 1);       // rhs / solution (n)
    __shared__ double Lkk[NB][NB + 1];
    __shared__ double yblk[NB];
    __shared__ int fail;
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += kCholThreads) y[i] = b[i];
    if (tid == 0) fail = 0;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += NB) {
        const int kb = min(NB, n - k0);
        const int k1 = k0 + kb;
        if (tid < 64) {
            // ---- diagonal block: lane r holds row r (identity padding beyond kb)
            const int r = tid;
            double row[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c)
                row[c] = (r < kb && c < kb) ? S[(size_t)(k0 + r) * n + k0 + c] : (r == c ? 1.0 : 0.0);
            bool bad = false;
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const double piv = readlane_d(row[c], c);
                bad |= !(piv > 0.0);
                const double lcc = sqrt(piv);
                if (r == c) row[c] = lcc;
                else if (r > c) row[c] = row[c] / lcc;
#pragma unroll
                for (int j = c + 1; j < NB; ++j) {
                    const double ljc = readlane_d(row[c], j);
                    if (r >= j) row[j] -= row[c] * ljc;
                }
            }
            // forward solve of this block of y: yb_c = (y_c - sum_{k<c} L_ck yb_k) / L_cc
            double yy = (r < kb) ? y[k0 + r] : 0.0;
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const double yc = readlane_d(yy, c) / readlane_d(row[c], c);
                if (r == c) yy = yc;
                else if (r > c) yy -= row[c] * yc;
            }
            if (r < NB) {
#pragma unroll
                for (int c = 0; c < NB; ++c) Lkk[r][c] = row[c];
                yblk[r] = yy;
            }
            if (r < kb) {
                y[k0 + r] = yy;
#pragma unroll
                for (int c = 0; c < NB; ++c)
                    if (c <= r && c < kb) S[(size_t)(k0 + r) * n + k0 + c] = row[c];
            }
            if (r == 0 && bad) fail = 1;
        }
        __syncthreads();
        // ---- panel: rows i >= k1 solve L[i, k0:k1] L_kk^T = S[i, k0:k1]; update y[i]
        const int m = n - k1;
        for (int t = tid; t < m; t += kCholThreads) {
            const int i = k1 + t;
            double v[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) v[c] = c < kb ? S[(size_t)i * n + k0 + c] : 0.0;
            double yi = y[i];
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                double s = v[c];
#pragma unroll
                for (int k = 0; k < c; ++k) s -= v[k] * Lkk[c][k];
                v[c] = s / Lkk[c][c];
                yi -= v[c] * yblk[c];
            }
            y[i] = yi;
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                P[(size_t)t * (NB + 1) + c] = v[c];
                if (c < kb) S[(size_t)i * n + k0 + c] = v[c];
            }
        }
        __syncthreads();
        // ---- trailing update of the lower triangle S[k1:n, k1:n] -= P P^T, 4x4 tiles
        const int nt = (m + 3) / 4;
        const int ntiles = nt * (nt + 1) / 2;
        for (int tt = tid; tt < ntiles; tt += kCholThreads) {
            // tile (ti, tj), tj <= ti, enumerated row by row
            int ti = (int)((sqrt(8.0 * tt + 1.0) - 1.0) * 0.5);
            while ((ti + 1) * (ti + 2) / 2 <= tt) ++ti;
            while (ti * (ti + 1) / 2 > tt) --ti;
            const int tj = tt - ti * (ti + 1) / 2;
            double acc[4][4];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[a][c] = 0;
            const int ia = 4 * ti, ja = 4 * tj;
#pragma unroll 4
            for (int k = 0; k < NB; ++k) {
                double pi[4], pj[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    pi[a] = (ia + a < m) ? P[(size_t)(ia + a) * (NB + 1) + k] : 0.0;
                    pj[a] = (ja + a < m) ? P[(size_t)(ja + a) * (NB + 1) + k] : 0.0;
                }
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[a][c] += pi[a] * pj[c];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int i = ia + a, j = ja + c;
                    if (i < m && j <= i) S[(size_t)(k1 + i) * n + k1 + j] -= acc[a][c];
                }
        }
        __syncthreads();
    }
    // ---- backward: L^T x = y, block by block from the bottom
    for (int k0 = ((n - 1) / NB) * NB; k0 >= 0; k0 -= NB) {
        const int kb = min(NB, n - k0);
        if (tid < 64) {
            const int c = tid;  // lane c holds column c of L_kk: L[k0 + r][k0 + c], r >= c
            double col[NB];
#pragma unroll
            for (int r = 0; r < NB; ++r)
                col[r] = (r < kb && c < kb && r >= c) ? S[(size_t)(k0 + r) * n + k0 + c] : (r == c ? 1.0 : 0.0);
            double yy = (c < kb) ? y[k0 + c] : 0.0;
#pragma unroll
            for (int r = NB - 1; r >= 0; --r) {
                const double xr = readlane_d(yy, r) / readlane_d(col[r], r);
                if (c == r) yy = xr;
                else if (c < r) yy -= col[r] * xr;
            }
            if (c < kb) {
                y[k0 + c] = yy;
                yblk[c] = yy;
            }
        }
        __syncthreads();
        // y[j] -= sum_c L[k0 + c][j] x_c for j < k0
        for (int j = tid; j < k0; j += kCholThreads) {
            double s = 0;
            for (int c = 0; c < kb; ++c) s += S[(size_t)(k0 + c) * n + j] * yblk[c];
            y[j] -= s;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += kCholThreads) x[i] = y[i];
    if (tid == 0) *status = fail;
}

// x_l = Dinv (b_l - sum_e Hpl_e^T x_pose(e))
__global__ __launch_bounds__(kT) void k_ba_backsub(int nl, int n, const int32_t* __restrict__ off,
                                                   const int32_t* __restrict__ eidx, const EdgeDev* __restrict__ edges,
                                                   const int32_t* __restrict__ pose_h, const double* __restrict__ hpl,
                                                   const double* __restrict__ bl, const double* __restrict__ dinv,
                                                   double* __restrict__ x) {
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l >= nl) return;
    double cl[3] = {bl[3 * (size_t)l], bl[3 * (size_t)l + 1], bl[3 * (size_t)l + 2]};
    for (int k = off[l]; k < off[l + 1]; ++k) {
        const int e = eidx[k];
        const double* H = hpl + 18 * (size_t)e;
        const double* xp = x + 6 * (size_t)pose_h[edges[e].pose];
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 6; ++r) cl[c] += H[3 * r + c] * -xp[r];
    }
    const double* Di = dinv + 9 * (size_t)l;
    for (int r = 0; r < 3; ++r) x[n + 3 * (size_t)l + r] = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
}

// push + oplus for every free vertex: threads [0, nf) poses, [nf, nf + nl) landmarks
__global__ __launch_bounds__(kT) void k_ba_update(int nf, int nl, int n, const int32_t* __restrict__ free_pose,
                                                  const int32_t* __restrict__ land_point, const double* __restrict__ x,
                                                  double* __restrict__ pose, double* __restrict__ pose_bak,
                                                  double* __restrict__ point, double* __restrict__ point_bak) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < nf) {
        double* T = pose + 7 * (size_t)free_pose[t];
        double* Tb = pose_bak + 7 * (size_t)free_pose[t];
        double v[7], u[6];
        for (int i = 0; i < 7; ++i) Tb[i] = v[i] = T[i];
        for (int i = 0; i < 6; ++i) u[i] = x[6 * (size_t)t + i];
        se3_oplus(v, u);
        for (int i = 0; i < 7; ++i) T[i] = v[i];
    } else if (t < nf + nl) {
        const int l = t - nf;
        double* X = point + 3 * (size_t)land_point[l];
        double* Xb = point_bak + 3 * (size_t)land_point[l];
        for (int i = 0; i < 3; ++i) {
            Xb[i] = X[i];
            X[i] += x[n + 3 * (size_t)l + i];
        }
    }
}

__global__ __launch_bounds__(kT) void k_ba_restore(int nf, int nl, const int32_t* __restrict__ free_pose,
                                                   const int32_t* __restrict__ land_point, double* __restrict__ pose,
                                                   const double* __restrict__ pose_bak, double* __restrict__ point,
                                                   const double* __restrict__ point_bak) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < nf) {
        for (int i = 0; i < 7; ++i) pose[7 * (size_t)free_pose[t] + i] = pose_bak[7 * (size_t)free_pose[t] + i];
    } else if (t < nf + nl) {
        const int l = t - nf;
        for (int i = 0; i < 3; ++i) point[3 * (size_t)land_point[l] + i] = point_bak[3 * (size_t)land_point[l] + i];
    }
}

// out[0] = sum rho0 (activeRobustChi2), out[1] = sum x (lambda x + b) (computeScale, before +1e-3)
__global__ __launch_bounds__(1024) void k_ba_sums(int ne, const double* __restrict__ rho0, int nx, double lambda,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  double* __restrict__ out) {
    __shared__ double r0[1024], r1[1024];
    double a = 0, c = 0;
    for (int i = threadIdx.x; i < ne; i += 1024) a += rho0[i];
    if (x)
        for (int i = threadIdx.x; i < nx; i += 1024) c += x[i] * (lambda * x[i] + b[i]);
    r0[threadIdx.x] = a;
    r1[threadIdx.x] = c;
    __syncthreads();
    for (int w = 512; w >= 1; w >>= 1) {
        if (threadIdx.x < w) {
            r0[threadIdx.x] += r0[threadIdx.x + w];
            r1[threadIdx.x] += r1[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = r0[0];
        out[1] = r1[0];
    }
}

__global__ __launch_bounds__(kT) void k_ba_final(int ne, const EdgeDev* __restrict__ edges, const double* __restrict__ pose,
                                                 const double* __restrict__ point, const double* __restrict__ err,
                                                 double* __restrict__ chi2, uint8_t* __restrict__ depth_ok) {
    const int e = blockIdx.x * kT + threadIdx.x;
    if (e >= ne) return;
    const EdgeDev E = edges[e];
    const double info = (double)E.inv_sigma2;
    const double* er = err + 3 * (size_t)e;
    double c = er[0] * info * er[0] + er[1] * info * er[1];
    if (E.stereo) c += er[2] * info * er[2];
    chi2[e] = c;
    const double* T = pose + 7 * (size_t)E.pose;
    const double q[4] = {T[3], T[4], T[5], T[6]};
    double Xc[3];
    qrotate(q, point + 3 * (size_t)E.point, Xc);
    depth_ok[e] = (Xc[2] + T[2]) > 0.0;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    bool grow(size_t n) {
        if (n <= cap) return true;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return false;
        cap = n;
        return true;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct orb_ba_s {
    hipStream_t stream = nullptr;
    DevBuf<double> pose, pose_bak, point, point_bak, err, rho0, ecl, hpl, ecp, hpp, hll, b, dinv, z, cb, S, bs, x, scal;
    DevBuf<EdgeDev> edges;
    DevBuf<orb_ba_camera_t> cams;
    DevBuf<int32_t> pose_h, free_pose, land_point, land_off, land_edge, landf_off, landf_edge, pose_off, pose_edge,
        blk_i, blk_j, blk_off, pair_a, pair_b, status;
    DevBuf<uint8_t> depth;
    double* h_scal = nullptr;  // pinned: [0] chi2, [1] scale, [2] status, [3] maxdiag
    float ms_total = 0;

    void release() {
        for (auto* d : {&pose, &pose_bak, &point, &point_bak, &err, &rho0, &ecl, &hpl, &ecp, &hpp, &hll, &b, &dinv, &z,
                        &cb, &S, &bs, &x, &scal})
            d->release();
        edges.release();
        cams.release();
        for (auto* d : {&pose_h, &free_pose, &land_point, &land_off, &land_edge, &landf_off, &landf_edge, &pose_off,
                        &pose_edge, &blk_i, &blk_j, &blk_off, &pair_a, &pair_b, &status})
            d->release();
        depth.release();
    }
};

namespace {

template <typename T>
bool upload(DevBuf<T>& d, const T* h, size_t n, hipStream_t s) {
    if (!d.grow(n)) return false;
    return n == 0 || hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s) == hipSuccess;
}

template <typename T>
bool upload(DevBuf<T>& d, const std::vector<T>& h, hipStream_t s) {
    return upload(d, h.data(), h.size(), s);
}

unsigned grid(size_t n, int t = kT) { return (unsigned)std::max<size_t>(1, (n + t - 1) / t); }

}  // namespace

extern "C" {

int orb_ba_create(orb_ba_t* out) {
    if (!out) return orbgpu_fail(ORB_ERR_ARG, "null handle pointer");
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) {
        (void)hipGetLastError();
        return orbgpu_fail(ORB_ERR_DEVICE, "no HIP device");
    }
    auto* h = new orb_ba_s();
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(&h->h_scal, 8 * sizeof(double), hipHostMallocDefault) != hipSuccess) {
        delete h;
        return orbgpu_fail(ORB_ERR_DEVICE, "BA handle allocation");
    }
    *out = h;
    return ORB_OK;
}

int orb_ba_destroy(orb_ba_t h) {
    if (!h) return ORB_OK;
    hipStreamSynchronize(h->stream);
    h->release();
    if (h->h_scal) hipHostFree(h->h_scal);
    hipStreamDestroy(h->stream);
    delete h;
    return ORB_OK;
}

int orb_ba_optimize(orb_ba_t h, orb_ba_problem_t* pr, const orb_ba_options_t* opt, double* edge_chi2,
                    uint8_t* edge_depth_ok, orb_ba_result_t* res) {
    if (!h || !pr || !opt || !res) return orbgpu_fail(ORB_ERR_ARG, "null BA argument");
    memset(res, 0, sizeof(*res));
    const int np = pr->n_poses, nq = pr->n_points, ne = pr->n_edges;
    if (np < 0 || nq < 0 || ne < 0 || (np && (!pr->pose || !pr->pose_id || !pr->pose_fixed || !pr->pose_camera)) ||
        (nq && (!pr->point || !pr->point_id)) || (ne && !pr->edges) || opt->iterations < 0)
        return orbgpu_fail(ORB_ERR_ARG, "invalid BA problem");
    for (int e = 0; e < ne; ++e) {
        const orb_ba_edge_t& E = pr->edges[e];
        if (E.point < 0 || E.point >= nq || E.pose < 0 || E.pose >= np || (E.stereo != 0 && E.stereo != 1))
            return orbgpu_fail(ORB_ERR_ARG, "BA edge references a missing vertex");
    }
    auto stop = [&]() { return opt->stop_flag && *opt->stop_flag; };

    // ---- structure (initializeOptimization + BlockSolver::buildStructure)
    std::vector<int> pdeg(np, 0), qdeg(nq, 0);
    for (int e = 0; e < ne; ++e) { pdeg[pr->edges[e].pose]++; qdeg[pr->edges[e].point]++; }
    std::vector<int> order(np);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return pr->pose_id[a] < pr->pose_id[b]; });
    std::vector<int32_t> pose_h(np, -1), free_pose;
    for (int i : order)
        if (pdeg[i] && !pr->pose_fixed[i]) { pose_h[i] = (int32_t)free_pose.size(); free_pose.push_back(i); }
    std::vector<int> qorder(nq);
    std::iota(qorder.begin(), qorder.end(), 0);
    std::sort(qorder.begin(), qorder.end(), [&](int a, int b) { return pr->point_id[a] < pr->point_id[b]; });
    std::vector<int32_t> point_l(nq, -1), land_point;
    for (int i : qorder)
        if (qdeg[i]) { point_l[i] = (int32_t)land_point.size(); land_point.push_back(i); }
    const int nf = (int)free_pose.size(), nl = (int)land_point.size();
    if (ne == 0 || nf + nl == 0) {  // SparseOptimizer::optimize returns -1: nothing to do
        for (int e = 0; e < ne; ++e) {
            if (edge_chi2) edge_chi2[e] = 0;
            if (edge_depth_ok) edge_depth_ok[e] = 0;
        }
        return ORB_OK;
    }
    if (stop()) { res->stopped = 1; return ORB_ERR_ABORTED; }
    const int n = 6 * nf, m = 3 * nl;
    if (n > 6 * 300) return orbgpu_fail(ORB_ERR_ARG, "more than 300 free keyframes in one local BA");

    // landmark -> all edges (edge order), landmark -> free-pose edges (pose row ascending), pose -> edges
    std::vector<int32_t> land_off(nl + 1, 0), land_edge(ne), landf_off(nl + 1, 0), landf_edge, pose_off(nf + 1, 0),
        pose_edge;
    for (int e = 0; e < ne; ++e) {
        land_off[point_l[pr->edges[e].point] + 1]++;
        if (pose_h[pr->edges[e].pose] >= 0) {
            landf_off[point_l[pr->edges[e].point] + 1]++;
            pose_off[pose_h[pr->edges[e].pose] + 1]++;
        }
    }
    for (int l = 0; l < nl; ++l) { land_off[l + 1] += land_off[l]; landf_off[l + 1] += landf_off[l]; }
    for (int p = 0; p < nf; ++p) pose_off[p + 1] += pose_off[p];
    landf_edge.resize(landf_off[nl]);
    pose_edge.resize(pose_off[nf]);
    {
        std::vector<int32_t> c1(land_off.begin(), land_off.end() - 1), c2(landf_off.begin(), landf_off.end() - 1),
            c3(pose_off.begin(), pose_off.end() - 1);
        for (int e = 0; e < ne; ++e) {
            const int l = point_l[pr->edges[e].point], p = pose_h[pr->edges[e].pose];
            land_edge[c1[l]++] = e;
            if (p >= 0) {
                landf_edge[c2[l]++] = e;
                pose_edge[c3[p]++] = e;
            }
        }
    }
    for (int l = 0; l < nl; ++l)
        std::stable_sort(landf_edge.begin() + landf_off[l], landf_edge.begin() + landf_off[l + 1],
                         [&](int a, int b) { return pose_h[pr->edges[a].pose] < pose_h[pr->edges[b].pose]; });
    // Schur block pattern: (row_a <= row_b) products per landmark, in landmark order
    std::vector<int32_t> blk_id((size_t)nf * nf, -1), blk_i, blk_j;
    std::vector<int32_t> cnt;
    for (int l = 0; l < nl; ++l)
        for (int a = landf_off[l]; a < landf_off[l + 1]; ++a)
            for (int b2 = a; b2 < landf_off[l + 1]; ++b2) {
                const int i = pose_h[pr->edges[landf_edge[a]].pose], j = pose_h[pr->edges[landf_edge[b2]].pose];
                int32_t& id = blk_id[(size_t)i * nf + j];
                if (id < 0) { id = (int32_t)blk_i.size(); blk_i.push_back(i); blk_j.push_back(j); cnt.push_back(0); }
                cnt[id]++;
            }
    const int nblk = (int)blk_i.size();
    std::vector<int32_t> blk_off(nblk + 1, 0);
    for (int k = 0; k < nblk; ++k) blk_off[k + 1] = blk_off[k] + cnt[k];
    std::vector<int32_t> pair_a(blk_off[nblk]), pair_b(blk_off[nblk]);
    {
        std::vector<int32_t> c(blk_off.begin(), blk_off.end() - 1);
        for (int l = 0; l < nl; ++l)
            for (int a = landf_off[l]; a < landf_off[l + 1]; ++a)
                for (int b2 = a; b2 < landf_off[l + 1]; ++b2) {
                    const int i = pose_h[pr->edges[landf_edge[a]].pose], j = pose_h[pr->edges[landf_edge[b2]].pose];
                    const int id = blk_id[(size_t)i * nf + j];
                    pair_a[c[id]] = landf_edge[a];
                    pair_b[c[id]++] = landf_edge[b2];
                }
    }
    // poses normalised as SE3Quat(q, t) does
    std::vector<double> pose(pr->pose, pr->pose + 7 * (size_t)np);
    for (int i = 0; i < np; ++i) {
        double* q = &pose[7 * (size_t)i + 3];
        if (q[3] < 0) for (int k = 0; k < 4; ++k) q[k] = -q[k];
        const double nn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        if (nn > 0) for (int k = 0; k < 4; ++k) q[k] /= nn;
    }

    hipStream_t s = h->stream;
    bool ok = upload(h->pose, pose, s) && h->pose_bak.grow(7 * (size_t)np) &&
              upload(h->point, pr->point, 3 * (size_t)nq, s) && h->point_bak.grow(3 * (size_t)nq) &&
              upload(h->edges, reinterpret_cast<const EdgeDev*>(pr->edges), ne, s) &&
              upload(h->cams, pr->pose_camera, np, s) && upload(h->pose_h, pose_h, s) &&
              upload(h->free_pose, free_pose, s) && upload(h->land_point, land_point, s) &&
              upload(h->land_off, land_off, s) && upload(h->land_edge, land_edge, s) &&
              upload(h->landf_off, landf_off, s) && upload(h->landf_edge, landf_edge, s) &&
              upload(h->pose_off, pose_off, s) && upload(h->pose_edge, pose_edge, s) && upload(h->blk_i, blk_i, s) &&
              upload(h->blk_j, blk_j, s) && upload(h->blk_off, blk_off, s) && upload(h->pair_a, pair_a, s) &&
              upload(h->pair_b, pair_b, s) && h->err.grow(3 * (size_t)ne) && h->rho0.grow(ne) &&
              h->ecl.grow(12 * (size_t)ne) && h->hpl.grow(18 * (size_t)ne) && h->ecp.grow(42 * (size_t)ne) &&
              h->hpp.grow(36 * (size_t)nf) && h->hll.grow(9 * (size_t)nl) && h->b.grow(n + m) &&
              h->dinv.grow(9 * (size_t)nl) && h->z.grow(18 * (size_t)ne) && h->cb.grow(6 * (size_t)ne) &&
              h->S.grow((size_t)n * n) && h->bs.grow(n) && h->x.grow(n + m) && h->scal.grow(8) && h->status.grow(1) &&
              h->depth.grow(ne);
    if (!ok) return orbgpu_fail(ORB_ERR_DEVICE, "BA device allocation / upload");
    hipMemsetAsync(h->x.p, 0, sizeof(double) * (n + m), s);  // g2o's _x starts zeroed

    const float dm = (float)std::sqrt(5.991), ds = (float)std::sqrt(7.815);  // src/Optimizer.cc:1957-1958
    const Huber2 hub{(double)dm, (double)ds, (float)((double)dm * (double)dm), (float)((double)ds * (double)ds)};
    // dynamic LDS of the Cholesky kernel: panel rows (n x (NB + 1)) + y (n)
    int nb = 32;
    size_t chol_lds = sizeof(double) * ((size_t)n * (nb + 1) + n);
    if (chol_lds > 150 * 1024) { nb = 16; chol_lds = sizeof(double) * ((size_t)n * (nb + 1) + n); }
    if (chol_lds > 150 * 1024) { nb = 8; chol_lds = sizeof(double) * ((size_t)n * (nb + 1) + n); }
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void*)k_ba_chol<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        hipFuncSetAttribute((const void*)k_ba_chol<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        hipFuncSetAttribute((const void*)k_ba_chol<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        attr_set = true;
    }
    double* bl = h->b.p + n;
    auto launch_edges = [&](bool build) {
        if (build)
            hipLaunchKernelGGL(k_ba_edges<true>, dim3(grid(ne)), dim3(kT), 0, s, ne, h->edges.p, h->cams.p, h->pose.p,
                               h->point.p, h->pose_h.p, hub, h->err.p, h->rho0.p, h->ecl.p, h->hpl.p, h->ecp.p);
        else
            hipLaunchKernelGGL(k_ba_edges<false>, dim3(grid(ne)), dim3(kT), 0, s, ne, h->edges.p, h->cams.p, h->pose.p,
                               h->point.p, h->pose_h.p, hub, h->err.p, h->rho0.p, h->ecl.p, h->hpl.p, h->ecp.p);
    };
    auto read_scalars = [&](double lambda, bool with_x) -> bool {
        hipLaunchKernelGGL(k_ba_sums, dim3(1), dim3(1024), 0, s, ne, h->rho0.p, n + m, lambda,
                           with_x ? h->x.p : nullptr, h->b.p, h->scal.p);
        hipMemcpyAsync(h->scal.p + 2, h->status.p, sizeof(int32_t), hipMemcpyDeviceToDevice, s);
        hipMemcpyAsync(h->h_scal, h->scal.p, 4 * sizeof(double), hipMemcpyDeviceToHost, s);
        return hipStreamSynchronize(s) == hipSuccess;
    };

    double lambda = 0, ni = 2;
    int nBad = 0, it = 0;
    const double tau = 1e-5;
    for (; it < opt->iterations && !stop(); ++it) {
        // computeActiveErrors + activeRobustChi2 + buildSystem
        launch_edges(true);
        hipLaunchKernelGGL(k_ba_reduce_land, dim3(grid(nl)), dim3(kT), 0, s, nl, h->land_off.p, h->land_edge.p,
                           h->ecl.p, h->hll.p, bl);
        if (nf)
            hipLaunchKernelGGL(k_ba_reduce_pose, dim3(nf), dim3(64), 0, s, h->pose_off.p, h->pose_edge.p, h->ecp.p,
                               h->hpp.p, h->b.p);
        if (it == 0)
            hipLaunchKernelGGL(k_ba_maxdiag, dim3(1), dim3(kT), 0, s, nf, nl, h->hpp.p, h->hll.p, h->scal.p + 3);
        if (!read_scalars(0.0, false)) return orbgpu_fail(ORB_ERR_DEVICE, "BA build failed");
        double currentChi = h->h_scal[0];
        const double iniChi = currentChi;
        if (it == 0) {
            res->initial_chi2 = currentChi;
            lambda = opt->user_lambda_init > 0 ? opt->user_lambda_init : tau * h->h_scal[3];
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            // setLambda + BlockSolver::solve
            hipLaunchKernelGGL(k_ba_schur_land, dim3(grid(nl)), dim3(kT), 0, s, nl, lambda, h->landf_off.p,
                               h->landf_edge.p, h->hll.p, bl, h->hpl.p, h->dinv.p, h->z.p, h->cb.p);
            if (nf) {
                hipMemsetAsync(h->S.p, 0, sizeof(double) * (size_t)n * n, s);
                hipLaunchKernelGGL(k_ba_schur_blocks, dim3((nblk + 3) / 4), dim3(256), 0, s, nblk, n, lambda,
                                   h->blk_i.p, h->blk_j.p, h->blk_off.p, h->pair_a.p, h->pair_b.p, h->z.p, h->hpl.p,
                                   h->hpp.p, h->S.p);
                hipLaunchKernelGGL(k_ba_schur_rhs, dim3(nf), dim3(64), 0, s, h->pose_off.p, h->pose_edge.p, h->cb.p,
                                   h->b.p, h->bs.p);
                if (nb == 32)
                    hipLaunchKernelGGL(k_ba_chol<32>, dim3(1), dim3(kCholThreads), chol_lds, s, n, h->S.p, h->bs.p,
                                       h->x.p, h->status.p);
                else if (nb == 16)
                    hipLaunchKernelGGL(k_ba_chol<16>, dim3(1), dim3(kCholThreads), chol_lds, s, n, h->S.p, h->bs.p,
                                       h->x.p, h->status.p);
                else
                    hipLaunchKernelGGL(k_ba_chol<8>, dim3(1), dim3(kCholThreads), chol_lds, s, n, h->S.p, h->bs.p,
                                       h->x.p, h->status.p);
            } else {
                hipMemsetAsync(h->status.p, 0, sizeof(int32_t), s);
            }
            hipLaunchKernelGGL(k_ba_backsub, dim3(grid(nl)), dim3(kT), 0, s, nl, n, h->landf_off.p, h->landf_edge.p,
                               h->edges.p, h->pose_h.p, h->hpl.p, bl, h->dinv.p, h->x.p);
            // SparseOptimizer::update (push first), then computeActiveErrors
            hipLaunchKernelGGL(k_ba_update, dim3(grid(nf + nl)), dim3(kT), 0, s, nf, nl, n, h->free_pose.p,
                               h->land_point.p, h->x.p, h->pose.p, h->pose_bak.p, h->point.p, h->point_bak.p);
            launch_edges(false);
            if (!read_scalars(lambda, true)) return orbgpu_fail(ORB_ERR_DEVICE, "BA trial failed");
            res->trials++;
            int32_t st;
            memcpy(&st, &h->h_scal[2], sizeof(st));
            double tempChi = h->h_scal[0];
            if (st) tempChi = std::numeric_limits<double>::max();  // solve failed (not positive definite)
            rho = currentChi - tempChi;
            double scale = h->h_scal[1] + 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                hipLaunchKernelGGL(k_ba_restore, dim3(grid(nf + nl)), dim3(kT), 0, s, nf, nl, h->free_pose.p,
                                   h->land_point.p, h->pose.p, h->pose_bak.p, h->point.p, h->point_bak.p);
            }
            qmax++;
        } while (rho < 0 && qmax < 10 && !stop());
        res->final_chi2 = currentChi;
        if (qmax == 10 || rho == 0) { res->terminated = 1; ++it; break; }
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) { res->terminated = 1; ++it; break; }
    }
    res->iterations = it;
    res->lambda = lambda;
    res->stopped = stop() ? 1 : 0;
    hipLaunchKernelGGL(k_ba_final, dim3(grid(ne)), dim3(kT), 0, s, ne, h->edges.p, h->pose.p, h->point.p, h->err.p,
                       h->rho0.p, h->depth.p);
    hipMemcpyAsync(pr->pose, h->pose.p, sizeof(double) * 7 * (size_t)np, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(pr->point, h->point.p, sizeof(double) * 3 * (size_t)nq, hipMemcpyDeviceToHost, s);
    if (edge_chi2) hipMemcpyAsync(edge_chi2, h->rho0.p, sizeof(double) * ne, hipMemcpyDeviceToHost, s);
    if (edge_depth_ok) hipMemcpyAsync(edge_depth_ok, h->depth.p, ne, hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "BA device error");
    return ORB_OK;
}

}  // extern "C"
