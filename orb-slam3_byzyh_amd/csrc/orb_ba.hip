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
// then landmarks by id), landmark -> edges CSR (pose rows ascending) and pose -> (landmark, edge)
// lists in landmark order; the landmarks two poses share are found on the device (k_ba_schur_blocks).
//
// One LM iteration = k_ba_build (per edge: error, Huber weight, Jacobians, quadratic form parts)
// -> k_ba_reduce_land / k_ba_reduce_pose (fixed-order reductions) -> per trial:
// k_ba_schur_edges (Dinv, Z, Hpl*db per edge) -> k_ba_schur_blocks (S = Hpp + lambda I - sum Z Hpl^T,
// one wave per 6x6 block) -> k_ba_schur_rhs -> k_ba_chol (single-workgroup blocked Cholesky + both
// triangular solves) -> k_ba_backsub (x_l) -> k_ba_update (push + oplus) -> k_ba_error -> k_ba_sums
// (robust chi2 and g2o's computeScale).  The host reads two scalars per trial and runs g2o's
// accept / reject logic (rejection restores the backup, like g2o's pop()).
//
// Reductions run in a fixed order, so results are deterministic; they differ from g2o's serial
// sums by rounding only (parity bar: 1e-6 RMSE on poses).  S is factored with Cholesky; Eigen's
// SimplicialLDLT differs only by rounding on the SPD matrices LM produces (H PSD, lambda > 0).
#include <dlfcn.h>
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

#include "ba_structure.h"
#include "orbgpu.h"
#include "orbgpu_internal.h"

// The BA path is judged at 1e-6 RMSE (not bitwise like the extractor): let products and sums
// contract into FMAs in this file despite the library-wide -ffp-contract=off.
#pragma clang fp contract(fast)
#include "orb_se3.h"  // (after the pragma: the helpers contract like the rest of this file)

namespace {

#ifndef ORB_BA_KT
#define ORB_BA_KT 64
#endif
// threads per block of the edge / landmark kernels: 64 (round 5) spreads a unit kernel over 4x the CUs,
// and the FP64 per-edge work runs faster one wave per CU than four (C5 0.169 -> 0.161 ms per added
// LM iteration; tools/ba_var_ab.sh)
constexpr int kT = ORB_BA_KT;

// The host structure's list entries (csrc/ba_structure.h): a free pose's (landmark, edge) observations
// and the Schur blocks' (Z edge, Hpl edge) products.
using orbgpu_ba::EdgePair;
using orbgpu_ba::LandEdge;


struct EdgeDev {  // == orb_ba_edge_t
    int32_t point, pose, stereo;
    float inv_sigma2;
    double obs[3];
};
static_assert(sizeof(EdgeDev) == sizeof(orb_ba_edge_t), "edge layout");

// ---- Levenberg-Marquardt state of the device-driven solve -----------------------------------------
// One process: the per-trial kernels read it to decide whether to run (the build only at the start
// of an iteration, nothing once the solve has ended); k_lm_build_done / k_lm_trial_done update it
// exactly as g2o's OptimizationAlgorithmLevenberg::solve does on the host.
struct LmState {
    double lambda, ni, current_chi, ini_chi, final_chi, initial_chi, user_lambda, tau;
    int32_t it, qmax, nbad, phase, done, reject, terminated, trials, iterations;
    int32_t lin;  // which half of the double-buffered Hpl holds the current linearisation
};
// what the host reads after each unit (pinned)
struct LmProgress {
    double final_chi, initial_chi, lambda;
    int32_t done, it, trials, terminated;
};
enum { kGateBuild = 0, kGateBuild0 = 1, kGateTrial = 2, kGateRestore = 3 };

// Hpl is double-buffered on the device-driven path: every trial linearises at its new estimate into
// the other half, which becomes current when the trial is accepted (the next iteration's build
// then has nothing left to compute).  Host-driven path (no state): the first half.
__device__ __forceinline__ size_t hpl_cur(const LmState* st, size_t alt) { return st && st->lin ? alt : 0; }

__device__ __forceinline__ bool lm_skip(const LmState* st, int kind) {
    if (!st) return false;
    if (kind == kGateRestore) return !st->reject;
    if (st->done) return true;
    if (kind == kGateBuild) return st->phase != 0;
    if (kind == kGateBuild0) return st->phase != 0 || st->it != 0;
    return false;
}

// The trial's pose update (push + VertexSE3Expmap::oplusImpl per free pose) for the landmark-major
// trial kernel (k_u_land_trial), which does it in LDS for up to kT free poses, and for
// k_u_pose_update, which moves more of them (tile-row Cholesky sizes) before it.  pose == nullptr: no
// pose kernel (launch_chol).  pscale: k_u_pose_update's computeScale part of the poses,
// sum_t x_t (lambda x_t + b_p) (rank 0 only when sharded: primary).
struct PoseTail {
    const int32_t* free_pose;
    double* pose;
    double* pose_bak;
    const double* bp;
    const double* lam;
    double* pscale;
    int nf, primary;
};

// pose t of the tail: from the backup when the previous trial was rejected (and not restored), the
// backup refreshed, exp(x_t) applied.  Returns pose t's computeScale part.
__device__ __forceinline__ double pose_tail_one(const PoseTail& pt, int t, int fp, const double* __restrict__ xt,
                                                bool rej) {
    double* T = pt.pose + 7 * (size_t)fp;
    double* Tb = pt.pose_bak + 7 * (size_t)fp;
    double v[7], u[6];
    for (int i = 0; i < 7; ++i) {
        v[i] = rej ? Tb[i] : T[i];
        Tb[i] = v[i];
    }
    for (int i = 0; i < 6; ++i) u[i] = xt[i];
    double c = 0.0;
    if (pt.primary) {
        const double lambda = *pt.lam;
        for (int i = 0; i < 6; ++i) c += u[i] * (lambda * u[i] + pt.bp[6 * (size_t)t + i]);
    }
    se3_oplus(v, u);
    for (int i = 0; i < 7; ++i) T[i] = v[i];
    return c;
}

// ---- per-edge error / linearisation ------------------------------------------------------------

// Error and robust chi2 of edge E at pose T and point X (computeError + the Huber kernel); Xc: the
// point in the camera frame.  Returns rho0.
__device__ __forceinline__ double ba_edge_err(const EdgeDev& E, const orb_ba_camera_t& cam, const double T[7],
                                              const double X[3], Huber2 hub, double Xc[3], double er[3], double& rho1) {
    const double q[4] = {T[3], T[4], T[5], T[6]};
    qrotate(q, X, Xc);
    Xc[0] += T[0]; Xc[1] += T[1]; Xc[2] += T[2];
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
    double rho0;
    if (E.stereo) huber(chi2, hub.delta_stereo, hub.dsqr_stereo, rho0, rho1);
    else huber(chi2, hub.delta_mono, hub.dsqr_mono, rho0, rho1);
    return rho0;
}

// kReg (k_u_land_build): the landmark part (Hll, b_l) and the edge's Hpl kept in registers (lo) instead
// of the ecl record; Hpl and the pose part still go to memory
struct LinOut {
    double pl[12], hx[18];
    bool free;
};
template <bool kBuild, bool kReg = false>
__device__ __forceinline__ double ba_edge(int e, const EdgeDev* __restrict__ edges,
                                                 const orb_ba_camera_t* __restrict__ cams,
                                                 const double* __restrict__ pose, const double* __restrict__ point,
                                                 const int32_t* __restrict__ pose_h, Huber2 hub,
                                                 double* __restrict__ err, double* __restrict__ rho0_out,
                                                 double* __restrict__ ecl, double* __restrict__ hpl,
                                                 double* __restrict__ ecp,
        int, LinOut* lo = nullptr) {
    const EdgeDev E = edges[e];
    const orb_ba_camera_t cam = cams[E.pose];
    double T[7], X[3], Xc[3];
    for (int i = 0; i < 7; ++i) T[i] = pose[7 * (size_t)E.pose + i];
    for (int i = 0; i < 3; ++i) X[i] = point[3 * (size_t)E.point + i];
    const double q[4] = {T[3], T[4], T[5], T[6]};
    double er[3], rho1;
    const double rho0 = ba_edge_err(E, cam, T, X, hub, Xc, er, rho1);
    const double info = (double)E.inv_sigma2;
    err[3 * (size_t)e] = er[0];
    err[3 * (size_t)e + 1] = er[1];
    err[3 * (size_t)e + 2] = er[2];
    rho0_out[e] = rho0;
    if (!kBuild) return rho0;

    // Jacobians: A = d e / d point (D x 3), B = d e / d pose (D x 6, rotation first)
    double R[9];
    qmatrix(q, R);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double fx = cam.fx, fy = cam.fy;
    constexpr int D = 3;  // mono edges have a zero third row and omega_r[2] = 0: adding +0.0 is exact
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
    double* pl = kReg ? lo->pl : ecl + 12 * (size_t)e;  // Hll part (3x3) + b_l part (3)
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
    if (kReg) lo->free = pose_h[E.pose] >= 0;
    if (pose_h[E.pose] < 0) return rho0;
    double* hx = hpl + 18 * (size_t)e;  // B^T W A (6 x 3)
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int r = 0; r < D; ++r) s += B[6 * r + i] * w * A[3 * r + j];
            hx[3 * i + j] = s;
            if (kReg) lo->hx[3 * i + j] = s;
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
    return rho0;
}

template <bool kBuild>
__global__ __launch_bounds__(kT) void k_ba_edges(int ne, const EdgeDev* __restrict__ edges,
                                                 const orb_ba_camera_t* __restrict__ cams,
                                                 const double* __restrict__ pose, const double* __restrict__ point,
                                                 const int32_t* __restrict__ pose_h, Huber2 hub,
                                                 double* __restrict__ err, double* __restrict__ rho0_out,
                                                 double* __restrict__ ecl, double* __restrict__ hpl,
                                                 double* __restrict__ ecp, const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    const int e = blockIdx.x * kT + threadIdx.x;
    if (e < ne) ba_edge<kBuild>(e, edges, cams, pose, point, pose_h, hub, err, rho0_out, ecl, hpl, ecp, 0);
}

// Hll and b_l per landmark: sum of its edges in edge order (g2o accumulates in edge id order)
__device__ __forceinline__ double ba_reduce_land(int l, const int32_t* __restrict__ off, const int32_t* __restrict__ eidx,
                                               const double* __restrict__ ecl, double* __restrict__ hll,
                                               double* __restrict__ bl) {
    double s[12] = {0};
    const int k0 = off[l], k1 = off[l + 1];
    for (int kb = k0; kb < k1; kb += 8) {  // the indices of 8 edges first, operands 4 at a time, same sum order
        int e[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) e[u] = eidx[min(kb + u, k1 - 1)];
#pragma unroll
        for (int h = 0; h < 8; h += 4) {
            if (kb + h >= k1) break;
            double v[4][12];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int i = 0; i < 12; ++i) v[u][i] = ecl[12 * (size_t)e[h + u] + i];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (kb + h + u < k1)
#pragma unroll
                    for (int i = 0; i < 12; ++i) s[i] += v[u][i];
        }
    }
    for (int i = 0; i < 9; ++i) hll[9 * (size_t)l + i] = s[i];
    for (int i = 0; i < 3; ++i) bl[3 * (size_t)l + i] = s[9 + i];
    return fmax(fmax(fabs(s[0]), fabs(s[4])), fabs(s[8]));  // computeLambdaInit's part of this landmark
}

__global__ __launch_bounds__(kT) void k_ba_reduce_land(int nl, const int32_t* __restrict__ off,
                                                       const int32_t* __restrict__ eidx, const double* __restrict__ ecl,
                                                       double* __restrict__ hll, double* __restrict__ bl,
                                                       const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    const int l = blockIdx.x * kT + threadIdx.x;
    if (l < nl) (void)ba_reduce_land(l, off, eidx, ecl, hll, bl);
}

// Sum of 64 lanes' partials of NC values, lane c < NC adding value c's partials in lane order
// (LDS transpose; one pass, no barrier-separated tree).  Returns value `lane`'s sum in lanes < NC.
template <int NC>
__device__ __forceinline__ double wave_sum_cols_in(const double (&v)[NC], int lane, double (*red)[65]) {
#pragma unroll
    for (int i = 0; i < NC; ++i) red[i][lane] = v[i];
    __syncthreads();
    double t = 0;
    if (lane < NC)
        for (int q = 0; q < 64; ++q) t += red[lane][q];
    return t;
}
template <int NC>
__device__ __forceinline__ double wave_sum_cols(const double (&v)[NC], int lane) {
    __shared__ double red[NC][65];
    return wave_sum_cols_in<NC>(v, lane, red);
}
// the caller's LDS buffer (kernels whose branches would otherwise each hold their own)
template <int NC, bool kExt>
__device__ __forceinline__ double wave_sum_cols_x(const double (&v)[NC], int lane, double (*red)[65]) {
    if constexpr (kExt) return wave_sum_cols_in<NC>(v, lane, red);
    else return wave_sum_cols<NC>(v, lane);
}

// Hpp and b_p per free pose: one wave; lane l sums the pose's edges l, l + 64, ... in order.  The
// indices of up to 8 edges per lane are loaded first, then two edges' 42 values at a time, so the
// usual pose (a few hundred edges) takes three rounds of loads instead of two per edge.
template <bool kExt = false>
__device__ __forceinline__ double ba_reduce_pose(int p, int lane, const int32_t* __restrict__ off,
                                               const LandEdge* __restrict__ eidx, const double* __restrict__ ecp,
                                               double* __restrict__ hpp, double* __restrict__ bp, double (*red)[65] = nullptr) {
    double s[42];
#pragma unroll
    for (int i = 0; i < 42; ++i) s[i] = 0;
    const int k0 = off[p] + lane, k1 = off[p + 1];
    int e[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) e[u] = k0 + 64 * u < k1 ? eidx[k0 + 64 * u].e : 0;
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
        if (k0 + 64 * u >= k1) break;
        const bool two = k0 + 64 * (u + 1) < k1;
        double a[42], b[42];
#pragma unroll
        for (int i = 0; i < 42; ++i) {
            a[i] = ecp[42 * (size_t)e[u] + i];
            b[i] = ecp[42 * (size_t)e[u + 1] + i];
        }
#pragma unroll
        for (int i = 0; i < 42; ++i) s[i] += a[i];
        if (two)
#pragma unroll
            for (int i = 0; i < 42; ++i) s[i] += b[i];
    }
    for (int k = k0 + 64 * 8; k < k1; k += 64) {  // poses of more than 512 edges
        const double* q = ecp + 42 * (size_t)eidx[k].e;
#pragma unroll
        for (int i = 0; i < 42; ++i) s[i] += q[i];
    }
    const double t = wave_sum_cols_x<42, kExt>(s, lane, red);
    if (lane < 36) hpp[36 * (size_t)p + lane] = t;
    else if (lane < 42) bp[6 * (size_t)p + lane - 36] = t;
    return t;  // value `lane`'s total (lanes < 42)
}

__global__ __launch_bounds__(64) void k_ba_reduce_pose(const int32_t* __restrict__ off, const LandEdge* __restrict__ eidx,
                                                       const double* __restrict__ ecp, double* __restrict__ hpp,
                                                       double* __restrict__ bp, const LmState* __restrict__ lm_st,
                                                       int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    ba_reduce_pose(blockIdx.x, threadIdx.x, off, eidx, ecp, hpp, bp);
}

// max |diag| over the free vertices' Hessian blocks (computeLambdaInit)
__global__ __launch_bounds__(kT) void k_ba_maxdiag(int nf, int nl, const double* __restrict__ hpp,
                                                   const double* __restrict__ hll, double* __restrict__ out,
        const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
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

// Dinv = (Hll_l + lambda I)^-1 (BlockSolver::solve: D->inverse() of the damped landmark block)
__device__ __forceinline__ void land_dinv(const double* __restrict__ hll, int l, double lambda, double Di[9]) {
    double D[9];
    for (int i = 0; i < 9; ++i) D[i] = hll[9 * (size_t)l + i] + (i % 4 == 0 ? lambda : 0.0);
    inverse3(D, Di);
}

// per free edge e of landmark l: Z_e = Hpl_e Dinv_l, cb_e = Hpl_e (Dinv_l b_l) (one thread per edge)
__global__ __launch_bounds__(kT) void k_ba_schur_edges(int nfe, const double* __restrict__ lam, const int32_t* __restrict__ fedge,
                                                       const int32_t* __restrict__ fland, const double* __restrict__ hll,
                                                       const double* __restrict__ bl, const double* __restrict__ hpl,
                                                       size_t hpl_alt, double* __restrict__ z, double* __restrict__ cb,
        const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    hpl += hpl_cur(lm_st, hpl_alt);
    const double lambda = *lam;
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t >= nfe) return;
    const int e = fedge[t], l = fland[t];
    double Di[9];
    land_dinv(hll, l, lambda, Di);
    const double b0 = bl[3 * (size_t)l], b1 = bl[3 * (size_t)l + 1], b2 = bl[3 * (size_t)l + 2];
    double db[3];
    for (int r = 0; r < 3; ++r) db[r] = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
    const double* H = hpl + 18 * (size_t)e;
    double* Z = z + 18 * (size_t)e;
    double* C = cb + 6 * (size_t)e;
    for (int r = 0; r < 6; ++r) {
        const double h0 = H[3 * r], h1 = H[3 * r + 1], h2 = H[3 * r + 2];
        for (int c = 0; c < 3; ++c) Z[3 * r + c] = h0 * Di[c] + h1 * Di[3 + c] + h2 * Di[6 + c];
        C[r] = h0 * db[0] + h1 * db[1] + h2 * db[2];
    }
}

// upper-triangle block number -> (i, j), i <= j, row-major: row i starts at i nf - i (i - 1) / 2
__device__ __forceinline__ void schur_block_ij(int blk, int nf, int& i, int& j) {
    auto cum = [nf](int r) { return r * nf - r * (r - 1) / 2; };
    const double T = 2.0 * nf + 1.0;
    int r = (int)floor((T - sqrt(T * T - 8.0 * blk)) * 0.5);
    r = max(0, min(r, nf - 1));
    while (r > 0 && cum(r) > blk) --r;
    while (r < nf - 1 && cum(r + 1) <= blk) ++r;
    i = r;
    j = r + (blk - cum(r));
}

constexpr int kSchurChunk = 512;  // landmarks of pose j's list staged in LDS per pass

// The product list of S block (i, j), i <= j, built on the device once per solve (one wave per block):
// the landmarks both poses see are found by searching each of pose i's observations in pose j's
// (sorted by landmark, staged in LDS); the (Z edge, Hpl edge) pairs go out compacted in pose i's
// list order (= landmark order) to pairs[blk_off[blk] ...], at most min(|i|, |j|) of them (a pose
// sees a landmark once: the host rejects repeated (pose, point) edges), and the count to cnt[blk].
__global__ __launch_bounds__(64) void k_ba_schur_pairs(int nf, const int32_t* __restrict__ pose_off,
                                                       const LandEdge* __restrict__ pose_fl,
                                                       const int32_t* __restrict__ blk_off, EdgePair* __restrict__ pairs,
                                                       int32_t* __restrict__ cnt) {
    __shared__ int32_t sl[kSchurChunk], se[kSchurChunk];
    const int blk = blockIdx.x, lane = threadIdx.x;
    int i, j;
    schur_block_ij(blk, nf, i, j);
    const int ib = pose_off[i], ie = pose_off[i + 1], jb = pose_off[j], je = pose_off[j + 1];
    EdgePair* out = pairs + blk_off[blk];
    int q = 0;  // pairs written (wave-uniform)
    for (int jc = jb; jc < je; jc += kSchurChunk) {
        const int jn = min(kSchurChunk, je - jc);
        __syncthreads();  // the previous chunk's searches are done
        for (int k = lane; k < jn; k += 64) {
            const LandEdge v = pose_fl[jc + k];
            sl[k] = v.l;
            se[k] = v.e;
        }
        __syncthreads();
        const int lmin = sl[0], lmax = sl[jn - 1];
        for (int k0 = ib; k0 < ie; k0 += 64) {
            const int k = k0 + lane;
            LandEdge v{-1, -1};
            if (k < ie) v = pose_fl[k];
            int lo = 0;
            bool has = false;
            if (k < ie && v.l >= lmin && v.l <= lmax) {
                int hi = jn;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sl[mid] < v.l) lo = mid + 1;
                    else hi = mid;
                }
                has = lo < jn && sl[lo] == v.l;
            }
            const uint64_t mask = __ballot(has);
            const int pos = q + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
            if (has) out[pos] = EdgePair{v.e, se[lo]};
            q += __popcll(mask);
        }
    }
    if (lane == 0) cnt[blk] = q;
}

// S block (i, j), i <= j, one wave: lanes split the block's (Z_a, Hpl_b) products (k_ba_schur_pairs),
// lane l taking products l, l + 64, ... in order and accumulating the full 6x6 partial sum; the pair
// indices of up to 4 rounds are loaded first, then two products' operands at a time.  Lane e < 36
// then adds the 64 partials in lane order.  S = [Hpp + lambda I] - sum Z_a Hpl_b^T, written to both
// triangles (every block of S, empty ones as 0).
__device__ __forceinline__ void schur_acc(double (&acc)[36], const double* __restrict__ Z, const double* __restrict__ H) {
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c)
            acc[6 * r + c] += Z[3 * r] * H[3 * c] + Z[3 * r + 1] * H[3 * c + 1] + Z[3 * r + 2] * H[3 * c + 2];
}

template <bool kExt = false>
__device__ __forceinline__ void ba_schur_block(int blk, int lane, int n, int nf, double lambda, int add_diag,
                                               const int32_t* __restrict__ blk_off, const EdgePair* __restrict__ pairs,
                                               const int32_t* __restrict__ cnt, const double* __restrict__ z,
                                               const double* __restrict__ hpl, const double* __restrict__ hpp,
                                               double* __restrict__ S, double (*red)[65] = nullptr) {
    int i, j;
    schur_block_ij(blk, nf, i, j);
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; ++k) acc[k] = 0;
    const EdgePair* pl = pairs + blk_off[blk];
    const int np = cnt[blk];
    EdgePair pr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) pr[u] = lane + 64 * u < np ? pl[lane + 64 * u] : EdgePair{0, 0};
#pragma unroll
    for (int u = 0; u < 4; u += 2) {
        if (lane + 64 * u >= np) break;
        double z0[18], h0[18], z1[18], h1[18];
#pragma unroll
        for (int q = 0; q < 18; ++q) {
            z0[q] = z[18 * (size_t)pr[u].a + q];
            h0[q] = hpl[18 * (size_t)pr[u].b + q];
            z1[q] = z[18 * (size_t)pr[u + 1].a + q];
            h1[q] = hpl[18 * (size_t)pr[u + 1].b + q];
        }
        schur_acc(acc, z0, h0);
        if (lane + 64 * (u + 1) < np) schur_acc(acc, z1, h1);
    }
    for (int k = lane + 256; k < np; k += 64) {  // blocks of more than 256 products
        const EdgePair p2 = pl[k];
        double zr[18], hr[18];
#pragma unroll
        for (int q = 0; q < 18; ++q) { zr[q] = z[18 * (size_t)p2.a + q]; hr[q] = hpl[18 * (size_t)p2.b + q]; }
        schur_acc(acc, zr, hr);
    }
    const double sum = wave_sum_cols_x<36, kExt>(acc, lane, red);
    if (lane >= 36) return;
    const int r = lane / 6, c = lane % 6;
    double v = 0.0 - sum;
    if (i == j && add_diag) v = (hpp[36 * (size_t)i + 6 * r + c] + (r == c ? lambda : 0.0)) - sum;
    S[(size_t)(6 * i + r) * n + 6 * j + c] = v;
    S[(size_t)(6 * j + c) * n + 6 * i + r] = v;
}


__global__ __launch_bounds__(64) void k_ba_schur_blocks(int n, int nf, const double* __restrict__ lam, int add_diag,
                                                        const int32_t* __restrict__ blk_off,
                                                        const EdgePair* __restrict__ pairs, const int32_t* __restrict__ cnt,
                                                        const double* __restrict__ z, const double* __restrict__ hpl,
                                                        const double* __restrict__ hpp, double* __restrict__ S,
                                                        const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    ba_schur_block(blockIdx.x, threadIdx.x, n, nf, *lam, add_diag, blk_off, pairs, cnt, z, hpl, hpp, S);
}

// b_S = b_p - sum over the pose's edges of Hpl_e db (one wave per free pose; the indices of up to 8
// edges per lane first, then their 6 values each, all in flight)
__device__ __forceinline__ void ba_schur_rhs(int p, int lane, const int32_t* __restrict__ off,
                                             const LandEdge* __restrict__ eidx, const double* __restrict__ cb,
                                             const double* __restrict__ bp, int use_bp, double* __restrict__ bs) {
    double s[6] = {0, 0, 0, 0, 0, 0};
    const int k0 = off[p] + lane, k1 = off[p + 1];
    int e[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) e[u] = k0 + 64 * u < k1 ? eidx[k0 + 64 * u].e : 0;
    double v[8][6];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int i = 0; i < 6; ++i) v[u][i] = cb[6 * (size_t)e[u] + i];
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (k0 + 64 * u < k1)
#pragma unroll
            for (int i = 0; i < 6; ++i) s[i] += v[u][i];
    for (int k = k0 + 64 * 8; k < k1; k += 64) {
        const double* q = cb + 6 * (size_t)eidx[k].e;
#pragma unroll
        for (int i = 0; i < 6; ++i) s[i] += q[i];
    }
    const double t = wave_sum_cols<6>(s, lane);
    if (lane < 6) bs[6 * (size_t)p + lane] = (use_bp ? bp[6 * (size_t)p + lane] : 0.0) - t;
}

__global__ __launch_bounds__(64) void k_ba_schur_rhs(const int32_t* __restrict__ off, const LandEdge* __restrict__ eidx,
                                                     const double* __restrict__ cb, const double* __restrict__ bp,
                                                     int use_bp, double* __restrict__ bs, const LmState* __restrict__ lm_st,
                                                     int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    ba_schur_rhs(blockIdx.x, threadIdx.x, off, eidx, cb, bp, use_bp, bs);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// ---- register-resident MFMA Cholesky + solve (n <= 288, one workgroup of 12 waves) -----------------
// The lower triangle of S is cut into 16x16 tiles that live in the waves' registers for the whole
// factorisation.  Each tile holds M in the operand layout O(M) of v_mfma_f64_16x16x4_f64: lane l,
// register q = M[l & 15][(l >> 4) + 4q].  That is the C/D layout of M^T, so with tiles kept
// transposed every product below takes its operands straight from registers or from one
// lane-linear LDS read:
//   trailing update  M_ij^T -= L_jk L_ik^T      A = O(L_jk) negated (blgp = neg A), B = O(L_ik)
//   panel            L_ik^T  = L_kk^-1 A_ik^T   A = O(L_kk^-1), B = the tile itself
// Right-looking over the 16-column block steps k.  One wave factors tile (k, k) (lane r = row r,
// cross-lane reads through DPP row broadcasts) and inverts L_kk, with a look-ahead: tile (k+1, k+1)
// is updated first in step k and factored while the other waves finish their updates.  The forward solve is folded in (y_k = L_kk^-1 b_k, then b_i -= L_ik y_k by the panel
// owners); the backward solve walks the tile rows kept in registers, pipelined through LDS
// flags: the diagonal wave publishes x_k once every L_kj^T x_j contribution has landed.  Tiles are dealt round-robin
// in order of decreasing column, so the active tiles of every step are a prefix of each wave's
// slots and the load stays balanced as the trailing matrix shrinks.  Every sum has a fixed order.
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kMf2TileWaves = 11, kMfMaxNT = 18;
// ORBGPU_BA_TRACE stamps (int64 clock64, kTraceLen entries): step k, wave w, point p at
// kTrStep + (k * 16 + w) * 4 + p (w = kMf2TileWaves is the diagonal wave); backward step j at
// kTrBack + j (start), kTrWaited + j (contributions in), kTrPub + j (x_j published); the diagonal
// factorisation of step k at kTrDiag + 4 k + {0: start, 1: factored, 2: L^-1 stored, 3: y_k}.
constexpr int kTrStep = 0, kTrEnd = 1199, kTrBack = 1200, kTrWaited = 1300, kTrPub = 1400, kTrDiag = 1500,
              kTrE = 1600, kTrC = 1640, kTrD = 2240, kTraceLen = 2304;  // kTrE + 2 j: e_j's contributions in, e_j formed;
                                                           // kTrC + 32 k + 2 w: wave w's row k contributions start / end
static_assert(kTrStep + (kMfMaxNT * 16) * 4 <= kTrEnd && kTrDiag + 4 * kMfMaxNT <= kTraceLen, "trace layout");

template <int N>
__device__ __forceinline__ double dpp_row_shr(double v) {  // lane l <- lane l - N of its 16-lane row, 0 at the edge
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x110 + N, 0xf, 0xf, true);
    const uint32_t hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x110 + N, 0xf, 0xf, true);
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// Sum over the 16 lanes of each DPP row (valid in lane 15 of the row), in a fixed order.
__device__ __forceinline__ double row16_sum(double v) {
    v += dpp_row_shr<1>(v);
    v += dpp_row_shr<2>(v);
    v += dpp_row_shr<4>(v);
    v += dpp_row_shr<8>(v);
    return v;
}

// Sum over the four 16-lane rows of a wave, ((p_0 + p_1) + (p_2 + p_3)), the same double in every lane:
// v_permlane16_swap then v_permlane32_swap (gfx950), a swap and an add each, no LDS round trip.  The
// operand order matches `p += shfl_xor(p, 16); p += shfl_xor(p, 32)` bit for bit.
__device__ __forceinline__ double group4_sum(double p) {
    const int2 a = __builtin_bit_cast(int2, p);
    const auto x = __builtin_amdgcn_permlane16_swap(a.x, a.x, false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(a.y, a.y, false, false);
    const double s = __builtin_bit_cast(double, int2{(int)x[0], (int)y[0]}) +
                     __builtin_bit_cast(double, int2{(int)x[1], (int)y[1]});
    const int2 b = __builtin_bit_cast(int2, s);
    const auto u = __builtin_amdgcn_permlane32_swap(b.x, b.x, false, false);
    const auto v = __builtin_amdgcn_permlane32_swap(b.y, b.y, false, false);
    return __builtin_bit_cast(double, int2{(int)u[0], (int)v[0]}) + __builtin_bit_cast(double, int2{(int)u[1], (int)v[1]});
}

__device__ __forceinline__ void mf_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 1/sqrt(x): v_rsq_f64 and two Newton steps (about 1 ulp; the factor need not be correctly rounded)
#ifndef ORB_BA_RSQ_NEWTON
#define ORB_BA_RSQ_NEWTON 2
#endif
__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
#pragma unroll
    for (int i = 0; i < ORB_BA_RSQ_NEWTON; ++i) y = y * __builtin_fma(-h, y * y, 1.5);
    return y;
}

// One wave: factor the 16x16 block in dk (row-major, stride 17) and write L_kk^-1 in operand layout
// to linv_k; replace yk[0 .. 16) (= b_k, already reduced by the earlier panels) by y_k = L_kk^-1 b_k.
// Lane r holds row r of the block and column r of L^-1.  Column step c: one rsqrt, then the values
// L[j][c] (j > c) are broadcast once and feed both the rank-1 update of the block and
// the substitution step of L^-1 (x_i -= L[i][c] x_c).  The updates run unconditionally: entries
// above the diagonal collect garbage that is never read.
// kColMajor: L^-1 stored column-major with stride 17 (L^-1[i][c] at c * 17 + i: conflict-free for the
// writes here and for every reader); otherwise in the MFMA operand layout.

// 64-bit DPP row broadcasts folded into the consuming instruction (gfx950 DPP64: v_mov_b64 and
// v_fmac_f64 take row_newbcast): one instruction per broadcast / per rank-1 update element instead of
// two 32-bit DPP moves, their old-value initialisations and a separate FMA.  Each starts with s_nop 1,
// the VALU-write -> DPP-read wait states, which the compiler cannot see inside inline asm.  j must
// fold to a constant.
#define MF_CASES(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
__device__ __forceinline__ double bcast64(double v, int j) {  // lane j of the 16-lane row
    double r = 0.0;
    switch (j) {
#define MF_B64(J)                                                                                        \
    case J:                                                                                              \
        asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v)); \
        break;
        MF_CASES(MF_B64)
#undef MF_B64
        default: break;
    }
    return r;
}
// acc = fma(-a_j, b, acc) = acc + a_j * (-b)  with a_j = a of lane j: the same rounding as fma(-a_j, b, acc)
__device__ __forceinline__ double fmac_bcast_negb(double acc, double a, double b, int j) {
    switch (j) {
#define MF_F64(J)                                                                                              \
    case J:                                                                                                    \
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) \
            : "v"(a), "v"(b));                                                                                 \
        break;
        MF_CASES(MF_F64)
#undef MF_F64
        default: break;
    }
    return acc;
}
// acc = fma(b, a_j, acc)
__device__ __forceinline__ double fmac_bcast(double acc, double a, double b, int j) {
    switch (j) {
#define MF_F64P(J)                                                                                            \
    case J:                                                                                                   \
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) \
            : "v"(a), "v"(b));                                                                                \
        break;
        MF_CASES(MF_F64P)
#undef MF_F64P
        default: break;
    }
    return acc;
}
// acc = fma(-a_j, b, acc) with the negation on the broadcast operand
__device__ __forceinline__ double fmac_negbcast(double acc, double a, double b, int j) {
    switch (j) {
#define MF_F64N(J)                                                                                             \
    case J:                                                                                                    \
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) \
            : "v"(a), "v"(b));                                                                                 \
        break;
        MF_CASES(MF_F64N)
#undef MF_F64N
        default: break;
    }
    return acc;
}

// The same three forms without the leading s_nop, for the factor's pivot steps: every DPP read there
// has its source (the column value lrc, or row[c+1]) written at least two VALU instructions earlier,
// which mf_diag guarantees by one s_nop per pivot (dpp_fence) and by the order of its volatile
// statements (volatile asm keeps its order; other instructions the compiler places between them only
// add wait states).
#define MF_DPP_NN(NAME, ASM)                                                                  \
    __device__ __forceinline__ double NAME(double acc, double a, double b, int j) {          \
        switch (j) { MF_CASES(ASM) default: break; }                                          \
        return acc;                                                                           \
    }
#define MF_NN_NEGB(J) \
    case J: asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b)); break;
#define MF_NN_NEGBC(J) \
    case J: asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b)); break;
MF_DPP_NN(fmac_bcast_negb_nn, MF_NN_NEGB)
MF_DPP_NN(fmac_negbcast_nn, MF_NN_NEGBC)
#undef MF_NN_NEGB
#undef MF_NN_NEGBC
#undef MF_DPP_NN
// v_mov_b64_dpp without the s_nop (the caller spaces it from the source's write)
__device__ __forceinline__ double bcast64_nn(double v, int j) {
    double r = 0.0;
    switch (j) {
#define MF_B64NN(J) \
    case J: asm volatile("v_mov_b64_dpp %0, %1 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v)); break;
        MF_CASES(MF_B64NN)
#undef MF_B64NN
        default: break;
    }
    return r;
}
// two wait states after the VALU write of v, before the DPP reads of it that follow (in program order)
__device__ __forceinline__ void dpp_fence(double v) { asm volatile("s_nop 1" ::"v"(v)); }

// acc[c & 3] += w[c] * src(lane c of the 16-lane row), c = 0..15 in order: the 16 DPP FMAs in one block
// with a single s_nop for the broadcast source (written before the block; no instruction inside
// writes it), instead of one per FMA.  The accumulators' own dependencies are interlocked.
#define MF_FMAC(C, A, W) "v_fmac_f64_dpp %" #A ", %4, %" #W " row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void fmac16_bcast(double acc[4], double src, const double w[16]) {
    asm("s_nop 1\n\t" MF_FMAC(0, 0, 5) MF_FMAC(1, 1, 6) MF_FMAC(2, 2, 7) MF_FMAC(3, 3, 8) MF_FMAC(4, 0, 9)
        MF_FMAC(5, 1, 10) MF_FMAC(6, 2, 11) MF_FMAC(7, 3, 12) MF_FMAC(8, 0, 13) MF_FMAC(9, 1, 14) MF_FMAC(10, 2, 15)
        MF_FMAC(11, 3, 16) MF_FMAC(12, 0, 17) MF_FMAC(13, 1, 18) MF_FMAC(14, 2, 19) MF_FMAC(15, 3, 20)
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
        : "v"(src), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]),
          "v"(w[8]), "v"(w[9]), "v"(w[10]), "v"(w[11]), "v"(w[12]), "v"(w[13]), "v"(w[14]), "v"(w[15]));
}
#undef MF_FMAC

// The same sum four terms at a time (c = C0 .. C0 + 3 into acc[0..3]), for callers short of registers;
// kNop: the first block after src's write carries the two wait states.
#define MF_FMAC4(C, A, W) "v_fmac_f64_dpp %" #A ", %4, %" #W " row_newbcast:" #C " row_mask:0xf bank_mask:0xf\n\t"
template <int C0, bool kNop>
__device__ __forceinline__ void fmac4_bcast(double acc[4], double src, double w0, double w1, double w2, double w3);
#define MF_FMAC4_DEF(C0, C1, C2, C3)                                                                          \
    template <>                                                                                               \
    __device__ __forceinline__ void fmac4_bcast<C0, true>(double acc[4], double src, double w0, double w1,    \
                                                          double w2, double w3) {                             \
        asm volatile("s_nop 1\n\t" MF_FMAC4(C0, 0, 5) MF_FMAC4(C1, 1, 6) MF_FMAC4(C2, 2, 7) MF_FMAC4(C3, 3, 8)  \
                     : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])                                  \
                     : "v"(src), "v"(w0), "v"(w1), "v"(w2), "v"(w3));                                         \
    }                                                                                                         \
    template <>                                                                                               \
    __device__ __forceinline__ void fmac4_bcast<C0, false>(double acc[4], double src, double w0, double w1,   \
                                                           double w2, double w3) {                            \
        asm volatile(MF_FMAC4(C0, 0, 5) MF_FMAC4(C1, 1, 6) MF_FMAC4(C2, 2, 7) MF_FMAC4(C3, 3, 8)               \
                     : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])                                  \
                     : "v"(src), "v"(w0), "v"(w1), "v"(w2), "v"(w3));                                         \
    }
MF_FMAC4_DEF(0, 1, 2, 3)
MF_FMAC4_DEF(4, 5, 6, 7)
MF_FMAC4_DEF(8, 9, 10, 11)
MF_FMAC4_DEF(12, 13, 14, 15)
#undef MF_FMAC4_DEF
#undef MF_FMAC4

// the rest of pivot C's rank-1 update, j = J .. 15
template <int C, int J>
__device__ __forceinline__ void mf_update(double (&row)[16], double (&xc)[16], double lrc) {
    if constexpr (J < 16) {
        row[J] = fmac_bcast_negb_nn(row[J], lrc, lrc, J);
        xc[J] = fmac_negbcast_nn(xc[J], lrc, xc[C], J);
        mf_update<C, J + 1>(row, xc, lrc);
    }
}

// Pivot C of mf_diag (and, recursively, the ones after it).  row[j] = fma(-L[r][C], L[j][C], row[j]),
// xc[j] = fma(-L[j][C], xc[C], xc[j]) for j > C, in the order and rounding of the column loop.
template <int C>
__device__ __forceinline__ void mf_pivot(double (&row)[16], double (&xc)[16], double inv, bool& bad) {
    const double lrc = row[C] * inv;  // L[r][C] for r > C
    xc[C] *= inv;                     // x_C of column r of L^-1
    if constexpr (C + 1 < 16) {
        dpp_fence(lrc);
        row[C + 1] = fmac_bcast_negb_nn(row[C + 1], lrc, lrc, C + 1);
        xc[C + 1] = fmac_negbcast_nn(xc[C + 1], lrc, xc[C], C + 1);
        if constexpr (C + 2 < 16) row[C + 2] = fmac_bcast_negb_nn(row[C + 2], lrc, lrc, C + 2);
        else asm volatile("s_nop 0");
        const double pn = bcast64_nn(row[C + 1], C + 1);  // two VALU writes after row[C+1]'s
        bad |= !(pn > 0.0);
        const double inv_next = rsqrt_nr(pn);
        if constexpr (C + 2 < 16) xc[C + 2] = fmac_negbcast_nn(xc[C + 2], lrc, xc[C], C + 2);
        mf_update<C, C + 3>(row, xc, lrc);
        mf_pivot<C + 1 < 16 ? C + 1 : 15>(row, xc, inv_next, bad);
    }
}

// The column values L[j][c] reach the other rows by DPP row broadcasts (every 16-lane row holds the
// same block, so each row broadcasts within itself).
template <bool kColMajor = false>
__device__ __forceinline__ void mf_diag(double* __restrict__ dk, double* __restrict__ linv_k,
                                        double* __restrict__ yk, int lane, int* fail, int64_t* tr = nullptr) {
    if (tr && lane == 0) tr[0] = clock64();
    const int r = lane & 15;
    double row[16], xc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        row[c] = dk[r * 17 + c];
        xc[c] = c == r ? 1.0 : 0.0;
    }
    // Software-pipelined: column c first updates row c+1 and starts column c+1's pivot chain
    // (broadcast, rsqrt, Newton) before its other updates, which then fill that chain's latency.  The
    // same operations on the same values as the column-by-column order.
    const double piv0 = bcast64(row[0], 0);
    bool bad = !(piv0 > 0.0);
    double inv = rsqrt_nr(piv0);  // 1 / L[c][c]
    // One s_nop per pivot (round 5): every DPP FMA of a pivot reads the same source lrc, so only the
    // first needs the two wait states after lrc's write; the next pivot's broadcast of row[c+1] is
    // spaced from its write by the two FMAs issued between them.  FP64 VALU on gfx950 is issue-bound
    // (a dependent v_fma_f64 costs its 4-5 issue cycles, tools/probe/f64_lat_probe.hip), so the
    // pivot's cost is its instruction count; the per-FMA s_nop had nearly doubled it.  The pivots are
    // instantiated one by one (mf_pivot<C>): with volatile asm inside, `#pragma unroll` left the loop
    // rolled and indexed the registers at run time.
    mf_pivot<0>(row, xc, inv, bad);
    bad = __ballot(bad) != 0;
    if (lane == 0 && bad) *fail = 1;
    if (tr && lane == 0) tr[1] = clock64();
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i)  // L^-1[i][r]
            linv_k[kColMajor ? r * 17 + i : (r >> 2) * 64 + i + 16 * (r & 3)] = xc[i];
    }
    mf_wave_sync();
    if (tr && lane == 0) tr[2] = clock64();
    // y_k row r = sum_c L^-1[r][c] b_k[c] (four partial sums)
    double y4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int cc = 0; cc < 16; ++cc)
        y4[cc & 3] = __builtin_fma(linv_k[kColMajor ? cc * 17 + r : (cc >> 2) * 64 + r + 16 * (cc & 3)], yk[cc],
                                   y4[cc & 3]);
    const double y = (y4[0] + y4[1]) + (y4[2] + y4[3]);
    mf_wave_sync();
    if (lane < 16) yk[r] = y;
    if (tr && lane == 0) tr[3] = clock64();
}

// ---- v2: the diagonal wave carries the whole critical chain ----------------------------------------
// The sequential part of every step runs in one wave without workgroup barriers:
//   diagonal wave, step k: wait for the "pre" tiles A_{k+1,k}, P_{k+1,k+1} (updated through panel
//   k-1, published by their owners in LDS); L_{k+1,k} = A L_kk^-T (4 MFMAs), b_{k+1} -= L y_k,
//   P -= L L^T (4 MFMAs), factor P (mf_diag), publish L_{k+1,k+1}^-1 and y_{k+1} (flag lk).
//   tile waves, step k: wait for lk >= k; panel tiles (i > k, k) into the double-buffered panel;
//   b_i -= L_ik y_k for i > k + 1; tile-wave barrier (LDS counter); trailing update, the next
//   step's two pre tiles first.  The diagonal tile (k+1, k+1) is left to the diagonal wave.
// Backward: the diagonal wave keeps every L_{k+1,k} (sub-diagonal tile) in LDS, so the chain
// x_{k+1} -> x_k never leaves it; the tile waves add the other rows' L_kj^T x_k contributions into
// per-tile slots (the panel buffers, free by then), summed in a fixed order.
constexpr size_t kMf2Lds = sizeof(double) * (2 * (size_t)kMfMaxNT * 256 + (size_t)kMfMaxNT * 272 +
                                             (kMfMaxNT - 1) * 256 + 4 * 256 + 16 * 17 + 2 * 16 * kMfMaxNT);

__device__ __forceinline__ void lds_flag_wait(int* f, int target, int lane, int* fail, int code) {
    for (int spin = 0; __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target; ++spin) {
        if (spin > (1 << 22)) {  // bounded: a missing hand-off fails the solve instead of hanging
            if (lane == 0) *fail = code;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int W>
__global__ __launch_bounds__((W + 1) * 64) void k_ba_chol_mf2(int n, const double* __restrict__ S,
                                                              const double* __restrict__ b, double* __restrict__ x,
                                                              int32_t* __restrict__ status, int64_t* __restrict__ trace,
                                                              const LmState* __restrict__ lm_st, int lm_gk,
                                                              const double* __restrict__ hpp_add, const double* __restrict__ lam_add) {
    if (lm_skip(lm_st, lm_gk)) return;
    constexpr int SL = (kMfMaxNT * (kMfMaxNT + 1) / 2 + W - 1) / W;
    // hpp_add (the fast unit, k_u_schur2): S holds -sum Z Hpl^T only; element (row, col) of a diagonal 6x6
    // block gains Hpp + lambda I here, in the value k_ba_schur_block would have stored there (its mirror
    // store, lane (col % 6, row % 6), is the one that lands): (0 - sum) + (Hpp + lambda) = (Hpp + lambda) - sum
    const double lam_d = hpp_add ? *lam_add : 0.0;
    // Only tiles (i, j) with i - j <= 1 hold diagonal 6x6 blocks (6 < 16), so only they read Hpp (a
    // wave-uniform choice per tile): S streams into the one CU at ~64 B per clock, and an Hpp load beside
    // every S element had doubled the load instructions before the first step (+8k cycles).  Within such
    // a tile the Hpp load is unconditional (an in-range index) and the sum a select.
    auto s_at = [&](int row, int col, bool near) {
        const double v = S[(size_t)row * n + col];
        if (!hpp_add || !near) return v;
        const bool dg = row / 6 == col / 6;
        const double h = hpp_add[36 * (size_t)(row / 6) + (dg ? 6 * (col % 6) : 0) + row % 6];
        return dg ? v + (h + (row == col ? lam_d : 0.0)) : v;
    };
    static_assert(SL <= 32, "slot dispatch covers 32 slots");
    extern __shared__ double lds[];
    double* pan = lds;                        // [2][NT][256] panel tiles O(L_ik), by step parity
    double* contrib = lds;                    // backward: [k (k - 1) / 2 + j][16] (aliases pan)
    double* linv = pan + 2 * kMfMaxNT * 256;  // [NT][272] L_kk^-1 column-major, stride 17
    double* sub = linv + kMfMaxNT * 272;      // [NT - 1][256] O(L_{k+1,k})
    double* pre = sub + (kMfMaxNT - 1) * 256;  // [2][2][256] A_{k+1,k}, P_{k+1,k+1} by step parity
    double* dk = pre + 4 * 256;               // [16][17]
    double* yv = dk + 16 * 17;                // [16 NT]
    double* xv = yv + 16 * kMfMaxNT;          // [16 NT]
    __shared__ int fail, lk, tbar, xready, pre_ready[kMfMaxNT], cnt[kMfMaxNT], wrdy[kMfMaxNT];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int NT = (n + 15) >> 4, ntt = NT * (NT + 1) / 2;
    const int r16 = lane & 15, g4 = lane >> 4;
    if (threadIdx.x == 0) {
        fail = 0;
        lk = -1;
        tbar = 0;
        xready = 0;  // number of x blocks published (x_{NT-1} first)
    }
    if (threadIdx.x < kMfMaxNT) {
        pre_ready[threadIdx.x] = 0;
        cnt[threadIdx.x] = 0;
        wrdy[threadIdx.x] = 0;  // W1_j / W2_j made (0, 1 or 2 of them)
    }
    for (int i = threadIdx.x; i < 16 * NT; i += (W + 1) * 64) yv[i] = i < n ? b[i] : 0.0;
    __syncthreads();  // the only workgroup barrier before the end
    if (w == W) {
        // ---------------- diagonal wave ----------------
        // It carries the critical chain and is the youngest wave of the workgroup: VALU / MFMA issue
        // is arbitrated by priority, then age (MI355X_MICROARCH.md, two waves per SIMD), so without a
        // priority the two tile waves on its SIMD take the issue slots first.
        __builtin_amdgcn_s_setprio(3);
        for (int t = lane; t < 256; t += 64) {
            const int r = t >> 4, c = t & 15;
            dk[r * 17 + c] = (r < n && c < n) ? s_at(r, c, true) : (r == c ? 1.0 : 0.0);
        }
        mf_wave_sync();
        mf_diag<true>(dk, linv, yv, lane, &fail);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&lk, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (int k = 0; k + 1 < NT; ++k) {
            if (trace && lane == 0) trace[kTrStep + (k * 16 + W) * 4 + 1] = clock64();
            lds_flag_wait(&pre_ready[k], 2, lane, &fail, 2);
            if (trace && lane == 0) trace[kTrStep + (k * 16 + W) * 4 + 2] = clock64();
            const double* A = pre + (k & 1) * 512;
            const double* P = A + 256;
            const double* lkk = linv + k * 272;
            f64x4 L = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 4; ++q)  // A operand O(L^-1): L^-1[r16][g4 + 4q]
                L = __builtin_amdgcn_mfma_f64_16x16x4f64(lkk[(g4 + 4 * q) * 17 + r16], A[q * 64 + lane], L, 0, 0, 0);
            f64x4 Pm = {P[lane], P[64 + lane], P[128 + lane], P[192 + lane]};
#pragma unroll
            for (int q = 0; q < 4; ++q) Pm = __builtin_amdgcn_mfma_f64_16x16x4f64(L[q], L[q], Pm, 0, 0, 1);
            double part = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                part = __builtin_fma(L[q], yv[16 * k + g4 + 4 * q], part);
                dk[r16 * 17 + g4 + 4 * q] = Pm[q];
            }
            part += __shfl_xor(part, 16);
            part += __shfl_xor(part, 32);
            if (lane < 16) yv[16 * (k + 1) + lane] -= part;  // b_{k+1} -= L_{k+1,k} y_k
            mf_wave_sync();
            mf_diag<true>(dk, linv + (k + 1) * 272, yv + 16 * (k + 1), lane, &fail, trace ? trace + kTrDiag + 4 * k : nullptr);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&lk, k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (trace && lane == 0) trace[kTrStep + (k * 16 + W) * 4 + 3] = clock64();
        }
        // backward (round 5): x_j = e_j - W1_j x_{j+1}, with W1_j = L_jj^-T L_{j+1,j}^T (16x16, formed by
        // the owner of tile (j+1, j) at its panel step) and e_j = L_jj^-T (y_j - sum_{k >= j+2} L_kj^T x_k):
        // the tile waves subtract the rows k >= j+2 from y_j in place as the x_k are published (row
        // j+2 one block before x_j is due), so this wave runs e_j's 16-term product, W1_j x_{j+1} and
        // the publication per block.  Round 4 summed every contribution here and applied two operators:
        // ~2.6k cycles per block, 48k for the backward of n = 288.
        double x1 = 0.0;  // x_{j+1}[r16]
        for (int j = NT - 1; j >= 0; --j) {
            if (trace && lane == 0) trace[kTrBack + j] = clock64();
            const double* lj = linv + j * 272 + r16 * 17;  // L_jj^-1[c][r16], c = 0..15
            double a1[16];
            if (j + 1 < NT) {  // W1_j row r16 (operand layout O(W))
                lds_flag_wait(&wrdy[j], 1, lane, &fail, 8);
#pragma unroll
                for (int c = 0; c < 16; ++c) a1[c] = sub[j * 256 + (c >> 2) * 64 + r16 + 16 * (c & 3)];
            }
            if (j + 2 < NT) lds_flag_wait(&cnt[j + 2], j + 1, lane, &fail, 3);  // row j+2 (and above) applied
            if (trace && lane == 0) trace[kTrE + 2 * j] = clock64();
            const double v = yv[16 * j + r16];
            double d4[4] = {0.0, 0.0, 0.0, 0.0};  // e_j = sum_c L_jj^-1[c][r16] v_c, four terms at a time
            fmac4_bcast<0, true>(d4, v, lj[0], lj[1], lj[2], lj[3]);
            fmac4_bcast<4, false>(d4, v, lj[4], lj[5], lj[6], lj[7]);
            fmac4_bcast<8, false>(d4, v, lj[8], lj[9], lj[10], lj[11]);
            fmac4_bcast<12, false>(d4, v, lj[12], lj[13], lj[14], lj[15]);
            const double e = (d4[0] + d4[1]) + (d4[2] + d4[3]);
            if (trace && lane == 0) trace[kTrE + 2 * j + 1] = clock64();
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
            if (j + 1 < NT) fmac16_bcast(s4, x1, a1);
            if (trace && lane == 0) trace[kTrWaited + j] = clock64();
            const double xj = e - ((s4[0] + s4[1]) + (s4[2] + s4[3]));
            if (lane < 16) xv[16 * j + r16] = xj;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&xready, NT - j, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (trace && lane == 0) trace[kTrPub + j] = clock64();
            x1 = xj;
        }
    } else {
        // ---------------- tile waves: slot s holds tile t = s W + w (packed i | j << 8) ----------------
        int tij[SL];
        f64x4 T[SL];
#pragma unroll
        for (int s = 0; s < SL; ++s) {
            const int t = s * W + w;
            tij[s] = -1;
            T[s] = f64x4{0.0, 0.0, 0.0, 0.0};
            if (t < ntt) {
                int c = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
                while ((c + 1) * (c + 2) / 2 <= t) ++c;
                while (c * (c + 1) / 2 > t) --c;
                const int j = NT - 1 - c, i = j + (t - c * (c + 1) / 2);
                tij[s] = i | (j << 8);
                double e[4];
                const bool near = i - j <= 1;  // (wave-uniform: the slot's tile)
#pragma unroll
                for (int q = 0; q < 4; ++q) {  // S symmetric: read as S[col block][row block], coalesced
                    const int row = 16 * j + g4 + 4 * q, col = 16 * i + r16;
                    const double v = s_at(min(row, n - 1), min(col, n - 1), near);
                    e[q] = (row < n && col < n) ? v : (row == col ? 1.0 : 0.0);
                }
                T[s] = f64x4{e[0], e[1], e[2], e[3]};
                if (NT > 1 && (tij[s] == (1 | (0 << 8)) || tij[s] == (1 | (1 << 8)))) {  // pre tiles of step 0
                    double* dst = pre + (tij[s] == 1 ? 0 : 256);
#pragma unroll
                    for (int q = 0; q < 4; ++q) dst[q * 64 + lane] = e[q];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) __hip_atomic_fetch_add(&pre_ready[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        // (range checks use `continue`, not `break`: a runtime exit stops the full unrolling that keeps
        // T[] in registers)
        // tiles are numbered by decreasing column: tiles with j > k are t < Tc(k) = (NT-1-k)(NT-k)/2,
        // column k is t in [Tc(k), Tc(k) + NT - k) (its first tile is the diagonal one); this
        // wave's slot s holds t = s W + w, so every phase below is a contiguous slot range
        auto Tc = [&](int k) { return (NT - 1 - k) * (NT - k) / 2; };
        auto slot_lo = [&](int t) { return t <= w ? 0 : (t - w + W - 1) / W; };  // first s with s W + w >= t
        for (int k = 0; k + 1 < NT; ++k) {
            if (trace && lane == 0) trace[kTrStep + (k * 16 + w) * 4] = clock64();
            lds_flag_wait(&lk, k, lane, &fail, 4);
            double* pk = pan + (k & 1) * kMfMaxNT * 256;
            const double* lkk = linv + k * 272;
            const int t_upd = Tc(k), s_upd = slot_lo(t_upd);  // update: s < s_upd
            const int s_pan_end = slot_lo(t_upd + NT - k);     // panel: s_upd <= s < s_pan_end
            // ---- panel: L_ik = A_ik L_kk^-T, i > k; forward b_i -= L_ik y_k for i > k + 1
#pragma unroll
            for (int s = 0; s < SL; ++s) {
                if (s < s_upd) continue;
                if (s >= s_pan_end) continue;
                const int i = tij[s] & 255;
                if (i > k) {
                    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(lkk[(g4 + 4 * q) * 17 + r16], T[s][q], acc, 0, 0, 0);
                    double part = 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        pk[i * 256 + q * 64 + lane] = acc[q];
                        part = __builtin_fma(acc[q], yv[16 * k + g4 + 4 * q], part);
                    }
                    if (i > k + 1) {
                        part = group4_sum(part);
                        // (the lane index laundered per step: the compiler otherwise hoists one address
                        // register per slot out of the step loop, which the tile waves cannot afford)
                        int lo = lane;
                        asm volatile("" : "+v"(lo));
                        if (lane < 16) yv[16 * i + lo] -= part;
                    } else {  // i = k + 1: the backward operator W1_k = L_kk^-T L_{k+1,k}^T = O^-1 form
                              // O(M X^T), X = L_{k+1,k} (A operand = acc), M = L_kk^-T (B from L_kk^-1)
                        f64x4 wv = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            wv = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[q], lkk[r16 * 17 + g4 + 4 * q], wv, 0, 0, 0);
#pragma unroll
                        for (int q = 0; q < 4; ++q) sub[k * 256 + q * 64 + lane] = wv[q];
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (lane == 0) __hip_atomic_store(&wrdy[k], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    // The tile is final (L_ik); the forward does not touch it again.  Keep it transposed,
                    // O(L_ik^T) = the D layout of L_ik = A (O(L_ik)) times the identity, so that the
                    // backward's L_ik^T x_i is four FMAs and a four-row sum per lane instead of four
                    // 16-lane reductions.
                    f64x4 tr = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        tr = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[q], (4 * q + g4 == r16) ? 1.0 : 0.0, tr, 0, 0, 0);
                    T[s] = tr;
                }
            }
            // ---- tile-wave barrier (the diagonal wave does not take part)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_fetch_add(&tbar, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            lds_flag_wait(&tbar, W * (k + 1), lane, &fail, 5);
            if (trace && lane == 0) trace[kTrStep + (k * 16 + w) * 4 + 1] = clock64();
            // ---- trailing update with panel k.  The next step's pre tiles first: A = (k+2, k+1) is
            // t = Tc(k+1) + 1, P = (k+2, k+2) is t = Tc(k+2); the diagonal wave takes (k+1, k+1) = Tc(k+1).
            const int t_diag = Tc(k + 1);
            const int t_pa = k + 2 < NT ? Tc(k + 1) + 1 : -1, t_pp = k + 2 < NT ? Tc(k + 2) : -1;
            const int s_pre_end = k + 2 < NT ? slot_lo(t_pa + 1) : 0;
#pragma unroll
            for (int s = 0; s < SL; ++s) {
                if (s >= s_pre_end) continue;
                const int t = s * W + w;
                if (t == t_pa || t == t_pp) {
                    const int i = tij[s] & 255, j = tij[s] >> 8;
                    const double* pi = pk + i * 256;
                    const double* pj = pk + j * 256;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        T[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(pj[q * 64 + lane], pi[q * 64 + lane], T[s], 0, 0, 1);
                    double* dst = pre + ((k + 1) & 1) * 512 + (t == t_pp ? 256 : 0);
#pragma unroll
                    for (int q = 0; q < 4; ++q) dst[q * 64 + lane] = T[s][q];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) __hip_atomic_fetch_add(&pre_ready[k + 1], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
#pragma unroll
            for (int s = 0; s < SL; ++s) {
                if (s >= s_upd) continue;
                const int t = s * W + w;
                if (t != t_diag && t != t_pa && t != t_pp) {
                    const int i = tij[s] & 255, j = tij[s] >> 8;
                    const double* pi = pk + i * 256;
                    const double* pj = pk + j * 256;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        T[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(pj[q * 64 + lane], pi[q * 64 + lane], T[s], 0, 0, 1);
                }
            }
            if (trace && lane == 0) trace[kTrStep + (k * 16 + w) * 4 + 3] = clock64();
        }
        // ---- backward: row k's tiles (k, m <= k - 2), kept transposed since their panel step, subtract
        // L_km^T x_k from y_m in place (the diagonal wave applies (k, k - 1) itself, through W1).  A tile
        // gives y_m[c] -= sum_r L_km[r][c] x_k[r]: lane (c, g) holds L_km[g + 4q][c] in register q, so
        // four FMAs with x_k[g + 4q] and a four-row sum.  cnt[k] counts row k's applied tiles, and row
        // k starts once row k + 1 is complete, so every y_m loses its rows in the order k = NT - 1,
        // NT - 2, ... (one read-modify-write each).
        auto mine = [&](int sl, int k) {  // slot sl holds a tile (k, m <= k - 2)
            return tij[sl] >= 0 && (tij[sl] & 255) == k && (tij[sl] >> 8) <= k - 2;
        };
        for (int k = NT - 1; k >= 2; --k) {
            int nown = 0;
#pragma unroll
            for (int sl = 0; sl < SL; ++sl) nown += mine(sl, k);
            if (!nown) continue;
            lds_flag_wait(&xready, NT - k, lane, &fail, 7);  // x_k published
            if (k + 1 < NT) lds_flag_wait(&cnt[k + 1], k, lane, &fail, 3);  // row k + 1's k tiles applied
            if (trace && lane == 0) trace[kTrC + 32 * k + 2 * w] = clock64();
            double xq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) xq[q] = xv[16 * k + g4 + 4 * q];
            if (trace && lane == 0 && k >= NT - 2) trace[kTrD + 32 * (NT - 1 - k) + 2 * w] = clock64();
#pragma unroll
            for (int sl = 0; sl < SL; ++sl)
                if (mine(sl, k)) {
                    const int m = tij[sl] >> 8;
                    double p = 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) p = __builtin_fma(T[sl][q], xq[q], p);
                    p = group4_sum(p);
                    int lo = lane;  // (laundered, as in the panel)
                    asm volatile("" : "+v"(lo));
                    if (lane < 16) yv[16 * m + lo] -= p;
                }
            // one release for the row's tiles (a fence and an LDS atomic cost ~250 cycles)
            if (trace && lane == 0 && k >= NT - 2) trace[kTrD + 32 * (NT - 1 - k) + 2 * w + 1] = clock64();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_fetch_add(&cnt[k], nown, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (trace && lane == 0) trace[kTrC + 32 * k + 2 * w + 1] = clock64();
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += (W + 1) * 64) x[i] = xv[i];
    if (threadIdx.x == 0) *status = fail;
    if (trace && threadIdx.x == 0) trace[kTrEnd] = clock64();
}

// The pose update after the tile-row Cholesky (PoseTail): one workgroup, poses in strides
__global__ __launch_bounds__(256) void k_u_pose_update(PoseTail pt, const double* __restrict__ x,
                                                       const LmState* __restrict__ st) {
    if (lm_skip(st, kGateTrial)) return;
    __shared__ double cs[256];
    const bool rej = st && st->reject;
    double c = 0.0;  // thread t: poses t, t + 256, ... in order
    for (int t = threadIdx.x; t < pt.nf; t += 256) c += pose_tail_one(pt, t, pt.free_pose[t], x + 6 * (size_t)t, rej);
    cs[threadIdx.x] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < 256; ++i) s += cs[i];
        *pt.pscale = s;
    }
}

// ---- tile-row Cholesky + solve over many workgroups (any n up to 16 x 256) ----------------------
// Workgroup i owns tile row i of S (tiles (i, j), j <= i, in the operand layout O of the kernels
// above) and runs the whole row left to right, eagerly:
//   step m < i: once row m has published L_mm^-1 and y_m, wave 0 turns its tile (i, m) into
//     L_im = A_im L_mm^-T (4 MFMAs), publishes it and folds the forward solve in (b_i -= L_im y_m);
//     then the four waves apply column m to the rest of the row, T_ij -= L_im L_jm^T for
//     m < j <= i, taking L_jm from row j as soon as row j has published it (tile (i, m+1), the
//     next step's panel tile, goes first).
//   diagonal: wave 0 factors T_ii (mf_diag), publishes L_ii^-1 and y_i = L_ii^-1 b_i.
// The critical chain per step is one hand-off (row m -> row m+1), one panel product, one update
// and one 16x16 factorisation.  The last row's workgroup, which has by then consumed every
// published tile, finishes with the backward solve L^T x = y.
// Hand-offs between workgroups (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the
// sc1 table): the payload (tiles, y) is stored with agent-scope relaxed 8-byte atomics (sc1
// write-through stores), each storing wave drains its stores (s_waitcnt vmcnt(0)) before one lane
// stores the flag (agent scope); the consumer wave polls the flag with agent-scope loads and reads
// every byte of the payload with agent-scope (sc1) loads; other waves of the consumer read only
// after a workgroup barrier the polling wave has joined.  Flags hold the launch's epoch (one more
// than the counter in cflag[0], which the last row advances when it finishes), so they never need
// clearing between launches; every spin is bounded and a timeout is reported as a failed solve.
// Rows are kept in LDS up to kRowLdsMaxNT tiles, in a private global scratch beyond.
constexpr int kRowThreads = 256, kRowLdsMaxNT = 72, kRowMaxNT = 256;
typedef __attribute__((address_space(1))) unsigned long long ba_gu64;
typedef __attribute__((address_space(1))) unsigned ba_gu32;

__device__ __forceinline__ double ld_agent(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((ba_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store((ba_gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// one wave polls one flag word until it holds `epoch` (or later); false after ~4 s
__device__ __forceinline__ bool flag_wait_agent(const unsigned* f, unsigned epoch, int limit = 1 << 22) {
    for (int spin = 0; spin < limit; ++spin) {
        if (__hip_atomic_load((ba_gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the payload loads below the poll
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}
__device__ __forceinline__ void flag_publish_agent(unsigned* f, unsigned epoch, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 payload stores have landed
    if (lane == 0) __hip_atomic_store((ba_gu32*)f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Forced-timeout hook (orb_debug_ba_chol_timeout, tests/test_ba_gpu.py): one row's first flag wait
// asks for a later epoch, so it times out and the launch must fail with status 6 (another row's
// timeout) while the next launch, at its own epoch, is clean.  One-shot: the armed row clears it.
__device__ int g_dbg_chol_row = -1;
__device__ unsigned g_dbg_chol_epoch = 0;
__device__ int g_dbg_chol_status = -1;

template <bool kLdsRow>
__global__ __launch_bounds__(kRowThreads) void k_ba_chol_rows(int n, const double* __restrict__ S,
                                                              const double* __restrict__ b, double* __restrict__ x,
                                                              int32_t* __restrict__ status, double* __restrict__ lpub,
                                                              double* __restrict__ ypub, unsigned* __restrict__ cflag,
                                                              double* __restrict__ racc,
                                                              const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int NT = (n + 15) >> 4;
    const int i = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, g4 = lane >> 4;
    double* R = kLdsRow ? lds : racc + (size_t)i * NT * 256;  // own row: tile j at R + 256 j
    double* dk = kLdsRow ? lds + (size_t)NT * 256 : lds;      // [16][17] diagonal block
    double* linv = dk + 272;                                   // [256] O(L_ii^-1)
    double* rv = linv + 256;                                   // [16] b_i -> y_i
    double* z = rv + 16;                                       // [16 NT] backward solve (last row)
    __shared__ int fail;
    unsigned* flags = cflag + 4;  // [row][col]: tile (row, col) published at this epoch
    const unsigned E = cflag[0] + 1;
    __shared__ unsigned dbg_bump;
    if (tid == 0) {
        fail = 0;
        dbg_bump = 0;
        if (__hip_atomic_load((ba_gu32*)&g_dbg_chol_row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i &&
            atomicCAS(&g_dbg_chol_row, i, -1) == i) {
            dbg_bump = 1000;
            __hip_atomic_store((ba_gu32*)&g_dbg_chol_epoch, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    for (int t = tid; t < (i + 1) * 256; t += kRowThreads) {  // S upper triangle read as S[col blk][row blk]
        const int j = t >> 8, e = t & 255, q = e >> 6, l = e & 63;
        const int row = 16 * j + (l >> 4) + 4 * q, col = 16 * i + (l & 15);
        const double v = S[(size_t)min(row, n - 1) * n + min(col, n - 1)];
        R[t] = (row < n && col < n) ? v : (row == col ? 1.0 : 0.0);
    }
    if (tid < 16) rv[tid] = 16 * i + tid < n ? b[16 * i + tid] : 0.0;
    __syncthreads();
    for (int m = 0; m < i; ++m) {
        if (w == 0) {  // panel tile (i, m) and the forward step
            // (the armed debug wait gives up after ~4k polls, long before any other row's bound)
            if (!flag_wait_agent(flags + m * NT + m, E + (m == 0 ? dbg_bump : 0u),
                                 m == 0 && dbg_bump ? 1 << 12 : 1 << 22) && lane == 0)
                fail = 4;
            const double* lp = lpub + ((size_t)m * NT + m) * 256;
            double lq[4], yq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                lq[q] = ld_agent(lp + q * 64 + lane);
                yq[q] = ld_agent(ypub + 16 * m + g4 + 4 * q);
            }
            double* Tm = R + m * 256;
            f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(lq[q], Tm[q * 64 + lane], acc, 0, 0, 0);
            double* dst = lpub + ((size_t)i * NT + m) * 256;
            double part = 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                Tm[q * 64 + lane] = acc[q];
                st_agent(dst + q * 64 + lane, acc[q]);
                part = __builtin_fma(acc[q], yq[q], part);
            }
            part += __shfl_xor(part, 16);
            part += __shfl_xor(part, 32);
            if (lane < 16) rv[lane] -= part;
            flag_publish_agent(flags + i * NT + m, E, lane);
        }
        __syncthreads();
        const double* Lim = R + m * 256;
        for (int j = m + 1 + w; j <= i; j += 4) {  // T_ij -= L_im L_jm^T
            double a[4];
            if (j < i) {
                if (!flag_wait_agent(flags + j * NT + m, E) && lane == 0) fail = 5;
                const double* lp = lpub + ((size_t)j * NT + m) * 256;
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = ld_agent(lp + q * 64 + lane);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) a[q] = Lim[q * 64 + lane];
            }
            double* T = R + j * 256;
            f64x4 t = {T[lane], T[64 + lane], T[128 + lane], T[192 + lane]};
#pragma unroll
            for (int q = 0; q < 4; ++q) t = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], Lim[q * 64 + lane], t, 0, 0, 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) T[q * 64 + lane] = t[q];
        }
        __syncthreads();
    }
    if (w == 0) {  // diagonal tile: L_ii^-1 and y_i
        const double* Ti = R + i * 256;
#pragma unroll
        for (int q = 0; q < 4; ++q) dk[r16 * 17 + g4 + 4 * q] = Ti[q * 64 + lane];
        mf_wave_sync();
        mf_diag<false>(dk, linv, rv, lane, &fail);
        mf_wave_sync();
        double* dst = lpub + ((size_t)i * NT + i) * 256;
#pragma unroll
        for (int q = 0; q < 4; ++q) st_agent(dst + q * 64 + lane, linv[q * 64 + lane]);
        if (lane < 16) st_agent(ypub + 16 * i + lane, rv[lane]);
        flag_publish_agent(flags + i * NT + i, E, lane);
    }
    __syncthreads();
    // a timed-out wait is reported to the last row tagged with this launch's epoch, so that it fails
    // this solve only (a later launch compares against its own epoch: no clearing needed)
    if (fail > 3 && tid == 0) __hip_atomic_store((ba_gu32*)(cflag + 1), E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (i != NT - 1) return;
    // ---- backward solve L^T x = y in the last row's workgroup: x_j = L_jj^-T (y_j - sum_{k>j} L_kj^T x_k),
    // right-looking: after x_j, every z_p (p < j) loses L_jp^T x_j
    __syncthreads();
    for (int t = tid; t < 16 * NT; t += kRowThreads) z[t] = t < 16 * (NT - 1) ? ld_agent(ypub + t) : rv[t - 16 * (NT - 1)];
    __syncthreads();
    for (int j = NT - 1; j >= 0; --j) {
        if (w == 0) {  // x_j[c] = sum_r L^-1[r][c] z_j[r]; L^-1[r][c] at (c >> 2) 64 + r + 16 (c & 3)
            const double* lj = lpub + ((size_t)j * NT + j) * 256;
            double v4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                const int o = (r16 >> 2) * 64 + rr + 16 * (r16 & 3);
                const double l = j == NT - 1 ? linv[o] : ld_agent(lj + o);
                v4[rr & 3] = __builtin_fma(l, z[16 * j + rr], v4[rr & 3]);
            }
            const double xj = (v4[0] + v4[1]) + (v4[2] + v4[3]);
            mf_wave_sync();
            if (lane < 16) z[16 * j + r16] = xj;
        }
        __syncthreads();
        for (int t = tid; t < 16 * j; t += kRowThreads) {  // z_p[c] -= sum_r L_jp[r][c] x_j[r]
            const int p = t >> 4, c = t & 15;
            const double* L = (j == NT - 1 ? R : lpub + (size_t)j * NT * 256) + p * 256 + (c >> 2) * 64 + 16 * (c & 3);
            double v4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int rr = 0; rr < 16; ++rr) {
                const double l = j == NT - 1 ? L[rr] : ld_agent(L + rr);
                v4[rr & 3] = __builtin_fma(l, z[16 * j + rr], v4[rr & 3]);
            }
            z[t] -= (v4[0] + v4[1]) + (v4[2] + v4[3]);
        }
        __syncthreads();
    }
    for (int t = tid; t < n; t += kRowThreads) x[t] = z[t];
    if (tid == 0) {
        const unsigned timeouts = __hip_atomic_load((ba_gu32*)(cflag + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *status = fail ? fail : (timeouts == E ? 6 : 0);
        if (__hip_atomic_load((ba_gu32*)&g_dbg_chol_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == E)
            __hip_atomic_store(&g_dbg_chol_status, *status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cflag[0] = E;  // every row read the epoch before publishing, and this row consumed all of them
    }
}

// x_l = Dinv (b_l - sum_e Hpl_e^T x_pose(e)).  The free edges' indices and pose rows (host-built
// erow) of up to 8 edges are loaded first, then the operands 4 edges at a time: two rounds of
// dependent loads for the usual landmark, not four per edge.  xl: x_l (also stored to x).
__device__ __forceinline__ void ba_backsub(int l, int n, double lambda, const int32_t* __restrict__ off,
                                           const int32_t* __restrict__ eidx, const int32_t* __restrict__ erow,
                                           const double* __restrict__ hpl, const double* __restrict__ bl,
                                           const double* __restrict__ hll, double* __restrict__ x, double xl[3]) {
    double cl[3] = {bl[3 * (size_t)l], bl[3 * (size_t)l + 1], bl[3 * (size_t)l + 2]};
    const int k0 = off[l], k1 = off[l + 1];
    // Dinv first: its loads and the 3x3 inverse overlap the rounds of the loop below
    double Di[9];
    land_dinv(hll, l, lambda, Di);
    for (int kb = k0; kb < k1; kb += 8) {
        int e[8], ph[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = min(kb + u, k1 - 1);
            e[u] = eidx[k];
            ph[u] = erow[k];
        }
#pragma unroll
        for (int h = 0; h < 8; h += 4) {
            if (kb + h >= k1) break;
            double H[4][18], xp[4][6];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int q = 0; q < 18; ++q) H[u][q] = hpl[18 * (size_t)e[h + u] + q];
#pragma unroll
                for (int q = 0; q < 6; ++q) xp[u][q] = x[6 * (size_t)ph[h + u] + q];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (kb + h + u < k1)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
#pragma unroll
                        for (int r = 0; r < 6; ++r) cl[c] += H[u][3 * r + c] * -xp[u][r];
        }
    }
    for (int r = 0; r < 3; ++r) {
        xl[r] = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
        x[n + 3 * (size_t)l + r] = xl[r];
    }
}

__global__ __launch_bounds__(kT) void k_ba_backsub(int nl, int n, const double* __restrict__ lam,
                                                   const int32_t* __restrict__ off, const int32_t* __restrict__ eidx,
                                                   const int32_t* __restrict__ erow, const double* __restrict__ hpl,
                                                   const double* __restrict__ bl, const double* __restrict__ hll,
                                                   double* __restrict__ x, const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    const int l = blockIdx.x * kT + threadIdx.x;
    double xl[3];
    if (l < nl) ba_backsub(l, n, *lam, off, eidx, erow, hpl, bl, hll, x, xl);
}

// push + oplus for every free vertex: threads [0, nf) poses, [nf, nf + nl) landmarks
// push + oplus for vertex t (poses first, then landmarks).  from_bak: the previous trial was
// rejected and not restored yet (device-driven loop): start from the backup and keep it.
__device__ __forceinline__ void ba_update(int t, int nf, int nl, int n, bool from_bak,
                                          const int32_t* __restrict__ free_pose, const int32_t* __restrict__ land_point,
                                          const double* __restrict__ x, double* __restrict__ pose,
                                          double* __restrict__ pose_bak, double* __restrict__ point,
                                          double* __restrict__ point_bak) {
    if (t < nf) {
        double* T = pose + 7 * (size_t)free_pose[t];
        double* Tb = pose_bak + 7 * (size_t)free_pose[t];
        double v[7], u[6];
        for (int i = 0; i < 7; ++i) {
            v[i] = from_bak ? Tb[i] : T[i];
            Tb[i] = v[i];
        }
        for (int i = 0; i < 6; ++i) u[i] = x[6 * (size_t)t + i];
        se3_oplus(v, u);
        for (int i = 0; i < 7; ++i) T[i] = v[i];
    } else if (t < nf + nl) {
        const int l = t - nf;
        double* X = point + 3 * (size_t)land_point[l];
        double* Xb = point_bak + 3 * (size_t)land_point[l];
        for (int i = 0; i < 3; ++i) {
            const double v = from_bak ? Xb[i] : X[i];
            Xb[i] = v;
            X[i] = v + x[n + 3 * (size_t)l + i];
        }
    }
}

__global__ __launch_bounds__(kT) void k_ba_update(int nf, int nl, int n, const int32_t* __restrict__ free_pose,
                                                  const int32_t* __restrict__ land_point, const double* __restrict__ x,
                                                  double* __restrict__ pose, double* __restrict__ pose_bak,
                                                  double* __restrict__ point, double* __restrict__ point_bak,
                                                  const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    ba_update(blockIdx.x * kT + threadIdx.x, nf, nl, n, false, free_pose, land_point, x, pose, pose_bak, point,
              point_bak);
}

__global__ __launch_bounds__(kT) void k_ba_restore(int nf, int nl, const int32_t* __restrict__ free_pose,
                                                   const int32_t* __restrict__ land_point, double* __restrict__ pose,
                                                   const double* __restrict__ pose_bak, double* __restrict__ point,
                                                   const double* __restrict__ point_bak,
        const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < nf) {
        for (int i = 0; i < 7; ++i) pose[7 * (size_t)free_pose[t] + i] = pose_bak[7 * (size_t)free_pose[t] + i];
    } else if (t < nf + nl) {
        const int l = t - nf;
        for (int i = 0; i < 3; ++i) point[3 * (size_t)land_point[l] + i] = point_bak[3 * (size_t)land_point[l] + i];
    }
}

// out[0] = sum rho0 (activeRobustChi2), out[1] = sum x (lambda x + b) (computeScale, before +1e-3)
// out: [0] robust chi2, [1] computeScale part, [2] factorisation status (as a double), [3] max diag
// (written earlier by k_ba_maxdiag).  host: optional pinned copy of out[0..3] (one process: the
// host reads it after the stream sync, no copy launches).
__global__ __launch_bounds__(1024) void k_ba_sums(int ne, const double* __restrict__ rho0, int x0, int nx, const double* __restrict__ lam,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  const int32_t* __restrict__ status, double* __restrict__ out,
                                                  double* __restrict__ host,
        const LmState* __restrict__ lm_st, int lm_gk) {
    if (lm_skip(lm_st, lm_gk)) return;
    const double lambda = *lam;
    __shared__ double r0[1024], r1[1024];
    double a = 0, c = 0;
    for (int i = threadIdx.x; i < ne; i += 1024) a += rho0[i];
    if (x)
        for (int i = x0 + threadIdx.x; i < nx; i += 1024) c += x[i] * (lambda * x[i] + b[i]);
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
        out[2] = (x && *status) ? 1.0 : 0.0;
        if (host) {
            host[0] = r0[0];
            host[1] = r1[0];
            host[2] = out[2];
            host[3] = out[3];
            __threadfence_system();
        }
    }
}

// The solve's results straight into the pinned host buffer (no device copies, one launch): poses
// [np][7], points [nq][3], then per edge chi2 (e^T Omega e) and the depth flag of src/Optimizer.cc:2115-2150.
__global__ __launch_bounds__(kT) void k_ba_results(int np, int nq, int ne, const EdgeDev* __restrict__ edges,
                                                   const double* __restrict__ pose, const double* __restrict__ point,
                                                   const double* __restrict__ err, double* __restrict__ h_pose,
                                                   double* __restrict__ h_point, double* __restrict__ h_chi2,
                                                   uint8_t* __restrict__ h_depth) {
    const int t = blockIdx.x * kT + threadIdx.x;
    if (t < 7 * np) h_pose[t] = pose[t];
    if (t < 3 * nq) h_point[t] = point[t];
    if (t >= ne) return;
    const EdgeDev E = edges[t];
    const double info = (double)E.inv_sigma2;
    const double* er = err + 3 * (size_t)t;
    double c = er[0] * info * er[0] + er[1] * info * er[1];
    if (E.stereo) c += er[2] * info * er[2];
    h_chi2[t] = c;
    const double* T = pose + 7 * (size_t)E.pose;
    const double q[4] = {T[3], T[4], T[5], T[6]};
    double Xc[3];
    qrotate(q, point + 3 * (size_t)E.point, Xc);
    h_depth[t] = (Xc[2] + T[2]) > 0.0;
}

// ---- LM controllers (one thread), g2o OptimizationAlgorithmLevenberg::solve ---------------------
// after the build: currentChi, iniChi; at iteration 0 the initial lambda (tau * max diag, or the
// user's)
__device__ void lm_build_done(LmState* st, double chi, double maxdiag) {
    st->current_chi = chi;
    st->ini_chi = chi;
    if (st->it == 0) {
        st->initial_chi = chi;
        st->lambda = st->user_lambda > 0 ? st->user_lambda : st->tau * maxdiag;
        st->ni = 2;
        st->nbad = 0;
    }
    st->qmax = 0;
    st->phase = 1;
}

// after a trial: accept (lambda shrinks) or reject (lambda grows; the next update starts from the
// backup, and a final restore launch undoes a rejected last trial); at the end of the trial loop
// the termination tests
// fast (the fast unit, no build controller): the trial loop's next unit skips the build (phase 1); at
// an iteration's end the next iteration's start is recorded here (ini_chi = the accepted chi2, qmax 0)
// and its unit builds (phase 0)
__device__ void lm_trial_done(LmState* st, double chi, double scale_part, bool failed, LmProgress* prog,
                              bool flip_lin = false, bool fast = false) {
    double tempChi = chi;
    if (failed) tempChi = DBL_MAX;
    double rho = st->current_chi - tempChi;
    const double scale = scale_part + 1e-3;
    rho /= scale;
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow(2 * rho - 1, 3.0);
        alpha = fmin(alpha, 2. / 3.);
        st->lambda *= fmax(1. / 3., alpha);
        st->ni = 2;
        st->current_chi = tempChi;
        st->reject = 0;
        if (flip_lin) st->lin ^= 1;  // the trial's linearisation (k_u_edges_trial<true>) is the next build's
    } else {
        st->lambda *= st->ni;
        st->ni *= 2;
        st->reject = 1;
    }
    st->qmax++;
    st->trials++;
    if (fast) st->phase = 1;
    if (!(rho < 0 && st->qmax < 10)) {  // the trial loop is over
        st->final_chi = st->current_chi;
        if (st->qmax == 10 || rho == 0) {
            st->terminated = 1;
            st->it++;
            st->done = 1;
        } else {
            if ((st->ini_chi - st->current_chi) * 1e3 < st->ini_chi) st->nbad++;
            else st->nbad = 0;
            st->it++;
            if (st->nbad >= 3) {
                st->terminated = 1;
                st->done = 1;
            } else {
                st->phase = 0;
                if (fast) {
                    st->ini_chi = st->current_chi;
                    st->qmax = 0;
                }
                if (st->it >= st->iterations) st->done = 1;
            }
        }
    }
    prog->final_chi = st->final_chi;
    prog->initial_chi = st->initial_chi;
    prog->lambda = st->lambda;
    prog->it = st->it;
    prog->trials = st->trials;
    prog->terminated = st->terminated;
    prog->done = st->done;
    __threadfence_system();
}

// ---- fused kernels of the device-driven unit ------------------------------------------------------
// fixed-order block sum of one value per thread (blockDim = NT); the result is valid in every thread
// (DPP row sums, the four row totals by v_readlane, then the wave totals through LDS: two barriers
// instead of a log2(NT)-level tree)
template <int NT>
__device__ __forceinline__ double block_sum(double v) {
    static_assert(NT % 64 == 0, "whole waves");
    __shared__ double red[NT / 64];
    v = row16_sum(v);  // row sums in lanes 15, 31, 47, 63
    const double w = (readlane_d(v, 15) + readlane_d(v, 31)) + (readlane_d(v, 47) + readlane_d(v, 63));
    __syncthreads();  // red may still be read by the previous call
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
    __syncthreads();
    double t = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    return t;
}

// true in the last block to finish (its predecessors' global writes are visible to it)
__device__ __forceinline__ bool last_block(unsigned* counter) {
    __shared__ bool last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(counter, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last) __threadfence();
    return last;
}

// unit step 1 (build): linearise every edge; per-block robust chi2 partials
__global__ __launch_bounds__(kT) void k_u_edges_build(int ne, const EdgeDev* __restrict__ edges,
                                                      const orb_ba_camera_t* __restrict__ cams,
                                                      const double* __restrict__ pose, const double* __restrict__ point,
                                                      const int32_t* __restrict__ pose_h, Huber2 hub,
                                                      double* __restrict__ err, double* __restrict__ rho0_out,
                                                      double* __restrict__ ecl, double* __restrict__ hpl,
                                                      double* __restrict__ ecp, double* __restrict__ part,
                                                      const LmState* __restrict__ st) {
    if (lm_skip(st, kGateBuild)) return;
    const int e = blockIdx.x * kT + threadIdx.x;
    double r = 0.0;
    if (e < ne) r = ba_edge<true>(e, edges, cams, pose, point, pose_h, hub, err, rho0_out, ecl, hpl, ecp, 0);
    const double bsum = block_sum<kT>(r);
    if (threadIdx.x == 0) part[blockIdx.x] = bsum;
}

// unit step 2 (build): Hpp/b_p (blocks [0, nf)), Hll/b_l (64 landmarks per block); the last block
// sums chi2, takes max diag at iteration 0 and runs the build controller.  Sharded (dist): hpp / bp are
// this rank's partial buffers, and the last block leaves its chi2 in sc_part[0] and its landmarks' max
// diag in the rank's slot sc_part[4 + rank] (zero elsewhere: the SUM all-reduce gathers the slots) for
// k_lm_build_ctl after the all-reduce
__global__ __launch_bounds__(64) void k_u_reduce_build(int nf, int nl, const int32_t* __restrict__ pose_off,
                                                       const LandEdge* __restrict__ pose_edge, const double* __restrict__ ecp,
                                                       double* __restrict__ hpp, double* __restrict__ bp,
                                                       const int32_t* __restrict__ land_off,
                                                       const int32_t* __restrict__ land_edge,
                                                       const double* __restrict__ ecl, double* __restrict__ hll,
                                                       double* __restrict__ bl, const double* __restrict__ part,
                                                       int nparts, unsigned* counter, double* __restrict__ scal,
                                                       LmState* st, int dist, double* __restrict__ sc_part, int rank,
                                                       double* __restrict__ pmax) {
    if (lm_skip(st, kGateBuild)) return;
    const int b = blockIdx.x, lane = threadIdx.x;
    // computeLambdaInit (iteration 0): each block's max |diag| of what it reduced, to pmax[block], so
    // the last block takes one max over the blocks instead of a pass over every Hpp / Hll (sharded:
    // the poses' part comes from the reduced Hpp, k_lm_build_ctl)
    double m = 0.0;
    if (b < nf) {
        const double t = ba_reduce_pose(b, lane, pose_off, pose_edge, ecp, hpp, bp);
        if (!dist && lane < 36 && lane % 7 == 0) m = fabs(t);
    } else {
        const int l = (b - nf) * 64 + lane;
        if (l < nl) m = ba_reduce_land(l, land_off, land_edge, ecl, hll, bl);
    }
    const bool first = st->it == 0;
    if (first) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o));
        if (lane == 0) pmax[b] = m;
    }
    if (!last_block(counter)) return;
    double c = 0.0;
    for (int i = lane; i < nparts; i += 64) c += part[i];
    const double chi = block_sum<64>(c);
    double md = 0.0;
    if (first) {  // (max is order-independent)
        double mm = 0.0;
        for (int i = lane; i < (int)gridDim.x; i += 64) mm = fmax(mm, pmax[i]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) mm = fmax(mm, __shfl_xor(mm, o));
        md = mm;
    }
    if (lane == 0) {
        if (dist) {
            sc_part[0] = chi;
            sc_part[4 + rank] = md;
        } else {
            scal[0] = chi;
            scal[3] = md;
            lm_build_done(st, chi, md);
        }
        *counter = 0;
    }
}

// sharded build controller, after the all-reduce of the build partials: chi2 = sc_red[0]; at iteration
// 0 max diag over the reduced Hpp and the ranks' landmark slots sc_red[4 .. 4 + world)
__global__ __launch_bounds__(64) void k_lm_build_ctl(int nf, const double* __restrict__ hpp,
                                                     const double* __restrict__ sc_red, int world,
                                                     double* __restrict__ scal, LmState* st) {
    if (lm_skip(st, kGateBuild)) return;
    const int lane = threadIdx.x;
    double md = 0.0;
    if (st->it == 0) {
        double m = 0;
        for (int i = lane; i < 6 * nf; i += 64) m = fmax(m, fabs(hpp[36 * (size_t)(i / 6) + 7 * (i % 6)]));
        for (int r = lane; r < world; r += 64) m = fmax(m, sc_red[4 + r]);
        __shared__ double mx[64];
        mx[lane] = m;
        __syncthreads();
        for (int w = 32; w >= 1; w >>= 1) {
            if (lane < w) mx[lane] = fmax(mx[lane], mx[lane + w]);
            __syncthreads();
        }
        md = mx[0];
    }
    if (lane == 0) {
        scal[0] = sc_red[0];
        scal[3] = md;
        lm_build_done(st, sc_red[0], md);
    }
}

// unit step 4 (trial): S blocks (blocks [0, nblk), the upper triangle) and b_S (one block per free pose).
// Sharded: S / bs are this rank's partials and only rank 0 (primary) adds Hpp + lambda I and b_p.
__global__ __launch_bounds__(64) void k_u_schur(int n, int nf, int nblk, const double* __restrict__ lam,
                                                const int32_t* __restrict__ blk_off, const EdgePair* __restrict__ pairs,
                                                const int32_t* __restrict__ cnt, const int32_t* __restrict__ pose_off,
                                                const LandEdge* __restrict__ pose_fl, const double* __restrict__ z,
                                                const double* __restrict__ hpl, size_t hpl_alt,
                                                const double* __restrict__ hpp, double* __restrict__ S,
                                                const double* __restrict__ cb, const double* __restrict__ bp,
                                                double* __restrict__ bs, const LmState* __restrict__ st, int primary) {
    if (lm_skip(st, kGateTrial)) return;
    hpl += hpl_cur(st, hpl_alt);
    if ((int)blockIdx.x < nblk)
        ba_schur_block(blockIdx.x, threadIdx.x, n, nf, *lam, primary, blk_off, pairs, cnt, z, hpl, hpp, S);
    else
        ba_schur_rhs(blockIdx.x - nblk, threadIdx.x, pose_off, pose_fl, cb, bp, primary, bs);
}

// unit step 6 (trial): x_l per landmark and its update, then the pose updates; a rejected previous
// trial is undone here (from the backup) instead of by a restore launch.  Each block also leaves its
// part of computeScale, sum x (lambda x + b) over its vertices' rows, in part2[block] (summed in
// block order by k_u_edges_trial: one load round there instead of a pass over x and b).
__global__ __launch_bounds__(kT) void k_u_backsub_update(int nl, int nf, int n, const double* __restrict__ lam,
                                                         const int32_t* __restrict__ off, const int32_t* __restrict__ eidx,
                                                         const int32_t* __restrict__ erow, const double* __restrict__ hpl,
                                                         size_t hpl_alt, const double* __restrict__ bl,
                                                         const double* __restrict__ hll, double* __restrict__ x,
                                                         const double* __restrict__ bp, const int32_t* __restrict__ free_pose,
                                                         const int32_t* __restrict__ land_point, double* __restrict__ pose,
                                                         double* __restrict__ pose_bak, double* __restrict__ point,
                                                         double* __restrict__ point_bak, double* __restrict__ part2,
                                                         const LmState* __restrict__ st, int pose_scale) {
    if (lm_skip(st, kGateTrial)) return;
    hpl += hpl_cur(st, hpl_alt);
    const bool rej = st->reject != 0;
    const double lambda = *lam;
    const int t = blockIdx.x * kT + threadIdx.x;
    double c = 0.0;
    if (t < nl) {
        double xl[3];
        ba_backsub(t, n, lambda, off, eidx, erow, hpl, bl, hll, x, xl);
        for (int r = 0; r < 3; ++r) c += xl[r] * (lambda * xl[r] + bl[3 * (size_t)t + r]);
        double* X = point + 3 * (size_t)land_point[t];
        double* Xb = point_bak + 3 * (size_t)land_point[t];
        for (int i = 0; i < 3; ++i) {
            const double v = rej ? Xb[i] : X[i];
            Xb[i] = v;
            X[i] = v + xl[i];
        }
    } else if (t < nl + nf) {
        const int p = t - nl;
        double* T = pose + 7 * (size_t)free_pose[p];
        double* Tb = pose_bak + 7 * (size_t)free_pose[p];
        double v[7], u[6];
        for (int i = 0; i < 6; ++i) u[i] = x[6 * (size_t)p + i];
        if (pose_scale)  // (sharded: the pose rows' computeScale part on rank 0 only)
            for (int i = 0; i < 6; ++i) c += u[i] * (lambda * u[i] + bp[6 * (size_t)p + i]);
        for (int i = 0; i < 7; ++i) {
            v[i] = rej ? Tb[i] : T[i];
            Tb[i] = v[i];
        }
        se3_oplus(v, u);
        for (int i = 0; i < 7; ++i) T[i] = v[i];
    }
    const double bsum = block_sum<kT>(c);
    if (threadIdx.x == 0) part2[blockIdx.x] = bsum;
}

// unit step 7 (trial): errors at the new estimate (with kLin also its linearisation: Hll/b_l and
// Hpp/b_p parts in place -- nothing reads them before the next build -- and Hpl into the other half);
// the last block sums chi2 and computeScale (part2, from k_u_backsub_update) and runs the trial
// controller, which on accept makes the kLin linearisation current: the next iteration's build at
// the same estimate would compute exactly these values
template <bool kLin>
__global__ __launch_bounds__(kT) void k_u_edges_trial(int ne, const EdgeDev* __restrict__ edges,
                                                      const orb_ba_camera_t* __restrict__ cams,
                                                      const double* __restrict__ pose, const double* __restrict__ point,
                                                      const int32_t* __restrict__ pose_h, Huber2 hub,
                                                      double* __restrict__ err, double* __restrict__ rho0_out,
                                                      double* __restrict__ ecl, double* __restrict__ hpl, size_t hpl_alt,
                                                      double* __restrict__ ecp, double* __restrict__ part,
                                                      unsigned* counter, const double* __restrict__ part2, int nparts2,
                                                      const int32_t* __restrict__ status, double* __restrict__ scal,
                                                      LmState* st, LmProgress* prog, int dist, double* __restrict__ sc_part,
                                                      const volatile int32_t* h_stop) {
    if (lm_skip(st, kGateTrial)) return;
    const int e = blockIdx.x * kT + threadIdx.x;
    double r = 0.0;
    if (e < ne)
        r = ba_edge<kLin>(e, edges, cams, pose, point, pose_h, hub, err, rho0_out, ecl, hpl + (st->lin ? 0 : hpl_alt),
                          ecp, 0);
    const double bsum = block_sum<kT>(r);
    if (threadIdx.x == 0) part[blockIdx.x] = bsum;
    if (!last_block(counter)) return;
    double c = 0.0, d = 0.0;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += kT) c += part[i];
    for (int i = threadIdx.x; i < nparts2; i += kT) d += part2[i];
    const double chi = block_sum<kT>(c);
    const double scale = block_sum<kT>(d);
    if (threadIdx.x == 0) {
        if (dist) {  // this rank's parts and its stop flag, for k_lm_trial_ctl after the all-reduce
            sc_part[0] = chi;
            sc_part[1] = scale;
            sc_part[2] = (h_stop && *h_stop) ? 1.0 : 0.0;
        } else {
            const bool failed = *status != 0;
            scal[0] = chi;
            scal[1] = scale;
            scal[2] = failed ? 1.0 : 0.0;
            lm_trial_done(st, chi, scale, failed, prog, kLin);
        }
        *counter = 0;
    }
}

// Fast unit (round 6; one process, the single-workgroup Cholesky): steps 1-3 in one landmark-major
// launch.  kLB lanes per landmark: at the start of an iteration (phase 0) lane j linearises the
// landmark's edges j, j + kLB, ... (ba_edge: error, Jacobians, Hpl and the pose part to memory) and
// keeps their landmark parts; the lanes' sums (a fixed xor tree) are the landmark's Hll and b_l.  A
// re-trial after a rejection (phase 1) reads Hll and b_l back.  Then every lane forms
// Dinv = (Hll + lambda I)^-1 and, for its free edges, Z_e = Hpl_e Dinv and cb_e = Hpl_e (Dinv b_l),
// as k_ba_schur_edges does.  The pose sums (Hpp, b_p) follow in k_u_schur2, lambda I and Hpp join S in
// the Cholesky's tile loads, and the iteration's current chi2 is the accepted trial's (the same
// estimate; g2o's build recomputes the same value).
constexpr int kLB = 8;
__global__ __launch_bounds__(kT) void k_u_land_build(int nl, const double* __restrict__ lam,
                                                     const int32_t* __restrict__ land_off,
                                                     const int32_t* __restrict__ land_edge, const EdgeDev* __restrict__ edges,
                                                     const orb_ba_camera_t* __restrict__ cams,
                                                     const double* __restrict__ pose, const double* __restrict__ point,
                                                     const int32_t* __restrict__ pose_h, Huber2 hub,
                                                     double* __restrict__ err, double* __restrict__ rho0_out,
                                                     double* __restrict__ hpl, double* __restrict__ ecp,
                                                     double* __restrict__ hll, double* __restrict__ bl,
                                                     double* __restrict__ z, double* __restrict__ cb,
                                                     const LmState* __restrict__ st) {
    if (lm_skip(st, kGateTrial)) return;
    static_assert(kT % kLB == 0, "landmark groups inside a block");
    const bool build = st->phase == 0;
    const double lambda = *lam;
    const int g = (blockIdx.x * kT + threadIdx.x) / kLB, j = threadIdx.x % kLB;
    const bool live = g < nl;
    const int k0 = live ? land_off[g] : 0, k1 = live ? land_off[g + 1] : 0;
    double H[12];  // Hll (9) and b_l (3)
    LinOut lo;
    lo.free = false;
    if (build) {
#pragma unroll
        for (int i = 0; i < 12; ++i) H[i] = 0.0;
        for (int k = k0 + j; k < k1; k += kLB) {
            ba_edge<true, true>(land_edge[k], edges, cams, pose, point, pose_h, hub, err, rho0_out, nullptr, hpl, ecp,
                                0, &lo);
#pragma unroll
            for (int i = 0; i < 12; ++i) H[i] += lo.pl[i];
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) {  // the group's sum, the same bits in its kLB lanes
            H[i] += __shfl_xor(H[i], 1);
            H[i] += __shfl_xor(H[i], 2);
            H[i] += __shfl_xor(H[i], 4);
        }
        if (live && j == 0) {
#pragma unroll
            for (int i = 0; i < 9; ++i) hll[9 * (size_t)g + i] = H[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) bl[3 * (size_t)g + i] = H[9 + i];
        }
    } else if (live) {
#pragma unroll
        for (int i = 0; i < 9; ++i) H[i] = hll[9 * (size_t)g + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) H[9 + i] = bl[3 * (size_t)g + i];
    }
    if (!live || k0 + j >= k1) return;
    double D[9], Di[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) D[i] = H[i] + (i % 4 == 0 ? lambda : 0.0);
    inverse3(D, Di);
    double db[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) db[r] = Di[3 * r] * H[9] + Di[3 * r + 1] * H[10] + Di[3 * r + 2] * H[11];
    for (int k = k0 + j; k < k1; k += kLB) {
        const int e = land_edge[k];
        double h[18];
        bool fr;
        if (build && k + kLB >= k1) {  // the lane's last edge: its Hpl is still in registers
            fr = lo.free;
#pragma unroll
            for (int q = 0; q < 18; ++q) h[q] = lo.hx[q];
        } else {  // (this lane wrote it, or an earlier build did)
            fr = pose_h[edges[e].pose] >= 0;
#pragma unroll
            for (int q = 0; q < 18; ++q) h[q] = fr ? hpl[18 * (size_t)e + q] : 0.0;
        }
        if (!fr) continue;
        double* Z = z + 18 * (size_t)e;
        double* C = cb + 6 * (size_t)e;
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            const double h0 = h[3 * r], h1 = h[3 * r + 1], h2 = h[3 * r + 2];
#pragma unroll
            for (int c = 0; c < 3; ++c) Z[3 * r + c] = h0 * Di[c] + h1 * Di[3 + c] + h2 * Di[6 + c];
            C[r] = h0 * db[0] + h1 * db[1] + h2 * db[2];
        }
    }
}

// Fast unit, step 4: the S blocks without Hpp + lambda I (the Cholesky adds them), b_S = b_p - sum cb per
// free pose with b_p summed here from the pose parts (ba_reduce_pose's order for its b_p), and per free
// pose Hpp and b_p (ba_reduce_pose) for the Cholesky and the trial.  Blocks: [0, nblk) S, then nf b_S,
// then nf Hpp.
__global__ __launch_bounds__(64) void k_u_schur2(int n, int nf, int nblk, const double* __restrict__ lam,
                                                 const int32_t* __restrict__ blk_off, const EdgePair* __restrict__ pairs,
                                                 const int32_t* __restrict__ cnt, const int32_t* __restrict__ pose_off,
                                                 const LandEdge* __restrict__ pose_fl, const double* __restrict__ z,
                                                 const double* __restrict__ hpl, const double* __restrict__ ecp,
                                                 double* __restrict__ hpp, double* __restrict__ bp, double* __restrict__ S,
                                                 const double* __restrict__ cb, double* __restrict__ bs,
                                                 const LmState* __restrict__ st) {
    if (lm_skip(st, kGateTrial)) return;
    __shared__ double red[42][65];  // the branches' column sums share one buffer
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b < nblk) {
        ba_schur_block<true>(b, lane, n, nf, *lam, 0, blk_off, pairs, cnt, z, hpl, hpp, S, red);
    } else if (b < nblk + nf) {
        const int p = b - nblk;
        double s[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // b_p part sums, then cb sums
        const int k0 = pose_off[p] + lane, k1 = pose_off[p + 1];
        for (int k = k0; k < k1; k += 64) {
            const int e = pose_fl[k].e;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                s[i] += ecp[42 * (size_t)e + 36 + i];
                s[6 + i] += cb[6 * (size_t)e + i];
            }
        }
        const double t = wave_sum_cols_in<12>(s, lane, red);
        __shared__ double bpv[6];
        if (lane < 6) bpv[lane] = t;
        __syncthreads();
        if (lane >= 6 && lane < 12) bs[6 * (size_t)p + lane - 6] = bpv[lane - 6] - t;
    } else if (b < nblk + 2 * nf) {
        (void)ba_reduce_pose<true>(b - nblk - nf, lane, pose_off, pose_fl, ecp, hpp, bp, red);
    }
}

// unit steps 6 + 7 in one launch, landmark-major: thread l computes x_l (back-substitution), pushes
// and moves landmark l, and evaluates the errors of the landmark's edges (all of them, in edge order)
// at the new estimate, with the new point from registers.  A block is two waves: wave 0 takes kT
// landmarks; wave 1 the poses (pose_mode 1, nf <= kT): every block computes the whole pose update into
// LDS (lane t: pose t from its base -- the backup when the previous trial was rejected -- and
// exp(x_t)) while wave 0 runs the back-substitution, so that no block waits for another; only the last
// block, once every other block has read the bases, writes the poses and their backups.  pose_mode 2:
// k_u_pose_update moved them before this launch (and left their computeScale part in *pscale); 0: no
// free pose.  Per block: the chi2 partial into part[block], the landmarks' computeScale partial into
// part2[block]; the last block sums both in block order, adds the poses' part (in pose order) and runs
// the trial controller, as k_u_edges_trial<false> does.  The sums are grouped by landmark instead of
// by edge block: the same terms, another rounding order.
constexpr int kLandEdgeBatch = 8;  // a landmark's edges evaluated 8 at a time (loads issued together; the
                                   // first batch's before the back-substitution)
constexpr int kLT = 2 * kT;        // k_u_land_trial's block: landmark wave + pose wave
static_assert(kT == 64, "k_u_land_trial: one wave of landmarks, one of poses");
__global__ __launch_bounds__(kLT) void k_u_land_trial(int nl, int n, const double* __restrict__ lam,
                                                     const int32_t* __restrict__ landf_off, const int32_t* __restrict__ landf_edge,
                                                     const int32_t* __restrict__ landf_row, const double* __restrict__ hpl,
                                                     size_t hpl_alt, const double* __restrict__ bl,
                                                     const double* __restrict__ hll, double* __restrict__ x,
                                                     const int32_t* __restrict__ land_point, double* __restrict__ point,
                                                     double* __restrict__ point_bak, const int32_t* __restrict__ land_off,
                                                     const int32_t* __restrict__ land_edge, const EdgeDev* __restrict__ edges,
                                                     const orb_ba_camera_t* __restrict__ cams, double* __restrict__ pose,
                                                     const int32_t* __restrict__ pose_h, PoseTail pt, int pose_mode,
                                                     Huber2 hub, double* __restrict__ err, double* __restrict__ rho0_out,
                                                     double* __restrict__ part, double* __restrict__ part2,
                                                     unsigned* counter, const int32_t* __restrict__ status,
                                                     double* __restrict__ scal, LmState* st, LmProgress* prog, int dist,
                                                     double* __restrict__ sc_part, const volatile int32_t* h_stop,
                                                     int fast) {
    if (lm_skip(st, kGateTrial)) return;
    __shared__ double s_new[kT][7], s_base[kT][7], s_pc[kT];
    hpl += hpl_cur(st, hpl_alt);
    const bool rej = st->reject != 0;
    const double lambda = *lam;
    const int tid = threadIdx.x, pw = tid - kT;  // pw: the pose wave's lane (wave 1)
    const int l = tid < kT ? blockIdx.x * kT + tid : nl;
    if (pose_mode == 1 && pw >= 0 && pw < pt.nf) {  // pose pw's trial update, into LDS only
        const int fp = pt.free_pose[pw];
        const double* src = (rej ? pt.pose_bak : pose) + 7 * (size_t)fp;
        double v[7], u[6];
        for (int i = 0; i < 7; ++i) v[i] = src[i];
        for (int i = 0; i < 6; ++i) u[i] = x[6 * (size_t)pw + i];
        double c = 0.0;
        if (pt.primary)
            for (int i = 0; i < 6; ++i) c += u[i] * (lambda * u[i] + pt.bp[6 * (size_t)pw + i]);
        for (int i = 0; i < 7; ++i) s_base[pw][i] = v[i];
        se3_oplus(v, u);
        for (int i = 0; i < 7; ++i) s_new[pw][i] = v[i];
        s_pc[pw] = c;
    }
    // the first edge batch's records (independent of the solve) are requested before the back-substitution
    int k0 = 0, k1 = 0;
    int e[kLandEdgeBatch], pr[kLandEdgeBatch];
    EdgeDev E[kLandEdgeBatch];
    orb_ba_camera_t cam[kLandEdgeBatch];
    auto load_batch = [&](int kb) {
#pragma unroll
        for (int u = 0; u < kLandEdgeBatch; ++u) {
            e[u] = land_edge[min(kb + u, k1 - 1)];
            E[u] = edges[e[u]];
            cam[u] = cams[E[u].pose];
            pr[u] = pose_mode == 1 ? pose_h[E[u].pose] : -1;
        }
    };
    if (l < nl) {
        k0 = land_off[l];
        k1 = land_off[l + 1];
        load_batch(k0);
    }
    double c = 0.0, r = 0.0;
    double Xn[3] = {0.0, 0.0, 0.0};
    if (l < nl) {
        // the landmark's base estimate is requested before the back-substitution (independent of it)
        double* X = point + 3 * (size_t)land_point[l];
        double* Xb = point_bak + 3 * (size_t)land_point[l];
        double v[3];
        for (int i = 0; i < 3; ++i) v[i] = rej ? Xb[i] : X[i];
        double xl[3];
        ba_backsub(l, n, lambda, landf_off, landf_edge, landf_row, hpl, bl, hll, x, xl);
        for (int i = 0; i < 3; ++i) c += xl[i] * (lambda * xl[i] + bl[3 * (size_t)l + i]);
        for (int i = 0; i < 3; ++i) {
            Xb[i] = v[i];
            Xn[i] = v[i] + xl[i];
            X[i] = Xn[i];
        }
    }
    if (pose_mode == 1) __syncthreads();  // s_new complete
    if (l < nl) {
        for (int kb = k0; kb < k1; kb += kLandEdgeBatch) {
            if (kb != k0) load_batch(kb);
            double T[kLandEdgeBatch][7];
#pragma unroll
            for (int u = 0; u < kLandEdgeBatch; ++u) {
                const double* ts = pr[u] >= 0 ? &s_new[pr[u]][0] : pose + 7 * (size_t)E[u].pose;
#pragma unroll
                for (int i = 0; i < 7; ++i) T[u][i] = ts[i];
            }
#pragma unroll
            for (int u = 0; u < kLandEdgeBatch; ++u) {
                if (kb + u >= k1) break;
                double Xc[3], er[3], rho1;
                const double rho0 = ba_edge_err(E[u], cam[u], T[u], Xn, hub, Xc, er, rho1);
                err[3 * (size_t)e[u]] = er[0];
                err[3 * (size_t)e[u] + 1] = er[1];
                err[3 * (size_t)e[u] + 2] = er[2];
                rho0_out[e[u]] = rho0;
                r += rho0;
            }
        }
    }
    const double rsum = block_sum<kLT>(r);
    const double csum = block_sum<kLT>(c);
    if (tid == 0) {
        part[blockIdx.x] = rsum;
        part2[blockIdx.x] = csum;
    }
    if (!last_block(counter)) return;
    if (pose_mode == 1 && pw >= 0 && pw < pt.nf) {  // every other block has read the bases: commit the poses
        const int fp = pt.free_pose[pw];
        for (int i = 0; i < 7; ++i) {
            pt.pose_bak[7 * (size_t)fp + i] = s_base[pw][i];
            pose[7 * (size_t)fp + i] = s_new[pw][i];
        }
    }
    double a = 0.0, d = 0.0;
    for (int i = tid; i < (int)gridDim.x; i += kLT) {
        a += part[i];
        d += part2[i];
    }
    const double chi = block_sum<kLT>(a);
    double scale = block_sum<kLT>(d);
    if (tid == 0) {
        if (pose_mode == 1)
            for (int p = 0; p < pt.nf; ++p) scale += s_pc[p];
        else if (pose_mode == 2)
            scale += *pt.pscale;
        if (dist) {  // this rank's parts and its stop flag, for k_lm_trial_ctl after the all-reduce
            sc_part[0] = chi;
            sc_part[1] = scale;
            sc_part[2] = (h_stop && *h_stop) ? 1.0 : 0.0;
        } else {
            const bool failed = *status != 0;
            scal[0] = chi;
            scal[1] = scale;
            scal[2] = failed ? 1.0 : 0.0;
            lm_trial_done(st, chi, scale, failed, prog, false, fast != 0);
        }
        *counter = 0;
    }
}

// sharded trial controller, after the all-reduce of the trial partials (sc_red: chi2, computeScale,
// the number of ranks whose stop flag is raised): every rank takes the same decision; a raised flag
// on any rank ends the solve after this trial (g2o's force-stop flag, tested between iterations)
template <bool kLin>
__global__ __launch_bounds__(64) void k_lm_trial_ctl(const double* __restrict__ sc_red, const int32_t* __restrict__ status,
                                                     double* __restrict__ scal, LmState* st, LmProgress* prog) {
    if (lm_skip(st, kGateTrial)) return;
    if (threadIdx.x != 0) return;
    const bool failed = *status != 0;
    scal[0] = sc_red[0];
    scal[1] = sc_red[1];
    scal[2] = failed ? 1.0 : 0.0;
    lm_trial_done(st, sc_red[0], sc_red[1], failed, prog, kLin);
    if (sc_red[2] > 0 && !st->done) {
        st->done = 1;
        prog->done = 1;
        __threadfence_system();
    }
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

// All per-solve inputs travel in one pinned staging buffer: one H2D copy, then k_ba_scatter moves
// every array to its device buffer (one launch instead of one copy per array).
struct ScatterItem {
    uint64_t dst, off, bytes;
};

constexpr uint64_t kScatterZero = ~0ull;  // ScatterItem::off of an item that zero-fills its buffer

__global__ __launch_bounds__(256) void k_ba_scatter(const uint8_t* __restrict__ src, const ScatterItem* __restrict__ items) {
    const ScatterItem it = items[blockIdx.y];
    uint8_t* dst = reinterpret_cast<uint8_t*>(it.dst);
    const size_t n16 = it.bytes / 16;
    if (it.off == kScatterZero) {
        for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
            reinterpret_cast<uint4*>(dst)[i] = make_uint4(0, 0, 0, 0);
        if (blockIdx.x == 0 && threadIdx.x < it.bytes % 16) dst[n16 * 16 + threadIdx.x] = 0;
        return;
    }
    const uint8_t* sp = src + it.off;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(sp)[i];
    if (blockIdx.x == 0 && threadIdx.x < it.bytes % 16) dst[n16 * 16 + threadIdx.x] = sp[n16 * 16 + threadIdx.x];
}

// Per-solve inputs: add() records (device buffer, host source, bytes), zero() a buffer to clear;
// pack() lays the sources out behind the item table in one pinned buffer (a single copy from each
// source), which goes up in one H2D copy and is spread by one k_ba_scatter launch (the clears too:
// no memset launches).
struct Stager {
    struct Src { const void* p; size_t off, bytes; };
    std::vector<ScatterItem> items;
    std::vector<Src> srcs;
    size_t data_bytes = 0;
    template <typename T>
    bool add(DevBuf<T>& d, const T* src, size_t n) {
        if (!d.grow(n)) return false;
        if (n == 0) return true;
        const size_t off = (data_bytes + 15) & ~size_t(15);
        data_bytes = off + n * sizeof(T);
        items.push_back({(uint64_t)(uintptr_t)d.p, off, n * sizeof(T)});
        srcs.push_back({src, off, n * sizeof(T)});
        return true;
    }
    template <typename T>
    bool add(DevBuf<T>& d, const std::vector<T>& v) {
        return add(d, v.data(), v.size());
    }
    template <typename T>
    bool zero(DevBuf<T>& d, size_t n) {
        if (!d.grow(n)) return false;
        if (n) items.push_back({(uint64_t)(uintptr_t)d.p, kScatterZero, n * sizeof(T)});
        return true;
    }
    size_t table_bytes() const { return (items.size() * sizeof(ScatterItem) + 255) & ~size_t(255); }
    void pack(uint8_t* dst) const {
        memcpy(dst, items.data(), items.size() * sizeof(ScatterItem));
        for (const Src& x : srcs) memcpy(dst + table_bytes() + x.off, x.p, x.bytes);
    }
};

struct orb_ba_s {
    orbgpu_ba::BaStructure st;  // the host structure of the last solve (vectors reused)
    hipStream_t stream = nullptr;
    hipStream_t tail = nullptr;  // the end of a device-driven solve, beside the queued no-op unit
    DevBuf<double> pose, pose_bak, point, point_bak, err, rho0, ecl, hpl, ecp, hpp, hll, b, z, cb, S, bs, x, scal;
    DevBuf<EdgeDev> edges;
    DevBuf<orb_ba_camera_t> cams;
    DevBuf<int32_t> pose_h, free_pose, land_point, land_off, land_edge, landf_off, landf_edge, landf_row, fland, pose_off,
        status;
    DevBuf<LandEdge> pose_fl;
    DevBuf<int32_t> blk_off, blk_cnt;  // Schur block product lists (k_ba_schur_pairs)
    DevBuf<EdgePair> pairs;
    DevBuf<uint8_t> depth;
    double* h_scal = nullptr;  // pinned: [0] chi2, [1] scale, [2] status, [3] maxdiag, [4] stop, [5] lambda
    DevBuf<LmState> lm;        // device-driven LM state
    DevBuf<double> part;       // per-block chi2 partials of the fused unit kernels
    DevBuf<unsigned> counters;  // last-block counters of the fused unit kernels
    uint8_t* h_stage = nullptr;  // pinned staging of the per-solve inputs
    size_t h_stage_cap = 0;
    uint8_t* h_stage0 = nullptr;  // one rank: the raw inputs, uploaded before the structure is built
    size_t h_stage0_cap = 0;
    DevBuf<uint8_t> d_stage0;
    uint8_t* h_dl = nullptr;     // pinned download of the per-solve results
    size_t h_dl_cap = 0;
    DevBuf<uint8_t> d_stage;
    LmProgress* h_prog = nullptr;  // pinned, written by k_lm_trial_done
    hipEvent_t unit_ev[2] = {nullptr, nullptr};
    // the LM unit (7 launches) captured as a HIP graph, reused while its launch arguments are unchanged
    hipGraph_t unit_graph = nullptr;
    hipGraphExec_t unit_exec = nullptr;
    std::vector<uintptr_t> unit_key;
    float ms_total = 0;
    // multi-GPU: ranks own landmark ranges; partial sums are all-reduced
    int world = 1, rank = 0;
    orb_ba_host_reduce_fn host_fn = nullptr;
    void* host_ctx = nullptr;
    void* nccl_comm = nullptr;
    double* h_red = nullptr;  // pinned staging of the host reducer
    size_t h_red_cap = 0;
    DevBuf<double> red_buf;
    // sharded device-driven loop: this rank's partials (all-reduced out of place into the solve's
    // buffers: a gated no-op unit re-reduces unchanged partials into unchanged sums) and the stop flag
    // the host raises for the trial controller (pinned)
    DevBuf<double> dpart;
    int32_t* h_stop = nullptr;
    bool force_dist = false;  // ORBGPU_BA_DIST_FORCE=1 with a one-rank RCCL communicator (tests)
    DevBuf<int64_t> trace;  // ORBGPU_BA_TRACE stamps (debug)
    // k_ba_chol_rows: published tiles / y, the epoch + flag words (zeroed when allocated), row scratch
    DevBuf<double> lpub, ypub, racc;
    DevBuf<unsigned> cflag;

    void release() {
        for (auto* d : {&pose, &pose_bak, &point, &point_bak, &err, &rho0, &ecl, &hpl, &ecp, &hpp, &hll, &b, &z,
                        &cb, &S, &bs, &x, &scal, &lpub, &ypub, &racc})
            d->release();
        cflag.release();
        edges.release();
        cams.release();
        for (auto* d : {&pose_h, &free_pose, &land_point, &land_off, &land_edge, &landf_off, &landf_edge, &landf_row, &fland,
                        &pose_off,
                        &status})
            d->release();
        pose_fl.release();
        blk_off.release();
        blk_cnt.release();
        pairs.release();
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

namespace {
std::atomic<bool> g_force_rows{false};  // orb_debug_ba_chol_timeout(force_rows, ...)
}

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
        hipStreamCreateWithFlags(&h->tail, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(&h->h_scal, 8 * sizeof(double), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&h->h_prog, sizeof(LmProgress), hipHostMallocDefault) != hipSuccess || !h->lm.grow(1) ||
        hipHostMalloc(&h->h_stop, sizeof(int32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&h->unit_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->unit_ev[1], hipEventDisableTiming) != hipSuccess) {
        delete h;
        return orbgpu_fail(ORB_ERR_DEVICE, "BA handle allocation");
    }
    *out = h;
    return ORB_OK;
}

int orb_ba_destroy(orb_ba_t h) {
    if (!h) return ORB_OK;
    hipStreamSynchronize(h->stream);
    hipStreamSynchronize(h->tail);
    h->release();
    h->red_buf.release();
    h->lm.release();
    h->part.release();
    h->counters.release();
    h->d_stage.release();
    if (h->h_stage) hipHostFree(h->h_stage);
    if (h->h_stage0) hipHostFree(h->h_stage0);
    if (h->h_dl) hipHostFree(h->h_dl);
    if (h->h_prog) hipHostFree(h->h_prog);
    if (h->h_stop) hipHostFree(h->h_stop);
    h->dpart.release();
    for (hipEvent_t e : h->unit_ev)
        if (e) hipEventDestroy(e);
    if (h->unit_exec) hipGraphExecDestroy(h->unit_exec);
    if (h->unit_graph) hipGraphDestroy(h->unit_graph);
    h->trace.release();
    if (h->h_scal) hipHostFree(h->h_scal);
    if (h->h_red) hipHostFree(h->h_red);
    if (h->stream) hipStreamDestroy(h->stream);
    if (h->tail) hipStreamDestroy(h->tail);
    delete h;
    return ORB_OK;
}

// ORBGPU_BA_TRACE: print the MFMA Cholesky's phase stamps (debug)
void dump_chol_trace(const int64_t* tr, int n, hipStream_t s) {
    std::vector<int64_t> ht(kTraceLen);
    hipMemcpyAsync(ht.data(), tr, kTraceLen * sizeof(int64_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    int64_t t0 = 0;  // the earliest stamp
    for (int64_t v : ht)
        if (v && (!t0 || v < t0)) t0 = v;
    const int NT = (n + 15) / 16;
    auto rel = [&](int i) { return (long long)(ht[i] ? ht[i] - t0 : -1); };
    for (int k = 0; k < NT; ++k)
        for (int w = 0; w <= kMf2TileWaves; ++w) {
            const int b = kTrStep + (k * 16 + w) * 4;
            fprintf(stderr, "MFTRACE k=%d w=%d %lld %lld %lld %lld\n", k, w, rel(b), rel(b + 1), rel(b + 2), rel(b + 3));
        }
    for (int k = NT - 1; k >= 0; --k) {
        long long c0 = -1, c1 = -1;  // row k's contributions: first wave in, last wave done
        for (int w = 0; w < kMf2TileWaves; ++w) {
            const long long a = rel(kTrC + 32 * k + 2 * w), b = rel(kTrC + 32 * k + 2 * w + 1);
            if (a >= 0 && (c0 < 0 || a < c0)) c0 = a;
            if (b > c1) c1 = b;
        }
        fprintf(stderr, "MFTRACE e k=%d in %lld formed %lld row_contrib %lld-%lld\n", k, rel(kTrE + 2 * k),
                rel(kTrE + 2 * k + 1), c0, c1);
        for (int w = 0; w < kMf2TileWaves; ++w)
            if (rel(kTrC + 32 * k + 2 * w) >= 0)
                fprintf(stderr, "MFTRACE rowc k=%d w=%d %lld %lld  (x loaded %lld, tiles done %lld)\n", k, w,
                        rel(kTrC + 32 * k + 2 * w), rel(kTrC + 32 * k + 2 * w + 1),
                        k >= NT - 2 ? rel(kTrD + 32 * (NT - 1 - k) + 2 * w) : -1,
                        k >= NT - 2 ? rel(kTrD + 32 * (NT - 1 - k) + 2 * w + 1) : -1);
        fprintf(stderr, "MFTRACE back k=%d %lld waited %lld published %lld\n", k, rel(kTrBack + k), rel(kTrWaited + k),
                rel(kTrPub + k));
    }
    fprintf(stderr, "MFTRACE end %lld\n", rel(kTrEnd));
    for (int k = 0; k + 1 < NT; ++k) {
        const int b = kTrDiag + 4 * k;
        fprintf(stderr, "MFTRACE diag k=%d factor %lld linv %lld y %lld\n", k, (long long)(ht[b + 1] - ht[b]),
                (long long)(ht[b + 2] - ht[b + 1]), (long long)(ht[b + 3] - ht[b + 2]));
    }
}

// ---- collectives of the sharded solve -------------------------------------------------------------
namespace {

// RCCL entry points, resolved from the librccl.so.1 already loaded in the process (torch's) or from
// /opt/rocm/lib: no link-time dependency, one RCCL instance per process.
struct NcclUniqueId {  // ncclUniqueId: 128 opaque bytes, passed BY VALUE to ncclCommInitRank
    char internal[128];
};
struct Rccl {
    typedef int (*GetUniqueId)(void*);
    typedef int (*CommInitRank)(void**, int, NcclUniqueId, int);
    typedef int (*AllReduce)(const void*, void*, size_t, int, int, void*, hipStream_t);
    typedef int (*CommDestroy)(void*);
    GetUniqueId get_id = nullptr;
    CommInitRank init = nullptr;
    AllReduce all_reduce = nullptr;
    CommDestroy destroy = nullptr;
    bool load() {
        if (all_reduce) return true;
        void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW);
        if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!lib) return false;
        get_id = (GetUniqueId)dlsym(lib, "ncclGetUniqueId");
        init = (CommInitRank)dlsym(lib, "ncclCommInitRank");
        all_reduce = (AllReduce)dlsym(lib, "ncclAllReduce");
        destroy = (CommDestroy)dlsym(lib, "ncclCommDestroy");
        return get_id && init && all_reduce && destroy;
    }
};
Rccl g_rccl;
constexpr int kNcclDouble = 8, kNcclSum = 0, kNcclMax = 2;  // ncclDataType_t / ncclRedOp_t values

// In-place all-reduce of n doubles at device address d (stream-ordered); no-op on one rank.
bool dev_reduce(orb_ba_s* h, double* d, size_t n, int op) {
    if ((h->world <= 1 && !h->force_dist) || n == 0) return true;
    if (h->nccl_comm)
        return g_rccl.all_reduce(d, d, n, kNcclDouble, op == ORB_BA_MAX ? kNcclMax : kNcclSum, h->nccl_comm,
                                 h->stream) == 0;
    if (n > h->h_red_cap) {
        if (h->h_red) hipHostFree(h->h_red);
        h->h_red = nullptr;
        h->h_red_cap = 0;
        if (hipHostMalloc(&h->h_red, n * sizeof(double), hipHostMallocDefault) != hipSuccess) return false;
        h->h_red_cap = n;
    }
    if (hipMemcpyAsync(h->h_red, d, n * sizeof(double), hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess)
        return false;
    if (h->host_fn(h->host_ctx, h->h_red, n, op) != 0) return false;
    return hipMemcpyAsync(d, h->h_red, n * sizeof(double), hipMemcpyHostToDevice, h->stream) == hipSuccess;
}

// Out-of-place all-reduce of n doubles, send -> recv (stream-ordered with RCCL; the host reducer
// synchronises the stream).
bool dev_reduce2(orb_ba_s* h, const double* send, double* recv, size_t n, int op) {
    if (n == 0) return true;
    if (h->nccl_comm)
        return g_rccl.all_reduce(send, recv, n, kNcclDouble, op == ORB_BA_MAX ? kNcclMax : kNcclSum, h->nccl_comm,
                                 h->stream) == 0;
    if (hipMemcpyAsync(recv, send, n * sizeof(double), hipMemcpyDeviceToDevice, h->stream) != hipSuccess) return false;
    return h->world <= 1 || dev_reduce(h, recv, n, op);
}

}  // namespace

int orb_ba_dist_unique_id(uint8_t id[128]) {
    if (!id) return orbgpu_fail(ORB_ERR_ARG, "null id");
    if (!g_rccl.load()) return orbgpu_fail(ORB_ERR_DEVICE, "librccl.so.1 not found");
    if (g_rccl.get_id(id) != 0) return orbgpu_fail(ORB_ERR_DEVICE, "ncclGetUniqueId failed");
    return ORB_OK;
}

int orb_ba_dist_init_rccl(orb_ba_t h, const uint8_t id[128], int world, int rank) {
    if (!h || !id || world < 1 || rank < 0 || rank >= world) return orbgpu_fail(ORB_ERR_ARG, "bad RCCL arguments");
    if (!g_rccl.load()) return orbgpu_fail(ORB_ERR_DEVICE, "librccl.so.1 not found");
    if (h->nccl_comm) g_rccl.destroy(h->nccl_comm);
    h->nccl_comm = nullptr;
    NcclUniqueId uid;
    memcpy(uid.internal, id, sizeof(uid.internal));
    if (g_rccl.init(&h->nccl_comm, world, uid, rank) != 0) {
        h->nccl_comm = nullptr;
        return orbgpu_fail(ORB_ERR_DEVICE, "ncclCommInitRank failed");
    }
    h->world = world;
    h->rank = rank;
    h->host_fn = nullptr;
    // ORBGPU_BA_DIST_FORCE=1: a one-rank communicator still takes the sharded path (its collectives are
    // RCCL calls on one rank), so the sharded device loop and RCCL run on a one-GPU box
    const char* fd = getenv("ORBGPU_BA_DIST_FORCE");
    h->force_dist = world == 1 && fd && !strcmp(fd, "1");
    return ORB_OK;
}

int orb_ba_dist_init_host(orb_ba_t h, orb_ba_host_reduce_fn fn, void* ctx, int world, int rank) {
    if (!h || (world > 1 && !fn) || world < 1 || rank < 0 || rank >= world)
        return orbgpu_fail(ORB_ERR_ARG, "bad host reducer arguments");
    if (h->nccl_comm) g_rccl.destroy(h->nccl_comm);
    h->nccl_comm = nullptr;
    h->force_dist = false;
    h->host_fn = fn;
    h->host_ctx = ctx;
    h->world = world;
    h->rank = rank;
    return ORB_OK;
}

static bool stop_requested(const orb_ba_options_t* opt) {
    return (opt->stop_flag && *opt->stop_flag) || (opt->stop_flag_bool && *opt->stop_flag_bool);
}

// Debug hook (not in the public header): force_rows selects k_ba_chol_rows for every n; row >= 0 arms
// the forced timeout of that tile row's first wait in the next k_ba_chol_rows launch.  Synchronous.
int orb_debug_ba_chol_timeout(int force_rows, int row) {
    g_force_rows.store(force_rows != 0, std::memory_order_relaxed);
    const int none = -1;
    const unsigned zero = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_chol_row), &row, sizeof(int)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_chol_epoch), &zero, sizeof(unsigned)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_chol_status), &none, sizeof(int)) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "debug symbol copy");
    return ORB_OK;
}

// The status the armed launch ended with (-1: no armed launch has finished).  Synchronous.
int orb_debug_ba_chol_timeout_status(int32_t* status) {
    if (!status) return orbgpu_fail(ORB_ERR_ARG, "null status");
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(status, HIP_SYMBOL(g_dbg_chol_status), sizeof(int32_t)) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "debug symbol read");
    return ORB_OK;
}

int orb_ba_optimize(orb_ba_t h, orb_ba_problem_t* pr, const orb_ba_options_t* opt, double* edge_chi2,
                    uint8_t* edge_depth_ok, orb_ba_result_t* res) {
    if (!h || !pr || !opt || !res) return orbgpu_fail(ORB_ERR_ARG, "null BA argument");
    memset(res, 0, sizeof(*res));
    // ORBGPU_BA_TRACE: host-side phase times of each solve on stderr (structure, upload+LM, results)
    static const bool trace = getenv("ORBGPU_BA_TRACE") != nullptr;
    using clk = std::chrono::steady_clock;
    const clk::time_point t_in = clk::now();
    clk::time_point t_struct = t_in, t_solve = t_in, t_order = t_in, t_csr = t_in, t_pairs = t_in, t_pack = t_in;
    double unit_t[32];  // (trace) when each unit launch was seen complete, from t_pack
    int n_unit_t = 0;
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    const int np = pr->n_poses, nq = pr->n_points, ne_all = pr->n_edges;
    if (np < 0 || nq < 0 || ne_all < 0 || (np && (!pr->pose || !pr->pose_id || !pr->pose_fixed || !pr->pose_camera)) ||
        (nq && (!pr->point || !pr->point_id)) || (ne_all && !pr->edges) || opt->iterations < 0)
        return orbgpu_fail(ORB_ERR_ARG, "invalid BA problem");
    for (int e = 0; e < ne_all; ++e) {
        const orb_ba_edge_t& E = pr->edges[e];
        if (E.point < 0 || E.point >= nq || E.pose < 0 || E.pose >= np || (E.stereo != 0 && E.stereo != 1))
            return orbgpu_fail(ORB_ERR_ARG, "BA edge references a missing vertex");
    }
    const bool dist = h->world > 1 || h->force_dist;
    const bool primary = h->rank == 0;
    hipStream_t s = h->stream;
    if (!h->scal.grow(16)) return orbgpu_fail(ORB_ERR_DEVICE, "BA scalar buffer");
    // the stop flag, agreed across the ranks (MAX) so that every rank takes the same path
    auto stop = [&]() -> bool {
        double f = stop_requested(opt) ? 1.0 : 0.0;
        if (!dist) return f != 0.0;
        h->h_scal[4] = f;
        hipMemcpyAsync(h->scal.p + 4, &h->h_scal[4], sizeof(double), hipMemcpyHostToDevice, s);
        dev_reduce(h, h->scal.p + 4, 1, ORB_BA_MAX);
        hipMemcpyAsync(&h->h_scal[4], h->scal.p + 4, sizeof(double), hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        return h->h_scal[4] != 0.0;
    };

    // A local failure before the solve must be agreed by every rank (MAX over the ranks), so that no
    // rank returns while the others block in the next collective.  Single process: the local value.
    auto agree_fail = [&](bool local_fail) -> bool {
        if (!dist) return local_fail;
        h->h_scal[6] = local_fail ? 1.0 : 0.0;
        hipMemcpyAsync(h->scal.p + 6, &h->h_scal[6], sizeof(double), hipMemcpyHostToDevice, s);
        const bool ok = dev_reduce(h, h->scal.p + 6, 1, ORB_BA_MAX);
        hipMemcpyAsync(&h->h_scal[6], h->scal.p + 6, sizeof(double), hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess || !ok) return true;
        return h->h_scal[6] != 0.0;
    };

    // [items table | data] of a Stager in one pinned buffer, one copy, one scatter launch
    auto upload_stage = [&](const Stager& sg, uint8_t*& hbuf, size_t& hcap, DevBuf<uint8_t>& dbuf) -> bool {
        if (sg.items.empty()) return true;
        const size_t data_off = sg.table_bytes(), total = data_off + sg.data_bytes;
        if (total > hcap) {
            if (hbuf) hipHostFree(hbuf);
            hbuf = nullptr;
            hcap = 0;
            if (hipHostMalloc(&hbuf, total, hipHostMallocDefault) != hipSuccess) return false;
            hcap = total;
        }
        if (!dbuf.grow(total)) return false;
        sg.pack(hbuf);
        if (hipMemcpyAsync(dbuf.p, hbuf, total, hipMemcpyHostToDevice, s) != hipSuccess) return false;
        size_t maxb = 0;
        for (const ScatterItem& it : sg.items) maxb = std::max<size_t>(maxb, it.bytes);
        const unsigned gx = (unsigned)std::min<size_t>(64, std::max<size_t>(1, (maxb / 16 + 255) / 256));
        hipLaunchKernelGGL(k_ba_scatter, dim3(gx, (unsigned)sg.items.size()), dim3(256), 0, s, dbuf.p + data_off,
                           (const ScatterItem*)dbuf.p);
        return hipGetLastError() == hipSuccess;
    };
    // poses normalised as SE3Quat(q, t) does
    std::vector<double> pose(pr->pose, pr->pose + 7 * (size_t)np);
    for (int i = 0; i < np; ++i) {
        double* q = &pose[7 * (size_t)i + 3];
        if (q[3] < 0) for (int k = 0; k < 4; ++k) q[k] = -q[k];
        const double nn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        if (nn > 0) for (int k = 0; k < 4; ++k) q[k] /= nn;
    }
    // One rank uses the problem's edges in place: the raw inputs (poses, points, edges, cameras) go up
    // now, and the copy runs while the host builds the structure below (it does not need them on the
    // device).  Sharded solves upload their rank's edge copy with the structure.
    const bool early = !dist && ne_all > 0;
    if (early) {
        Stager s0;
        const bool ok0 = s0.add(h->pose, pose) && s0.add(h->point, pr->point, 3 * (size_t)nq) &&
                         s0.add(h->edges, reinterpret_cast<const EdgeDev*>(pr->edges), (size_t)ne_all) &&
                         s0.add(h->cams, pr->pose_camera, np) &&
                         upload_stage(s0, h->h_stage0, h->h_stage0_cap, h->d_stage0);
        if (!ok0) return orbgpu_fail(ORB_ERR_DEVICE, "BA device allocation / upload");
    }

    // ---- structure (initializeOptimization + BlockSolver::buildStructure), csrc/ba_structure.h
    orbgpu_ba::BaStructure& T = h->st;
    if (!orbgpu_ba::ba_build_structure(pr, h->world, h->rank, T)) {  // SparseOptimizer::optimize returns -1: nothing to do
        if (early) (void)hipStreamSynchronize(s);  // the raw upload reads the pinned staging the next call rewrites
        for (int e = 0; e < ne_all; ++e) {
            if (edge_chi2) edge_chi2[e] = 0;
            if (edge_depth_ok) edge_depth_ok[e] = 0;
        }
        return ORB_OK;
    }
    t_order = t_csr = clk::now();
    if (stop()) {
        if (early) (void)hipStreamSynchronize(s);
        res->stopped = 1;
        return ORB_ERR_ABORTED;
    }
    if (agree_fail(T.dup_edge) || agree_fail(T.n_products > INT32_MAX)) {
        if (early) (void)hipStreamSynchronize(s);
        return orbgpu_fail(ORB_ERR_ARG, T.dup_edge ? "two edges between one keyframe and one map point"
                                                   : "BA window too large");
    }
    static_assert(sizeof(EdgeDev) == sizeof(orb_ba_edge_t), "EdgeDev mirrors orb_ba_edge_t");
    const EdgeDev* ledges = reinterpret_cast<const EdgeDev*>(T.ledges);
    const int nf = T.nf, ne = T.ne, nl = T.nl, nfe = T.nfe, nblk = T.nblk;
    const int n = 6 * nf, m = 3 * nl;
    const std::vector<int32_t>& point_l = T.point_l;
    const std::vector<int32_t>& qdeg = T.qdeg;
    const std::vector<int32_t>& lmap = T.lmap;
    t_pairs = clk::now();

    const double tau = 1e-5;
    LmState lm_init{};  // the device-driven loop's start (g2o's Levenberg state before iteration 0)
    lm_init.ni = 2;
    lm_init.user_lambda = opt->user_lambda_init;
    lm_init.tau = tau;
    lm_init.iterations = opt->iterations;
    lm_init.done = opt->iterations <= 0;

    t_struct = clk::now();
    const size_t ne1 = std::max(ne, 1);
    Stager st;
    bool ok = (early || (st.add(h->pose, pose) && st.add(h->point, pr->point, 3 * (size_t)nq) &&
                         st.add(h->edges, ledges, (size_t)ne) && st.add(h->cams, pr->pose_camera, np))) &&
              h->pose_bak.grow(7 * (size_t)np) && h->point_bak.grow(3 * (size_t)nq) && st.add(h->pose_h, T.pose_h) && st.add(h->free_pose, T.free_pose) && st.add(h->land_point, T.land_point) &&
              st.add(h->land_off, T.land_off) && st.add(h->land_edge, T.land_edge) &&
              st.add(h->landf_off, T.landf_off) && st.add(h->landf_edge, T.landf_edge) && st.add(h->fland, T.fland) &&
              st.add(h->landf_row, T.landf_row) && st.add(h->pose_off, T.pose_off) && st.add(h->pose_fl, T.pose_fl) &&
              st.add(h->blk_off, T.blk_off) && h->blk_cnt.grow(std::max(nblk, 1)) &&
              h->pairs.grow(std::max<size_t>(1, (size_t)T.blk_off[nblk])) &&
              h->err.grow(3 * ne1) && h->rho0.grow(ne1) && h->ecl.grow(12 * ne1) && h->hpl.grow(36 * ne1) &&
              h->ecp.grow(42 * ne1) && h->hpp.grow(36 * (size_t)nf + n + m) && h->hll.grow(9 * (size_t)nl) &&
              h->z.grow(18 * ne1) && h->cb.grow(6 * ne1) && h->S.grow((size_t)n * n + n) &&
              h->depth.grow(ne1) && h->part.grow(grid(ne) + grid(nl + nf) + nf + grid(nl, 64)) &&
              // cleared by the scatter launch: g2o's _x starts zeroed, the scalars, the factorisation
              // status, the last-block counters of the unit kernels; and the device LM state's start
              st.zero(h->x, n + m) && st.zero(h->scal, 8) && st.zero(h->status, 1) && st.zero(h->counters, 2) &&
              st.add(h->lm, &lm_init, 1);
    if (ok && !st.items.empty()) {
        ok = upload_stage(st, h->h_stage, h->h_stage_cap, h->d_stage);
        t_pack = clk::now();
        if (ok && nblk)  // the Schur blocks' product lists, for every trial of the solve
            hipLaunchKernelGGL(k_ba_schur_pairs, dim3(nblk), dim3(64), 0, s, nf, h->pose_off.p, h->pose_fl.p,
                               h->blk_off.p, h->pairs.p, h->blk_cnt.p);
    }
    // the pinned result buffer too, before the solve: [poses | points | edge chi2 | depth flags]
    const size_t dl_bytes = sizeof(double) * (7 * (size_t)np + 3 * (size_t)nq + ne1) + ne1;
    if (ok && dl_bytes > h->h_dl_cap) {
        if (h->h_dl) hipHostFree(h->h_dl);
        h->h_dl = nullptr;
        h->h_dl_cap = 0;
        ok = hipHostMalloc(&h->h_dl, dl_bytes, hipHostMallocDefault) == hipSuccess;
        if (ok) h->h_dl_cap = dl_bytes;
    }
    if (agree_fail(!ok)) return orbgpu_fail(ORB_ERR_DEVICE, "BA device allocation / upload");
    // [Hpp | b_p | b_l] and [S | b_S] are contiguous: a sharded solve all-reduces [Hpp | b_p] and
    // [S | b_S] in one collective each
    double* const HPP = h->hpp.p;
    double* const BV = HPP + 36 * (size_t)nf;
    double* const SS = h->S.p;
    double* const BSV = SS + (size_t)n * n;

    const float dm = (float)std::sqrt(5.991), ds = (float)std::sqrt(7.815);  // src/Optimizer.cc:1957-1958
    const Huber2 hub{(double)dm, (double)ds, (float)((double)dm * (double)dm), (float)((double)ds * (double)ds)};
    // Cholesky + solves of the reduced camera system: the register-resident single-workgroup kernel
    // (k_ba_chol_mf2) for n <= 16 x kMfMaxNT = 288, the tile-row kernel (k_ba_chol_rows, one workgroup
    // per 16-row tile row) above that and for any n with ORBGPU_BA_CHOL=rows (tests/test_ba_gpu.py).
    const int NT = (n + 15) / 16;
    if (NT > kRowMaxNT) {
        agree_fail(true);
        return orbgpu_fail(ORB_ERR_ARG, "more than 682 free keyframes in the local window");
    }
    static const char* chol_env = getenv("ORBGPU_BA_CHOL");
    const bool use_rows = n > 0 && (n > 16 * kMfMaxNT || (chol_env && !strcmp(chol_env, "rows")) ||
                                    g_force_rows.load(std::memory_order_relaxed));
    const bool rows_lds = NT <= kRowLdsMaxNT;
    const size_t rows_lds_bytes =
        sizeof(double) * ((rows_lds ? (size_t)NT * 256 : 0) + 272 + 256 + 16 + 16 * (size_t)NT);
    if (use_rows) {
        const size_t nflag = 4 + (size_t)NT * NT;
        bool ok2 = h->lpub.grow((size_t)NT * NT * 256) && h->ypub.grow(16 * (size_t)NT) &&
                   (rows_lds || h->racc.grow((size_t)NT * NT * 256));
        if (ok2 && nflag > h->cflag.cap) {  // (re)allocated: epoch and every flag start at 0
            ok2 = h->cflag.grow(nflag) && hipMemsetAsync(h->cflag.p, 0, nflag * sizeof(unsigned), s) == hipSuccess;
        }
        if (agree_fail(!ok2)) return orbgpu_fail(ORB_ERR_DEVICE, "BA Cholesky buffers");
    }
    static bool attr_set = false;
    if (!attr_set) {
        hipFuncSetAttribute((const void*)k_ba_chol_mf2<kMf2TileWaves>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMf2Lds);
        hipFuncSetAttribute((const void*)k_ba_chol_rows<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)k_ba_chol_rows<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        (void)hipGetLastError();
        attr_set = true;
    }
    // ORBGPU_BA_TRACE: the first Cholesky of the process records its phase stamps (dump_chol_trace)
    static int trace_left = getenv("ORBGPU_BA_TRACE") ? 1 : 0;
    auto launch_chol = [&](const LmState* g, const PoseTail& pt, const double* hpp_add = nullptr,
                           const double* lam_add = nullptr) {
        if (use_rows) {
            if (rows_lds)
                hipLaunchKernelGGL(k_ba_chol_rows<true>, dim3(NT), dim3(kRowThreads), rows_lds_bytes, s, n, SS,
                                   BSV, h->x.p, h->status.p, h->lpub.p, h->ypub.p, h->cflag.p, h->racc.p, g,
                                   (int)kGateTrial);
            else
                hipLaunchKernelGGL(k_ba_chol_rows<false>, dim3(NT), dim3(kRowThreads), rows_lds_bytes, s, n, SS,
                                   BSV, h->x.p, h->status.p, h->lpub.p, h->ypub.p, h->cflag.p, h->racc.p, g,
                                   (int)kGateTrial);
            if (pt.pose) hipLaunchKernelGGL(k_u_pose_update, dim3(1), dim3(256), 0, s, pt, (const double*)h->x.p, g);
            return;
        }
        int64_t* tr = nullptr;
        if (trace_left && h->trace.grow(kTraceLen)) {
            hipMemsetAsync(h->trace.p, 0, kTraceLen * sizeof(int64_t), s);
            tr = h->trace.p;
        }
        hipLaunchKernelGGL((k_ba_chol_mf2<kMf2TileWaves>), dim3(1), dim3((kMf2TileWaves + 1) * 64), kMf2Lds, s, n,
                           SS, BSV, h->x.p, h->status.p, tr, g, (int)kGateTrial, hpp_add, lam_add);
        if (tr) {
            trace_left = 0;
            dump_chol_trace(tr, n, s);
        }
    };
    double* bl = BV + n;
    const size_t hpl_alt = 18 * ne1;  // the second half of the double-buffered Hpl
    // The device-driven LM loop: no host round trip per trial.  Sharded, its all-reduces are
    // stream-ordered RCCL calls between the unit's launches (every rank reduces to the same values and
    // takes the same LM decisions).  The host-driven loop serves ORBGPU_BA_HOST_LM=1 (tested in
    // tests/test_ba_gpu.py against the oracle).
    static const bool host_lm_env = getenv("ORBGPU_BA_HOST_LM") != nullptr;
    const bool dev_lm = !host_lm_env;
    const LmState* G = dev_lm ? h->lm.p : nullptr;            // gate source for every per-trial kernel
    const double* lam = dev_lm ? &h->lm.p->lambda : h->h_scal + 5;  // the trial's lambda (device / pinned)
    // ---- computeActiveErrors + activeRobustChi2 + buildSystem
    auto launch_build = [&](bool first) -> bool {
        if (ne)
            hipLaunchKernelGGL(k_ba_edges<true>, dim3(grid(ne)), dim3(kT), 0, s, ne, h->edges.p, h->cams.p, h->pose.p,
                               h->point.p, h->pose_h.p, hub, h->err.p, h->rho0.p, h->ecl.p, h->hpl.p, h->ecp.p, G,
                               (int)kGateBuild);
        if (nl)
            hipLaunchKernelGGL(k_ba_reduce_land, dim3(grid(nl)), dim3(kT), 0, s, nl, h->land_off.p, h->land_edge.p,
                               h->ecl.p, h->hll.p, bl, G, (int)kGateBuild);
        if (nf) {
            hipLaunchKernelGGL(k_ba_reduce_pose, dim3(nf), dim3(64), 0, s, h->pose_off.p, h->pose_fl.p, h->ecp.p,
                               HPP, BV, G, (int)kGateBuild);
            if (!dev_reduce(h, HPP, 36 * (size_t)nf, ORB_BA_SUM) || !dev_reduce(h, BV, n, ORB_BA_SUM))
                return false;
        }
        if (first)  // (on the device path the gate limits it to iteration 0)
            hipLaunchKernelGGL(k_ba_maxdiag, dim3(1), dim3(kT), 0, s, nf, nl, HPP, h->hll.p, h->scal.p + 3, G,
                               (int)kGateBuild0);
        hipLaunchKernelGGL(k_ba_sums, dim3(1), dim3(1024), 0, s, ne, h->rho0.p, primary ? 0 : n, n + m, lam,
                           (const double*)nullptr, BV, h->status.p, h->scal.p, dev_lm || dist ? nullptr : h->h_scal,
                           G, (int)kGateBuild);
        return true;
    };
    // ---- setLambda + BlockSolver::solve + SparseOptimizer::update + computeActiveErrors + computeScale
    auto launch_trial = [&]() -> bool {
        if (nfe)
            hipLaunchKernelGGL(k_ba_schur_edges, dim3(grid(nfe)), dim3(kT), 0, s, nfe, lam, h->landf_edge.p, h->fland.p,
                               h->hll.p, bl, h->hpl.p, hpl_alt, h->z.p, h->cb.p, G, (int)kGateTrial);
        if (nf) {
            hipLaunchKernelGGL(k_ba_schur_blocks, dim3(nblk), dim3(64), 0, s, n, nf, lam, primary ? 1 : 0, h->blk_off.p,
                               h->pairs.p, h->blk_cnt.p, h->z.p, h->hpl.p, HPP, SS, G, (int)kGateTrial);
            hipLaunchKernelGGL(k_ba_schur_rhs, dim3(nf), dim3(64), 0, s, h->pose_off.p, h->pose_fl.p, h->cb.p, BV,
                               primary ? 1 : 0, BSV, G, (int)kGateTrial);
            if (!dev_reduce(h, SS, (size_t)n * n, ORB_BA_SUM) || !dev_reduce(h, BSV, n, ORB_BA_SUM))
                return false;
            launch_chol(G, PoseTail{});
        } else if (!dev_lm) {
            hipMemsetAsync(h->status.p, 0, sizeof(int32_t), s);
        }
        if (nl)
            hipLaunchKernelGGL(k_ba_backsub, dim3(grid(nl)), dim3(kT), 0, s, nl, n, lam, h->landf_off.p, h->landf_edge.p,
                               h->landf_row.p, h->hpl.p, bl, h->hll.p, h->x.p, G, (int)kGateTrial);
        hipLaunchKernelGGL(k_ba_update, dim3(grid(nf + nl)), dim3(kT), 0, s, nf, nl, n, h->free_pose.p, h->land_point.p,
                           h->x.p, h->pose.p, h->pose_bak.p, h->point.p, h->point_bak.p, G, (int)kGateTrial);
        if (ne)
            hipLaunchKernelGGL(k_ba_edges<false>, dim3(grid(ne)), dim3(kT), 0, s, ne, h->edges.p, h->cams.p, h->pose.p,
                               h->point.p, h->pose_h.p, hub, h->err.p, h->rho0.p, h->ecl.p, h->hpl.p, h->ecp.p, G,
                               (int)kGateTrial);
        hipLaunchKernelGGL(k_ba_sums, dim3(1), dim3(1024), 0, s, ne, h->rho0.p, primary ? 0 : n, n + m, lam,
                           (const double*)h->x.p, BV, h->status.p, h->scal.p,
                           dev_lm || dist ? nullptr : h->h_scal, G, (int)kGateTrial);
        return true;
    };
    hipStream_t rs = s;  // the stream of the restore and the results (see the device-driven loop)
    auto launch_restore = [&]() {
        hipLaunchKernelGGL(k_ba_restore, dim3(grid(nf + nl)), dim3(kT), 0, rs, nf, nl, h->free_pose.p, h->land_point.p,
                           h->pose.p, h->pose_bak.p, h->point.p, h->point_bak.p, G, (int)kGateRestore);
    };
    // the host loop reads [0] chi2, [1] computeScale, [2] status, [3] max diag (reduced over the ranks)
    auto read_scalars = [&]() -> bool {
        if (dist) {
            if (!dev_reduce(h, h->scal.p, 2, ORB_BA_SUM) || !dev_reduce(h, h->scal.p + 3, 1, ORB_BA_MAX)) return false;
            hipMemcpyAsync(h->h_scal, h->scal.p, 4 * sizeof(double), hipMemcpyDeviceToHost, s);
        }
        return hipStreamSynchronize(s) == hipSuccess;
    };

    if (dev_lm) {
        // One unit per trial: the build's reductions and controller (gated to the start of an
        // iteration; the linearisation itself comes from the accepted trial, or from the one build
        // launch before the first unit), the trial, the trial controller, restore on reject.  The host
        // keeps one unit queued behind the running one and reads the pinned progress after each
        // unit's event; once the solve is done the queued unit is a run of no-op launches.
        // (the state's start, the counters and the status went up with the inputs)
        memset(h->h_prog, 0, sizeof(LmProgress));
        *h->h_stop = 0;
        if (dist) {  // the partial buffers; the scalar slots must start at zero (the ranks' max diag slots)
            const size_t nd = 2 * (36 * (size_t)nf + n + 4 + h->world) + (size_t)n * n + n + 2 * 4;
            const bool okp = h->dpart.grow(nd) && hipMemsetAsync(h->dpart.p, 0, nd * sizeof(double), s) == hipSuccess;
            if (agree_fail(!okp)) return orbgpu_fail(ORB_ERR_DEVICE, "BA sharded buffers");
        }
        const int nparts = (int)grid(ne), nparts2 = (int)grid(nl + nf);  // partials: edge blocks, vertex blocks
        double* const pmax = h->part.p + nparts + nparts2;  // k_u_reduce_build's per-block max |diag|
        LmState* L = h->lm.p;
        // one unit = 6 launches: reductions (+ chi2, max diag, build controller), Schur edges, Schur
        // blocks + rhs, Cholesky + solves, back-substitution + update, errors and linearisation at the
        // new estimate (+ chi2, computeScale, trial controller)
        // ORBGPU_BA_TRIAL_LIN=1: every trial also linearises at its new estimate, so an accepted
        // trial leaves nothing for the next build (default off: on MI355X the trial then costs what
        // the build launch saves, C5 1.590 vs 1.582 ms per solve)
        static const char* tl_env = getenv("ORBGPU_BA_TRIAL_LIN");
        const bool trial_lin = tl_env && !strcmp(tl_env, "1");
        // The trial's back-substitution, update and error pass in one launch instead of two (round 6):
        // k_u_land_trial moves the poses (each block in LDS, the last one in memory) and the landmarks,
        // then evaluates the landmarks' edges.  Beyond kT free poses (tile-row Cholesky sizes)
        // k_u_pose_update moves the poses first.  ORBGPU_BA_FUSED_TRIAL=0: k_u_backsub_update +
        // k_u_edges_trial.
        static const char* ft_env = getenv("ORBGPU_BA_FUSED_TRIAL");
        const bool fused = !trial_lin && !(ft_env && !strcmp(ft_env, "0"));
        const int pose_mode = nf == 0 ? 0 : nf <= kT ? 1 : 2;
        const PoseTail pt_unit = PoseTail{h->free_pose.p, h->pose.p, h->pose_bak.p, BV, lam, h->scal.p + 8, nf,
                                          primary ? 1 : 0};
        auto launch_edges_build = [&]() {
            hipLaunchKernelGGL(k_u_edges_build, dim3(nparts), dim3(kT), 0, s, ne, h->edges.p, h->cams.p, h->pose.p,
                               h->point.p, h->pose_h.p, hub, h->err.p, h->rho0.p, h->ecl.p, h->hpl.p, h->ecp.p,
                               h->part.p, (const LmState*)L);
        };
        if (trial_lin) launch_edges_build();
        // sharded: the partials [Hpp | b_p | build scalars] (chi2, slots of the ranks' max diag at
        // 4 + r: one payload, one collective), their sums, [S | b_S], the trial scalars (chi2,
        // computeScale, stop) and their sums
        const int nsb = 4 + h->world;
        const size_t nhb = 36 * (size_t)nf + n;
        double* const p_hb = dist ? h->dpart.p : nullptr;
        double* const p_scb = dist ? p_hb + nhb : nullptr;
        double* const r_hb = dist ? p_scb + nsb : nullptr;
        double* const r_scb = dist ? r_hb + nhb : nullptr;
        double* const p_sb = dist ? r_scb + nsb : nullptr;
        double* const p_sct = dist ? p_sb + (size_t)n * n + n : nullptr;
        double* const r_sct = dist ? p_sct + 4 : nullptr;
        bool coll_ok = true;
        // The fast unit (one process, the single-workgroup Cholesky, the fused trial): 4 launches per trial
        // instead of 6 -- k_u_land_build (linearisation, Hll / b_l, Z and cb), k_u_schur2 (S without its
        // diagonal Hpp + lambda I, b_S, Hpp / b_p), the Cholesky (adding Hpp + lambda I as it loads S),
        // k_u_land_trial.  The solve's first build (lambda from max diag) runs once before the units,
        // with the build controller.  ORBGPU_BA_FAST_UNIT=0: the 6-launch unit.
        static const char* fu_env = getenv("ORBGPU_BA_FAST_UNIT");
        const bool fast = fused && !dist && !use_rows && !(fu_env && !strcmp(fu_env, "0"));
        auto launch_reduce_build = [&]() {
            hipLaunchKernelGGL(k_u_reduce_build, dim3(nf + grid(nl, 64)), dim3(64), 0, s, nf, nl, h->pose_off.p,
                               h->pose_fl.p, h->ecp.p, HPP, BV, h->land_off.p, h->land_edge.p, h->ecl.p, h->hll.p, bl,
                               h->part.p, nparts, h->counters.p, h->scal.p, L, 0, (double*)nullptr, h->rank, pmax);
        };
        if (fast) {  // the solve's first build (gated to phase 0, i.e. before any unit has run)
            launch_edges_build();
            launch_reduce_build();
        }
        auto unit_launches = [&]() {
            if (fast) {
                hipLaunchKernelGGL(k_u_land_build, dim3(grid((size_t)nl * kLB)), dim3(kT), 0, s, nl, lam, h->land_off.p,
                                   h->land_edge.p, h->edges.p, h->cams.p, h->pose.p, h->point.p, h->pose_h.p, hub,
                                   h->err.p, h->rho0.p, h->hpl.p, h->ecp.p, h->hll.p, bl, h->z.p, h->cb.p,
                                   (const LmState*)L);
                if (nf) {
                    hipLaunchKernelGGL(k_u_schur2, dim3(nblk + 2 * nf), dim3(64), 0, s, n, nf, nblk, lam, h->blk_off.p,
                                       h->pairs.p, h->blk_cnt.p, h->pose_off.p, h->pose_fl.p, h->z.p, h->hpl.p, h->ecp.p,
                                       HPP, BV, SS, h->cb.p, BSV, (const LmState*)L);
                    launch_chol((const LmState*)L, PoseTail{}, HPP, lam);
                }
                hipLaunchKernelGGL(k_u_land_trial, dim3(grid(nl)), dim3(kLT), 0, s, nl, n, lam, h->landf_off.p,
                                   h->landf_edge.p, h->landf_row.p, h->hpl.p, hpl_alt, bl, h->hll.p, h->x.p,
                                   h->land_point.p, h->point.p, h->point_bak.p, h->land_off.p, h->land_edge.p,
                                   h->edges.p, h->cams.p, h->pose.p, h->pose_h.p, pt_unit, pose_mode, hub, h->err.p,
                                   h->rho0.p, h->part.p, h->part.p + nparts, h->counters.p + 1, h->status.p, h->scal.p,
                                   L, h->h_prog, 0, (double*)nullptr, (const volatile int32_t*)h->h_stop, 1);
                return;
            }
            if (!trial_lin) launch_edges_build();
            hipLaunchKernelGGL(k_u_reduce_build, dim3(nf + grid(nl, 64)), dim3(64), 0, s, nf, nl, h->pose_off.p,
                               h->pose_fl.p, h->ecp.p, dist ? p_hb : HPP, dist ? p_hb + 36 * (size_t)nf : BV,
                               h->land_off.p, h->land_edge.p, h->ecl.p, h->hll.p, bl, h->part.p, nparts, h->counters.p,
                               h->scal.p, L, dist ? 1 : 0, p_scb, h->rank, pmax);
            if (dist) {  // one collective for [Hpp | b_p | build scalars], then the sums into place
                coll_ok = coll_ok && dev_reduce2(h, p_hb, r_hb, nhb + nsb, ORB_BA_SUM) &&
                          hipMemcpyAsync(HPP, r_hb, nhb * sizeof(double), hipMemcpyDeviceToDevice, s) == hipSuccess;
                hipLaunchKernelGGL(k_lm_build_ctl, dim3(1), dim3(64), 0, s, nf, (const double*)HPP, (const double*)r_scb,
                                   h->world, h->scal.p, L);
            }
            if (nfe)
                hipLaunchKernelGGL(k_ba_schur_edges, dim3(grid(nfe)), dim3(kT), 0, s, nfe, lam, h->landf_edge.p,
                                   h->fland.p, h->hll.p, bl, h->hpl.p, hpl_alt, h->z.p, h->cb.p, (const LmState*)L,
                                   (int)kGateTrial);
            if (nf) {
                hipLaunchKernelGGL(k_u_schur, dim3(nblk + nf), dim3(64), 0, s, n, nf, nblk, lam, h->blk_off.p,
                                   h->pairs.p, h->blk_cnt.p, h->pose_off.p, h->pose_fl.p, h->z.p, h->hpl.p, hpl_alt, HPP,
                                   dist ? p_sb : SS, h->cb.p, BV, dist ? p_sb + (size_t)n * n : BSV, (const LmState*)L,
                                   primary ? 1 : 0);
                if (dist) coll_ok = coll_ok && dev_reduce2(h, p_sb, SS, (size_t)n * n + n, ORB_BA_SUM);
                launch_chol((const LmState*)L, fused && pose_mode == 2 ? pt_unit : PoseTail{});
            }
            if (fused) {
                hipLaunchKernelGGL(k_u_land_trial, dim3(grid(nl)), dim3(kLT), 0, s, nl, n, lam, h->landf_off.p,
                                   h->landf_edge.p, h->landf_row.p, h->hpl.p, hpl_alt, bl, h->hll.p, h->x.p,
                                   h->land_point.p, h->point.p, h->point_bak.p, h->land_off.p, h->land_edge.p,
                                   h->edges.p, h->cams.p, h->pose.p, h->pose_h.p, pt_unit, pose_mode, hub, h->err.p,
                                   h->rho0.p, h->part.p, h->part.p + nparts, h->counters.p + 1, h->status.p, h->scal.p,
                                   L, h->h_prog, dist ? 1 : 0, p_sct,
                                   (const volatile int32_t*)h->h_stop, 0);
            } else {
            hipLaunchKernelGGL(k_u_backsub_update, dim3(nparts2), dim3(kT), 0, s, nl, nf, n, lam, h->landf_off.p,
                               h->landf_edge.p, h->landf_row.p, h->hpl.p, hpl_alt, bl, h->hll.p, h->x.p, BV,
                               h->free_pose.p, h->land_point.p, h->pose.p, h->pose_bak.p, h->point.p, h->point_bak.p,
                               h->part.p + nparts, (const LmState*)L, primary ? 1 : 0);
            hipLaunchKernelGGL(trial_lin ? k_u_edges_trial<true> : k_u_edges_trial<false>, dim3(nparts), dim3(kT), 0, s,
                               ne, h->edges.p, h->cams.p, h->pose.p, h->point.p, h->pose_h.p, hub, h->err.p, h->rho0.p,
                               h->ecl.p, h->hpl.p, hpl_alt, h->ecp.p, h->part.p, h->counters.p + 1, h->part.p + nparts,
                               nparts2, h->status.p, h->scal.p, L, h->h_prog, dist ? 1 : 0, p_sct,
                               (const volatile int32_t*)h->h_stop);
            }
            if (dist) {
                coll_ok = coll_ok && dev_reduce2(h, p_sct, r_sct, 4, ORB_BA_SUM);
                hipLaunchKernelGGL(trial_lin ? k_lm_trial_ctl<true> : k_lm_trial_ctl<false>, dim3(1), dim3(64), 0, s,
                                   (const double*)r_sct, (const int32_t*)h->status.p, h->scal.p, L, h->h_prog);
            }
        };
        // Every unit launches the same kernels with the same arguments (the device state gates them),
        // so the unit is captured once as a graph and replayed: one graph launch instead of 7 kernel
        // launches per trial.  The capture is kept while the arguments (sizes, buffers) are unchanged.
        auto dbits = [](double v) { uintptr_t u; memcpy(&u, &v, sizeof(u)); return u; };
        bool use_graph = !trace_left && !dist;  // (the trace dump synchronises the stream: not capturable;
                                                // sharded, the collectives stay direct calls)
        // four units per graph launch: each launch boundary costs ~13 us on the device, a gated no-op
        // unit behind the last trial about as much (round 6, the 4-launch fast unit, C5 mono solve:
        // 2 units 1.410 / 1.436 ms, 3: 1.397 / 1.377, 4: 1.368 / 1.381, 8: 1.356 / 1.360; 4 keeps the
        // waste of a 9-12-trial solve small, profiles/r06/ba_units_ab_r06.txt)
        // With a stop flag, one unit per launch: the host polls the flag after every launch, so at
        // most two trials (the running and the queued unit) follow a raised flag, as before.
        static const char* upl_env = getenv("ORBGPU_BA_UNITS");  // (A/B of the units per graph launch)
        const int upl_default = upl_env ? std::max(1, std::min(16, atoi(upl_env))) : 4;
        const int units_per_launch = (opt->stop_flag || opt->stop_flag_bool) ? 1 : upl_default;
        if (use_graph) {
            const std::vector<uintptr_t> key = {
                (uintptr_t)s, (uintptr_t)n, (uintptr_t)m, (uintptr_t)ne, (uintptr_t)nf, (uintptr_t)nl, (uintptr_t)nfe,
                (uintptr_t)nblk, (uintptr_t)nparts, (uintptr_t)units_per_launch, dbits(hub.delta_mono), dbits(hub.delta_stereo), (uintptr_t)bl,
                (uintptr_t)h->edges.p, (uintptr_t)h->cams.p, (uintptr_t)h->pose.p, (uintptr_t)h->point.p,
                (uintptr_t)h->pose_h.p, (uintptr_t)h->err.p, (uintptr_t)h->rho0.p, (uintptr_t)h->ecl.p,
                (uintptr_t)h->hpl.p, (uintptr_t)h->ecp.p, (uintptr_t)h->part.p, (uintptr_t)h->pose_off.p,
                (uintptr_t)h->pose_fl.p, (uintptr_t)HPP, (uintptr_t)BV, (uintptr_t)h->land_off.p,
                (uintptr_t)h->land_edge.p, (uintptr_t)h->hll.p, (uintptr_t)h->counters.p, (uintptr_t)h->scal.p,
                (uintptr_t)L, (uintptr_t)lam, (uintptr_t)h->landf_edge.p, (uintptr_t)h->fland.p, (uintptr_t)h->z.p,
                (uintptr_t)h->cb.p, (uintptr_t)SS, (uintptr_t)h->blk_off.p, (uintptr_t)h->pairs.p,
                (uintptr_t)h->blk_cnt.p, (uintptr_t)BSV,
                (uintptr_t)h->x.p, (uintptr_t)h->status.p, (uintptr_t)h->landf_off.p, (uintptr_t)h->landf_row.p, (uintptr_t)h->free_pose.p,
                (uintptr_t)h->land_point.p, (uintptr_t)h->pose_bak.p, (uintptr_t)h->point_bak.p, (uintptr_t)h->h_prog,
                (uintptr_t)use_rows, (uintptr_t)trial_lin, (uintptr_t)fused, (uintptr_t)fast, (uintptr_t)h->lpub.p, (uintptr_t)h->ypub.p, (uintptr_t)h->cflag.p,
                (uintptr_t)h->racc.p};
            if (!h->unit_exec || key != h->unit_key) {
                if (h->unit_exec) { hipGraphExecDestroy(h->unit_exec); h->unit_exec = nullptr; }
                if (h->unit_graph) { hipGraphDestroy(h->unit_graph); h->unit_graph = nullptr; }
                bool ok = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess;
                if (ok) {
                    for (int r = 0; r < units_per_launch; ++r) unit_launches();
                    ok = hipStreamEndCapture(s, &h->unit_graph) == hipSuccess && h->unit_graph &&
                         hipGraphInstantiate(&h->unit_exec, h->unit_graph, nullptr, nullptr, 0) == hipSuccess;
                }
                if (!ok) {  // fall back to direct launches
                    (void)hipGetLastError();
                    if (h->unit_graph) { hipGraphDestroy(h->unit_graph); h->unit_graph = nullptr; }
                    h->unit_exec = nullptr;
                    use_graph = false;
                } else {
                    h->unit_key = key;
                }
            }
        }
        auto unit = [&](int u) -> bool {
            if (dist) *h->h_stop = stop_requested(opt) ? 1 : 0;  // read by the trial's last block
            if (use_graph) {
                if (hipGraphLaunch(h->unit_exec, s) != hipSuccess) return false;
            } else {
                for (int r = 0; r < units_per_launch; ++r) unit_launches();
            }
            return hipEventRecord(h->unit_ev[u & 1], s) == hipSuccess;
        };
        const int max_units = (std::max(0, opt->iterations) * 10 + units_per_launch - 1) / units_per_launch;
        if (max_units > 0) {
            if (!unit(0)) return orbgpu_fail(ORB_ERR_DEVICE, "BA launch failed");
            for (int u = 1;; ++u) {
                const bool more = u < max_units;
                if (more && !unit(u)) return orbgpu_fail(ORB_ERR_DEVICE, "BA launch failed");
                if (hipEventSynchronize(h->unit_ev[(u - 1) & 1]) != hipSuccess)
                    return orbgpu_fail(ORB_ERR_DEVICE, "BA device error");
                if (trace && n_unit_t < 32) unit_t[n_unit_t++] = us(t_pack, clk::now());
                if (h->h_prog->done && more) {
                    // the solve ended inside unit u-1 and unit u, queued behind it, is a run of gated
                    // no-op launches: the restore and the results go on the tail stream beside it
                    if (hipStreamWaitEvent(h->tail, h->unit_ev[(u - 1) & 1], 0) != hipSuccess)
                        return orbgpu_fail(ORB_ERR_DEVICE, "BA device error");
                    rs = h->tail;
                }
                if (!coll_ok) return orbgpu_fail(ORB_ERR_DEVICE, "BA collective failed");
                if (h->h_prog->done || !more) break;
                // (the queued unit is live: the tail stays on s; sharded, the ranks agree on the stop on
                // the device instead, so that every rank launches the same collectives)
                if (!dist && stop_requested(opt)) break;
            }
        }
        launch_restore();  // undo a rejected last trial (gated on the device state)
        // (the progress record is read after the results' synchronisation below)
    } else {
        double lambda = 0, ni = 2;
        int nBad = 0, it = 0;
        for (; it < opt->iterations && !stop(); ++it) {
            if (!launch_build(it == 0) || !read_scalars()) return orbgpu_fail(ORB_ERR_DEVICE, "BA build failed");
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
                h->h_scal[5] = lambda;  // read by the trial kernels (the stream is idle here)
                if (!launch_trial() || !read_scalars()) return orbgpu_fail(ORB_ERR_DEVICE, "BA trial failed");
                res->trials++;
                double tempChi = h->h_scal[0];
                if (h->h_scal[2] != 0.0) tempChi = std::numeric_limits<double>::max();  // not positive definite
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
                    launch_restore();
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
    }
    res->stopped = stop() ? 1 : 0;
    t_solve = clk::now();
    // results through the pinned buffer sized before the solve, written by one kernel (edge chi2 / depth
    // flags, the poses and points): no device-to-host copies
    double* const dpose = reinterpret_cast<double*>(h->h_dl);
    double* const pts = dpose + 7 * (size_t)np;
    double* const lchi = pts + 3 * (size_t)nq;
    uint8_t* const ldep = reinterpret_cast<uint8_t*>(lchi + ne1);
    {
        const int nt = std::max(std::max(7 * np, 3 * nq), ne);
        if (nt > 0)
            hipLaunchKernelGGL(k_ba_results, dim3(grid(nt)), dim3(kT), 0, rs, np, nq, ne, h->edges.p, h->pose.p,
                               h->point.p, h->err.p, dpose, pts, lchi, ldep);
    }
    if (hipStreamSynchronize(rs) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "BA device error");
    if (dev_lm) {
        const LmProgress pg = *h->h_prog;
        res->iterations = pg.it;
        res->trials = pg.trials;
        res->terminated = pg.terminated;
        res->initial_chi2 = pg.initial_chi;
        res->final_chi2 = pg.final_chi;
        res->lambda = pg.lambda;
    }
    memcpy(pr->pose, dpose, sizeof(double) * 7 * (size_t)np);
    if (!dist) {
        memcpy(pr->point, pts, sizeof(double) * 3 * (size_t)nq);
        for (int e = 0; e < ne; ++e) {
            if (edge_chi2) edge_chi2[e] = lchi[e];
            if (edge_depth_ok) edge_depth_ok[e] = ldep[e];
        }
        if (trace)
            fprintf(stderr, "[ba] structure %.1f us (order %.1f, csr %.1f, pairs %.1f, rest %.1f), pack %.1f us, upload+LM %.1f us, "
                            "results %.1f us, it %d trials %d\n",
                    us(t_in, t_struct), us(t_in, t_order), us(t_order, t_csr), us(t_csr, t_pairs), us(t_pairs, t_struct),
                    us(t_struct, t_pack), us(t_pack, t_solve), us(t_solve, clk::now()), res->iterations, res->trials);
        if (trace && n_unit_t) {
            fprintf(stderr, "[ba] launches seen done at");
            for (int i = 0; i < n_unit_t; ++i) fprintf(stderr, " %.1f", unit_t[i]);
            fprintf(stderr, " us\n");
        }
        return ORB_OK;
    }
    // gather: each rank contributes its landmarks (rank 0 also the points without edges) and its
    // edges' chi2 / depth flags; one SUM all-reduce of the zero-padded arrays
    const size_t nred = 3 * (size_t)nq + 2 * (size_t)ne_all;
    std::vector<double> contrib(nred, 0.0);
    for (int q = 0; q < nq; ++q)
        if (point_l[q] >= 0 || (primary && qdeg[q] == 0))
            for (int k = 0; k < 3; ++k) contrib[3 * (size_t)q + k] = pts[3 * (size_t)q + k];
    for (int e = 0; e < ne; ++e) {
        const int ge = lmap.empty() ? e : lmap[e];  // (one rank: the structure keeps the edge order)
        contrib[3 * (size_t)nq + ge] = lchi[e];
        contrib[3 * (size_t)nq + ne_all + ge] = ldep[e] ? 1.0 : 0.0;
    }
    if (!h->red_buf.grow(nred) ||
        hipMemcpyAsync(h->red_buf.p, contrib.data(), nred * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
        !dev_reduce(h, h->red_buf.p, nred, ORB_BA_SUM) ||
        hipMemcpyAsync(contrib.data(), h->red_buf.p, nred * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "BA result all-reduce failed");
    memcpy(pr->point, contrib.data(), sizeof(double) * 3 * (size_t)nq);
    for (int e = 0; e < ne_all; ++e) {
        if (edge_chi2) edge_chi2[e] = contrib[3 * (size_t)nq + e];
        if (edge_depth_ok) edge_depth_ok[e] = contrib[3 * (size_t)nq + ne_all + e] != 0.0;
    }
    return ORB_OK;
}

}  // extern "C"
