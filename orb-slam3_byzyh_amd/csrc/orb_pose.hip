// MI355X Optimizer::PoseOptimization (reference src/Optimizer.cc:55-415): tracking's motion-only
// bundle adjustment, batched over frames, FP64.
//
// One 256-thread workgroup per frame runs the whole optimisation: 4 rounds of g2o's optimize(10)
// (OptimizationAlgorithmLevenberg::solve, core/optimization_algorithm_levenberg.cpp:61-194, with
// LinearSolverDense on the single 6x6 pose block), each round restarting from the frame's pose and
// followed by the chi2 re-classification of every edge.  Per LM trial:
//   solve  thread 0 factors H + lambda I (LDL^T), exponentiates and applies the step
//   pass   threads evaluate their active (level-0) edges at the trial pose -- error, Huber weight,
//          Jacobian (EdgeSE3ProjectXYZOnlyPose: -projectJac * SE3deriv;
//          EdgeStereoSE3ProjectXYZOnlyPose: types_six_dof_expmap.cpp:375-404) -- and keep every
//          edge's chi2 (g2o classifies the active edges on the error of the LAST evaluated state,
//          even a rejected one); the 21 + 6 entries of J^T W J / -J^T W e and the robust chi2 are
//          reduced in a fixed order (a transposed butterfly in each wave, then the waves in order)
//   decide thread 0 runs g2o's accept / reject rule, restores the pose on a rejection, and on an
//          acceptance takes the pass's sums as the next iteration's system (g2o rebuilds it at the
//          accepted state), then solves the next trial
// No MFMA: a 6x6 system per frame; the work is the per-edge linearisation and reductions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

// parity bar: 1e-6 pose RMSE (like the local BA): products may contract into FMAs
#pragma clang fp contract(fast)
#include "orb_se3.h"

namespace {

#ifndef ORB_POSE_THREADS
#define ORB_POSE_THREADS 256
#endif
constexpr int kPT = ORB_POSE_THREADS;  // threads per frame
constexpr int kPW = kPT / 64;          // waves
constexpr int kCap = 2048;             // edges per frame held in LDS (beyond: read from memory every pass)
constexpr int kPair = 2 * kPT;         // edge positions per pair step of the pass
constexpr int kDualMinFrames = 512;    // batches from this size run two frames per CU (launch site)
static_assert(kPT % 64 == 0 && kCap % kPair == 0 && kPW <= 32, "pose workgroup shape");

static_assert(sizeof(orb_pose_edge_t) == 56, "pose edge layout");

struct EdgeEval {
    double er[3];
    double chi2;
    int stereo;
};

// error of edge E at pose T (EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose::computeError)
__device__ __forceinline__ void pose_edge_error(const orb_pose_edge_t& E, const double T[7], const orb_ba_camera_t& c,
                                                double Xc[3], EdgeEval& ev) {
    const double q[4] = {T[3], T[4], T[5], T[6]};
    qrotate(q, E.xw, Xc);
    Xc[0] += T[0]; Xc[1] += T[1]; Xc[2] += T[2];
    if (!E.stereo) {  // Pinhole::project(Vector3d)
        ev.er[0] = E.obs[0] - ((double)c.fx * Xc[0] / Xc[2] + (double)c.cx);
        ev.er[1] = E.obs[1] - ((double)c.fy * Xc[1] / Xc[2] + (double)c.cy);
        ev.er[2] = 0.0;
    } else {  // cam_project: float invz, double fx, fy, cx, cy, bf members
        const float invz = (float)(1.0f / Xc[2]);
        const double u = Xc[0] * invz * (double)c.fx + (double)c.cx;
        const double v = Xc[1] * invz * (double)c.fy + (double)c.cy;
        ev.er[0] = E.obs[0] - u;
        ev.er[1] = E.obs[1] - v;
        ev.er[2] = E.obs[2] - (u - (double)c.bf * invz);
    }
    const double info = (double)E.inv_sigma2;
    ev.chi2 = ev.er[0] * info * ev.er[0] + ev.er[1] * info * ev.er[1];
    if (E.stereo) ev.chi2 += ev.er[2] * info * ev.er[2];
    ev.stereo = E.stereo;
}

__device__ __forceinline__ double robust_rho(const EdgeEval& ev, bool robust, Huber2 hub, double& rho1) {
    if (!robust) {
        rho1 = 1.0;
        return ev.chi2;
    }
    double rho0;
    if (ev.stereo) huber(ev.chi2, hub.delta_stereo, hub.dsqr_stereo, rho0, rho1);
    else huber(ev.chi2, hub.delta_mono, hub.dsqr_mono, rho0, rho1);
    return rho0;
}

// Partner exchanges of a double for the transposed butterfly below.  Pairs differ in lane bit M:
// M = 32 ds_bpermute, 16 ds_swizzle (xor 16 in each half), 8 DPP row_mirror (i <-> 15 - i), 4 DPP
// row_half_mirror (i <-> 7 - i), 2 / 1 DPP quad_perm; only the last four stay in the VALU.
template <int M>
__device__ __forceinline__ double xchg(double v) {
    if constexpr (M == 32) {
        return __shfl_xor(v, 32, 64);
    } else {
        const int2 h = __builtin_bit_cast(int2, v);
        int2 r;
        if constexpr (M == 16) {
            r.x = __builtin_amdgcn_ds_swizzle(h.x, 0x401F);
            r.y = __builtin_amdgcn_ds_swizzle(h.y, 0x401F);
        } else {
            constexpr int ctl = M == 8 ? 0x140 : M == 4 ? 0x141 : M == 2 ? 0x4E : 0xB1;
            r.x = __builtin_amdgcn_update_dpp(0, h.x, ctl, 0xF, 0xF, false);
            r.y = __builtin_amdgcn_update_dpp(0, h.y, ctl, 0xF, 0xF, false);
        }
        return __builtin_bit_cast(double, r);
    }
}
// One transposed butterfly step: lanes with bit M set keep values [C, 2C) and send [0, C), their
// partners the reverse, so the partner's half arrives with one exchange per kept value.  Partners
// hold the same value set before each step (they agree in every lane bit above M).
template <int C, int M>
__device__ __forceinline__ void tb_step(double (&v)[32], int lane) {
    if constexpr (M == 32 || M == 16) {
        // v_permlane32_swap / v_permlane16_swap (gfx950): the upper half-wave (odd 16-lane row) of
        // v[i] trades places with the lower half (even row) of v[i + C], so each lane then holds its
        // kept value in one register and its partner's sent value in the other: one add, no LDS
        // (the sum is keep + recv in either order, the same double)
#pragma unroll
        for (int i = 0; i < C; ++i) {
            int2 a = __builtin_bit_cast(int2, v[i]), b = __builtin_bit_cast(int2, v[i + C]);
            if constexpr (M == 32) {
                const auto rx = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
                const auto ry = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
                a.x = rx[0]; b.x = rx[1]; a.y = ry[0]; b.y = ry[1];
            } else {
                const auto rx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
                const auto ry = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
                a.x = rx[0]; b.x = rx[1]; a.y = ry[0]; b.y = ry[1];
            }
            v[i] = __builtin_bit_cast(double, a) + __builtin_bit_cast(double, b);
        }
    } else {
        const bool up = (lane & M) != 0;
#pragma unroll
        for (int i = 0; i < C; ++i) {
            const double send = up ? v[i] : v[i + C];
            const double keep = up ? v[i + C] : v[i];
            v[i] = keep + xchg<M>(send);
        }
    }
}
// Wave sums of 32 per-lane doubles in 32 exchanges (16 + 8 + 4 + 2 + 1, then the pair) instead of
// 32 x 6 shuffles: afterwards v[0] of lanes 2k and 2k + 1 is the wave's sum of value k, also stored
// to part[wave * 32 + k].  The workgroup total of value k is ((p0 + p1) + p2) + p3 over the waves.
__device__ __forceinline__ void wave_partials32(double (&v)[32], double* part) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    tb_step<16, 32>(v, lane);
    tb_step<8, 16>(v, lane);
    tb_step<4, 8>(v, lane);
    tb_step<2, 4>(v, lane);
    tb_step<1, 2>(v, lane);
    v[0] += xchg<1>(v[0]);
    if (!(lane & 1)) part[wv * 32 + (lane >> 1)] = v[0];
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// 1 / d from v_rcp_f64 and two Newton steps (within an ulp; d finite and nonzero): five dependent
// operations instead of the IEEE division sequence, on thread 0's serial chain
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

// 1 / sqrt(x) from v_rsq_f64 and two Newton steps (x > 0 finite)
__device__ __forceinline__ double rsq_nr(double x) {
    double r = __builtin_amdgcn_rsq(x);
    double h = 0.5 * x;
    r = r * fma(-h * r, r, 1.5);
    return r * fma(-h * r, r, 1.5);
}

// (H + lambda I) x = b for the 6x6 symmetric H given as its upper triangle row by row
// (LinearSolverDense: Eigen::LDLT; the same solution up to rounding).  As 3x3 blocks [A B; B^T C]:
// A^-1 and the Schur complement's inverse by cofactors (no pivot chain: the cofactors are independent
// products, one reciprocal per block), so the serial depth is about half of a 6-pivot LDL^T.  Returns
// LDLT::isPositive's answer by Sylvester's criterion: the leading minors of A, and those of the Schur
// complement (det of H's leading k x k for k > 3 is det A times them), are all positive.
__device__ __forceinline__ bool inv3sym(const double (&a)[6], double (&ai)[6], double& m2, double& det) {
    // a = (a00, a01, a02, a11, a12, a22)
    const double c00 = a[3] * a[5] - a[4] * a[4], c01 = a[2] * a[4] - a[1] * a[5], c02 = a[1] * a[4] - a[2] * a[3];
    const double c11 = a[0] * a[5] - a[2] * a[2], c12 = a[1] * a[2] - a[0] * a[4], c22 = a[0] * a[3] - a[1] * a[1];
    det = a[0] * c00 + a[1] * c01 + a[2] * c02;
    m2 = c22;
    const double id = rcp_nr(det);
    ai[0] = c00 * id; ai[1] = c01 * id; ai[2] = c02 * id; ai[3] = c11 * id; ai[4] = c12 * id; ai[5] = c22 * id;
    return a[0] > 0 && c22 > 0 && det > 0;
}
__device__ __forceinline__ void sym3_mul(const double (&s)[6], const double (&v)[3], double (&o)[3]) {
    o[0] = s[0] * v[0] + s[1] * v[1] + s[2] * v[2];
    o[1] = s[1] * v[0] + s[3] * v[1] + s[4] * v[2];
    o[2] = s[2] * v[0] + s[4] * v[1] + s[5] * v[2];
}
__device__ __forceinline__ bool solve6(const double (&U)[21], double lambda, const double (&b)[6], double (&x)[6]) {
    // U rows: (0,0..5) = 0..5, (1,1..5) = 6..10, (2,2..5) = 11..14, (3,3..5) = 15..17, (4,4..5) = 18, 19, (5,5) = 20
    const double A[6] = {U[0] + lambda, U[1], U[2], U[6] + lambda, U[7], U[11] + lambda};
    const double B[3][3] = {{U[3], U[4], U[5]}, {U[8], U[9], U[10]}, {U[12], U[13], U[14]}};  // B[i][j] = H[i][3 + j]
    double Ai[6], mA2, dA;
    const bool okA = inv3sym(A, Ai, mA2, dA);
    double X[3][3];  // A^-1 B
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double col[3] = {B[0][j], B[1][j], B[2][j]};
        double o[3];
        sym3_mul(Ai, col, o);
        X[0][j] = o[0]; X[1][j] = o[1]; X[2][j] = o[2];
    }
    // Schur complement C - B^T A^-1 B (symmetric)
    auto btx = [&](int i, int j) { return B[0][i] * X[0][j] + B[1][i] * X[1][j] + B[2][i] * X[2][j]; };
    const double Sc[6] = {U[15] + lambda - btx(0, 0), U[16] - btx(0, 1), U[17] - btx(0, 2),
                          U[18] + lambda - btx(1, 1), U[19] - btx(1, 2), U[20] + lambda - btx(2, 2)};
    double Si[6], mS2, dS;
    const bool okS = inv3sym(Sc, Si, mS2, dS);
    const double b1[3] = {b[0], b[1], b[2]};
    double y1[3];
    sym3_mul(Ai, b1, y1);
    const double r2[3] = {b[3] - (B[0][0] * y1[0] + B[1][0] * y1[1] + B[2][0] * y1[2]),
                          b[4] - (B[0][1] * y1[0] + B[1][1] * y1[1] + B[2][1] * y1[2]),
                          b[5] - (B[0][2] * y1[0] + B[1][2] * y1[1] + B[2][2] * y1[2])};
    double x2[3];
    sym3_mul(Si, r2, x2);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        x[3 + i] = x2[i];
        x[i] = y1[i] - (X[i][0] * x2[0] + X[i][1] * x2[1] + X[i][2] * x2[2]);
    }
    return okA && okS;
}

__device__ __forceinline__ void qnormalize_r(double q[4]) {  // SE3Quat::normalizeRotation, one reciprocal root
    if (q[3] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
    const double n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    if (n2 > 0) {
        const double in = rsq_nr(n2);
        for (int i = 0; i < 4; ++i) q[i] *= in;
    }
}

// sin / cos of h >= 0.25 (a step of more than half a radian: rare): h / 2^k below 0.25 by its
// exponent, the Taylor series there, then k double-angle steps -- a few ulps per step, far inside the
// pose bar, and without the library's large register footprint (Payne-Hanek reduction) in this kernel
__device__ __forceinline__ void sincos_halving(double h, double& sn, double& cs) {
    int e;
    (void)frexp(h, &e);  // h = m 2^e, 0.5 <= m < 1
    const int k = min(max(e + 2, 0), 64);
    const double a = ldexp(h, -k), a2 = a * a;
    double s = a * (1 + a2 * (-1. / 6 + a2 * (1. / 120 + a2 * (-1. / 5040 + a2 * (1. / 362880 + a2 * (-1. / 39916800 +
               a2 * (1. / 6227020800. + a2 * (-1. / 1307674368000.))))))));
    double c = 1 + a2 * (-1. / 2 + a2 * (1. / 24 + a2 * (-1. / 720 + a2 * (1. / 40320 + a2 * (-1. / 3628800 +
               a2 * (1. / 479001600. + a2 * (-1. / 87178291200. + a2 * (1. / 20922789888000.))))))));
    for (int i = 0; i < k; ++i) {
        const double s2 = 2 * s * c;
        c = (c - s) * (c + s);
        s = s2;
    }
    sn = s;
    cs = c;
}

// pose <- exp(u) * pose (VertexSE3Expmap::oplusImpl, SE3Quat::exp then operator*), as orb_se3.h's
// se3_oplus with reciprocal roots instead of divisions (the pose bar is 1e-6 RMSE), written with
// Omega^2 = w w^T - theta^2 I so that no product with a zero entry is issued: V = a I + b Omega + c w w^T
// and V u = a u + b (w x u) + c w (w . u).
//   theta < 0.00001 (g2o's small-angle branch): R = V = I + Omega + Omega^2 (a = 1 - theta^2, b = c = 1)
//     and Quaterniond(R) by its trace branch, normalised: R - R^T = 2 Omega gives the vector part
//     w / s with s = sqrt(tr R + 1) = sqrt(4 - 2 theta^2), the scalar part s / 2;
//   theta < 0.5: the Rodrigues quaternion (sin(theta/2) / theta w, cos(theta/2)) and the coefficients
//     (1 - cos) / theta^2, (theta - sin) / theta^3 as Taylor series in theta^2 (no sqrt, no sincos);
//   beyond: sincos of the half angle.
__device__ __forceinline__ void se3_oplus_r(double (&T)[7], const double (&u)[6]) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double t2 = w0 * w0 + w1 * w1 + w2 * w2;
    double eq[4], va, vb, vc;
    if (t2 < 1e-10) {
        const double tr1 = 4.0 - 2.0 * t2;  // tr R + 1
        const double rs = rsq_nr(tr1);
        const double f = rs;                // (R[7] - R[5]) * (0.5 / s) = 2 w0 * 0.5 / s
        eq[0] = f * w0; eq[1] = f * w1; eq[2] = f * w2; eq[3] = 0.5 * (tr1 * rs);
        qnormalize_r(eq);
        va = 1.0 - t2; vb = 1.0; vc = 1.0;
    } else {
        double f, c, b, d;
        if (t2 < 0.25) {
            const double s = t2;  // theta^2; half angle h^2 = s / 4
            // sin(h) / theta = (1/2) sum (-1)^k h^2k / (2k+1)!,  cos(h) = sum (-1)^k h^2k / (2k)!
            const double hh = 0.25 * s;
            f = 0.5 * (1 + hh * (-1. / 6 + hh * (1. / 120 + hh * (-1. / 5040 + hh * (1. / 362880 +
                  hh * (-1. / 39916800 + hh * (1. / 6227020800. + hh * (-1. / 1307674368000.))))))));
            c = 1 + hh * (-1. / 2 + hh * (1. / 24 + hh * (-1. / 720 + hh * (1. / 40320 + hh * (-1. / 3628800 +
                  hh * (1. / 479001600. + hh * (-1. / 87178291200.)))))));
            // (1 - cos theta) / theta^2 = sum (-1)^k s^k / (2k+2)!,  (theta - sin theta) / theta^3 = sum (-1)^k s^k / (2k+3)!
            b = 1. / 2 + s * (-1. / 24 + s * (1. / 720 + s * (-1. / 40320 + s * (1. / 3628800 + s * (-1. / 479001600. +
                  s * (1. / 87178291200. + s * (-1. / 20922789888000.)))))));
            d = 1. / 6 + s * (-1. / 120 + s * (1. / 5040 + s * (-1. / 362880 + s * (1. / 39916800 + s * (-1. / 6227020800. +
                  s * (1. / 1307674368000. + s * (-1. / 355687428096000.)))))));
        } else {
            const double theta = sqrt(t2);
            double sh, chh;
            sincos_halving(0.5 * theta, sh, chh);
            const double it = rcp_nr(theta), it2 = it * it;
            const double sn = 2 * sh * chh, omc = 2 * sh * sh;
            b = omc * it2;
            d = (theta - sn) * (it2 * it);
            f = sh * it;
            c = chh;
        }
        eq[0] = f * w0; eq[1] = f * w1; eq[2] = f * w2; eq[3] = c;
        va = 1.0 - d * t2; vb = b; vc = d;
    }
    // V upsilon
    const double wu = w0 * u[3] + w1 * u[4] + w2 * u[5];
    const double x0 = w1 * u[5] - w2 * u[4], x1 = w2 * u[3] - w0 * u[5], x2 = w0 * u[4] - w1 * u[3];
    const double cw = vc * wu;
    const double et[3] = {va * u[3] + vb * x0 + cw * w0, va * u[4] + vb * x1 + cw * w1, va * u[5] + vb * x2 + cw * w2};
    const double q[4] = {T[3], T[4], T[5], T[6]};
    double rt[3];
    qrotate(eq, T, rt);
    double nq[4] = {eq[3] * q[0] + eq[0] * q[3] + eq[1] * q[2] - eq[2] * q[1],
                    eq[3] * q[1] + eq[1] * q[3] + eq[2] * q[0] - eq[0] * q[2],
                    eq[3] * q[2] + eq[2] * q[3] + eq[0] * q[1] - eq[1] * q[0],
                    eq[3] * q[3] - eq[0] * q[0] - eq[1] * q[1] - eq[2] * q[2]};
    qnormalize_r(nq);
    T[0] = et[0] + rt[0];
    T[1] = et[1] + rt[1];
    T[2] = et[2] + rt[2];
    for (int i = 0; i < 4; ++i) T[3 + i] = nq[i];
}

// The pose as a rotation matrix and translation, once per pass (SE3Quat::map = R x + t)
struct PoseRT {
    double r[9], t[3];
};
__device__ __forceinline__ PoseRT pose_rt(const double (&T)[7]) {
    PoseRT P;
    const double q[4] = {T[3], T[4], T[5], T[6]};
    qmatrix(q, P.r);
    P.t[0] = T[0]; P.t[1] = T[1]; P.t[2] = T[2];
    return P;
}

// Error, robust chi2 and the J^T W J / -J^T W e contributions of one edge at pose P, added to acc:
// acc[0..21) the upper triangle of H row by row, acc[21..27) b, acc[27] the robust chi2.  Returns the
// edge's chi2.  The Jacobian rows of EdgeSE3ProjectXYZOnlyPose (two) and EdgeStereoSE3ProjectXYZOnlyPose
// (three; types_six_dof_expmap.cpp:375-404) share their zero pattern: row 0 (and the stereo row 2) has
// column 4 zero, row 1 column 3; the products with those zeros are skipped.  The stereo row is a
// separate block, so a wave of one edge type runs only its own path (edges are sorted by type).  One
// reciprocal of the depth replaces the divisions.  An edge with `on` false contributes exactly zero
// (zero information and a zero depth reciprocal; its values must be finite).
__device__ __forceinline__ double linearize_edge(const orb_pose_edge_t& Ed, const PoseRT& P, const orb_ba_camera_t& cam,
                                                 bool robust, Huber2 hub, double (&acc)[32], bool on) {
    const double X = Ed.xw[0], Y = Ed.xw[1], Z = Ed.xw[2];
    const double x = P.r[0] * X + P.r[1] * Y + P.r[2] * Z + P.t[0];
    const double y = P.r[3] * X + P.r[4] * Y + P.r[5] * Z + P.t[1];
    const double z = P.r[6] * X + P.r[7] * Y + P.r[8] * Z + P.t[2];
    const double fx = cam.fx, fy = cam.fy;
    const double iz = on ? rcp_nr(z) : 0.0, iz2 = iz * iz;
    const bool st = Ed.stereo != 0;
    double r0[6], r1[6], r2[6], e0, e1, e2 = 0.0;
    if (!st) {
        e0 = Ed.obs[0] - (fx * x * iz + (double)cam.cx);
        e1 = Ed.obs[1] - (fy * y * iz + (double)cam.cy);
        const double j00 = -(fx * iz), j02 = fx * x * iz2, j11 = -(fy * iz), j12 = fy * y * iz2;
        r0[0] = j02 * y; r0[1] = j00 * z - j02 * x; r0[2] = -j00 * y; r0[3] = j00; r0[4] = 0; r0[5] = j02;
        r1[0] = -j11 * z + j12 * y; r1[1] = -j12 * x; r1[2] = j11 * x; r1[3] = 0; r1[4] = j11; r1[5] = j12;
    } else {  // cam_project: float invz, double fx, fy, cx, cy, bf members
        const float finvz = (float)iz;
        const double u = x * finvz * fx + (double)cam.cx;
        const double v = y * finvz * fy + (double)cam.cy;
        e0 = Ed.obs[0] - u;
        e1 = Ed.obs[1] - v;
        e2 = Ed.obs[2] - (u - (double)cam.bf * finvz);
        const double bf = cam.bf;
        r0[0] = x * y * iz2 * fx; r0[1] = -(1 + (x * x * iz2)) * fx; r0[2] = y * iz * fx;
        r0[3] = -iz * fx; r0[4] = 0; r0[5] = x * iz2 * fx;
        r1[0] = (1 + y * y * iz2) * fy; r1[1] = -x * y * iz2 * fy; r1[2] = -x * iz * fy;
        r1[3] = 0; r1[4] = -iz * fy; r1[5] = y * iz2 * fy;
        r2[0] = r0[0] - bf * y * iz2; r2[1] = r0[1] + bf * x * iz2; r2[2] = r0[2];
        r2[3] = r0[3]; r2[4] = 0; r2[5] = r0[5] - bf * iz2;
    }
    const double info = on ? (double)Ed.inv_sigma2 : 0.0;
    double chi2 = e0 * info * e0 + e1 * info * e1;
    if (st) chi2 += e2 * info * e2;
    double rho0 = chi2, rho1 = 1.0;
    if (robust) {  // RobustKernelHuber with its float dsqr (robust_kernel_impl.cpp:78-91)
        const double dsq = (double)(st ? hub.dsqr_stereo : hub.dsqr_mono);
        if (!(chi2 <= dsq)) {
            const double delta = st ? hub.delta_stereo : hub.delta_mono;
            const double rs = rsq_nr(chi2);
            rho0 = 2 * (chi2 * rs) * delta - dsq;
            rho1 = delta * rs;
        }
    }
    acc[27] += rho0;
    const double w = rho1 * info;
    constexpr bool nz0[6] = {true, true, true, true, false, true};   // rows 0 and 2
    constexpr bool nz1[6] = {true, true, true, false, true, true};   // row 1
    double w0[6], w1[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        w0[i] = w * r0[i];
        w1[i] = w * r1[i];
    }
    {
        int k = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 6; ++j, ++k) {
                if (nz0[i] && nz0[j]) acc[k] += w0[i] * r0[j];
                if (nz1[i] && nz1[j]) acc[k] += w1[i] * r1[j];
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (nz0[i]) acc[21 + i] -= w0[i] * e0;
            if (nz1[i]) acc[21 + i] -= w1[i] * e1;
        }
    }
    if (st) {
        double w2[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) w2[i] = w * r2[i];
        int k = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 6; ++j, ++k)
                if (nz0[i] && nz0[j]) acc[k] += w2[i] * r2[j];
#pragma unroll
        for (int i = 0; i < 6; ++i)
            if (nz0[i]) acc[21 + i] -= w2[i] * e2;
    }
    return chi2;
}

// linearize_edge for one edge type known at compile time, without branches (the Huber weight by
// selects; a non-robust pass passes an infinite dsq), split in two: lin_front computes the error, the
// Jacobian rows and the weight, lin_accum adds the products to the sums.  A pair step runs both fronts
// before both accumulations, so that the scheduler can overlap the two edges' dependent chains (one
// wave per SIMD cannot hide a single edge's).  Same arithmetic as linearize_edge.
struct EdgeLin {
    double r0[6], r1[6], r2[6], e0, e1, e2, w, rho0, chi2;
};
template <bool St>
__device__ __forceinline__ EdgeLin lin_front(double X, double Y, double Z, double o0, double o1, double o2, float isg,
                                             const PoseRT& P, const orb_ba_camera_t& cam, double delta, double dsq,
                                             bool on) {
    EdgeLin L;
    const double x = P.r[0] * X + P.r[1] * Y + P.r[2] * Z + P.t[0];
    const double y = P.r[3] * X + P.r[4] * Y + P.r[5] * Z + P.t[1];
    const double z = P.r[6] * X + P.r[7] * Y + P.r[8] * Z + P.t[2];
    const double fx = cam.fx, fy = cam.fy;
    const double iz = on ? rcp_nr(z) : 0.0, iz2 = iz * iz;
    L.e2 = 0.0;
    if constexpr (!St) {
        L.e0 = o0 - (fx * x * iz + (double)cam.cx);
        L.e1 = o1 - (fy * y * iz + (double)cam.cy);
        const double j00 = -(fx * iz), j02 = fx * x * iz2, j11 = -(fy * iz), j12 = fy * y * iz2;
        L.r0[0] = j02 * y; L.r0[1] = j00 * z - j02 * x; L.r0[2] = -j00 * y; L.r0[3] = j00; L.r0[4] = 0; L.r0[5] = j02;
        L.r1[0] = -j11 * z + j12 * y; L.r1[1] = -j12 * x; L.r1[2] = j11 * x; L.r1[3] = 0; L.r1[4] = j11; L.r1[5] = j12;
    } else {
        const float finvz = (float)iz;
        const double u = x * finvz * fx + (double)cam.cx;
        const double v = y * finvz * fy + (double)cam.cy;
        L.e0 = o0 - u;
        L.e1 = o1 - v;
        L.e2 = o2 - (u - (double)cam.bf * finvz);
        const double bf = cam.bf;
        L.r0[0] = x * y * iz2 * fx; L.r0[1] = -(1 + (x * x * iz2)) * fx; L.r0[2] = y * iz * fx;
        L.r0[3] = -iz * fx; L.r0[4] = 0; L.r0[5] = x * iz2 * fx;
        L.r1[0] = (1 + y * y * iz2) * fy; L.r1[1] = -x * y * iz2 * fy; L.r1[2] = -x * iz * fy;
        L.r1[3] = 0; L.r1[4] = -iz * fy; L.r1[5] = y * iz2 * fy;
        L.r2[0] = L.r0[0] - bf * y * iz2; L.r2[1] = L.r0[1] + bf * x * iz2; L.r2[2] = L.r0[2];
        L.r2[3] = L.r0[3]; L.r2[4] = 0; L.r2[5] = L.r0[5] - bf * iz2;
    }
    const double info = on ? (double)isg : 0.0;
    double chi2 = L.e0 * info * L.e0 + L.e1 * info * L.e1;
    if constexpr (St) chi2 += L.e2 * info * L.e2;
    const double rs = rsq_nr(chi2);  // unused (possibly not finite) unless the edge is beyond dsq
    const bool big = !(chi2 <= dsq);
    L.rho0 = big ? 2 * (chi2 * rs) * delta - dsq : chi2;
    const double rho1 = big ? delta * rs : 1.0;
    L.w = rho1 * info;
    L.chi2 = chi2;
    return L;
}
template <bool St>
__device__ __forceinline__ void lin_accum(const EdgeLin& L, double (&acc)[32]) {
    acc[27] += L.rho0;
    constexpr bool nz0[6] = {true, true, true, true, false, true};   // rows 0 and 2
    constexpr bool nz1[6] = {true, true, true, false, true, true};   // row 1
    double w0[6], w1[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        w0[i] = L.w * L.r0[i];
        w1[i] = L.w * L.r1[i];
    }
    {
        int k = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 6; ++j, ++k) {
                if (nz0[i] && nz0[j]) acc[k] += w0[i] * L.r0[j];
                if (nz1[i] && nz1[j]) acc[k] += w1[i] * L.r1[j];
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (nz0[i]) acc[21 + i] -= w0[i] * L.e0;
            if (nz1[i]) acc[21 + i] -= w1[i] * L.e1;
        }
    }
    if constexpr (St) {
        double w2[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) w2[i] = L.w * L.r2[i];
        int k = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 6; ++j, ++k)
                if (nz0[i] && nz0[j]) acc[k] += w2[i] * L.r2[j];
#pragma unroll
        for (int i = 0; i < 6; ++i)
            if (nz0[i]) acc[21 + i] -= w2[i] * L.e2;
    }
}
// both edges of a pair step of one type: both fronts, then both accumulations
template <bool St>
__device__ __forceinline__ void lin_pair(const double2 (&xw)[3], const double2 (&ob)[3], float2 is, const PoseRT& P,
                                         const orb_ba_camera_t& cam, double delta, double dsq, double (&acc)[32],
                                         bool on0, bool on1, double& c0, double& c1) {
    const EdgeLin a = lin_front<St>(xw[0].x, xw[1].x, xw[2].x, ob[0].x, ob[1].x, ob[2].x, is.x, P, cam, delta, dsq, on0);
    const EdgeLin b = lin_front<St>(xw[0].y, xw[1].y, xw[2].y, ob[0].y, ob[1].y, ob[2].y, is.y, P, cam, delta, dsq, on1);
    lin_accum<St>(a, acc);
    lin_accum<St>(b, acc);
    c0 = a.chi2;
    c1 = b.chi2;
}

// Phase stamps of frame 0 (orb_debug_pose_trace, tools/pose_trace.py): per LM trial, s_memtime at the
// pass start, after the pass's reduction, after the totals reached thread 0, after its decision and
// solve, after the barrier that ends the trial, and inside the solve: its start, after the LDL^T,
// after the exponential.
__device__ long long* g_pose_trace = nullptr;
__device__ int g_pose_trace_cap = 0;
// Cost probe (built with -DORB_POSE_PROBE; orb_debug_pose_extra, tools/pose_trace.py): bit 0 runs the
// block solve once more and bit 1 the exponential once more, each on the dependent path of the real
// one, so the kernel-time difference is that step's latency.  Off by default: its branches cost ~3 %.
#ifdef ORB_POSE_PROBE
__device__ int g_pose_extra = 0;
#endif

// LM state of a frame's optimize(10), kept in registers of the workgroup's thread 0
struct LmState {
    double iscale;  // 1 / computeScale of the trial's step (x . (lambda x + b) + 1e-3), known at its solve
    double lambda, ni, current, ini;
    int nbad, qmax, it, ok, cur;  // cur: the buffer of sys holding the system
};

// One workgroup per frame.  The frame's first kCap edges live in LDS for the whole optimisation,
// field by field (structure of arrays), sorted by type -- the monocular edges first, then the stereo
// ones, each in index order -- with their outlier flag and last chi2; edges beyond are read from memory
// on every pass.  A pass steps over the positions in pairs: thread t takes positions 2t and 2t + 1 of
// each 2 kPT block, both of one type in every wave but the one at the type boundary, so that the two
// linearisations are straight-line code of one type that the scheduler interleaves (one wave per SIMD
// cannot hide a single edge's dependent FP64 chain).  Every trial evaluates the new pose and linearises
// there in the same pass: g2o rebuilds the system at the accepted state before the next iteration, and
// a rejected trial keeps the old linearisation, so the next iteration's build is this pass's sums.
// Thread 0 holds the LM state; per trial it takes the totals, decides, and solves the next trial,
// between two barriers.
template <int kCapT, int kOcc>
__global__ __launch_bounds__(kPT, kOcc) void k_pose_opt_t(const orb_pose_frame_t* __restrict__ frames,
                                                  const orb_pose_edge_t* __restrict__ edges,
                                                  double* __restrict__ pose_out, uint8_t* __restrict__ level,
                                                  int32_t* __restrict__ inliers, double* __restrict__ echi2, Huber2 hub) {
    __shared__ double part[kPW * 32];
    __shared__ double T[7];
    __shared__ int s_state;  // 1: evaluate the trial pose in T, 2: the round's optimize() is done
    constexpr int kA = kCapT / kPT;  // edges ranked per thread by the type sort
    __shared__ int perm[kCapT];      // position -> edge index
    __shared__ int scan[kPT];
    __shared__ double lxw[3][kCapT], lob[3][kCapT];  // xw, obs by position
    __shared__ float lis[kCapT];                    // inv_sigma2
    __shared__ double lch[kCapT];                   // last chi2
    __shared__ uint8_t llv[kCapT];                  // level (1: outlier)
    const int tid = threadIdx.x, f = blockIdx.x;
    long long* const tr = f == 0 ? g_pose_trace : nullptr;
    const int tr_cap = g_pose_trace_cap;
    int tr_n = 0;  // trials stamped
    auto stamp = [&](int k) {
        if (tr && tid == 0 && tr_n < tr_cap) tr[16 * tr_n + k] = clock64();
    };
    const orb_pose_frame_t F = frames[f];
    const int n = F.n_edges;
    const orb_pose_edge_t* E = edges + F.edge_begin;
    uint8_t* lev = level + F.edge_begin;
    double* ech = echi2 + F.edge_begin;
    if (n < 3) {  // nInitialCorrespondences < 3: return 0, pose untouched
        for (int e = tid; e < n; e += kPT) lev[e] = 0;
        if (tid < 7) pose_out[7 * (size_t)f + tid] = frames[f].pose[tid];
        if (tid == 0) inliers[f] = 0;
        return;
    }
    // ---- the LDS edges sorted by type: thread t ranks edges [kA t, kA t + kA).  The monocular edges
    // take positions [0, nmono), the stereo ones start at s0 (nmono rounded up to a wave's 128 positions
    // of a pair step, the gap filled with dummies), so every wave of a pair step runs one edge type.
    const int nr = min(n, kCapT - 128);
    int nmono, s0, npos;
    {
        int mono = 0;
        bool st[kA];
#pragma unroll
        for (int s = 0; s < kA; ++s) {
            const int e = kA * tid + s;
            st[s] = e < nr ? E[e].stereo != 0 : true;
            mono += e < nr && !st[s];
        }
        scan[tid] = mono;
        __syncthreads();
        for (int o = 1; o < kPT; o <<= 1) {
            const int v = tid >= o ? scan[tid - o] : 0;
            __syncthreads();
            scan[tid] += v;
            __syncthreads();
        }
        nmono = scan[kPT - 1];
        s0 = (nmono + 127) & ~127;
        npos = s0 + nr - nmono;
        int rm = scan[tid] - mono;       // monocular edges before this thread's
        int rs = kA * tid - rm;          // stereo edges before this thread's (of the e < nr ones)
#pragma unroll
        for (int s = 0; s < kA; ++s) {
            const int e = kA * tid + s;
            if (e < nr) perm[st[s] ? s0 + rs++ : rm++] = e;
        }
        __syncthreads();
    }
    // the gap and the positions up to the pair step's round-up hold finite dummies (level 2: never
    // active, computed with zero information)
    const int nfill = (npos + kPair - 1) / kPair * kPair;
    for (int q = tid; q < nfill; q += kPT) {
        const bool real = q < nmono || (q >= s0 && q < npos);
        if (real) {
            const orb_pose_edge_t Ed = E[perm[q]];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                lxw[i][q] = Ed.xw[i];
                lob[i][q] = Ed.obs[i];
            }
            lis[q] = Ed.inv_sigma2;
        } else {
            lxw[0][q] = 0; lxw[1][q] = 0; lxw[2][q] = 1.0;
            lob[0][q] = 0; lob[1][q] = 0; lob[2][q] = 0;
            lis[q] = 0;
        }
        llv[q] = real ? 0 : 2;  // mvbOutlier[i] = false at edge creation
        lch[q] = 0;
    }
    for (int e = tid + nr; e < n; e += kPT) lev[e] = 0;
    __syncthreads();
    // fn(edge index, LDS position or -1, outlier flag, last chi2) over this thread's edges
    auto visit = [&](auto&& fn) {
        for (int q = tid; q < npos; q += kPT) {
            int l = llv[q];
            if (l == 2) continue;
            double c = lch[q];
            fn(perm[q], q, l, c);
            llv[q] = (uint8_t)l;
            lch[q] = c;
        }
        for (int e = tid + nr; e < n; e += kPT) {
            int l = lev[e];
            double c = ech[e];
            fn(e, -1, l, c);
            lev[e] = (uint8_t)l;
            ech[e] = c;
        }
    };
    // a linearisation pass at T over the active edges (chi2 kept when `keep`), reduced: wave 0's lane
    // 2k ends with the workgroup total of value k.  A wave skips the pair steps past the frame's edges.
    auto pass = [&](bool robust, bool keep, double (&acc)[32]) {
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = 0;
        double Tl[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) Tl[i] = T[i];
        const PoseRT P = pose_rt(Tl);
        const int wv = tid >> 6;
        const double dsqm = robust ? (double)hub.dsqr_mono : INFINITY;
        const double dsqs = robust ? (double)hub.dsqr_stereo : INFINITY;
        stamp(8);
        for (int jb = 0; jb < npos; jb += kPair) {
            const int wlo = jb + 128 * wv;  // the wave's first position (wave-uniform)
            if (wlo >= npos) continue;
            const int p = jb + 2 * tid;
            double2 xw[3], ob[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                xw[i] = *reinterpret_cast<const double2*>(&lxw[i][p]);
                ob[i] = *reinterpret_cast<const double2*>(&lob[i][p]);
            }
            const float2 is = *reinterpret_cast<const float2*>(&lis[p]);
            const bool on0 = !llv[p], on1 = !llv[p + 1];
            double c0, c1;
            if (wlo < s0) lin_pair<false>(xw, ob, is, P, F.cam, hub.delta_mono, dsqm, acc, on0, on1, c0, c1);
            else lin_pair<true>(xw, ob, is, P, F.cam, hub.delta_stereo, dsqs, acc, on0, on1, c0, c1);
            if (keep) {
                if (on0) lch[p] = c0;
                if (on1) lch[p + 1] = c1;
            }
        }
        for (int e = tid + nr; e < n; e += kPT) {
            if (lev[e]) continue;
            const double c2 = linearize_edge(E[e], P, F.cam, robust, hub, acc, true);
            if (keep) ech[e] = c2;
        }
        stamp(11);
        wave_partials32(acc, part);
        stamp(12);
        __syncthreads();
        stamp(13);
        if (tid < 64) {
            const int k = (tid >> 1) & 31;
#pragma unroll
            for (int w = 1; w < kPW; ++w) acc[0] += part[32 * w + k];  // the waves in order
        }
    };
    // the 28 workgroup totals (wave 0's lane 2k holds total k) into sys[buf]: the linear system and
    // chi2 live in LDS, double-buffered -- an accepted trial's pass becomes the system by a buffer swap
    __shared__ double sys[2][28];
    __shared__ double Tb[7];  // the pose before the trial step (restored on a rejection)
    auto totals = [&](const double (&acc)[32], int buf) {
        if (tid < 56 && !(tid & 1)) sys[buf][tid >> 1] = acc[0];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto solve = [&](LmState& S) {  // thread 0: the damped system sys[cur], the trial pose into T
        stamp(5);
        double U[21], b[6], Tn[7];
#pragma unroll
        for (int k = 0; k < 21; ++k) U[k] = sys[S.cur][k];
#pragma unroll
        for (int i = 0; i < 6; ++i) b[i] = sys[S.cur][21 + i];
#pragma unroll
        for (int i = 0; i < 7; ++i) Tn[i] = T[i];
#pragma unroll
        for (int i = 0; i < 7; ++i) Tb[i] = Tn[i];
        double x[6];
#ifdef ORB_POSE_PROBE
        const int extra = g_pose_extra;
#else
        constexpr int extra = 0;
#endif
        double lam = S.lambda;
        if (extra & 1) {
            double xd[6];
            (void)solve6(U, lam, b, xd);
            double z = xd[5];
            asm volatile("" : "+v"(z));
            lam += z * 0.0;
        }
        S.ok = solve6(U, lam, b, x);
        if (!S.ok)
#pragma unroll
            for (int i = 0; i < 6; ++i) x[i] = 0;
        // the decision's computeScale needs only this step: computed here (beside the exponential's
        // chain) instead of on the path from the pass to the decision
        double scale = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) scale += x[i] * (S.lambda * x[i] + b[i]);
        scale += 1e-3;
        S.iscale = rcp_nr(scale);
        stamp(6);
        if (extra & 2) {
            double Td[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) Td[i] = Tn[i];
            se3_oplus_r(Td, x);
            double z = Td[6];
            asm volatile("" : "+v"(z));
            x[0] += z * 0.0;
        }
        se3_oplus_r(Tn, x);
        stamp(7);
#pragma unroll
        for (int i = 0; i < 7; ++i) T[i] = Tn[i];
    };
    bool robust = true;
    int nBad = 0;
    // thread 0's LM state, in its registers for the whole optimisation
    LmState S;
    for (int round = 0; round < 4; ++round) {
        // vSE3->setEstimate(pFrame->GetPose()); read from global: a lane-indexed read of the copy F
        // would put F in scratch
        if (tid < 7) T[tid] = frames[f].pose[tid];
        __syncthreads();
        // ---- optimizer.initializeOptimization(0); optimizer.optimize(10)
        int active = 0;
        visit([&](int, int, int& l, double&) { active += l == 0; });
        active = __syncthreads_or(active);
        if (active) {
            int cur = 0;  // every thread tracks the system buffer
            double acc[32];
            pass(robust, false, acc);  // computeActiveErrors + buildSystem at the round's start pose
            totals(acc, cur);
            if (tid == 0) {
                S.cur = cur;
                S.current = S.ini = sys[cur][27];
                double m = 0;  // computeLambdaInit: tau * max |diag H|
                constexpr int kDiag[6] = {0, 6, 11, 15, 18, 20};
#pragma unroll
                for (int i = 0; i < 6; ++i) m = fmax(fabs(sys[cur][kDiag[i]]), m);
                S.lambda = 1e-5 * m;
                S.ni = 2;
                S.nbad = 0;
                S.qmax = 0;
                S.it = 0;
                solve(S);
            }
            __syncthreads();
            for (;;) {
                // evaluate (and linearise) at the trial pose; every active edge's chi2 is kept, since
                // g2o classifies on the last evaluated state even when it was rejected
                const int wb = cur ^ 1;
                stamp(0);
                pass(robust, true, acc);
                stamp(1);
                totals(acc, wb);
                stamp(2);
                if (tid == 0) {
                    double tempChi = sys[wb][27];
                    if (!S.ok) tempChi = DBL_MAX;
                    double r = S.current - tempChi;
                    r *= S.iscale;
                    const bool accept = r > 0 && isfinite(tempChi);
                    if (accept) {
                        const double c = 2 * r - 1;
                        double alpha = 1. - c * c * c;  // 1 - pow(2 rho - 1, 3)
                        alpha = fmin(alpha, 2. / 3.);
                        S.lambda *= fmax(1. / 3., alpha);
                        S.ni = 2;
                        S.current = tempChi;
                    } else {
                        S.lambda *= S.ni;
                        S.ni *= 2;
#pragma unroll
                        for (int i = 0; i < 7; ++i) T[i] = Tb[i];
                    }
                    S.qmax++;
                    int st = 1, swap = 0;
                    if (!(r < 0 && S.qmax < 10)) {
                        // the iteration ends; optimize()'s loop stops on qmax == 10 or rho == 0, after
                        // 10 iterations, or on the third consecutive small chi2 decrease
                        if (S.qmax == 10 || r == 0) {
                            st = 2;
                        } else {
                            if ((S.ini - S.current) * 1e3 < S.ini) S.nbad++;
                            else S.nbad = 0;
                            if (S.nbad >= 3 || ++S.it == 10) st = 2;
                        }
                        if (st == 1) {  // accepted: the next iteration's system is this pass's linearisation
                            swap = 1;
                            S.cur = wb;
                            S.ini = S.current;
                            S.qmax = 0;
                        }
                    }
                    if (st == 1) solve(S);
                    s_state = st | (swap << 2);
                }
                stamp(3);
                __syncthreads();
                stamp(4);
                ++tr_n;
                const int ss = s_state;
                if (ss & 4) cur = wb;
                if ((ss & 3) == 2) break;
            }
        }
        // ---- re-classification (src/Optimizer.cc:285-386)
        int bad = 0;
        visit([&](int e, int q, int& l, double& c) {
            const bool stereo = q >= 0 ? q >= s0 : E[e].stereo != 0;
            double c2 = c;
            if (l) {  // an outlier's error at the round's final pose
                orb_pose_edge_t Ed;
                if (q >= 0) {
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        Ed.xw[i] = lxw[i][q];
                        Ed.obs[i] = lob[i][q];
                    }
                    Ed.inv_sigma2 = lis[q];
                    Ed.stereo = stereo;
                } else {
                    Ed = E[e];
                }
                double Xc[3];
                EdgeEval ev;
                pose_edge_error(Ed, T, F.cam, Xc, ev);
                c2 = ev.chi2;
            }
            const float chi2 = (float)c2;
            l = chi2 > (stereo ? 7.815f : 5.991f);
            bad += l;
        });
        {
            const double wb = wave_sum_d((double)bad);
            if ((tid & 63) == 0) part[tid >> 6] = wb;
            __syncthreads();
            double nb = part[0];
#pragma unroll
            for (int w = 1; w < kPW; ++w) nb += part[w];
            nBad = (int)nb;
            __syncthreads();  // part is rewritten by the next round
        }
        if (round == 2) robust = false;
        if (n < 10) break;  // optimizer.edges().size() < 10
    }
    for (int q = tid; q < npos; q += kPT)
        if (llv[q] != 2) lev[perm[q]] = llv[q];
    if (tid < 7) pose_out[7 * (size_t)f + tid] = T[tid];
    if (tid == 0) inliers[f] = n - nBad;
}


Huber2 make_huber() {
    Huber2 h;
    const float dm = std::sqrt(5.991), ds = std::sqrt(7.815);  // const float deltaMono = sqrt(5.991)
    h.delta_mono = dm;
    h.delta_stereo = ds;
    h.dsqr_mono = (float)((double)dm * (double)dm);  // RobustKernel::setDelta: float dsqr = delta * delta
    h.dsqr_stereo = (float)((double)ds * (double)ds);
    return h;
}

}  // namespace

extern "C" {

int orb_pose_optimization_device(int n_frames, const orb_pose_frame_t* d_frames, int n_edges,
                                 const orb_pose_edge_t* d_edges, double* d_pose_out, uint8_t* d_outlier,
                                 int32_t* d_inliers, void* stream) {
    return orbgpu_pose_optimization_device_scratch(n_frames, d_frames, n_edges, d_edges, d_pose_out, d_outlier, d_inliers,
                                                   stream, nullptr);
}

}  // extern "C"

// d_chi: max(n_edges, 1) doubles of the caller's, or NULL: the chi2 of edges beyond the LDS (only frames
// of more than kCap - 128 edges use it) in stream-ordered scratch (allocated and freed on the call's
// stream), so calls on different streams may run concurrently
int orbgpu_pose_optimization_device_scratch(int n_frames, const orb_pose_frame_t* d_frames, int n_edges,
                                            const orb_pose_edge_t* d_edges, double* d_pose_out, uint8_t* d_outlier,
                                            int32_t* d_inliers, void* stream, double* d_chi) {
    if (n_frames < 0 || n_edges < 0 || (n_frames && (!d_frames || !d_pose_out || !d_inliers)) ||
        (n_edges && (!d_edges || !d_outlier)))
        return orbgpu_fail(ORB_ERR_ARG, "invalid pose optimisation arguments");
    if (n_frames == 0) return ORB_OK;
    double* chi = d_chi;
    if (!chi && hipMallocAsync(reinterpret_cast<void**>(&chi), std::max<size_t>(1, (size_t)n_edges) * sizeof(double),
                               (hipStream_t)stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    // Large batches (the batched tracking chain: 2 x 512 frames per call) run two frames per CU: the
    // kernel with a 1024-edge LDS room (69 KB) at two waves per SIMD (its registers spill more); a frame
    // beyond ~900 edges reads the rest from memory every pass.  ORBGPU_POSE_DUAL=0 / 1 forces one form.
    const char* fc = getenv("ORBGPU_POSE_DUAL");
    const int forced = fc ? atoi(fc) : -1;
    if (forced == 1 || (forced < 0 && n_frames >= kDualMinFrames))
        hipLaunchKernelGGL((k_pose_opt_t<1024, 2>), dim3(n_frames), dim3(kPT), 0, (hipStream_t)stream, d_frames, d_edges,
                           d_pose_out, d_outlier, d_inliers, chi, make_huber());
    else
        hipLaunchKernelGGL((k_pose_opt_t<kCap, 1>), dim3(n_frames), dim3(kPT), 0, (hipStream_t)stream, d_frames, d_edges,
                           d_pose_out, d_outlier, d_inliers, chi, make_huber());
    const bool launched = hipGetLastError() == hipSuccess;
    if ((!d_chi && hipFreeAsync(chi, (hipStream_t)stream) != hipSuccess) || !launched)
        return orbgpu_fail(ORB_ERR_DEVICE, "pose kernel launch failed");
    return ORB_OK;
}

extern "C" {

// Debug hook (not in the public header): stamp frame 0's LM trials into d_buf (16 int64 per trial, up
// to `cap` trials; NULL turns it off).  Synchronous.
int orb_debug_pose_trace(long long* d_buf, int cap) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_trace), &d_buf, sizeof(d_buf)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_pose_trace_cap), &cap, sizeof(cap)) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "debug symbol copy");
    return ORB_OK;
}

// Debug hook (not in the public header): the cost probe's mode (g_pose_extra).  Synchronous.
int orb_debug_pose_extra(int mode) {
#ifdef ORB_POSE_PROBE
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_extra), &mode, sizeof(mode)) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "debug symbol copy");
    return ORB_OK;
#else
    (void)mode;
    return orbgpu_fail(ORB_ERR_ARG, "built without ORB_POSE_PROBE");
#endif
}

int orb_pose_optimization(int n_frames, const orb_pose_frame_t* frames, int n_edges, const orb_pose_edge_t* edges,
                          double* pose_out, uint8_t* outlier, int32_t* inliers) {
    if (n_frames < 0 || n_edges < 0 || (n_frames && (!frames || !pose_out || !inliers)) ||
        (n_edges && (!edges || !outlier)))
        return orbgpu_fail(ORB_ERR_ARG, "invalid pose optimisation arguments");
    for (int f = 0; f < n_frames; ++f)
        if (frames[f].n_edges < 0 || frames[f].edge_begin < 0 || (long long)frames[f].edge_begin + frames[f].n_edges > n_edges)
            return orbgpu_fail(ORB_ERR_ARG, "frame edge range outside the edge array");
    if (n_frames == 0) return ORB_OK;
    if (orb_device_count() <= 0) return orbgpu_fail(ORB_ERR_DEVICE, "no HIP device visible");
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_f = 0, o_e = al(sizeof(orb_pose_frame_t) * n_frames), o_p = o_e + al(sizeof(orb_pose_edge_t) * std::max(n_edges, 1));
    const size_t o_o = o_p + al(56 * (size_t)n_frames), o_i = o_o + al(std::max(n_edges, 1)), total = o_i + al(4 * (size_t)n_frames);
    uint8_t* d = nullptr;
    if (hipMalloc(&d, total) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
    int rc = ORB_OK;
    if (hipMemcpy(d + o_f, frames, sizeof(orb_pose_frame_t) * n_frames, hipMemcpyHostToDevice) != hipSuccess ||
        (n_edges && hipMemcpy(d + o_e, edges, sizeof(orb_pose_edge_t) * n_edges, hipMemcpyHostToDevice) != hipSuccess))
        rc = orbgpu_fail(ORB_ERR_DEVICE, "pose upload failed");
    if (rc == ORB_OK)
        rc = orb_pose_optimization_device(n_frames, reinterpret_cast<const orb_pose_frame_t*>(d + o_f), n_edges,
                                          reinterpret_cast<const orb_pose_edge_t*>(d + o_e), reinterpret_cast<double*>(d + o_p),
                                          d + o_o, reinterpret_cast<int32_t*>(d + o_i), nullptr);
    if (rc == ORB_OK &&
        (hipMemcpy(pose_out, d + o_p, 56 * (size_t)n_frames, hipMemcpyDeviceToHost) != hipSuccess ||
         (n_edges && hipMemcpy(outlier, d + o_o, n_edges, hipMemcpyDeviceToHost) != hipSuccess) ||
         hipMemcpy(inliers, d + o_i, 4 * (size_t)n_frames, hipMemcpyDeviceToHost) != hipSuccess))
        rc = orbgpu_fail(ORB_ERR_DEVICE, "pose download failed");
    (void)hipFree(d);
    return rc;
}

}  // extern "C"
