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
constexpr int kEdgeSlots = 512 / kPT;  // edges per thread kept in registers (512 per frame)
static_assert(kPT % 64 == 0 && kEdgeSlots >= 1 && kPW <= 32, "pose workgroup shape");

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

// LDL^T of the 6x6 symmetric matrix given as its upper triangle row by row (LinearSolverDense:
// Eigen::LDLT; the same solution up to rounding); one reciprocal per pivot
__device__ __forceinline__ bool ldlt6(const double (&U)[21], double lambda, const double (&b)[6], double (&x)[6]) {
    double A[36];
    {
        int k = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = i; j < 6; ++j) { A[6 * i + j] = A[6 * j + i] = U[k]; ++k; }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) A[7 * i] += lambda;
    double L[36] = {0}, d[6], id[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double dj = A[7 * j];
#pragma unroll
        for (int k = 0; k < j; ++k) dj -= L[6 * j + k] * L[6 * j + k] * d[k];
        if (!(dj > 0)) return false;  // LDLT::isPositive (the damped system is SPD unless degenerate)
        d[j] = dj;
        id[j] = rcp_nr(dj);
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double v = A[6 * j + i];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[6 * i + k] * L[6 * j + k] * d[k];
            L[6 * i + j] = v * id[j];
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        x[i] = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) x[i] -= L[6 * i + k] * x[k];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] *= id[i];
#pragma unroll
    for (int i = 5; i >= 0; --i)
#pragma unroll
        for (int k = i + 1; k < 6; ++k) x[i] -= L[6 * k + i] * x[k];
    return true;
}

__device__ __forceinline__ void qnormalize_r(double q[4]) {  // SE3Quat::normalizeRotation, one reciprocal
    if (q[3] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (n > 0) {
        const double in = rcp_nr(n);
        for (int i = 0; i < 4; ++i) q[i] *= in;
    }
}

// pose <- exp(u) * pose (VertexSE3Expmap::oplusImpl, SE3Quat::exp then operator*), as orb_se3.h's
// se3_oplus with reciprocals instead of divisions and, above g2o's small-angle threshold, the rotation's
// quaternion in closed form instead of Quaterniond(R) (the pose bar is 1e-6 RMSE)
__device__ __forceinline__ void se3_oplus_r(double (&T)[7], const double (&u)[6]) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    double V[9], eq[4], et[3];
    if (theta < 0.00001) {  // g2o's small-angle branch: R = V = I + Omega + Omega^2, then Quaterniond(R)
        double R[9];
        for (int k = 0; k < 9; ++k) R[k] = V[k] = (k % 4 == 0 ? 1.0 : 0.0) + O[k] + O2[k];
        qfrom_matrix(R, eq);
        qnormalize_r(eq);
    } else {
        // Quaterniond(R) of the Rodrigues R is (sin(theta/2) w / theta, cos(theta/2)), already unit:
        // one sincos of the half angle gives it, and sin(theta) = 2 s c, 1 - cos(theta) = 2 s^2 for V
        double sh, chh;
        sincos(0.5 * theta, &sh, &chh);
        const double it = rcp_nr(theta), it2 = it * it;
        const double sn = 2 * sh * chh, omc = 2 * sh * sh;
        const double b = omc * it2, d = (theta - sn) * (it2 * it);
        for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0 ? 1.0 : 0.0) + b * O[k] + d * O2[k];
        const double f = sh * it;
        eq[0] = f * w0; eq[1] = f * w1; eq[2] = f * w2; eq[3] = chh;
    }
    for (int i = 0; i < 3; ++i) et[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
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

// Error, robust chi2 and the J^T W J / -J^T W e contributions of one edge at pose T, added to acc:
// acc[0..21) the upper triangle of H row by row, acc[21..27) b, acc[27] the robust chi2.  Returns the
// edge's chi2.  One reciprocal of the depth replaces the divisions of computeError / linearizeOplus.
// An edge with `on` false contributes exactly zero (zero information, and a zero depth reciprocal so
// that no product is infinite).
__device__ __forceinline__ double linearize_edge(const orb_pose_edge_t& Ed, const double* T, const orb_ba_camera_t& cam,
                                                 bool robust, Huber2 hub, double (&acc)[32], bool on = true) {
    const double q[4] = {T[3], T[4], T[5], T[6]};
    double Xc[3];
    qrotate(q, Ed.xw, Xc);
    Xc[0] += T[0]; Xc[1] += T[1]; Xc[2] += T[2];
    const double x = Xc[0], y = Xc[1], z = Xc[2], fx = cam.fx, fy = cam.fy;
    const double iz = on ? 1.0 / z : 0.0, iz2 = iz * iz;
    EdgeEval ev;
    double B[18];
    if (!Ed.stereo) {
        ev.er[0] = Ed.obs[0] - (fx * x * iz + (double)cam.cx);
        ev.er[1] = Ed.obs[1] - (fy * y * iz + (double)cam.cy);
        ev.er[2] = 0.0;
        const double j00 = -(fx * iz), j02 = fx * x * iz2, j11 = -(fy * iz), j12 = fy * y * iz2;
        B[0] = j02 * y;  B[1] = j00 * z - j02 * x; B[2] = -j00 * y; B[3] = j00; B[4] = 0;   B[5] = j02;
        B[6] = -j11 * z + j12 * y; B[7] = -j12 * x; B[8] = j11 * x;  B[9] = 0;  B[10] = j11; B[11] = j12;
        for (int k = 12; k < 18; ++k) B[k] = 0;
    } else {  // cam_project: float invz, double fx, fy, cx, cy, bf members
        const float finvz = (float)(1.0f / z);
        const double u = x * finvz * fx + (double)cam.cx;
        const double v = y * finvz * fy + (double)cam.cy;
        ev.er[0] = Ed.obs[0] - u;
        ev.er[1] = Ed.obs[1] - v;
        ev.er[2] = Ed.obs[2] - (u - (double)cam.bf * finvz);
        const double bf = cam.bf;
        B[0] = x * y * iz2 * fx;    B[1] = -(1 + (x * x * iz2)) * fx; B[2] = y * iz * fx;
        B[3] = -iz * fx;            B[4] = 0;                         B[5] = x * iz2 * fx;
        B[6] = (1 + y * y * iz2) * fy; B[7] = -x * y * iz2 * fy;      B[8] = -x * iz * fy;
        B[9] = 0;                   B[10] = -iz * fy;                 B[11] = y * iz2 * fy;
        B[12] = B[0] - bf * y * iz2; B[13] = B[1] + bf * x * iz2;     B[14] = B[2];
        B[15] = B[3];               B[16] = 0;                        B[17] = B[5] - bf * iz2;
    }
    const double info = on ? (double)Ed.inv_sigma2 : 0.0;
    ev.chi2 = ev.er[0] * info * ev.er[0] + ev.er[1] * info * ev.er[1];
    if (Ed.stereo) ev.chi2 += ev.er[2] * info * ev.er[2];
    ev.stereo = Ed.stereo;
    double rho1;
    acc[27] += robust_rho(ev, robust, hub, rho1);
    const double w = rho1 * info;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
#pragma unroll
        for (int j = i; j < 6; ++j) {
            double s = B[i] * w * B[j] + B[6 + i] * w * B[6 + j];
            if (Ed.stereo) s += B[12 + i] * w * B[12 + j];
            acc[k++] += s;
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double bs = B[i] * info * ev.er[0] + B[6 + i] * info * ev.er[1];
        if (Ed.stereo) bs += B[12 + i] * info * ev.er[2];
        acc[21 + i] -= rho1 * bs;
    }
    return ev.chi2;
}

// Phase stamps of frame 0 (orb_debug_pose_trace, tools/pose_trace.py): per LM trial, s_memtime at the
// pass start, after the pass's reduction, after the totals reached thread 0, after its decision and
// solve, after the barrier that ends the trial, and inside the solve: its start, after the LDL^T,
// after the exponential.
__device__ long long* g_pose_trace = nullptr;
__device__ int g_pose_trace_cap = 0;

// LM state of a frame's optimize(10), kept in registers of the workgroup's thread 0
struct LmState {
    double H[21], b[6], x[6], Tb[7];
    double lambda, ni, current, ini;
    int nbad, qmax, it, ok;
};

// One 256-thread workgroup per frame.  The first kS * kPT edges of the frame (and their outlier flag
// and last chi2) stay in registers for the whole optimisation; edges beyond are read from memory on
// every pass.  Every trial evaluates the new pose and linearises there in the same pass: g2o rebuilds
// the system at the accepted state before the next iteration, and a rejected trial keeps the old
// linearisation, so the next iteration's build is this pass's sums.  Thread 0 holds the LM state; per
// trial it takes the totals, decides, and solves the next trial, between two barriers.
template <int kS>
__global__ __launch_bounds__(kPT) void k_pose_opt(const orb_pose_frame_t* __restrict__ frames,
                                                  const orb_pose_edge_t* __restrict__ edges,
                                                  double* __restrict__ pose_out, uint8_t* __restrict__ level,
                                                  int32_t* __restrict__ inliers, double* __restrict__ echi2, Huber2 hub) {
    __shared__ double part[kPW * 32];
    __shared__ double tot[28];
    __shared__ double T[7];
    __shared__ int s_state;  // 1: evaluate the trial pose in T, 2: the round's optimize() is done
    const int tid = threadIdx.x, f = blockIdx.x;
    long long* const tr = f == 0 ? g_pose_trace : nullptr;
    const int tr_cap = g_pose_trace_cap;
    int tr_n = 0;  // trials stamped
    auto stamp = [&](int k) {
        if (tr && tid == 0 && tr_n < tr_cap) tr[8 * tr_n + k] = clock64();
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
    orb_pose_edge_t ed[kS];
    int lv[kS];
    double ch[kS];
#pragma unroll
    for (int s = 0; s < kS; ++s) {
        const int e = tid + s * kPT;
        if (e < n) ed[s] = E[e];
        lv[s] = 0;  // mvbOutlier[i] = false at edge creation
        ch[s] = 0;
    }
    for (int e = tid + kS * kPT; e < n; e += kPT) lev[e] = 0;
    // fn(edge, outlier flag, last chi2) over this thread's edges
    auto visit = [&](auto&& fn) {
#pragma unroll
        for (int s = 0; s < kS; ++s)
            if (tid + s * kPT < n) fn(ed[s], lv[s], ch[s]);
        for (int e = tid + kS * kPT; e < n; e += kPT) {
            int l = lev[e];
            double c = ech[e];
            fn(E[e], l, c);
            lev[e] = (uint8_t)l;
            ech[e] = c;
        }
    };
    // a linearisation pass at T over the active edges (chi2 kept when `keep`), reduced: wave 0's lane
    // 2k ends with the workgroup total of value k.  The register slots are linearised without branches
    // (an inactive slot computes a zero-information dummy edge), so their latency chains interleave.
    orb_pose_edge_t dummy{};
    dummy.xw[2] = 1.0;
    auto pass = [&](bool robust, bool keep, double (&acc)[32]) {
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = 0;
        double Tl[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) Tl[i] = T[i];
#pragma unroll
        for (int s = 0; s < kS; ++s) {
            const bool on = tid + s * kPT < n && !lv[s];
            const double c2 = linearize_edge(on ? ed[s] : dummy, Tl, F.cam, robust, hub, acc, on);
            if (keep && on) ch[s] = c2;
        }
        for (int e = tid + kS * kPT; e < n; e += kPT) {
            if (lev[e]) continue;
            const double c2 = linearize_edge(E[e], Tl, F.cam, robust, hub, acc);
            if (keep) ech[e] = c2;
        }
        wave_partials32(acc, part);
        __syncthreads();
        if (tid < 64) {
            const int k = (tid >> 1) & 31;
#pragma unroll
            for (int w = 1; w < kPW; ++w) acc[0] += part[32 * w + k];  // the waves in order
        }
    };
    // the 28 workgroup totals to thread 0: wave 0's lane 2k holds total k; they go through LDS (one
    // store, thread 0's loads issued together) instead of 56 v_readlane in every lane of wave 0
    auto totals = [&](const double (&acc)[32], double (&t)[28]) {
        if (tid < 56 && !(tid & 1)) tot[tid >> 1] = acc[0];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 28; ++k) t[k] = tot[k];
        }
    };
    auto solve = [&](LmState& S) {  // thread 0: the damped system, the trial pose into T
        stamp(5);
        for (int i = 0; i < 7; ++i) S.Tb[i] = T[i];
        S.ok = ldlt6(S.H, S.lambda, S.b, S.x);
        if (!S.ok) for (int i = 0; i < 6; ++i) S.x[i] = 0;
        stamp(6);
        double Tn[7];
        for (int i = 0; i < 7; ++i) Tn[i] = S.Tb[i];
        se3_oplus_r(Tn, S.x);
        stamp(7);
        for (int i = 0; i < 7; ++i) T[i] = Tn[i];
    };
    bool robust = true;
    int nBad = 0;
    LmState S;
    for (int round = 0; round < 4; ++round) {
        // vSE3->setEstimate(pFrame->GetPose()); read from global: a lane-indexed read of the copy F
        // would put F in scratch
        if (tid < 7) T[tid] = frames[f].pose[tid];
        __syncthreads();
        // ---- optimizer.initializeOptimization(0); optimizer.optimize(10)
        int active = 0;
        visit([&](const orb_pose_edge_t&, int& l, double&) { active += l == 0; });
        active = __syncthreads_or(active);
        if (active) {
            double acc[32];
            pass(robust, false, acc);  // computeActiveErrors + buildSystem at the round's start pose
            double t[28];
            totals(acc, t);
            if (tid == 0) {
#pragma unroll
                for (int k = 0; k < 21; ++k) S.H[k] = t[k];
#pragma unroll
                for (int i = 0; i < 6; ++i) S.b[i] = t[21 + i];
                S.current = S.ini = t[27];
                double m = 0;  // computeLambdaInit: tau * max |diag H|
                constexpr int kDiag[6] = {0, 6, 11, 15, 18, 20};
#pragma unroll
                for (int i = 0; i < 6; ++i) m = fmax(fabs(S.H[kDiag[i]]), m);
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
                stamp(0);
                pass(robust, true, acc);
                stamp(1);
                totals(acc, t);
                stamp(2);
                if (tid == 0) {
                    double tempChi = t[27];
                    if (!S.ok) tempChi = DBL_MAX;
                    double r = S.current - tempChi;
                    double scale = 0;
                    for (int i = 0; i < 6; ++i) scale += S.x[i] * (S.lambda * S.x[i] + S.b[i]);
                    scale += 1e-3;
                    r *= rcp_nr(scale);
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
                        for (int i = 0; i < 7; ++i) T[i] = S.Tb[i];
                    }
                    S.qmax++;
                    int st = 1;
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
#pragma unroll
                            for (int k = 0; k < 21; ++k) S.H[k] = t[k];
#pragma unroll
                            for (int i = 0; i < 6; ++i) S.b[i] = t[21 + i];
                            S.ini = S.current;
                            S.qmax = 0;
                        }
                    }
                    if (st == 1) solve(S);
                    s_state = st;
                }
                stamp(3);
                __syncthreads();
                stamp(4);
                ++tr_n;
                if (s_state == 2) break;
            }
        }
        // ---- re-classification (src/Optimizer.cc:285-386)
        int bad = 0;
        visit([&](const orb_pose_edge_t& Ed, int& l, double& c) {
            double c2 = c;
            if (l) {
                double Xc[3];
                EdgeEval ev;
                pose_edge_error(Ed, T, F.cam, Xc, ev);
                c2 = ev.chi2;
            }
            const float chi2 = (float)c2;
            l = chi2 > (Ed.stereo ? 7.815f : 5.991f);
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
#pragma unroll
    for (int s = 0; s < kS; ++s) {
        const int e = tid + s * kPT;
        if (e < n) lev[e] = (uint8_t)lv[s];
    }
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
    if (n_frames < 0 || n_edges < 0 || (n_frames && (!d_frames || !d_pose_out || !d_inliers)) ||
        (n_edges && (!d_edges || !d_outlier)))
        return orbgpu_fail(ORB_ERR_ARG, "invalid pose optimisation arguments");
    if (n_frames == 0) return ORB_OK;
    // the chi2 of edges beyond the register slots: stream-ordered scratch (allocated and freed on the
    // call's stream), so calls on different streams may run concurrently
    double* chi = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&chi), std::max<size_t>(1, (size_t)n_edges) * sizeof(double),
                       (hipStream_t)stream) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "hipMallocAsync failed");
    hipLaunchKernelGGL(k_pose_opt<kEdgeSlots>, dim3(n_frames), dim3(kPT), 0, (hipStream_t)stream, d_frames, d_edges,
                       d_pose_out, d_outlier, d_inliers, chi, make_huber());
    const bool launched = hipGetLastError() == hipSuccess;
    if (hipFreeAsync(chi, (hipStream_t)stream) != hipSuccess || !launched)
        return orbgpu_fail(ORB_ERR_DEVICE, "pose kernel launch failed");
    return ORB_OK;
}

// Debug hook (not in the public header): stamp frame 0's LM trials into d_buf (8 int64 per trial, up
// to `cap` trials; NULL turns it off).  Synchronous.
int orb_debug_pose_trace(long long* d_buf, int cap) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pose_trace), &d_buf, sizeof(d_buf)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_pose_trace_cap), &cap, sizeof(cap)) != hipSuccess)
        return orbgpu_fail(ORB_ERR_DEVICE, "debug symbol copy");
    return ORB_OK;
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
