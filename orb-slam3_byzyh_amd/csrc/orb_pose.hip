// MI355X Optimizer::PoseOptimization (reference src/Optimizer.cc:55-415): tracking's motion-only
// bundle adjustment, batched over frames, FP64.
//
// One 256-thread workgroup per frame runs the whole optimisation: 4 rounds of g2o's optimize(10)
// (OptimizationAlgorithmLevenberg::solve, core/optimization_algorithm_levenberg.cpp:61-194, with
// LinearSolverDense on the single 6x6 pose block), each round restarting from the frame's pose and
// followed by the chi2 re-classification of every edge.  Per LM step:
//   build  threads stride over the active (level-0) edges: error, Huber weight, Jacobian
//          (EdgeSE3ProjectXYZOnlyPose: -projectJac * SE3deriv; EdgeStereoSE3ProjectXYZOnlyPose:
//          types_six_dof_expmap.cpp:375-404), the 21 + 6 entries of J^T W J / -J^T W e and the
//          robust chi2, reduced over the workgroup in a fixed order (wave shuffles, then LDS)
//   trial  lane 0 of wave 0 factors H + lambda I (LDL^T), exponentiates and applies the step; the
//          workgroup evaluates the new robust chi2 (storing every edge's chi2: g2o classifies the
//          active edges on the error of the LAST evaluated state, even a rejected one); lane 0 runs
//          g2o's accept / reject rule and restores the pose on a rejection
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

constexpr int kPT = 256;               // threads per frame
constexpr int kPW = kPT / 64;          // waves
constexpr int kNV = 28;                // reduced values: H upper (21), b (6), chi2

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

// fixed-order workgroup sum of N doubles per thread; result in red[0..N) for every thread
template <int N>
__device__ __forceinline__ void block_reduce(double (&v)[N], double* red) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < N; ++k)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    __syncthreads();  // red may still be read from the previous reduction
    if (lane < N) {
        double mine = 0;
#pragma unroll
        for (int k = 0; k < N; ++k) mine = lane == k ? v[k] : mine;
        red[wv * N + lane] = mine;
    }
    __syncthreads();
    if (threadIdx.x < N) {
        double s = 0;
        for (int w = 0; w < kPW; ++w) s += red[w * N + threadIdx.x];
        red[kPW * N + threadIdx.x] = s;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = red[kPW * N + k];
}

// LDL^T of the 6x6 symmetric matrix (LinearSolverDense: Eigen::LDLT; same solution up to rounding)
__device__ bool ldlt6(const double A[36], const double b[6], double x[6]) {
    double L[36] = {0}, d[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double dj = A[7 * j];
#pragma unroll
        for (int k = 0; k < j; ++k) dj -= L[6 * j + k] * L[6 * j + k] * d[k];
        if (!(dj > 0)) return false;  // LDLT::isPositive (the damped system is SPD unless degenerate)
        d[j] = dj;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
            double v = A[6 * j + i];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[6 * i + k] * L[6 * j + k] * d[k];
            L[6 * i + j] = v / dj;
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        x[i] = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) x[i] -= L[6 * i + k] * x[k];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] /= d[i];
#pragma unroll
    for (int i = 5; i >= 0; --i)
#pragma unroll
        for (int k = i + 1; k < 6; ++k) x[i] -= L[6 * k + i] * x[k];
    return true;
}

__global__ __launch_bounds__(kPT) void k_pose_opt(const orb_pose_frame_t* __restrict__ frames,
                                                  const orb_pose_edge_t* __restrict__ edges,
                                                  double* __restrict__ pose_out, uint8_t* __restrict__ level,
                                                  int32_t* __restrict__ inliers, double* __restrict__ echi2, Huber2 hub) {
    __shared__ double red[(kPW + 1) * kNV];
    __shared__ double T[7], Tb[7];
    __shared__ double H[36], bvec[6];
    __shared__ double s_lambda, s_ni, s_current, s_ini, s_temp;
    __shared__ int s_go, s_qmax, s_nbad, s_trial_go;
    const int tid = threadIdx.x, f = blockIdx.x;
    const orb_pose_frame_t F = frames[f];
    const int n = F.n_edges;
    const orb_pose_edge_t* E = edges + F.edge_begin;
    uint8_t* lev = level + F.edge_begin;
    double* ech = echi2 + F.edge_begin;
    for (int e = tid; e < n; e += kPT) lev[e] = 0;  // mvbOutlier[i] = false at edge creation
    if (n < 3) {  // nInitialCorrespondences < 3: return 0, pose untouched
        if (tid < 7) pose_out[7 * (size_t)f + tid] = frames[f].pose[tid];
        if (tid == 0) inliers[f] = 0;
        return;
    }
    const orb_ba_camera_t cam = F.cam;
    bool robust = true;
    int nBad = 0;
    for (int round = 0; round < 4; ++round) {
        // vSE3->setEstimate(pFrame->GetPose()); read from global: a lane-indexed read of the copy F
        // would put F in scratch
        if (tid < 7) T[tid] = frames[f].pose[tid];
        __syncthreads();
        // ---- optimizer.initializeOptimization(0); optimizer.optimize(10)
        int active = 0;
        for (int e = tid; e < n; e += kPT) active += lev[e] == 0;
        active = __syncthreads_or(active);
        for (int it = 0; it < 10 && active; ++it) {
            // computeActiveErrors + buildSystem at T
            double acc[kNV];
#pragma unroll
            for (int k = 0; k < kNV; ++k) acc[k] = 0;
            for (int e = tid; e < n; e += kPT) {
                if (lev[e]) continue;
                const orb_pose_edge_t Ed = E[e];
                double Xc[3];
                EdgeEval ev;
                pose_edge_error(Ed, T, cam, Xc, ev);
                double rho1;
                acc[27] += robust_rho(ev, robust, hub, rho1);
                const double x = Xc[0], y = Xc[1], z = Xc[2], fx = cam.fx, fy = cam.fy;
                double B[18];
                if (!Ed.stereo) {
                    const double j00 = -(fx / z), j02 = -(-fx * x / (z * z)), j11 = -(fy / z), j12 = -(-fy * y / (z * z));
                    B[0] = j02 * y;  B[1] = j00 * z - j02 * x; B[2] = -j00 * y; B[3] = j00; B[4] = 0;   B[5] = j02;
                    B[6] = -j11 * z + j12 * y; B[7] = -j12 * x; B[8] = j11 * x;  B[9] = 0;  B[10] = j11; B[11] = j12;
                    for (int k = 12; k < 18; ++k) B[k] = 0;
                } else {
                    const double bf = cam.bf, invz = 1.0 / z, invz_2 = invz * invz;
                    B[0] = x * y * invz_2 * fx;    B[1] = -(1 + (x * x * invz_2)) * fx; B[2] = y * invz * fx;
                    B[3] = -invz * fx;             B[4] = 0;                            B[5] = x * invz_2 * fx;
                    B[6] = (1 + y * y * invz_2) * fy; B[7] = -x * y * invz_2 * fy;      B[8] = -x * invz * fy;
                    B[9] = 0;                      B[10] = -invz * fy;                  B[11] = y * invz_2 * fy;
                    B[12] = B[0] - bf * y * invz_2; B[13] = B[1] + bf * x * invz_2;     B[14] = B[2];
                    B[15] = B[3];                  B[16] = 0;                           B[17] = B[5] - bf * invz_2;
                }
                const double info = (double)Ed.inv_sigma2, w = rho1 * info;
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
            }
            block_reduce<kNV>(acc, red);
            if (tid == 0) {
                int k = 0;
                for (int i = 0; i < 6; ++i)
                    for (int j = i; j < 6; ++j) H[6 * i + j] = H[6 * j + i] = acc[k++];
                for (int i = 0; i < 6; ++i) bvec[i] = acc[21 + i];
                s_current = s_ini = acc[27];
                if (it == 0) {  // computeLambdaInit: tau * max |diag H|
                    double m = 0;
                    for (int i = 0; i < 6; ++i) m = fmax(fabs(H[7 * i]), m);
                    s_lambda = 1e-5 * m;
                    s_ni = 2;
                    s_nbad = 0;
                }
                s_qmax = 0;
                s_trial_go = 1;
            }
            __syncthreads();
            double rho = 0;
            while (s_trial_go) {
                __shared__ int s_ok2;
                __shared__ double s_x[6];
                if (tid == 0) {
                    for (int i = 0; i < 7; ++i) Tb[i] = T[i];
                    double A[36];
                    for (int i = 0; i < 36; ++i) A[i] = H[i];
                    for (int i = 0; i < 6; ++i) A[7 * i] += s_lambda;
                    double x[6];
                    s_ok2 = ldlt6(A, bvec, x);
                    if (!s_ok2) for (int i = 0; i < 6; ++i) x[i] = 0;
                    for (int i = 0; i < 6; ++i) s_x[i] = x[i];
                    double Tn[7];
                    for (int i = 0; i < 7; ++i) Tn[i] = T[i];
                    se3_oplus(Tn, x);
                    for (int i = 0; i < 7; ++i) T[i] = Tn[i];
                }
                __syncthreads();
                double tc[1] = {0};
                for (int e = tid; e < n; e += kPT) {
                    if (lev[e]) continue;
                    double Xc[3];
                    EdgeEval ev;
                    pose_edge_error(E[e], T, cam, Xc, ev);
                    ech[e] = ev.chi2;  // the last evaluated state's chi2 (read by the classification)
                    double rho1;
                    tc[0] += robust_rho(ev, robust, hub, rho1);
                }
                block_reduce<1>(tc, red);
                if (tid == 0) {
                    double tempChi = tc[0];
                    if (!s_ok2) tempChi = DBL_MAX;
                    double r = s_current - tempChi;
                    double scale = 0;
                    for (int i = 0; i < 6; ++i) scale += s_x[i] * (s_lambda * s_x[i] + bvec[i]);
                    scale += 1e-3;
                    r /= scale;
                    if (r > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * r - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        s_lambda *= fmax(1. / 3., alpha);
                        s_ni = 2;
                        s_current = tempChi;
                    } else {
                        s_lambda *= s_ni;
                        s_ni *= 2;
                        for (int i = 0; i < 7; ++i) T[i] = Tb[i];
                    }
                    s_qmax++;
                    s_temp = r;
                    s_trial_go = (r < 0 && s_qmax < 10);
                }
                __syncthreads();
                rho = s_temp;
            }
            // termination (uniform: every thread read the same shared values)
            if (s_qmax == 10 || rho == 0) break;
            if (tid == 0) {
                if ((s_ini - s_current) * 1e3 < s_ini) s_nbad++;
                else s_nbad = 0;
                s_go = s_nbad < 3;
            }
            __syncthreads();
            if (!s_go) break;
        }
        __syncthreads();
        // ---- re-classification (src/Optimizer.cc:285-386)
        int bad = 0;
        for (int e = tid; e < n; e += kPT) {
            double c2;
            if (lev[e]) {
                double Xc[3];
                EdgeEval ev;
                pose_edge_error(E[e], T, cam, Xc, ev);
                c2 = ev.chi2;
            } else {
                c2 = ech[e];
            }
            const float chi2 = (float)c2;
            const bool out = chi2 > (E[e].stereo ? 7.815f : 5.991f);
            lev[e] = out;
            bad += out;
        }
        {
            double nb[1] = {(double)bad};
            block_reduce<1>(nb, red);
            nBad = (int)nb[0];
        }
        if (round == 2) robust = false;
        if (n < 10) break;  // optimizer.edges().size() < 10
    }
    __syncthreads();
    if (tid < 7) pose_out[7 * (size_t)f + tid] = T[tid];
    if (tid == 0) inliers[f] = n - nBad;
}

std::mutex g_mu;
double* g_chi = nullptr;
size_t g_chi_cap = 0;

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
    std::lock_guard<std::mutex> lk(g_mu);
    const size_t need = std::max<size_t>(1, (size_t)n_edges);
    if (need > g_chi_cap) {
        if (g_chi) (void)hipFree(g_chi);
        g_chi = nullptr;
        g_chi_cap = 0;
        if (hipMalloc(&g_chi, need * sizeof(double)) != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "hipMalloc failed");
        g_chi_cap = need;
    }
    hipLaunchKernelGGL(k_pose_opt, dim3(n_frames), dim3(kPT), 0, (hipStream_t)stream, d_frames, d_edges, d_pose_out,
                       d_outlier, d_inliers, g_chi, make_huber());
    if (hipGetLastError() != hipSuccess) return orbgpu_fail(ORB_ERR_DEVICE, "pose kernel launch failed");
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
