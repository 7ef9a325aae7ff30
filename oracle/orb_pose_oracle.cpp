// ORACLE -- TEST INFRASTRUCTURE ONLY.  CPU restatement (double precision, single thread) of
// ORB_SLAM3::Optimizer::PoseOptimization (reference src/Optimizer.cc:55-415) on the vendored g2o:
//   - one VertexSE3Expmap, unary edges EdgeSE3ProjectXYZOnlyPose (include/OptimizableTypes.h:32-60,
//     src/OptimizableTypes.cpp:58-73, Pinhole::project / projectJac) and
//     EdgeStereoSE3ProjectXYZOnlyPose (types/types_six_dof_expmap.h:208-236, .cpp:339-404:
//     float invz, double bf), information I * invSigma2, Huber sqrt(5.991) / sqrt(7.815)
//   - BaseUnaryEdge::constructQuadraticForm (core/base_unary_edge.hpp), LinearSolverDense's LDLT
//     (solvers/linear_solver_dense.h: replaced by a dense LDL^T, same solution up to rounding)
//   - OptimizationAlgorithmLevenberg::solve (core/optimization_algorithm_levenberg.cpp:61-194) inside
//     SparseOptimizer::optimize(10), 4 rounds re-classifying outliers (src/Optimizer.cc:278-386):
//     each round restarts from the frame pose; active edges are classified on the error of the last
//     evaluated state (g2o keeps a rejected trial's errors), outliers on a fresh computeError();
//     robust kernels are dropped after round 2; the loop stops after a round if < 10 edges exist.
// Summation follows g2o's edge order.  Parity with the GPU is judged at 1e-6 pose RMSE.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/orbgpu.h"
#include "g2o_common.h"

using namespace oracle_g2o;

namespace {

struct PoseFrame {
    const orb_pose_frame_t& f;
    const orb_pose_edge_t* E;
    SE3 T;
    std::vector<double> err;  // 3 per edge: the last evaluated error
    std::vector<uint8_t> level;
    bool robust = true;
    Huber hmono{(float)std::sqrt(5.991)}, hstereo{(float)std::sqrt(7.815)};  // const float delta = sqrt(double)
    PoseFrame(const orb_pose_frame_t& fr, const orb_pose_edge_t* edges) : f(fr), E(edges + fr.edge_begin) {}
    int n() const { return f.n_edges; }

    void compute_error(int e) {  // EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose::computeError
        const orb_pose_edge_t& ed = E[e];
        double Xc[3];
        T.map(ed.xw, Xc);
        double* er = &err[3 * e];
        const orb_ba_camera_t& c = f.cam;
        if (!ed.stereo) {  // Pinhole::project(Vector3d): float parameters promoted
            er[0] = ed.obs[0] - ((double)c.fx * Xc[0] / Xc[2] + (double)c.cx);
            er[1] = ed.obs[1] - ((double)c.fy * Xc[1] / Xc[2] + (double)c.cy);
            er[2] = 0;
        } else {  // cam_project: const float invz = 1.0f / z; double fx, fy, cx, cy, bf members
            const float invz = (float)(1.0f / Xc[2]);
            const double u = Xc[0] * invz * (double)c.fx + (double)c.cx;
            const double v = Xc[1] * invz * (double)c.fy + (double)c.cy;
            er[0] = ed.obs[0] - u;
            er[1] = ed.obs[1] - v;
            er[2] = ed.obs[2] - (u - (double)c.bf * invz);
        }
    }
    double chi2(int e) const {
        const double* er = &err[3 * e];
        const double info = (double)E[e].inv_sigma2;
        double c = er[0] * info * er[0] + er[1] * info * er[1];
        if (E[e].stereo) c += er[2] * info * er[2];
        return c;
    }
    double robust_chi2() const {  // SparseOptimizer::activeRobustChi2 (level-0 edges)
        double s = 0, rho[3];
        for (int e = 0; e < n(); ++e) {
            if (level[e]) continue;
            if (robust) {
                (E[e].stereo ? hstereo : hmono).robustify(chi2(e), rho);
                s += rho[0];
            } else {
                s += chi2(e);
            }
        }
        return s;
    }
    void compute_active_errors() {
        for (int e = 0; e < n(); ++e)
            if (!level[e]) compute_error(e);
    }
    // d e / d pose (D x 6, rotation first)
    void jacobian(int e, double B[18]) const {
        const orb_pose_edge_t& ed = E[e];
        double Xc[3];
        T.map(ed.xw, Xc);
        const double x = Xc[0], y = Xc[1], z = Xc[2];
        const double fx = f.cam.fx, fy = f.cam.fy;
        if (!ed.stereo) {  // -projectJac * SE3deriv, src/OptimizableTypes.cpp:58-73
            const double J[6] = {-(fx / z), -0.0, -(-fx * x / (z * z)), -0.0, -(fy / z), -(-fy * y / (z * z))};
            const double D[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
            for (int r = 0; r < 2; ++r)
                for (int c = 0; c < 6; ++c)
                    B[6 * r + c] = J[3 * r] * D[c] + J[3 * r + 1] * D[6 + c] + J[3 * r + 2] * D[12 + c];
            for (int c = 12; c < 18; ++c) B[c] = 0;
        } else {  // types_six_dof_expmap.cpp:375-404
            const double bf = f.cam.bf, invz = 1.0 / z, invz_2 = invz * invz;
            B[0] = x * y * invz_2 * fx;    B[1] = -(1 + (x * x * invz_2)) * fx; B[2] = y * invz * fx;
            B[3] = -invz * fx;             B[4] = 0;                            B[5] = x * invz_2 * fx;
            B[6] = (1 + y * y * invz_2) * fy; B[7] = -x * y * invz_2 * fy;      B[8] = -x * invz * fy;
            B[9] = 0;                      B[10] = -invz * fy;                  B[11] = y * invz_2 * fy;
            B[12] = B[0] - bf * y * invz_2; B[13] = B[1] + bf * x * invz_2;     B[14] = B[2];
            B[15] = B[3];                  B[16] = 0;                           B[17] = B[5] - bf * invz_2;
        }
    }
    // BaseUnaryEdge::constructQuadraticForm over the active edges (errors already current)
    void build(double H[36], double b[6]) const {
        for (int k = 0; k < 36; ++k) H[k] = 0;
        for (int k = 0; k < 6; ++k) b[k] = 0;
        for (int e = 0; e < n(); ++e) {
            if (level[e]) continue;
            double B[18];
            jacobian(e, B);
            const int D = E[e].stereo ? 3 : 2;
            const double info = (double)E[e].inv_sigma2;
            double rho1 = 1.0;
            if (robust) {
                double rho[3];
                (E[e].stereo ? hstereo : hmono).robustify(chi2(e), rho);
                rho1 = rho[1];
            }
            const double* er = &err[3 * e];
            for (int i = 0; i < 6; ++i) {
                for (int j = 0; j < 6; ++j) {
                    double s = 0;
                    for (int r = 0; r < D; ++r) s += B[6 * r + i] * (rho1 * info) * B[6 * r + j];
                    H[6 * i + j] += s;
                }
                double bs = 0;
                for (int r = 0; r < D; ++r) bs += B[6 * r + i] * info * er[r];
                b[i] -= rho1 * bs;
            }
        }
    }

    // SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg
    void optimize(int iterations) {
        bool any = false;
        for (int e = 0; e < n(); ++e) any |= !level[e];
        if (!any) return;  // no active vertex: optimize() returns at once
        double lambda = 0, ni = 2;
        int nbad = 0;
        for (int it = 0; it < iterations; ++it) {
            compute_active_errors();
            double currentChi = robust_chi2();
            const double iniChi = currentChi;
            double H[36], b[6];
            build(H, b);
            if (it == 0) {  // computeLambdaInit: tau * max |diag H|, tau = 1e-5
                double m = 0;
                for (int k = 0; k < 6; ++k) m = std::max(std::fabs(H[7 * k]), m);
                lambda = 1e-5 * m;
                ni = 2;
                nbad = 0;
            }
            double rho = 0;
            int qmax = 0;
            do {
                const SE3 backup = T;
                std::vector<double> S(H, H + 36), bv(b, b + 6), x(6);
                for (int k = 0; k < 6; ++k) S[7 * k] += lambda;
                const bool ok2 = ldlt_solve(S, 6, bv, x);
                T = se3_mul(se3_exp(x.data()), T);
                compute_active_errors();
                double tempChi = robust_chi2();
                if (!ok2) tempChi = std::numeric_limits<double>::max();
                rho = currentChi - tempChi;
                double scale = 0;
                for (int k = 0; k < 6; ++k) scale += x[k] * (lambda * x[k] + b[k]);
                scale += 1e-3;
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
                    T = backup;
                }
                qmax++;
            } while (rho < 0 && qmax < 10);
            if (qmax == 10 || rho == 0) return;  // Terminate
            if ((iniChi - currentChi) * 1e3 < iniChi) nbad++;
            else nbad = 0;
            if (nbad >= 3) return;
        }
    }
};

}  // namespace

extern "C" int oracle_pose_optimization(int n_frames, const orb_pose_frame_t* frames, const orb_pose_edge_t* edges,
                                        double* pose_out, uint8_t* outlier, int32_t* inliers) {
    for (int fi = 0; fi < n_frames; ++fi) {
        const orb_pose_frame_t& F = frames[fi];
        PoseFrame P(F, edges);
        const double* p0 = F.pose;
        SE3 T0;
        T0.t[0] = p0[0]; T0.t[1] = p0[1]; T0.t[2] = p0[2];
        T0.r = Quat{p0[3], p0[4], p0[5], p0[6]};
        const int n = F.n_edges;
        P.err.assign(3 * (size_t)n, 0.0);
        P.level.assign(n, 0);
        for (int e = 0; e < n; ++e) outlier[F.edge_begin + e] = 0;  // mvbOutlier[i] = false at edge creation
        for (int k = 0; k < 7; ++k) pose_out[7 * fi + k] = p0[k];
        if (n < 3) {  // nInitialCorrespondences < 3: return 0, pose untouched
            inliers[fi] = 0;
            continue;
        }
        const float chi2Mono[4] = {5.991, 5.991, 5.991, 5.991};
        const float chi2Stereo[4] = {7.815, 7.815, 7.815, 7.815};
        int nBad = 0;
        for (int it = 0; it < 4; ++it) {
            P.T = T0;  // vSE3->setEstimate(pFrame->GetPose())
            P.optimize(10);
            nBad = 0;
            // mono edges first, then stereo (the reference's two loops; classification is per edge)
            for (int pass = 0; pass < 2; ++pass)
                for (int e = 0; e < n; ++e) {
                    if (P.E[e].stereo != pass) continue;
                    if (P.level[e]) P.compute_error(e);
                    const float chi2 = (float)P.chi2(e);
                    if (chi2 > (pass ? chi2Stereo[it] : chi2Mono[it])) {
                        P.level[e] = 1;
                        nBad++;
                    } else {
                        P.level[e] = 0;
                    }
                }
            if (it == 2) P.robust = false;
            if (n < 10) break;  // optimizer.edges().size() < 10
        }
        const double out[7] = {P.T.t[0], P.T.t[1], P.T.t[2], P.T.r.x, P.T.r.y, P.T.r.z, P.T.r.w};
        for (int k = 0; k < 7; ++k) pose_out[7 * fi + k] = out[k];
        for (int e = 0; e < n; ++e) outlier[F.edge_begin + e] = P.level[e];
        inliers[fi] = n - nBad;
    }
    return 0;
}
