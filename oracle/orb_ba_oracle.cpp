// ORACLE -- TEST INFRASTRUCTURE ONLY.  CPU restatement (double precision, single thread) of the
// optimisation ORB_SLAM3::Optimizer::LocalBundleAdjustment runs (src/Optimizer.cc:1740-2188) on the
// g2o it vendors: SparseOptimizer::initializeOptimization/optimize (core/sparse_optimizer.cpp),
// OptimizationAlgorithmLevenberg::solve (core/optimization_algorithm_levenberg.cpp:61-194),
// BlockSolver_6_3 buildSystem / setLambda / Schur solve (core/block_solver.hpp:143-560),
// BaseBinaryEdge::constructQuadraticForm (core/base_binary_edge.hpp:55-120), RobustKernelHuber
// (core/robust_kernel_impl.cpp:65-91), EdgeSE3ProjectXYZ (include/OptimizableTypes.h:108-121,
// src/OptimizableTypes.cpp:175-197, src/CameraModels/Pinhole.cpp:47-54,119-130),
// EdgeStereoSE3ProjectXYZ (types/types_six_dof_expmap.h:156-172, .cpp:190-274) and SE3Quat
// (types/se3quat.h).  Only tests/ and bench.py's cpu_baseline use it.
//
// Summation orders follow g2o (edges in id order into each vertex, landmarks in order into the
// Schur complement).  Eigen's SimplicialLDLT with AMD ordering is replaced by a dense LDL^T of the
// same matrix (same solution up to rounding; it fails only on a zero pivot, as Eigen reports).
// Eigen SIMD code paths (quaternion product, small products) are restated as scalar formulas, so
// agreement with a real g2o build is to rounding, not bitwise: parity is judged at 1e-6 RMSE.
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

void inverse3(const double m[9], double out[9]) {  // Eigen closed-form 3x3 inverse
    auto at = [&](int r, int c) { return m[3 * r + c]; };
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return at(i1, j1) * at(i2, j2) - at(i1, j2) * at(i2, j1);
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double det = c0 * at(0, 0) + c1 * at(1, 0) + c2 * at(2, 0);
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out[3 * i + j] = cof(j, i) * invdet;
}

struct Problem {
    const orb_ba_problem_t& p;
    std::vector<SE3> pose;
    std::vector<double> point;  // 3 per point
    std::vector<int> pose_hidx;   // -1 fixed / inactive
    std::vector<int> point_lidx;  // landmark index or -1
    int n_free = 0, n_land = 0;
    std::vector<double> err;      // 3 per edge
    Huber hmono{(float)std::sqrt(5.991)}, hstereo{(float)std::sqrt(7.815)};  // const float thHuber = sqrt(double) (src/Optimizer.cc:1957-1958)
    explicit Problem(const orb_ba_problem_t& pr) : p(pr) {}
};

void compute_error(Problem& P, int e) {
    const orb_ba_edge_t& E = P.p.edges[e];
    const orb_ba_camera_t& cam = P.p.pose_camera[E.pose];
    double Xc[3];
    P.pose[E.pose].map(&P.point[3 * E.point], Xc);
    double* er = &P.err[3 * e];
    if (!E.stereo) {  // obs - Pinhole::project (double path, float parameters)
        const double u = (double)cam.fx * Xc[0] / Xc[2] + (double)cam.cx;
        const double v = (double)cam.fy * Xc[1] / Xc[2] + (double)cam.cy;
        er[0] = E.obs[0] - u;
        er[1] = E.obs[1] - v;
        er[2] = 0;
    } else {  // EdgeStereoSE3ProjectXYZ::cam_project: float invz, float bf
        const float invz = (float)(1.0f / Xc[2]);
        const float bf = (float)(double)cam.bf;
        const double u = Xc[0] * invz * (double)cam.fx + (double)cam.cx;
        const double v = Xc[1] * invz * (double)cam.fy + (double)cam.cy;
        const double ur = u - (double)(bf * invz);
        er[0] = E.obs[0] - u;
        er[1] = E.obs[1] - v;
        er[2] = E.obs[2] - ur;
    }
}

double edge_chi2(const Problem& P, int e) {
    const orb_ba_edge_t& E = P.p.edges[e];
    const double* er = &P.err[3 * e];
    const double info = (double)E.inv_sigma2;
    double c = er[0] * info * er[0] + er[1] * info * er[1];
    if (E.stereo) c += er[2] * info * er[2];
    return c;
}

double robust_chi2(const Problem& P) {  // SparseOptimizer::activeRobustChi2
    double chi = 0;
    double rho[3];
    for (int e = 0; e < P.p.n_edges; ++e) {
        (P.p.edges[e].stereo ? P.hstereo : P.hmono).robustify(edge_chi2(P, e), rho);
        chi += rho[0];
    }
    return chi;
}

// EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::linearizeOplus: A = d e / d point (D x 3),
// B = d e / d pose (D x 6, rotation first)
void linearize(const Problem& P, int e, double A[9], double B[18]) {
    const orb_ba_edge_t& E = P.p.edges[e];
    const orb_ba_camera_t& cam = P.p.pose_camera[E.pose];
    const SE3& T = P.pose[E.pose];
    double Xc[3];
    T.map(&P.point[3 * E.point], Xc);
    double R[9];
    qmatrix(T.r, R);
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double fx = cam.fx, fy = cam.fy;
    if (!E.stereo) {
        // -Pinhole::projectJac
        const double J[6] = {-(fx / z), -0.0, -(-fx * x / (z * z)), -0.0, -(fy / z), -(-fy * y / (z * z))};
        for (int r = 0; r < 2; ++r)
            for (int c = 0; c < 3; ++c) A[3 * r + c] = J[3 * r] * R[c] + J[3 * r + 1] * R[3 + c] + J[3 * r + 2] * R[6 + c];
        const double D[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
        for (int r = 0; r < 2; ++r)
            for (int c = 0; c < 6; ++c)
                B[6 * r + c] = J[3 * r] * D[c] + J[3 * r + 1] * D[6 + c] + J[3 * r + 2] * D[12 + c];
    } else {
        const double bf = cam.bf, z2 = z * z;
        for (int c = 0; c < 3; ++c) {
            A[c] = -fx * R[c] / z + fx * x * R[6 + c] / z2;
            A[3 + c] = -fy * R[3 + c] / z + fy * y * R[6 + c] / z2;
            A[6 + c] = A[c] - bf * R[6 + c] / z2;
        }
        B[0] = x * y / z2 * fx; B[1] = -(1 + (x * x / z2)) * fx; B[2] = y / z * fx;
        B[3] = -1. / z * fx;    B[4] = 0;                        B[5] = x / z2 * fx;
        B[6] = (1 + y * y / z2) * fy; B[7] = -x * y / z2 * fy; B[8] = -x / z * fy;
        B[9] = 0;                     B[10] = -1. / z * fy;    B[11] = y / z2 * fy;
        B[12] = B[0] - bf * y / z2; B[13] = B[1] + bf * x / z2; B[14] = B[2];
        B[15] = B[3];               B[16] = 0;                  B[17] = B[5] - bf / z2;
    }
}

}  // namespace

namespace {
// Test hook (oracle_local_ba_stop_after): the solve behaves as if the caller's stop flag went up right
// after trial `stop_after_trials` (0: before the first iteration).
int g_stop_after = -1;
}  // namespace

extern "C" int oracle_local_ba(orb_ba_problem_t* prob, const orb_ba_options_t* opt, double* edge_chi2_out,
                               uint8_t* depth_ok_out, orb_ba_result_t* res) {
    Problem P(*prob);
    const int np = prob->n_poses, nq = prob->n_points, ne = prob->n_edges;
    memset(res, 0, sizeof(*res));
    auto stop = [&]() {
        return (opt->stop_flag && *opt->stop_flag) || (opt->stop_flag_bool && *opt->stop_flag_bool) ||
               (g_stop_after >= 0 && res->trials >= g_stop_after);
    };
    P.pose.resize(np);
    for (int i = 0; i < np; ++i) {
        const double* v = prob->pose + 7 * i;
        P.pose[i].t[0] = v[0]; P.pose[i].t[1] = v[1]; P.pose[i].t[2] = v[2];
        P.pose[i].r = Quat{v[3], v[4], v[5], v[6]};
        normalize_rotation(P.pose[i].r);  // SE3Quat(q, t) constructor
    }
    P.point.assign(prob->point, prob->point + 3 * nq);
    P.err.assign(3 * (size_t)ne, 0.0);

    // initializeOptimization: every edge is active (points are never fixed); active vertices are
    // the ones with an edge; Hessian indices: free poses by id, then points by id (buildIndexMapping)
    std::vector<int> pose_deg(np, 0), point_deg(nq, 0);
    for (int e = 0; e < ne; ++e) { pose_deg[prob->edges[e].pose]++; point_deg[prob->edges[e].point]++; }
    std::vector<int> order(np);
    for (int i = 0; i < np; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return prob->pose_id[a] < prob->pose_id[b]; });
    P.pose_hidx.assign(np, -1);
    for (int i : order)
        if (pose_deg[i] && !prob->pose_fixed[i]) P.pose_hidx[i] = P.n_free++;
    std::vector<int> porder(nq);
    for (int i = 0; i < nq; ++i) porder[i] = i;
    std::sort(porder.begin(), porder.end(), [&](int a, int b) { return prob->point_id[a] < prob->point_id[b]; });
    P.point_lidx.assign(nq, -1);
    std::vector<int> land_point;
    for (int i : porder)
        if (point_deg[i]) { P.point_lidx[i] = P.n_land++; land_point.push_back(i); }
    if (ne == 0 || P.n_free + P.n_land == 0) {  // optimize() returns -1 without a free vertex
        for (int e = 0; e < ne; ++e) { if (edge_chi2_out) edge_chi2_out[e] = 0; }
        return 0;
    }
    if (stop()) { res->stopped = 1; return ORB_ERR_ABORTED; }

    const int n = 6 * P.n_free, m = 3 * P.n_land;
    // per landmark column of Hpl: the edges sorted by pose row (CCS structure, rows ascending)
    std::vector<std::vector<int>> land_edges(P.n_land);
    for (int e = 0; e < ne; ++e) {
        const orb_ba_edge_t& E = prob->edges[e];
        if (P.pose_hidx[E.pose] >= 0) land_edges[P.point_lidx[E.point]].push_back(e);
    }
    for (auto& v : land_edges)
        std::stable_sort(v.begin(), v.end(), [&](int a, int b) {
            return P.pose_hidx[prob->edges[a].pose] < P.pose_hidx[prob->edges[b].pose];
        });

    std::vector<double> Hpp((size_t)P.n_free * 36), Hll((size_t)P.n_land * 9), Hpl((size_t)ne * 18), b(n + m);
    std::vector<double> x(n + m), S((size_t)n * n), bs(n), coeff(n), Dinv((size_t)P.n_land * 9);
    double lambda = 0, ni = 2;
    int nBad = 0;
    const double tau = 1e-5;
    std::vector<SE3> pose_bak;
    std::vector<double> point_bak;

    int it = 0;
    for (; it < opt->iterations && !stop(); ++it) {
        // ---- computeActiveErrors, activeRobustChi2
        for (int e = 0; e < ne; ++e) compute_error(P, e);
        double currentChi = robust_chi2(P);
        const double iniChi = currentChi;
        if (it == 0) res->initial_chi2 = currentChi;
        // ---- buildSystem
        std::fill(Hpp.begin(), Hpp.end(), 0.0);
        std::fill(Hll.begin(), Hll.end(), 0.0);
        std::fill(b.begin(), b.end(), 0.0);
        for (int e = 0; e < ne; ++e) {
            const orb_ba_edge_t& E = prob->edges[e];
            const int D = E.stereo ? 3 : 2;
            double A[9], B[18], rho[3];
            linearize(P, e, A, B);
            const double info = E.inv_sigma2;
            (E.stereo ? P.hstereo : P.hmono).robustify(edge_chi2(P, e), rho);
            const double w = rho[1] * info;  // robustInformation = rho[1] * Omega
            double omr[3];
            for (int r = 0; r < D; ++r) omr[r] = -info * P.err[3 * e + r] * rho[1];
            const int li = P.point_lidx[E.point], pi = P.pose_hidx[E.pose];
            // from = point (always free), to = pose
            double* bl = &b[n + 3 * li];
            double* Hl = &Hll[9 * li];
            for (int i = 0; i < 3; ++i) {
                for (int r = 0; r < D; ++r) bl[i] += A[3 * r + i] * omr[r];
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int r = 0; r < D; ++r) s += A[3 * r + i] * w * A[3 * r + j];
                    Hl[3 * i + j] += s;
                }
            }
            if (pi >= 0) {
                double* Hx = &Hpl[18 * e];  // B^T W A, 6 x 3 (transposed block of the edge)
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 3; ++j) {
                        double s = 0;
                        for (int r = 0; r < D; ++r) s += B[6 * r + i] * w * A[3 * r + j];
                        Hx[3 * i + j] = s;
                    }
                double* bp = &b[6 * pi];
                double* Hp = &Hpp[36 * pi];
                for (int i = 0; i < 6; ++i) {
                    for (int r = 0; r < D; ++r) bp[i] += B[6 * r + i] * omr[r];
                    for (int j = 0; j < 6; ++j) {
                        double s = 0;
                        for (int r = 0; r < D; ++r) s += B[6 * r + i] * w * B[6 * r + j];
                        Hp[6 * i + j] += s;
                    }
                }
            }
        }
        if (it == 0) {  // computeLambdaInit
            if (opt->user_lambda_init > 0) {
                lambda = opt->user_lambda_init;
            } else {
                double maxDiagonal = 0;
                for (int i = 0; i < P.n_free; ++i)
                    for (int j = 0; j < 6; ++j) maxDiagonal = std::max(std::fabs(Hpp[36 * i + 7 * j]), maxDiagonal);
                for (int i = 0; i < P.n_land; ++i)
                    for (int j = 0; j < 3; ++j) maxDiagonal = std::max(std::fabs(Hll[9 * i + 4 * j]), maxDiagonal);
                lambda = tau * maxDiagonal;
            }
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            pose_bak = P.pose;  // push
            point_bak = P.point;
            // ---- setLambda + Schur complement (BlockSolver::solve)
            std::fill(S.begin(), S.end(), 0.0);
            for (int i = 0; i < P.n_free; ++i)
                for (int r = 0; r < 6; ++r)
                    for (int c = 0; c < 6; ++c)
                        S[(size_t)(6 * i + r) * n + 6 * i + c] = Hpp[36 * i + 6 * r + c] + (r == c ? lambda : 0.0);
            std::fill(coeff.begin(), coeff.end(), 0.0);
            for (int l = 0; l < P.n_land; ++l) {
                double Dm[9];
                for (int k = 0; k < 9; ++k) Dm[k] = Hll[9 * l + k] + (k % 4 == 0 ? lambda : 0.0);
                double* Di = &Dinv[9 * l];
                inverse3(Dm, Di);
                double db[3];
                for (int r = 0; r < 3; ++r)
                    db[r] = Di[3 * r] * b[n + 3 * l] + Di[3 * r + 1] * b[n + 3 * l + 1] + Di[3 * r + 2] * b[n + 3 * l + 2];
                const auto& col = land_edges[l];
                for (size_t a = 0; a < col.size(); ++a) {
                    const int i1 = P.pose_hidx[prob->edges[col[a]].pose];
                    const double* Bi = &Hpl[18 * col[a]];
                    double BDinv[18];
                    for (int r = 0; r < 6; ++r)
                        for (int c = 0; c < 3; ++c)
                            BDinv[3 * r + c] = Bi[3 * r] * Di[c] + Bi[3 * r + 1] * Di[3 + c] + Bi[3 * r + 2] * Di[6 + c];
                    for (int r = 0; r < 6; ++r)
                        coeff[6 * i1 + r] += Bi[3 * r] * db[0] + Bi[3 * r + 1] * db[1] + Bi[3 * r + 2] * db[2];
                    for (size_t bb = a; bb < col.size(); ++bb) {
                        const int i2 = P.pose_hidx[prob->edges[col[bb]].pose];
                        const double* Bj = &Hpl[18 * col[bb]];
                        for (int r = 0; r < 6; ++r)
                            for (int c = 0; c < 6; ++c)
                                S[(size_t)(6 * i1 + r) * n + 6 * i2 + c] -= BDinv[3 * r] * Bj[3 * c] +
                                                                            BDinv[3 * r + 1] * Bj[3 * c + 1] +
                                                                            BDinv[3 * r + 2] * Bj[3 * c + 2];
                    }
                }
            }
            for (int i = 0; i < n; ++i) bs[i] = b[i] - coeff[i];
            std::vector<double> xp;
            bool ok2 = true;
            if (n > 0) ok2 = ldlt_solve(S, n, bs, xp);
            if (ok2) {
                for (int i = 0; i < n; ++i) x[i] = xp[i];
                // x_l = Dinv (b_l - Hpl^T x_p)
                for (int l = 0; l < P.n_land; ++l) {
                    double cl[3] = {b[n + 3 * l], b[n + 3 * l + 1], b[n + 3 * l + 2]};
                    for (int e : land_edges[l]) {
                        const int i1 = P.pose_hidx[prob->edges[e].pose];
                        const double* Bi = &Hpl[18 * e];
                        for (int c = 0; c < 3; ++c)
                            for (int r = 0; r < 6; ++r) cl[c] += Bi[3 * r + c] * -x[6 * i1 + r];
                    }
                    const double* Di = &Dinv[9 * l];
                    for (int r = 0; r < 3; ++r)
                        x[n + 3 * l + r] = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
                }
                // ---- SparseOptimizer::update (x after the solve; on failure g2o applies a stale x)
            }
            for (int i = 0; i < np; ++i)
                if (P.pose_hidx[i] >= 0) P.pose[i] = se3_mul(se3_exp(&x[6 * P.pose_hidx[i]]), P.pose[i]);
            for (int q = 0; q < nq; ++q)
                if (P.point_lidx[q] >= 0)
                    for (int k = 0; k < 3; ++k) P.point[3 * q + k] += x[n + 3 * P.point_lidx[q] + k];
            res->trials++;
            for (int e = 0; e < ne; ++e) compute_error(P, e);
            double tempChi = robust_chi2(P);
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;  // computeScale
            for (int j = 0; j < n + m; ++j) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                P.pose = pose_bak;  // pop
                P.point = point_bak;
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
    // outputs: estimates, e->chi2() of the last computed errors, isDepthPositive of the final state
    for (int i = 0; i < np; ++i) {
        double* v = prob->pose + 7 * i;
        v[0] = P.pose[i].t[0]; v[1] = P.pose[i].t[1]; v[2] = P.pose[i].t[2];
        v[3] = P.pose[i].r.x; v[4] = P.pose[i].r.y; v[5] = P.pose[i].r.z; v[6] = P.pose[i].r.w;
    }
    memcpy(prob->point, P.point.data(), sizeof(double) * 3 * nq);
    for (int e = 0; e < ne; ++e) {
        if (edge_chi2_out) edge_chi2_out[e] = edge_chi2(P, e);
        if (depth_ok_out) {
            double Xc[3];
            P.pose[prob->edges[e].pose].map(&P.point[3 * prob->edges[e].point], Xc);
            depth_ok_out[e] = Xc[2] > 0.0;
        }
    }
    return 0;
}

// oracle_local_ba with the stop flag raised right after `stop_after_trials` LM trials (g2o polls the
// flag after each trial and before each iteration: optimization_algorithm_levenberg.cpp:149,
// sparse_optimizer.cpp:376).  Used to check a GPU solve interrupted by a real flag.
extern "C" int oracle_local_ba_stop_after(orb_ba_problem_t* prob, const orb_ba_options_t* opt, int stop_after_trials,
                                          double* edge_chi2_out, uint8_t* depth_ok_out, orb_ba_result_t* res) {
    g_stop_after = stop_after_trials;
    const int rc = oracle_local_ba(prob, opt, edge_chi2_out, depth_ok_out, res);
    g_stop_after = -1;
    return rc;
}
