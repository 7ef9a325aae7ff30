/*
 * orbgpu_optimizer.hpp -- header-only drop-in for ORB_SLAM3::Optimizer::LocalBundleAdjustment
 * (include/Optimizer.h:57, src/Optimizer.cc:1740-2188) on top of the C ABI (orbgpu.h).
 *
 * The reference keeps the graph gather (B1) and the culling / write-back (B10) on the host and only
 * the g2o solve (initializeOptimization + optimize(10), src/Optimizer.cc:2099-2100) moves to the GPU
 * through orb_ba_optimize.  This header restates B1 and B10 over an accessor type A, so that the
 * same code runs on the reference's KeyFrame / MapPoint / Map (orbgpu::ORBSLAM3Access below, compiled
 * inside the reference build) and on a mock graph in this repository's CPU tests
 * (tests/native/local_ba_shim_check.cpp):
 *
 *   struct A {
 *     using KeyFrame = ...; using MapPoint = ...; using Map = ...;
 *     // graph reads
 *     static unsigned long Id(KeyFrame*);  static unsigned long Id(MapPoint*);        // mnId
 *     static unsigned long& BALocalForKF(KeyFrame*); static unsigned long& BAFixedForKF(KeyFrame*);
 *     static unsigned long& BALocalForKF(MapPoint*);                                  // mnBA*ForKF marks
 *     static bool IsBad(KeyFrame*);  static bool IsBad(MapPoint*);
 *     static Map* GetMap(KeyFrame*); static Map* GetMap(MapPoint*);
 *     static std::vector<KeyFrame*> Covisible(KeyFrame*);        // GetVectorCovisibleKeyFrames()
 *     static std::vector<MapPoint*> MapPointMatches(KeyFrame*);  // GetMapPointMatches()
 *     static std::map<KeyFrame*, std::tuple<int, int>> Observations(MapPoint*);
 *     static unsigned long InitKFid(Map*);  static bool IsInertial(Map*);
 *     static bool HasCamera2(KeyFrame*);                         // mpCamera2 != NULL
 *     static void Pose(KeyFrame*, double q_xyzw[4], double t[3]);  // GetPose(): unit_quaternion, translation
 *     static orb_ba_camera_t Camera(KeyFrame*);                   // fx, fy, cx, cy, mbf
 *     static float URight(KeyFrame*, int idx);                    // mvuRight[idx]
 *     static void KeyUn(KeyFrame*, int idx, double* x, double* y, int* octave);  // mvKeysUn[idx]
 *     static float InvLevelSigma2(KeyFrame*, int octave);         // mvInvLevelSigma2[octave]
 *     static void WorldPos(MapPoint*, double X[3]);               // GetWorldPos().cast<double>()
 *     // writes (B10)
 *     static void DebugWindow(Map*, const std::set<unsigned long>& opt, const std::set<unsigned long>& fixed);
 *     static std::mutex& MapUpdateMutex(Map*);                    // mMutexMapUpdate
 *     static void EraseObservation(KeyFrame*, MapPoint*);         // EraseMapPointMatch + EraseObservation
 *     static void SetPose(KeyFrame*, const double q_xyzw[4], const double t[3]);
 *     static void SetWorldPos(MapPoint*, const double X[3]);      // SetWorldPos + UpdateNormalAndDepth
 *     static void IncreaseChangeIndex(Map*);
 *   };
 *
 * The two-camera fisheye rig (KeyFrame::mpCamera2, EdgeSE3ProjectXYZToBody) is outside this path:
 * Gather reports kCamera2, and LocalBundleAdjustment returns kFallback (1) so that the caller runs the
 * reference's own body.  So does a window the device cannot take or a device failure.  Before such a
 * return every mnBALocalForKF / mnBAFixedForKF mark Gather wrote is restored to its previous value:
 * the reference body sets and tests the same marks (src/Optimizer.cc:1748-1803) and would otherwise
 * find every neighbour already marked, collect no local map point and no fixed keyframe, and stop at
 * "LBA aborted" (:1851-1855).
 */
#ifndef ORBGPU_OPTIMIZER_HPP
#define ORBGPU_OPTIMIZER_HPP

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <list>
#include <map>
#include <mutex>
#include <chrono>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "orbgpu.h"

namespace orbgpu {

// Thresholds of the reference (src/Optimizer.cc:1957-1958, 2115, 2145).
constexpr double kChi2Mono = 5.991, kChi2Stereo = 7.815;

// One LocalBundleAdjustment window, flattened into orb_ba_problem_t arrays in the reference's order.
template <class A>
struct LocalBAWindow {
    using KF = typename A::KeyFrame;
    using MP = typename A::MapPoint;
    enum Status { kOk = 0, kNoFixed = 1, kCamera2 = 2 };

    std::vector<KF*> local_kfs;   // lLocalKeyFrames (pKF first, then its covisible KFs)
    std::vector<KF*> fixed_kfs;   // lFixedCameras
    std::vector<MP*> local_mps;   // lLocalMapPoints
    unsigned long max_kf_id = 0;  // maxKFid (src/Optimizer.cc:1876-1915)
    int num_fixed_kf = 0;

    // vertices: local KFs then fixed KFs (addVertex order), then points; edges in addEdge order
    std::vector<double> pose;                 // [7] per KF: SE3Quat::toVector (tx ty tz qx qy qz qw)
    std::vector<int64_t> pose_id;             // KeyFrame::mnId
    std::vector<uint8_t> pose_fixed;          // setFixed
    std::vector<orb_ba_camera_t> pose_camera;
    std::vector<double> point;                // [3] per point
    std::vector<int64_t> point_id;            // mnId + maxKFid + 1
    std::vector<orb_ba_edge_t> edges;
    std::vector<KF*> edge_kf;                 // vpEdgeKFMono / vpEdgeKFStereo, per edge
    std::vector<MP*> edge_mp;                 // vpMapPointEdgeMono / vpMapPointEdgeStereo, per edge
    // every mark Gather wrote, with its value before (restored in reverse order by RestoreMarks)
    std::vector<std::pair<unsigned long*, unsigned long>> mark_log;

    void Mark(unsigned long& m, unsigned long v) {
        mark_log.emplace_back(&m, m);
        m = v;
    }
    // Undo Gather's marks, so that the reference body can build the same window itself.
    void RestoreMarks() {
        for (auto it = mark_log.rbegin(); it != mark_log.rend(); ++it) *it->first = it->second;
        mark_log.clear();
    }

    orb_ba_problem_t Problem() {
        orb_ba_problem_t p{};
        p.n_poses = (int32_t)pose_id.size();
        p.n_points = (int32_t)point_id.size();
        p.n_edges = (int32_t)edges.size();
        p.pose = pose.data();
        p.pose_id = pose_id.data();
        p.pose_fixed = pose_fixed.data();
        p.pose_camera = pose_camera.data();
        p.point = point.data();
        p.point_id = point_id.data();
        p.edges = edges.data();
        return p;
    }

    // B1: src/Optimizer.cc:1744-1855 (window), 1884-2092 (vertices and edges)
    Status Gather(KF* pKF, typename A::Map* pMap) {
        *this = LocalBAWindow();
        const unsigned long kfid = A::Id(pKF);
        // local keyframes: pKF and its covisible keyframes (:1744-1760); the mark is set before the
        // bad / other-map test, so such a neighbour is neither local nor fixed
        local_kfs.push_back(pKF);
        Mark(A::BALocalForKF(pKF), kfid);
        auto* cur_map = A::GetMap(pKF);
        for (KF* pKFi : A::Covisible(pKF)) {
            Mark(A::BALocalForKF(pKFi), kfid);
            if (!A::IsBad(pKFi) && A::GetMap(pKFi) == cur_map) local_kfs.push_back(pKFi);
        }
        // local map points (:1762-1789)
        num_fixed_kf = 0;
        for (KF* pKFi : local_kfs) {
            if (A::Id(pKFi) == A::InitKFid(pMap)) num_fixed_kf = 1;
            for (MP* pMP : A::MapPointMatches(pKFi)) {
                if (!pMP || A::IsBad(pMP) || A::GetMap(pMP) != cur_map) continue;
                if (A::BALocalForKF(pMP) != kfid) {
                    local_mps.push_back(pMP);
                    Mark(A::BALocalForKF(pMP), kfid);
                }
            }
        }
        // fixed keyframes: observers of the local points outside the window (:1791-1808)
        for (MP* pMP : local_mps)
            for (const auto& ob : A::Observations(pMP)) {
                KF* pKFi = ob.first;
                if (A::BALocalForKF(pKFi) != kfid && A::BAFixedForKF(pKFi) != kfid) {
                    Mark(A::BAFixedForKF(pKFi), kfid);
                    if (!A::IsBad(pKFi) && A::GetMap(pKFi) == cur_map) fixed_kfs.push_back(pKFi);
                }
            }
        num_fixed_kf += (int)fixed_kfs.size();  // (:1810)
        if (num_fixed_kf == 0) return kNoFixed;  // "LBA aborted" (:1851-1855)
        for (KF* k : local_kfs)
            if (A::HasCamera2(k)) return kCamera2;
        for (KF* k : fixed_kfs)
            if (A::HasCamera2(k)) return kCamera2;

        // keyframe vertices (:1882-1915): local (fixed only if it is the map's initial KF), then fixed
        std::map<KF*, int> pose_index;
        auto add_kf = [&](KF* k, bool fixed) {
            double q[4], t[3];
            A::Pose(k, q, t);
            pose_index[k] = (int)pose_id.size();
            pose.insert(pose.end(), {t[0], t[1], t[2], q[0], q[1], q[2], q[3]});
            pose_id.push_back((int64_t)A::Id(k));
            pose_fixed.push_back(fixed ? 1 : 0);
            pose_camera.push_back(A::Camera(k));
            if (A::Id(k) > max_kf_id) max_kf_id = A::Id(k);
        };
        for (KF* k : local_kfs) add_kf(k, A::Id(k) == A::InitKFid(pMap));
        for (KF* k : fixed_kfs) add_kf(k, true);
        // point vertices and their edges (:1964-2091): observations in std::map order
        for (MP* pMP : local_mps) {
            double X[3];
            A::WorldPos(pMP, X);
            const int pi = (int)point_id.size();
            point.insert(point.end(), {X[0], X[1], X[2]});
            point_id.push_back((int64_t)(A::Id(pMP) + max_kf_id + 1));
            for (const auto& ob : A::Observations(pMP)) {
                KF* pKFi = ob.first;
                if (A::IsBad(pKFi) || A::GetMap(pKFi) != cur_map) continue;
                const int left = std::get<0>(ob.second);
                if (left == -1) continue;
                const auto it = pose_index.find(pKFi);
                if (it == pose_index.end()) continue;  // (cannot happen: every such observer is a vertex)
                double x, y;
                int octave;
                A::KeyUn(pKFi, left, &x, &y, &octave);
                const float ur = A::URight(pKFi, left);
                orb_ba_edge_t e{};
                e.point = pi;
                e.pose = it->second;
                e.stereo = ur >= 0 ? 1 : 0;  // mono (:1991) / stereo (:2018)
                e.inv_sigma2 = A::InvLevelSigma2(pKFi, octave);
                e.obs[0] = x;
                e.obs[1] = y;
                e.obs[2] = e.stereo ? (double)ur : 0.0;
                edges.push_back(e);
                edge_kf.push_back(pKFi);
                edge_mp.push_back(pMP);
            }
        }
        return kOk;
    }

    // B10: src/Optimizer.cc:2102-2187.  chi2 / depth_ok per edge (orb_ba_optimize's outputs); the
    // problem's pose / point arrays hold the optimised estimates.
    void CullAndWriteBack(typename A::Map* pMap, const double* chi2, const uint8_t* depth_ok) {
        std::vector<std::pair<KF*, MP*>> to_erase;
        to_erase.reserve(edges.size());
        // mono edges first, then stereo edges, each in insertion order (vToErase order, :2107-2150)
        for (int pass = 0; pass < 2; ++pass)
            for (size_t i = 0; i < edges.size(); ++i) {
                if (edges[i].stereo != pass) continue;
                if (A::IsBad(edge_mp[i])) continue;
                const double th = pass ? kChi2Stereo : kChi2Mono;
                if (chi2[i] > th || !depth_ok[i]) to_erase.emplace_back(edge_kf[i], edge_mp[i]);
            }
        std::unique_lock<std::mutex> lock(A::MapUpdateMutex(pMap));  // (:2153)
        for (auto& p : to_erase) A::EraseObservation(p.first, p.second);
        for (size_t k = 0; k < local_kfs.size(); ++k)  // local keyframes only (:2169-2176)
            A::SetPose(local_kfs[k], &pose[7 * k + 3], &pose[7 * k]);
        for (size_t k = 0; k < local_mps.size(); ++k)  // (:2179-2185)
            A::SetWorldPos(local_mps[k], &point[3 * k]);
        A::IncreaseChangeIndex(pMap);
    }
};

// z of SE3Quat(q, t).map(X) > 0 (EdgeSE3ProjectXYZ::isDepthPositive, include/OptimizableTypes.h:116-120);
// T = (tx ty tz qx qy qz qw), q normalised as SE3Quat does
inline bool DepthPositive(const double* T, const double* X) {
    double x = T[3], y = T[4], z = T[5], w = T[6];
    const double nn = std::sqrt(x * x + y * y + z * z + w * w);
    x /= nn; y /= nn; z /= nn; w /= nn;
    // third row of the rotation matrix of (w, x, y, z)
    const double r20 = 2 * (x * z - w * y), r21 = 2 * (y * z + w * x), r22 = 1 - 2 * (x * x + y * y);
    return r20 * X[0] + r21 * X[1] + r22 * X[2] + T[2] > 0.0;
}

// LocalBundleAdjustment's return value when the caller must run the reference's own body.
constexpr int kFallback = 1;

// Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap, num_fixedKF, num_OptKF, num_MPs, num_edges)
// on a GPU BA handle.  Returns ORB_OK (also for the reference's silent early returns) or kFallback:
// the window holds a two-camera keyframe, or the library could not solve it (a window beyond the
// device's limits, a device error; orb_last_error() says which).  On kFallback nothing in the map has
// been changed and Gather's marks are restored, so the caller runs the reference body (:1742-2187)
// on the same arguments, as INTEGRATION.md shows; the reference is slower there, never wrong.
// num_MPs is left untouched, as in the reference.
template <class A>
int LocalBundleAdjustmentBody(orb_ba_t h, typename A::KeyFrame* pKF, bool* pbStopFlag, typename A::Map* pMap,
                              int& num_fixedKF, int& num_OptKF, int& num_edges) {
    LocalBAWindow<A> w;
    const auto st = w.Gather(pKF, pMap);
    if (st == LocalBAWindow<A>::kCamera2) {
        w.RestoreMarks();
        return kFallback;
    }
    num_fixedKF = w.num_fixed_kf;
    if (st == LocalBAWindow<A>::kNoFixed) return ORB_OK;  // the reference keeps its marks here too
    {  // DEBUG LBA sets of the current map (:1879-1880, 1896, 1914)
        std::set<unsigned long> opt, fixed;
        for (auto* k : w.local_kfs) opt.insert(A::Id(k));
        for (auto* k : w.fixed_kfs) fixed.insert(A::Id(k));
        A::DebugWindow(A::GetMap(pKF), opt, fixed);
    }
    num_OptKF = (int)w.local_kfs.size();
    num_edges = (int)w.edges.size();
    if (pbStopFlag && *pbStopFlag) return ORB_OK;  // (:2094-2096)
    orb_ba_problem_t prob = w.Problem();
    orb_ba_options_t opt{};
    opt.iterations = 10;                                         // optimizer.optimize(10)
    opt.user_lambda_init = A::IsInertial(pMap) ? 100.0 : 0.0;   // setUserLambdaInit(100) (:1867-1868)
    opt.stop_flag = nullptr;
    opt.stop_flag_bool = reinterpret_cast<const volatile uint8_t*>(pbStopFlag);
    std::vector<double> chi2(w.edges.size());
    std::vector<uint8_t> depth(w.edges.size());
    orb_ba_result_t res{};
    const int rc = orb_ba_optimize(h, &prob, &opt, chi2.data(), depth.data(), &res);
    if (rc != ORB_OK && rc != ORB_ERR_ABORTED) {  // nothing written back: the reference body takes over
        w.RestoreMarks();
        return kFallback;
    }
    // a flag raised before the first iteration: g2o's optimize() returns without an update and the
    // reference still culls and writes back the unchanged estimates
    if (rc == ORB_ERR_ABORTED) {
        // no iteration ran: the estimates are the initial ones and no edge error was ever computed
        // (g2o leaves _error as constructed), so only isDepthPositive can cull: Xc = R X + t, z > 0
        std::fill(chi2.begin(), chi2.end(), 0.0);
        for (size_t e = 0; e < w.edges.size(); ++e) {
            const double* T = &w.pose[7 * (size_t)w.edges[e].pose];
            const double* X = &w.point[3 * (size_t)w.edges[e].point];
            depth[e] = DepthPositive(T, X) ? 1 : 0;
        }
    }
    w.CullAndWriteBack(pMap, chi2.data(), depth.data());
    return ORB_OK;
}

// REGISTER_TIMES: the "LBA" sample covers the whole call as vdLBA_ms does (src/LocalMapping.cc:208-219),
// recorded when the library's timers are on (orb_timers_enabled) and the call did not fall back.
struct LbaTimer {
    const bool on = orb_timers_enabled() != 0;
    const std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    bool record = true;
    ~LbaTimer() {
        if (on && record)
            orb_timer_add("LBA", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

template <class A>
int LocalBundleAdjustment(orb_ba_t h, typename A::KeyFrame* pKF, bool* pbStopFlag, typename A::Map* pMap,
                          int& num_fixedKF, int& num_OptKF, int& /*num_MPs*/, int& num_edges) {
    LbaTimer timer;
    const int rc = LocalBundleAdjustmentBody<A>(h, pKF, pbStopFlag, pMap, num_fixedKF, num_OptKF, num_edges);
    timer.record = rc != kFallback;  // the reference body's own run is the caller's to time
    return rc;
}

}  // namespace orbgpu

// ---- the reference's own types (compile inside the ORB-SLAM3 build: define ORBGPU_WITH_ORBSLAM3 and
// include after KeyFrame.h, MapPoint.h and Map.h) --------------------------------------------------
#ifdef ORBGPU_WITH_ORBSLAM3
namespace orbgpu {

struct ORBSLAM3Access {
    using KeyFrame = ORB_SLAM3::KeyFrame;
    using MapPoint = ORB_SLAM3::MapPoint;
    using Map = ORB_SLAM3::Map;
    static unsigned long Id(KeyFrame* k) { return k->mnId; }
    static unsigned long Id(MapPoint* p) { return p->mnId; }
    static unsigned long& BALocalForKF(KeyFrame* k) { return k->mnBALocalForKF; }
    static unsigned long& BAFixedForKF(KeyFrame* k) { return k->mnBAFixedForKF; }
    static unsigned long& BALocalForKF(MapPoint* p) { return p->mnBALocalForKF; }
    static bool IsBad(KeyFrame* k) { return k->isBad(); }
    static bool IsBad(MapPoint* p) { return p->isBad(); }
    static Map* GetMap(KeyFrame* k) { return k->GetMap(); }
    static Map* GetMap(MapPoint* p) { return p->GetMap(); }
    static std::vector<KeyFrame*> Covisible(KeyFrame* k) { return k->GetVectorCovisibleKeyFrames(); }
    static std::vector<MapPoint*> MapPointMatches(KeyFrame* k) { return k->GetMapPointMatches(); }
    static std::map<KeyFrame*, std::tuple<int, int>> Observations(MapPoint* p) { return p->GetObservations(); }
    static unsigned long InitKFid(Map* m) { return m->GetInitKFid(); }
    static bool IsInertial(Map* m) { return m->IsInertial(); }
    static bool HasCamera2(KeyFrame* k) { return k->mpCamera2 != nullptr; }
    static void Pose(KeyFrame* k, double q[4], double t[3]) {
        const Sophus::SE3f Tcw = k->GetPose();
        const Eigen::Quaterniond qd = Tcw.unit_quaternion().cast<double>();
        const Eigen::Vector3d td = Tcw.translation().cast<double>();
        q[0] = qd.x(); q[1] = qd.y(); q[2] = qd.z(); q[3] = qd.w();
        t[0] = td(0); t[1] = td(1); t[2] = td(2);
    }
    static orb_ba_camera_t Camera(KeyFrame* k) { return {k->fx, k->fy, k->cx, k->cy, k->mbf}; }
    static float URight(KeyFrame* k, int i) { return k->mvuRight[i]; }
    static void KeyUn(KeyFrame* k, int i, double* x, double* y, int* octave) {
        const cv::KeyPoint& kp = k->mvKeysUn[i];
        *x = kp.pt.x; *y = kp.pt.y; *octave = kp.octave;
    }
    static float InvLevelSigma2(KeyFrame* k, int octave) { return k->mvInvLevelSigma2[octave]; }
    static void WorldPos(MapPoint* p, double X[3]) {
        const Eigen::Vector3d x = p->GetWorldPos().cast<double>();
        X[0] = x(0); X[1] = x(1); X[2] = x(2);
    }
    static void DebugWindow(Map* m, const std::set<unsigned long>& opt, const std::set<unsigned long>& fixed) {
        m->msOptKFs = opt;
        m->msFixedKFs = fixed;
    }
    static std::mutex& MapUpdateMutex(Map* m) { return m->mMutexMapUpdate; }
    static void EraseObservation(KeyFrame* k, MapPoint* p) {
        k->EraseMapPointMatch(p);
        p->EraseObservation(k);
    }
    static void SetPose(KeyFrame* k, const double q[4], const double t[3]) {
        // Sophus::SE3f Tiw(SE3quat.rotation().cast<float>(), SE3quat.translation().cast<float>()) (:2174)
        const Eigen::Quaterniond qd(q[3], q[0], q[1], q[2]);
        k->SetPose(Sophus::SE3f(qd.cast<float>(), Eigen::Vector3d(t[0], t[1], t[2]).cast<float>()));
    }
    static void SetWorldPos(MapPoint* p, const double X[3]) {
        p->SetWorldPos(Eigen::Vector3d(X[0], X[1], X[2]).cast<float>());
        p->UpdateNormalAndDepth();
    }
    static void IncreaseChangeIndex(Map* m) { m->IncreaseChangeIndex(); }
};

}  // namespace orbgpu
#endif  // ORBGPU_WITH_ORBSLAM3

#endif  // ORBGPU_OPTIMIZER_HPP
