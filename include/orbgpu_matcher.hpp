/*
 * orbgpu_matcher.hpp -- header-only drop-in for the ORB_SLAM3::ORBmatcher methods on the GPU path
 * (include/ORBmatcher.h:40-76, src/ORBmatcher.cc) over the C ABI (orbgpu.h):
 *
 *   ORBmatcher(float nnratio = 0.6, bool checkOri = true)                       (:41)
 *   static int DescriptorDistance(a, b)                                          (:2384-2404)
 *   int SearchForTriangulation(KeyFrame*, KeyFrame*, vector<pair<size_t,size_t>>&, bOnlyStereo, bCoarse)
 *                                                                                (:1046-1324)
 *   int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)   (:1951-2185)
 *   int SearchByProjection(Frame& F, const vector<MapPoint*>&, th, bFarPoints, thFarPoints) (:46-240)
 *
 * The class translates the reference's KeyFrame / Frame / MapPoint objects into the ABI's flat views
 * (orb_kf_view_t, orb_frame_view_t, orb_last_points_t, orb_local_points_t), calls the HIP matcher,
 * and writes the results back exactly where the reference writes them (vMatchedPairs,
 * CurrentFrame.mvpMapPoints, F.mvpMapPoints).  The object graph is reached through an accessor type A
 * so that the same code runs on the reference's classes (orbgpu::ORBSLAM3MatcherAccess below, compiled
 * inside the reference build) and on a mock graph in this repository's CPU test
 * (tests/native/matcher_shim_check.cpp):
 *
 *   struct A {
 *     using KeyFrame = ...; using Frame = ...; using MapPoint = ...;
 *     // keyframes (SearchForTriangulation)
 *     static int N(KeyFrame*);                          static const orb_keypoint_t* KeysUn(KeyFrame*);
 *     static const uint8_t* Descriptors(KeyFrame*);     static const float* URight(KeyFrame*);
 *     static std::vector<MapPoint*> MapPointMatches(KeyFrame*);
 *     static const FeatureVector& FeatVec(KeyFrame*);   // std::map<node id, std::vector<unsigned>>
 *     static void Pinhole(KeyFrame*, float K[4]);       // fx, fy, cx, cy of mpCamera
 *     static int Levels(KeyFrame*);  static const float* ScaleFactors(KeyFrame*);
 *     static const float* LevelSigma2(KeyFrame*);
 *     static orb_kf_pair_geom_t PairGeometry(KeyFrame* pKF1, KeyFrame* pKF2);   // :1054-1072
 *     static bool SingleCamera(KeyFrame*);              // mpCamera2 == NULL (and NLeft == -1)
 *     // frames (SearchByProjection)
 *     static orb_frame_view_t View(const Frame&);       // keypoints, grid, camera, levels, GetPose()
 *     static bool SingleCamera(const Frame&);           // Nleft == -1
 *     static std::vector<MapPoint*>& MapPoints(Frame&); // mvpMapPoints
 *     static const std::vector<MapPoint*>& MapPoints(const Frame&);
 *     static bool Outlier(const Frame&, int i);         // mvbOutlier[i]
 *     // map points
 *     static int Observations(MapPoint*);  static bool IsBad(MapPoint*);
 *     static void WorldPos(MapPoint*, float X[3]);  static void Descriptor(MapPoint*, uint8_t d[32]);
 *     static void Track(MapPoint*, orbgpu::TrackFields*);   // mbTrackInView, mTrackProjX/Y/XR, ...
 *   };
 *
 * Scope: pinhole single-camera frames and keyframes (the configuration the ABI covers).  For the
 * two-camera fisheye rig (mpCamera2 / Nleft != -1) Supports() is false and the caller keeps the
 * reference's CPU body.
 *
 * Failures (orbgpu_status.hpp): nothing here throws.  A library failure returns the reference's result
 * for a search that matches nothing -- 0, vMatchedPairs empty, no map point written -- and a failed
 * ComputeDistinctiveDescriptors leaves every descriptor as it was; orbgpu::LastShimError() reports it.
 */
#ifndef ORBGPU_MATCHER_HPP
#define ORBGPU_MATCHER_HPP

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_status.hpp"

namespace orbgpu {

// The tracking fields Frame::isInFrustum leaves in a map point (src/Frame.cc:667-773).
struct TrackFields {
    bool in_view = false;      // mbTrackInView
    float proj[3] = {0, 0, 0}; // mTrackProjX, mTrackProjY, mTrackProjXR
    float view_cos = 0;        // mTrackViewCos
    float depth = 0;           // mTrackDepth
    int level = 0;             // mnTrackScaleLevel
};

namespace detail {

// One device matcher handle per (thread, nnratio, checkOri): the reference constructs ORBmatcher
// objects on the stack per call site (e.g. src/LocalMapping.cc:536, src/Tracking.cc:4120), and a
// handle owns a HIP stream and staging buffers that should outlive them.
class HandleCache {
public:
    orb_matcher_t Get(float nnratio, bool check_ori) {
        const auto key = std::make_pair(nnratio, check_ori);
        auto it = handles_.find(key);
        if (it != handles_.end()) return it->second;
        orb_matcher_t h = nullptr;
        if (Failed(orb_matcher_create(nnratio, check_ori ? 1 : 0, &h), "orb_matcher_create"))
            return nullptr;  // not cached: the next call tries again
        handles_[key] = h;
        return h;
    }
    ~HandleCache() {
        for (auto& kv : handles_) orb_matcher_destroy(kv.second);
    }

private:
    std::map<std::pair<float, bool>, orb_matcher_t> handles_;
};

inline orb_matcher_t ThreadHandle(float nnratio, bool check_ori) {
    thread_local HandleCache cache;
    return cache.Get(nnratio, check_ori);
}

// A keyframe's orb_kf_view_t and the arrays it points into.
template <class A>
struct KfViewStore {
    orb_kf_view_t view{};
    std::vector<uint8_t> has_mp;
    std::vector<uint32_t> node;
    std::vector<int32_t> offset, index;

    explicit KfViewStore(typename A::KeyFrame* k) {
        const int n = A::N(k);
        const auto mps = A::MapPointMatches(k);
        has_mp.resize(n);
        for (int i = 0; i < n; ++i) has_mp[i] = (i < (int)mps.size() && mps[i]) ? 1 : 0;  // GetMapPoint(i) != NULL
        const auto& fv = A::FeatVec(k);
        node.reserve(fv.size());
        offset.reserve(fv.size() + 1);
        offset.push_back(0);
        for (const auto& kv : fv) {  // std::map: node ids ascending, each node's indices in insertion order
            node.push_back((uint32_t)kv.first);
            for (auto idx : kv.second) index.push_back((int32_t)idx);
            offset.push_back((int32_t)index.size());
        }
        float K[4];
        A::Pinhole(k, K);
        view.n = n;
        view.kps_un = A::KeysUn(k);
        view.desc = A::Descriptors(k);
        view.u_right = A::URight(k);
        view.has_mappoint = has_mp.data();
        view.n_nodes = (int32_t)node.size();
        view.fv_node = node.data();
        view.fv_offset = offset.data();
        view.fv_index = index.data();
        view.fx = K[0];
        view.fy = K[1];
        view.cx = K[2];
        view.cy = K[3];
        view.nlevels = A::Levels(k);
        view.scale_factors = A::ScaleFactors(k);
        view.level_sigma2 = A::LevelSigma2(k);
    }
    KfViewStore(const KfViewStore&) = delete;
    KfViewStore& operator=(const KfViewStore&) = delete;
};
}  // namespace detail

template <class A>
class ORBmatcher {
public:
    using KeyFrame = typename A::KeyFrame;
    using Frame = typename A::Frame;
    using MapPoint = typename A::MapPoint;

    static const int TH_LOW = 50;        // src/ORBmatcher.cc:36-38
    static const int TH_HIGH = 100;
    static const int HISTO_LENGTH = 30;

    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orb_descriptor_distance(a, b); }

    static bool Supports(KeyFrame* a, KeyFrame* b) { return A::SingleCamera(a) && A::SingleCamera(b); }
    static bool Supports(const Frame& f) { return A::SingleCamera(f); }

    // src/ORBmatcher.cc:1046-1324.  vMatchedPairs = (idx1, idx2) in increasing idx1 (:1313-1321).
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<std::pair<size_t, size_t>>& vMatchedPairs,
                               const bool bOnlyStereo, const bool bCoarse = false) {
        std::vector<std::vector<std::pair<size_t, size_t>>> all;
        const std::vector<int> n = SearchForTriangulation(pKF1, std::vector<KeyFrame*>{pKF2}, all, bOnlyStereo, bCoarse);
        vMatchedPairs = std::move(all[0]);
        return n[0];
    }

    // The loop of LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:565-610) in one launch: pKF1
    // against every neighbour, all against pKF1's map points as they are at the call.  The loop adds
    // map points to pKF1 while it walks the neighbours (AddMapPoint(pMP, idx1)), so a caller that
    // triangulates neighbour p's pairs after neighbour q < p must drop the pairs whose idx1 received
    // a map point meanwhile; with checkOri == false (LocalMapping's ORBmatcher(0.6, false)) every other
    // pair equals what the per-neighbour call would return, since vbMatched2 is never set (:1256-1257).
    std::vector<int> SearchForTriangulation(KeyFrame* pKF1, const std::vector<KeyFrame*>& vpKF2,
                                            std::vector<std::vector<std::pair<size_t, size_t>>>& vvMatchedPairs,
                                            const bool bOnlyStereo, const bool bCoarse = false) {
        const size_t p = vpKF2.size();
        vvMatchedPairs.assign(p, {});
        std::vector<int> counts(p, 0);
        if (p == 0) return counts;
        detail::KfViewStore<A> v1(pKF1);
        std::vector<std::unique_ptr<detail::KfViewStore<A>>> v2;
        std::vector<orb_kf_view_t> views(p);
        std::vector<orb_kf_pair_geom_t> geoms(p);
        for (size_t i = 0; i < p; ++i) {
            v2.emplace_back(new detail::KfViewStore<A>(vpKF2[i]));
            views[i] = v2.back()->view;
            geoms[i] = A::PairGeometry(pKF1, vpKF2[i]);
        }
        const int n1 = v1.view.n;
        std::vector<int32_t> m12((size_t)p * (n1 > 0 ? n1 : 1), -1), cnt(p, 0);
        if (Failed(orb_search_for_triangulation(Handle(), &v1.view, views.data(), geoms.data(), (int)p,
                                                bOnlyStereo ? 1 : 0, bCoarse ? 1 : 0, m12.data(), cnt.data()),
                   "orb_search_for_triangulation"))
            return counts;  // no pairs, 0 matches
        for (size_t k = 0; k < p; ++k) {
            auto& out = vvMatchedPairs[k];
            out.reserve(cnt[k]);
            for (int i = 0; i < n1; ++i) {
                const int32_t j = m12[k * n1 + i];
                if (j >= 0) out.emplace_back((size_t)i, (size_t)j);
            }
            counts[k] = cnt[k];
        }
        return counts;
    }

    // src/ORBmatcher.cc:1951-2185.  The matches are written into CurrentFrame.mvpMapPoints as the
    // reference does (CurrentFrame.mvpMapPoints[i2] = LastFrame.mvpMapPoints[i]); entries it does not
    // match keep what they held.  Tracking clears the vector before every call (src/Tracking.cc:4137,
    // 4156); a keypoint that already holds a map point with observations is skipped by every candidate
    // search (:2038-2041), so the shim hides it from the grid (its copy of the keypoint is moved out of
    // the frame bounds), which is the same skip for every last-frame point.
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
        auto& cur_mps = A::MapPoints(CurrentFrame);
        orb_frame_view_t cur = A::View(CurrentFrame);
        std::vector<orb_keypoint_t> hidden;
        for (int i2 = 0; i2 < cur.n && i2 < (int)cur_mps.size(); ++i2) {
            if (!cur_mps[i2] || A::Observations(cur_mps[i2]) <= 0) continue;
            if (hidden.empty()) hidden.assign(cur.kps_un, cur.kps_un + cur.n);
            hidden[i2].x = cur.min_x - 1e6f;  // outside every grid cell (Frame::PosInGrid fails)
        }
        if (!hidden.empty()) cur.kps_un = hidden.data();
        const orb_frame_view_t lastv = A::View(LastFrame);
        const auto& last_mps = A::MapPoints(LastFrame);
        const int nl = lastv.n;
        std::vector<uint8_t> valid(nl, 0), observed(nl, 0), desc((size_t)nl * 32, 0);
        std::vector<float> xyz((size_t)nl * 3, 0.f);
        for (int i = 0; i < nl; ++i) {
            MapPoint* pMP = i < (int)last_mps.size() ? last_mps[i] : nullptr;
            if (!pMP || A::Outlier(LastFrame, i)) continue;  // (:1980-1984)
            valid[i] = 1;
            observed[i] = A::Observations(pMP) > 0 ? 1 : 0;
            A::WorldPos(pMP, &xyz[3 * (size_t)i]);
            A::Descriptor(pMP, &desc[32 * (size_t)i]);
        }
        orb_last_points_t last{};
        last.n = nl;
        last.valid = valid.data();
        last.observed = observed.data();
        last.xyz = xyz.data();
        last.desc = desc.data();
        last.kps_un = lastv.kps_un;
        for (int k = 0; k < 12; ++k) last.Tcw[k] = lastv.Tcw[k];
        std::vector<int32_t> match(cur.n > 0 ? cur.n : 1, -1);
        int32_t n = 0;
        if (Failed(orb_search_by_projection_frame(Handle(), &cur, &last, th, bMono ? 1 : 0, match.data(), &n),
                   "orb_search_by_projection_frame"))
            return 0;
        for (int i2 = 0; i2 < cur.n; ++i2)
            if (match[i2] >= 0) cur_mps[i2] = last_mps[match[i2]];
        return n;
    }

    // src/ORBmatcher.cc:46-240 (Tracking::SearchLocalPoints, src/Tracking.cc:4825), after
    // Frame::isInFrustum has set the tracking fields of vpMapPoints.
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3,
                           const bool bFarPoints = false, const float thFarPoints = 50.0f) {
        const orb_frame_view_t fv = A::View(F);
        auto& fmps = A::MapPoints(F);
        std::vector<uint8_t> taken(fv.n > 0 ? fv.n : 1, 0);
        for (int i = 0; i < fv.n && i < (int)fmps.size(); ++i)
            taken[i] = (fmps[i] && A::Observations(fmps[i]) > 0) ? 1 : 0;  // (:103-105)
        const int np = (int)vpMapPoints.size();
        std::vector<uint8_t> in_view(np), bad(np), observed(np), desc((size_t)np * 32, 0);
        std::vector<float> proj((size_t)np * 3), view_cos(np), depth(np);
        std::vector<int32_t> level(np);
        for (int i = 0; i < np; ++i) {
            MapPoint* pMP = vpMapPoints[i];
            TrackFields t;
            A::Track(pMP, &t);
            in_view[i] = t.in_view ? 1 : 0;
            bad[i] = A::IsBad(pMP) ? 1 : 0;
            observed[i] = A::Observations(pMP) > 0 ? 1 : 0;
            for (int k = 0; k < 3; ++k) proj[3 * (size_t)i + k] = t.proj[k];
            view_cos[i] = t.view_cos;
            depth[i] = t.depth;
            level[i] = t.level;
            if (t.in_view && !bad[i]) A::Descriptor(pMP, &desc[32 * (size_t)i]);
        }
        orb_local_points_t pts{};
        pts.n = np;
        pts.track_in_view = in_view.data();
        pts.is_bad = bad.data();
        pts.observed = observed.data();
        pts.track_proj = proj.data();
        pts.track_view_cos = view_cos.data();
        pts.track_depth = depth.data();
        pts.track_level = level.data();
        pts.desc = desc.data();
        std::vector<int32_t> match(fv.n > 0 ? fv.n : 1, -1);
        int32_t n = 0;
        if (Failed(orb_search_by_projection_local(Handle(), &fv, taken.data(), &pts, th, bFarPoints ? 1 : 0,
                                                  thFarPoints, match.data(), &n),
                   "orb_search_by_projection_local"))
            return 0;
        for (int i = 0; i < fv.n; ++i)
            if (match[i] >= 0) fmps[i] = vpMapPoints[match[i]];  // F.mvpMapPoints[bestIdx] = pMP (:156)
        return n;
    }

    float mfNNratio;
    bool mbCheckOrientation;

private:
    orb_matcher_t Handle() const { return detail::ThreadHandle(mfNNratio, mbCheckOrientation); }
    static bool Failed(int rc, const char* what) { return detail::Failed(rc, what); }
};

// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:438-529) for a batch of map points in one
// launch, e.g. the loops of LocalMapping::SearchInNeighbors (src/LocalMapping.cc:1045-1060) and
// ProcessNewKeyFrame (:400-416): each point's result depends only on its own observations, so the
// batch equals the per-point calls.  Per point, as the reference: skipped when bad or without
// observations; rows = the observations in std::map order, left then right index, bad keyframes
// skipped; skipped when no row; otherwise mDescriptor = the row with the least median distance.
// Accessor members used (besides those above):
//   static std::map<KeyFrame*, std::tuple<int, int>> ObservationMap(MapPoint*); // GetObservations()
//   static bool IsBad(KeyFrame*);
//   static const uint8_t* DescriptorRow(KeyFrame*, int idx);                    // mDescriptors.row(idx)
//   static void SetDescriptor(MapPoint*, const uint8_t d[32]);                  // mDescriptor = row.clone()
template <class A>
void ComputeDistinctiveDescriptors(const std::vector<typename A::MapPoint*>& points) {
    std::vector<uint8_t> rows;
    std::vector<int32_t> offsets{0};
    std::vector<typename A::MapPoint*> todo;
    for (auto* pMP : points) {
        if (!pMP || A::IsBad(pMP)) continue;
        const auto observations = A::ObservationMap(pMP);
        if (observations.empty()) continue;
        const size_t before = rows.size();
        for (const auto& ob : observations) {
            if (A::IsBad(ob.first)) continue;
            const int l = std::get<0>(ob.second), r = std::get<1>(ob.second);
            if (l != -1) rows.insert(rows.end(), A::DescriptorRow(ob.first, l), A::DescriptorRow(ob.first, l) + 32);
            if (r != -1) rows.insert(rows.end(), A::DescriptorRow(ob.first, r), A::DescriptorRow(ob.first, r) + 32);
        }
        if (rows.size() == before) continue;
        offsets.push_back((int32_t)(rows.size() / 32));
        todo.push_back(pMP);
    }
    if (todo.empty()) return;
    std::vector<int32_t> best(todo.size());
    std::vector<uint8_t> out(32 * todo.size());
    if (detail::Failed(orb_compute_distinctive_descriptors(detail::ThreadHandle(0.6f, false), rows.data(), offsets.data(),
                                                           (int)todo.size(), best.data(), out.data()),
                       "orb_compute_distinctive_descriptors"))
        return;  // descriptors left as they were
    for (size_t p = 0; p < todo.size(); ++p) A::SetDescriptor(todo[p], &out[32 * p]);
}

}  // namespace orbgpu

// ---- the reference's own types (compile inside the ORB-SLAM3 build: define ORBGPU_WITH_ORBSLAM3 and
// include after Frame.h, KeyFrame.h and MapPoint.h) ------------------------------------------------
#ifdef ORBGPU_WITH_ORBSLAM3
namespace orbgpu {

struct ORBSLAM3MatcherAccess {
    using KeyFrame = ORB_SLAM3::KeyFrame;
    using Frame = ORB_SLAM3::Frame;
    using MapPoint = ORB_SLAM3::MapPoint;
    static_assert(sizeof(cv::KeyPoint) == sizeof(orb_keypoint_t), "cv::KeyPoint layout");

    static int N(KeyFrame* k) { return k->N; }
    static const orb_keypoint_t* KeysUn(KeyFrame* k) { return reinterpret_cast<const orb_keypoint_t*>(k->mvKeysUn.data()); }
    static const uint8_t* Descriptors(KeyFrame* k) { return k->mDescriptors.empty() ? nullptr : k->mDescriptors.ptr<uint8_t>(); }
    static const float* URight(KeyFrame* k) { return k->mvuRight.data(); }
    static std::vector<MapPoint*> MapPointMatches(KeyFrame* k) { return k->GetMapPointMatches(); }
    static const DBoW2::FeatureVector& FeatVec(KeyFrame* k) { return k->mFeatVec; }
    static void Pinhole(KeyFrame* k, float K[4]) {
        for (int i = 0; i < 4; ++i) K[i] = k->mpCamera->getParameter(i);  // Pinhole mvParameters: fx, fy, cx, cy
    }
    static int Levels(KeyFrame* k) { return k->mnScaleLevels; }
    static const float* ScaleFactors(KeyFrame* k) { return k->mvScaleFactors.data(); }
    static const float* LevelSigma2(KeyFrame* k) { return k->mvLevelSigma2.data(); }
    static bool SingleCamera(KeyFrame* k) { return k->mpCamera2 == nullptr && k->NLeft == -1; }
    static orb_kf_pair_geom_t PairGeometry(KeyFrame* pKF1, KeyFrame* pKF2) {  // src/ORBmatcher.cc:1054-1072
        const Sophus::SE3f T1w = pKF1->GetPose(), T2w = pKF2->GetPose(), Tw2 = pKF2->GetPoseInverse();
        const Eigen::Vector3f C2 = T2w * pKF1->GetCameraCenter();
        const Eigen::Vector2f ep = pKF2->mpCamera->project(C2);
        const Sophus::SE3f T12 = T1w * Tw2;
        const Eigen::Matrix3f R12 = T12.rotationMatrix();
        const Eigen::Vector3f t12 = T12.translation();
        orb_kf_pair_geom_t g;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) g.R12[3 * r + c] = R12(r, c);
            g.t12[r] = t12(r);
        }
        g.ep[0] = ep(0);
        g.ep[1] = ep(1);
        return g;
    }

    static orb_frame_view_t View(const Frame& f) {
        orb_frame_view_t v{};
        v.n = f.N;
        v.kps_un = reinterpret_cast<const orb_keypoint_t*>(f.mvKeysUn.data());
        v.desc = f.mDescriptors.empty() ? nullptr : f.mDescriptors.ptr<uint8_t>();
        v.u_right = f.mvuRight.data();
        v.min_x = Frame::mnMinX; v.max_x = Frame::mnMaxX; v.min_y = Frame::mnMinY; v.max_y = Frame::mnMaxY;
        v.grid_inv_w = Frame::mfGridElementWidthInv;
        v.grid_inv_h = Frame::mfGridElementHeightInv;
        v.fx = f.fx; v.fy = f.fy; v.cx = f.cx; v.cy = f.cy;
        v.bf = f.mbf; v.b = f.mb;
        v.nlevels = f.mnScaleLevels;
        v.scale_factors = f.mvScaleFactors.data();
        const Eigen::Matrix<float, 3, 4> T = f.GetPose().matrix3x4();
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) v.Tcw[4 * r + c] = T(r, c);
        return v;
    }
    static bool SingleCamera(const Frame& f) { return f.Nleft == -1 && f.mpCamera2 == nullptr; }
    static std::vector<MapPoint*>& MapPoints(Frame& f) { return f.mvpMapPoints; }
    static const std::vector<MapPoint*>& MapPoints(const Frame& f) { return f.mvpMapPoints; }
    static bool Outlier(const Frame& f, int i) { return f.mvbOutlier[i]; }

    static int Observations(MapPoint* p) { return p->Observations(); }
    static bool IsBad(MapPoint* p) { return p->isBad(); }
    static void WorldPos(MapPoint* p, float X[3]) {
        const Eigen::Vector3f x = p->GetWorldPos();
        X[0] = x(0); X[1] = x(1); X[2] = x(2);
    }
    static void Descriptor(MapPoint* p, uint8_t d[32]) {
        const cv::Mat m = p->GetDescriptor();
        for (int i = 0; i < 32; ++i) d[i] = m.ptr<uint8_t>()[i];
    }
    static std::map<KeyFrame*, std::tuple<int, int>> ObservationMap(MapPoint* p) { return p->GetObservations(); }
    static bool IsBad(KeyFrame* k) { return k->isBad(); }
    static const uint8_t* DescriptorRow(KeyFrame* k, int idx) { return k->mDescriptors.ptr<uint8_t>(idx); }
    // mDescriptor is protected in MapPoint: the integration adds `friend struct orbgpu::ORBSLAM3MatcherAccess;`
    static void SetDescriptor(MapPoint* p, const uint8_t d[32]) {
        std::unique_lock<std::mutex> lock(p->mMutexFeatures);
        p->mDescriptor = cv::Mat(1, 32, CV_8U, const_cast<uint8_t*>(d)).clone();
    }
    static void Track(MapPoint* p, TrackFields* t) {
        t->in_view = p->mbTrackInView;
        t->proj[0] = p->mTrackProjX; t->proj[1] = p->mTrackProjY; t->proj[2] = p->mTrackProjXR;
        t->view_cos = p->mTrackViewCos;
        t->depth = p->mTrackDepth;
        t->level = p->mnTrackScaleLevel;
    }
};

using GpuORBmatcher = ORBmatcher<ORBSLAM3MatcherAccess>;

}  // namespace orbgpu
#endif  // ORBGPU_WITH_ORBSLAM3

#endif  // ORBGPU_MATCHER_HPP
