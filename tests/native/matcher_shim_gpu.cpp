// GPU check of include/orbgpu_matcher.hpp (the ORBmatcher drop-in) linked to the real liborbgpu.so.
// Mock KeyFrame / Frame / MapPoint objects are built from the arrays tests/test_shims_gpu.py writes,
// together with the oracle's answers for the same inputs (oracle/, test infrastructure).  Checked:
//   * SearchForTriangulation, batched over the neighbours and single-pair (src/ORBmatcher.cc:1046-1324):
//     vMatchedPairs = the oracle's vMatches12 as (idx1, idx2) pairs in increasing idx1, and the counts;
//   * SearchByProjection(Frame, Frame) (:1951-2185): CurrentFrame.mvpMapPoints[i2] = the LastFrame map
//     point the oracle assigns, from LastFrame objects with NULL slots, outliers and unobserved points;
//   * SearchByProjection(Frame, vector<MapPoint*>) (:46-240): F.mvpMapPoints after the call (slots that
//     held an observed map point untouched), from map points with their isInFrustum tracking fields;
//   * ComputeDistinctiveDescriptors over map points (src/MapPoint.cc:438-529): each mDescriptor = the
//     oracle's choice among the point's rows (bad keyframes and bad / unobserved points skipped).
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "orbgpu_matcher.hpp"
#include "shim_records.h"

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

struct MockKF;
struct MockMP {
    int obs = 0;
    bool bad = false;
    float X[3] = {0, 0, 0};
    uint8_t desc[32] = {};
    orbgpu::TrackFields track;
    std::map<MockKF*, std::tuple<int, int>> obsmap;
    bool desc_set = false;
};

struct MockKF {
    std::vector<orb_keypoint_t> kps;
    std::vector<uint8_t> desc;
    std::vector<float> ur;
    std::vector<MockMP*> mps;
    std::map<unsigned int, std::vector<unsigned int>> fv;
    float K[4] = {0, 0, 0, 0};
    std::vector<float> scale, sigma2;
    bool bad = false;
};

struct MockFrame {
    std::vector<orb_keypoint_t> kps;
    std::vector<uint8_t> desc;
    std::vector<float> ur;
    std::vector<MockMP*> mps;
    std::vector<bool> outlier;
    std::vector<float> scale;
    float scal[12] = {};  // min_x max_x min_y max_y grid_inv_w grid_inv_h fx fy cx cy bf b
    float Tcw[12] = {};
};

static std::map<std::pair<MockKF*, MockKF*>, orb_kf_pair_geom_t> g_geom;

struct Access {
    using KeyFrame = MockKF;
    using Frame = MockFrame;
    using MapPoint = MockMP;
    static int N(KeyFrame* k) { return (int)k->kps.size(); }
    static const orb_keypoint_t* KeysUn(KeyFrame* k) { return k->kps.data(); }
    static const uint8_t* Descriptors(KeyFrame* k) { return k->desc.data(); }
    static const float* URight(KeyFrame* k) { return k->ur.empty() ? nullptr : k->ur.data(); }
    static std::vector<MapPoint*> MapPointMatches(KeyFrame* k) { return k->mps; }
    static const std::map<unsigned int, std::vector<unsigned int>>& FeatVec(KeyFrame* k) { return k->fv; }
    static void Pinhole(KeyFrame* k, float K[4]) { std::memcpy(K, k->K, sizeof k->K); }
    static int Levels(KeyFrame* k) { return (int)k->scale.size(); }
    static const float* ScaleFactors(KeyFrame* k) { return k->scale.data(); }
    static const float* LevelSigma2(KeyFrame* k) { return k->sigma2.data(); }
    static bool SingleCamera(KeyFrame*) { return true; }
    static orb_kf_pair_geom_t PairGeometry(KeyFrame* a, KeyFrame* b) { return g_geom.at({a, b}); }
    static orb_frame_view_t View(const Frame& f) {
        orb_frame_view_t v{};
        v.n = (int)f.kps.size();
        v.kps_un = f.kps.data();
        v.desc = f.desc.data();
        v.u_right = f.ur.empty() ? nullptr : f.ur.data();
        v.min_x = f.scal[0]; v.max_x = f.scal[1]; v.min_y = f.scal[2]; v.max_y = f.scal[3];
        v.grid_inv_w = f.scal[4]; v.grid_inv_h = f.scal[5];
        v.fx = f.scal[6]; v.fy = f.scal[7]; v.cx = f.scal[8]; v.cy = f.scal[9];
        v.bf = f.scal[10]; v.b = f.scal[11];
        v.nlevels = (int)f.scale.size();
        v.scale_factors = f.scale.data();
        std::memcpy(v.Tcw, f.Tcw, sizeof v.Tcw);
        return v;
    }
    static bool SingleCamera(const Frame&) { return true; }
    static std::vector<MapPoint*>& MapPoints(Frame& f) { return f.mps; }
    static const std::vector<MapPoint*>& MapPoints(const Frame& f) { return f.mps; }
    static bool Outlier(const Frame& f, int i) { return f.outlier[i]; }
    static int Observations(MapPoint* p) { return p->obs; }
    static bool IsBad(MapPoint* p) { return p->bad; }
    static void WorldPos(MapPoint* p, float X[3]) { std::memcpy(X, p->X, sizeof p->X); }
    static void Descriptor(MapPoint* p, uint8_t d[32]) { std::memcpy(d, p->desc, 32); }
    static void Track(MapPoint* p, orbgpu::TrackFields* t) { *t = p->track; }
    static std::map<KeyFrame*, std::tuple<int, int>> ObservationMap(MapPoint* p) { return p->obsmap; }
    static bool IsBad(KeyFrame* k) { return k->bad; }
    static const uint8_t* DescriptorRow(KeyFrame* k, int idx) { return k->desc.data() + 32 * (size_t)idx; }
    static void SetDescriptor(MapPoint* p, const uint8_t d[32]) {
        std::memcpy(p->desc, d, 32);
        p->desc_set = true;
    }
};
using Matcher = orbgpu::ORBmatcher<Access>;

static MockMP g_dummy;  // the map point held by KF slots flagged has_mappoint

static void load_kf(const Records& r, const std::string& p, MockKF& k) {
    k.kps = r.Get<orb_keypoint_t>(p + ".kps");
    k.desc = r.Get<uint8_t>(p + ".desc");
    if (r.Has(p + ".ur")) k.ur = r.Get<float>(p + ".ur");
    const auto has = r.Get<uint8_t>(p + ".has_mp");
    k.mps.assign(k.kps.size(), nullptr);
    for (size_t i = 0; i < has.size() && i < k.mps.size(); ++i)
        if (has[i]) k.mps[i] = &g_dummy;
    const auto node = r.Get<uint32_t>(p + ".fv_node");
    const auto off = r.Get<int32_t>(p + ".fv_off");
    const auto idx = r.Get<int32_t>(p + ".fv_idx");
    for (size_t n = 0; n < node.size(); ++n)
        for (int j = off[n]; j < off[n + 1]; ++j) k.fv[node[n]].push_back((unsigned)idx[j]);
    const auto cam = r.Get<float>(p + ".cam");
    std::memcpy(k.K, cam.data(), sizeof k.K);
    k.scale = r.Get<float>(p + ".scale");
    k.sigma2 = r.Get<float>(p + ".sigma2");
}

static void load_frame(const Records& r, const std::string& p, MockFrame& f) {
    f.kps = r.Get<orb_keypoint_t>(p + ".kps");
    f.desc = r.Get<uint8_t>(p + ".desc");
    if (r.Has(p + ".ur")) f.ur = r.Get<float>(p + ".ur");
    f.scale = r.Get<float>(p + ".scale");
    const auto s = r.Get<float>(p + ".scal");
    std::memcpy(f.scal, s.data(), sizeof f.scal);
    const auto T = r.Get<float>(p + ".Tcw");
    std::memcpy(f.Tcw, T.data(), sizeof f.Tcw);
    f.mps.assign(f.kps.size(), nullptr);
    f.outlier.assign(f.kps.size(), false);
}

static void test_sft(const Records& r) {
    const int P = r.Scalar<int32_t>("sft.n_pairs");
    std::vector<MockKF> K(P + 1);
    for (int k = 0; k <= P; ++k) load_kf(r, "kf" + std::to_string(k), K[k]);
    std::vector<MockKF*> nb;
    for (int p = 0; p < P; ++p) {
        const auto g = r.Get<orb_kf_pair_geom_t>("geom" + std::to_string(p));
        g_geom[{&K[0], &K[p + 1]}] = g[0];
        nb.push_back(&K[p + 1]);
    }
    const int n1 = (int)K[0].kps.size();
    for (int c = 0; r.Has("sft" + std::to_string(c) + ".m12"); ++c) {
        const std::string s = "sft" + std::to_string(c);
        const bool only_stereo = r.Scalar<int32_t>(s + ".only_stereo") != 0;
        const bool coarse = r.Scalar<int32_t>(s + ".coarse") != 0;
        const bool check_ori = r.Scalar<int32_t>(s + ".check_ori") != 0;
        const auto m12 = r.Get<int32_t>(s + ".m12");
        const auto cnt = r.Get<int32_t>(s + ".cnt");
        Matcher matcher(0.6f, check_ori);
        std::vector<std::vector<std::pair<size_t, size_t>>> all;
        const std::vector<int> ns = matcher.SearchForTriangulation(&K[0], nb, all, only_stereo, coarse);
        int total = 0, bad = 0;
        for (int p = 0; p < P; ++p) {
            std::vector<std::pair<size_t, size_t>> want;
            for (int i = 0; i < n1; ++i)
                if (m12[(size_t)p * n1 + i] >= 0) want.emplace_back((size_t)i, (size_t)m12[(size_t)p * n1 + i]);
            if (ns[p] != cnt[p] || all[p] != want) ++bad;
            total += ns[p];
        }
        std::printf("SearchForTriangulation (onlyStereo %d, coarse %d, checkOri %d): %d pairs, %d matches, %d "
                    "neighbours differ\n",
                    (int)only_stereo, (int)coarse, (int)check_ori, P, total, bad);
        CHECK(bad == 0 && total > 0);
        // the single-pair overload on the first neighbour
        std::vector<std::pair<size_t, size_t>> pairs;
        const int n = matcher.SearchForTriangulation(&K[0], nb[0], pairs, only_stereo, coarse);
        CHECK(n == cnt[0] && pairs == all[0]);
    }
}

static void test_sbp_frame(const Records& r) {
    MockFrame cur, last;
    load_frame(r, "cur", cur);
    load_frame(r, "last", last);
    const auto kind = r.Get<uint8_t>("last.mp_kind");
    const auto obs = r.Get<int32_t>("last.mp_obs");
    const auto xyz = r.Get<float>("last.mp_xyz");
    const auto desc = r.Get<uint8_t>("last.mp_desc");
    std::vector<MockMP> pts(kind.size());
    for (size_t i = 0; i < kind.size(); ++i) {
        if (kind[i] == 0) continue;  // NULL slot
        pts[i].obs = obs[i];
        std::memcpy(pts[i].X, &xyz[3 * i], sizeof pts[i].X);
        std::memcpy(pts[i].desc, &desc[32 * i], 32);
        last.mps[i] = &pts[i];
        last.outlier[i] = kind[i] == 2;
    }
    for (int c = 0; r.Has("sbpf" + std::to_string(c) + ".match"); ++c) {
        const std::string s = "sbpf" + std::to_string(c);
        const float th = r.Scalar<float>(s + ".th");
        const bool mono = r.Scalar<int32_t>(s + ".mono") != 0;
        const bool ori = r.Scalar<int32_t>(s + ".check_ori") != 0;
        const auto match = r.Get<int32_t>(s + ".match");
        std::fill(cur.mps.begin(), cur.mps.end(), nullptr);  // Tracking clears it first (src/Tracking.cc:4137)
        Matcher matcher(0.9f, ori);
        const int n = matcher.SearchByProjection(cur, last, th, mono);
        int bad = 0, assigned = 0;
        for (size_t i = 0; i < cur.mps.size(); ++i) {
            MockMP* want = match[i] >= 0 ? last.mps[match[i]] : nullptr;
            if (cur.mps[i] != want) ++bad;
            assigned += cur.mps[i] != nullptr;
        }
        std::printf("SearchByProjection(Frame, Frame) th %.0f mono %d checkOri %d: %d matches (oracle %d), %d "
                    "keypoints hold a point, %d differ\n",
                    th, (int)mono, (int)ori, n, r.Scalar<int32_t>(s + ".n"), assigned, bad);
        CHECK(n == r.Scalar<int32_t>(s + ".n") && bad == 0 && n > 0);
    }
}

static void test_sbp_local(const Records& r) {
    MockFrame F;
    load_frame(r, "F", F);
    const auto taken_kind = r.Get<uint8_t>("F.taken_kind");
    std::vector<MockMP> held(F.kps.size());
    for (size_t i = 0; i < F.kps.size(); ++i)
        if (taken_kind[i]) {
            held[i].obs = taken_kind[i] == 1 ? 2 : 0;
            F.mps[i] = &held[i];
        }
    const auto in_view = r.Get<uint8_t>("lp.in_view");
    const auto bad = r.Get<uint8_t>("lp.bad");
    const auto obs = r.Get<int32_t>("lp.obs");
    const auto proj = r.Get<float>("lp.proj");
    const auto vcos = r.Get<float>("lp.view_cos");
    const auto depth = r.Get<float>("lp.depth");
    const auto level = r.Get<int32_t>("lp.level");
    const auto desc = r.Get<uint8_t>("lp.desc");
    std::vector<MockMP> P(in_view.size());
    std::vector<MockMP*> vp;
    for (size_t i = 0; i < P.size(); ++i) {
        P[i].track.in_view = in_view[i] != 0;
        P[i].bad = bad[i] != 0;
        P[i].obs = obs[i];
        for (int k = 0; k < 3; ++k) P[i].track.proj[k] = proj[3 * i + k];
        P[i].track.view_cos = vcos[i];
        P[i].track.depth = depth[i];
        P[i].track.level = level[i];
        std::memcpy(P[i].desc, &desc[32 * i], 32);
        vp.push_back(&P[i]);
    }
    const auto before = F.mps;
    const float th = r.Scalar<float>("sbpl.th"), th_far = r.Scalar<float>("sbpl.th_far");
    const bool far = r.Scalar<int32_t>("sbpl.far") != 0;
    const float ratio = r.Scalar<float>("sbpl.ratio");
    const auto match = r.Get<int32_t>("sbpl.match");
    Matcher matcher(ratio, true);
    const int n = matcher.SearchByProjection(F, vp, th, far, th_far);
    int differ = 0;
    for (size_t i = 0; i < F.mps.size(); ++i) {
        MockMP* want = match[i] >= 0 ? vp[match[i]] : before[i];
        if (F.mps[i] != want) ++differ;
    }
    std::printf("SearchByProjection(Frame, %zu MapPoints) th %.0f: %d matches (oracle %d), %d slots differ\n", vp.size(),
                th, n, r.Scalar<int32_t>("sbpl.n"), differ);
    CHECK(n == r.Scalar<int32_t>("sbpl.n") && differ == 0 && n > 0);
}

static void test_distinctive(const Records& r) {
    const int nk = r.Scalar<int32_t>("dd.n_kf");
    std::vector<MockKF> K(nk);
    const auto kbad = r.Get<uint8_t>("dd.kf_bad");
    for (int k = 0; k < nk; ++k) {
        K[k].desc = r.Get<uint8_t>("dd.kf_desc" + std::to_string(k));
        K[k].bad = kbad[k] != 0;
    }
    const auto pbad = r.Get<uint8_t>("dd.pt_bad");
    const auto off = r.Get<int32_t>("dd.obs_off");
    const auto ob = r.Get<int32_t>("dd.obs");
    const auto want = r.Get<uint8_t>("dd.best_desc");
    const auto has = r.Get<uint8_t>("dd.has");
    std::vector<MockMP> P(pbad.size());
    std::vector<MockMP*> vp;
    for (size_t p = 0; p < P.size(); ++p) {
        P[p].bad = pbad[p] != 0;
        for (int j = off[p]; j < off[p + 1]; ++j)
            P[p].obsmap[&K[ob[3 * j]]] = std::make_tuple(ob[3 * j + 1], ob[3 * j + 2]);
        vp.push_back(&P[p]);
        if (p % 7 == 3) vp.push_back(nullptr);  // NULL entries are skipped
    }
    orbgpu::ComputeDistinctiveDescriptors<Access>(vp);
    int differ = 0, set = 0;
    for (size_t p = 0; p < P.size(); ++p) {
        set += P[p].desc_set;
        if (P[p].desc_set != (has[p] != 0) || (has[p] && std::memcmp(P[p].desc, &want[32 * p], 32) != 0)) ++differ;
    }
    std::printf("ComputeDistinctiveDescriptors: %zu points, %d descriptors set, %d differ from the oracle\n", P.size(),
                set, differ);
    CHECK(differ == 0 && set > 0);
}

int main(int argc, char** argv) {
    Records r;
    if (argc < 2 || !r.Load(argv[1])) {
        std::printf("usage: %s records.bin\n", argv[0]);
        return 2;
    }
    try {
        test_sft(r);
        test_sbp_frame(r);
        test_sbp_local(r);
        test_distinctive(r);
    } catch (const std::exception& e) {
        std::printf("FAIL exception: %s\n", e.what());
        return 1;
    }
    if (orbgpu::LastShimError() != ORB_OK) {  // failures do not throw: every call must have succeeded
        std::printf("FAIL shim error %d: %s\n", orbgpu::LastShimError(), orbgpu::LastShimMessage().c_str());
        return 1;
    }
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK matcher_shim_gpu\n");
    return 0;
}
