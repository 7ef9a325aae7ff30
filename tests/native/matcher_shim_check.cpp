// CPU check of include/orbgpu_matcher.hpp (the ORBmatcher drop-in) on mock KeyFrame / Frame / MapPoint
// objects.  The C ABI is replaced by test doubles defined below that record the flat views the shim
// builds and return chosen results, so this runs without a GPU; the HIP matchers themselves are
// compared with the oracle in tests/test_matcher_gpu.py and tests/test_projection_gpu.py.  Checked:
//   * SearchForTriangulation (src/ORBmatcher.cc:1046-1324): has-map-point flags (GetMapPoint != NULL),
//     the FeatureVector as sorted node ids + CSR indices in each node's order, pinhole / levels, the
//     pair geometry; vMatchedPairs in increasing idx1 (:1313-1321) and the returned count; the batched
//     form over several neighbours;
//   * SearchByProjection(Frame, Frame) (:1951-2185): last-frame points valid only when non-NULL and
//     not outliers (:1980-1984), their Observations() > 0, world positions, descriptors; the write of
//     CurrentFrame.mvpMapPoints; a frame that still holds map points: the ones with observations
//     hidden from every candidate search (:2038-2041), the unmatched entries kept;
//   * SearchByProjection(Frame, vector<MapPoint*>) (:46-240): keypoints already holding a map point
//     with observations (:103-105), the tracking fields, the write of F.mvpMapPoints;
//   * a library error never throws (orbgpu_status.hpp): every entry point returns the reference's
//     empty result, leaves its outputs untouched and reports the ORB_ERR_* code through
//     orbgpu::LastShimError(); a handle that cannot be created is retried on the next call; one
//     device handle per (thread, nnratio, checkOri).
#include <cstdio>
#include <cstring>
#include <map>
#include <tuple>
#include <string>
#include <vector>

#include "orbgpu_matcher.hpp"

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

// ---- mock reference objects ------------------------------------------------------------------------
struct MockKF;
struct MockMP {
    int obs = 1;
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
    float K[4] = {458.654f, 457.296f, 367.215f, 248.375f};
    std::vector<float> scale{1.f, 1.2f, 1.44f}, sigma2{1.f, 1.44f, 2.0736f};
    bool cam2 = false, bad = false;
    int tag = 0;  // identifies the keyframe in PairGeometry
};

struct MockFrame {
    std::vector<orb_keypoint_t> kps;
    std::vector<uint8_t> desc;
    std::vector<float> ur;
    std::vector<MockMP*> mps;
    std::vector<bool> outlier;
    std::vector<float> scale{1.f, 1.2f, 1.44f};
    float Tcw[12] = {1, 0, 0, 0.5f, 0, 1, 0, 0, 0, 0, 1, 0};
    int nleft = -1;
};

struct Access {
    using KeyFrame = MockKF;
    using Frame = MockFrame;
    using MapPoint = MockMP;
    static int N(KeyFrame* k) { return (int)k->kps.size(); }
    static const orb_keypoint_t* KeysUn(KeyFrame* k) { return k->kps.data(); }
    static const uint8_t* Descriptors(KeyFrame* k) { return k->desc.data(); }
    static const float* URight(KeyFrame* k) { return k->ur.data(); }
    static std::vector<MapPoint*> MapPointMatches(KeyFrame* k) { return k->mps; }
    static const std::map<unsigned int, std::vector<unsigned int>>& FeatVec(KeyFrame* k) { return k->fv; }
    static void Pinhole(KeyFrame* k, float K[4]) { std::memcpy(K, k->K, sizeof k->K); }
    static int Levels(KeyFrame* k) { return (int)k->scale.size(); }
    static const float* ScaleFactors(KeyFrame* k) { return k->scale.data(); }
    static const float* LevelSigma2(KeyFrame* k) { return k->sigma2.data(); }
    static bool SingleCamera(KeyFrame* k) { return !k->cam2; }
    static orb_kf_pair_geom_t PairGeometry(KeyFrame* a, KeyFrame* b) {
        orb_kf_pair_geom_t g{};
        g.ep[0] = (float)a->tag;
        g.ep[1] = (float)b->tag;
        g.R12[0] = g.R12[4] = g.R12[8] = 1.f;
        return g;
    }
    static orb_frame_view_t View(const Frame& f) {
        orb_frame_view_t v{};
        v.n = (int)f.kps.size();
        v.kps_un = f.kps.data();
        v.desc = f.desc.data();
        v.u_right = f.ur.data();
        v.min_x = 0; v.max_x = 752; v.min_y = 0; v.max_y = 480;
        v.grid_inv_w = 64.f / 752; v.grid_inv_h = 48.f / 480;
        v.fx = 458.654f; v.fy = 457.296f; v.cx = 367.215f; v.cy = 248.375f;
        v.bf = 47.9f; v.b = 0.11f;
        v.nlevels = (int)f.scale.size();
        v.scale_factors = f.scale.data();
        std::memcpy(v.Tcw, f.Tcw, sizeof v.Tcw);
        return v;
    }
    static bool SingleCamera(const Frame& f) { return f.nleft == -1; }
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
    static const uint8_t* DescriptorRow(KeyFrame* k, int idx) { return k->desc.data() + 32 * idx; }
    static void SetDescriptor(MapPoint* p, const uint8_t d[32]) {
        std::memcpy(p->desc, d, 32);
        p->desc_set = true;
    }
};
using Matcher = orbgpu::ORBmatcher<Access>;

// ---- test doubles of the C ABI -------------------------------------------------------------------
struct FakeHandle {
    float nnratio;
    int check_ori;
};
static int g_creates = 0, g_rc = 0, g_create_rc = 0;
static std::string g_err;
// what the last call saw
static struct {
    int n_pairs = 0, only_stereo = -1, coarse = -1;
    orb_kf_view_t kf1{};
    std::vector<uint8_t> kf1_has_mp;
    std::vector<uint32_t> kf1_nodes;
    std::vector<int32_t> kf1_offset, kf1_index;
    std::vector<orb_kf_pair_geom_t> geoms;
    std::vector<int> kf2_n;
    FakeHandle* h = nullptr;
    orb_frame_view_t cur{};
    std::vector<uint8_t> valid, observed, taken, in_view, bad, desc;
    std::vector<float> xyz, proj, cur_x;
    std::vector<int32_t> level;
    float th = 0, th_far = 0;
    int mono = -1, far = -1;
} g_seen;
static std::vector<int32_t> g_match;  // result row(s) the doubles return
static std::vector<int32_t> g_counts;

extern "C" {
const char* orb_last_error(void) { return g_err.c_str(); }
int orb_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; ++i) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}
static std::vector<uint8_t> g_dd_rows;
static std::vector<int32_t> g_dd_off;
int orb_compute_distinctive_descriptors(orb_matcher_t, const uint8_t* desc, const int32_t* offsets, int n_points,
                                        int32_t* best, uint8_t* out) {
    if (g_rc) {
        g_err = "fake failure";
        return g_rc;
    }
    g_dd_off.assign(offsets, offsets + n_points + 1);
    g_dd_rows.assign(desc, desc + 32 * (size_t)offsets[n_points]);
    for (int p = 0; p < n_points; ++p) {  // the double picks each point's last row
        best[p] = offsets[p + 1] - offsets[p] - 1;
        std::memcpy(out + 32 * p, desc + 32 * (size_t)(offsets[p + 1] - 1), 32);
    }
    return ORB_OK;
}
int orb_matcher_create(float nnratio, int check_orientation, orb_matcher_t* out) {
    if (g_create_rc) {
        g_err = "fake create failure";
        return g_create_rc;
    }
    ++g_creates;
    *out = reinterpret_cast<orb_matcher_t>(new FakeHandle{nnratio, check_orientation});
    return ORB_OK;
}
int orb_matcher_destroy(orb_matcher_t m) {
    delete reinterpret_cast<FakeHandle*>(m);
    return ORB_OK;
}
int orb_search_for_triangulation(orb_matcher_t m, const orb_kf_view_t* kf1, const orb_kf_view_t* kf2s,
                                 const orb_kf_pair_geom_t* geoms, int n_pairs, int only_stereo, int coarse,
                                 int32_t* matches12, int32_t* n_matches) {
    if (g_rc) {
        g_err = "fake failure";
        return g_rc;
    }
    g_seen.h = reinterpret_cast<FakeHandle*>(m);
    g_seen.n_pairs = n_pairs;
    g_seen.only_stereo = only_stereo;
    g_seen.coarse = coarse;
    g_seen.kf1 = *kf1;
    g_seen.kf1_has_mp.assign(kf1->has_mappoint, kf1->has_mappoint + kf1->n);
    g_seen.kf1_nodes.assign(kf1->fv_node, kf1->fv_node + kf1->n_nodes);
    g_seen.kf1_offset.assign(kf1->fv_offset, kf1->fv_offset + kf1->n_nodes + 1);
    g_seen.kf1_index.assign(kf1->fv_index, kf1->fv_index + kf1->fv_offset[kf1->n_nodes]);
    g_seen.geoms.assign(geoms, geoms + n_pairs);
    g_seen.kf2_n.clear();
    for (int p = 0; p < n_pairs; ++p) g_seen.kf2_n.push_back(kf2s[p].n);
    std::memcpy(matches12, g_match.data(), sizeof(int32_t) * (size_t)n_pairs * kf1->n);
    std::memcpy(n_matches, g_counts.data(), sizeof(int32_t) * n_pairs);
    return ORB_OK;
}
int orb_search_by_projection_frame(orb_matcher_t m, const orb_frame_view_t* cur, const orb_last_points_t* last,
                                   float th, int mono, int32_t* match, int32_t* n_matches) {
    if (g_rc || !m) {
        g_err = "fake failure";
        return g_rc ? g_rc : ORB_ERR_ARG;
    }
    g_seen.h = reinterpret_cast<FakeHandle*>(m);
    g_seen.cur = *cur;
    g_seen.cur_x.clear();
    for (int i = 0; i < cur->n; ++i) g_seen.cur_x.push_back(cur->kps_un[i].x);
    g_seen.th = th;
    g_seen.mono = mono;
    g_seen.valid.assign(last->valid, last->valid + last->n);
    g_seen.observed.assign(last->observed, last->observed + last->n);
    g_seen.xyz.assign(last->xyz, last->xyz + 3 * last->n);
    g_seen.desc.assign(last->desc, last->desc + 32 * last->n);
    std::memcpy(match, g_match.data(), sizeof(int32_t) * cur->n);
    *n_matches = g_counts[0];
    return ORB_OK;
}
int orb_search_by_projection_local(orb_matcher_t m, const orb_frame_view_t* F, const uint8_t* frame_taken,
                                   const orb_local_points_t* pts, float th, int far_points, float th_far_points,
                                   int32_t* match, int32_t* n_matches) {
    if (g_rc) {
        g_err = "fake failure";
        return g_rc;
    }
    g_seen.h = reinterpret_cast<FakeHandle*>(m);
    g_seen.cur = *F;
    g_seen.taken.assign(frame_taken, frame_taken + F->n);
    g_seen.in_view.assign(pts->track_in_view, pts->track_in_view + pts->n);
    g_seen.bad.assign(pts->is_bad, pts->is_bad + pts->n);
    g_seen.observed.assign(pts->observed, pts->observed + pts->n);
    g_seen.proj.assign(pts->track_proj, pts->track_proj + 3 * pts->n);
    g_seen.level.assign(pts->track_level, pts->track_level + pts->n);
    g_seen.desc.assign(pts->desc, pts->desc + 32 * pts->n);
    g_seen.th = th;
    g_seen.far = far_points;
    g_seen.th_far = th_far_points;
    std::memcpy(match, g_match.data(), sizeof(int32_t) * F->n);
    *n_matches = g_counts[0];
    return ORB_OK;
}
}

static MockKF make_kf(int n, int tag) {
    MockKF k;
    k.tag = tag;
    for (int i = 0; i < n; ++i) {
        orb_keypoint_t kp{};
        kp.x = 10.f * i;
        kp.y = 5.f * i;
        kp.octave = i % 3;
        k.kps.push_back(kp);
        for (int b = 0; b < 32; ++b) k.desc.push_back((uint8_t)(i * 7 + b));
        k.ur.push_back(i % 2 ? 30.f : -1.f);
    }
    k.mps.assign(n, nullptr);
    return k;
}

static void test_search_for_triangulation() {
    MockMP mp;
    MockKF k1 = make_kf(6, 1), k2 = make_kf(5, 2), k3 = make_kf(4, 3);
    k1.mps[2] = &mp;
    k1.mps[4] = &mp;
    k1.fv[40] = {3, 1};
    k1.fv[7] = {0, 5, 2};
    k1.fv[12] = {4};
    Matcher matcher(0.6f, false);
    // single neighbour: m12 row, count
    g_match = {-1, 3, -1, 0, -1, 1};
    g_counts = {3};
    std::vector<std::pair<size_t, size_t>> pairs{{99, 99}};
    const int n = matcher.SearchForTriangulation(&k1, &k2, pairs, false, true);
    CHECK(n == 3);
    CHECK((pairs == std::vector<std::pair<size_t, size_t>>{{1, 3}, {3, 0}, {5, 1}}));
    CHECK(g_seen.n_pairs == 1 && g_seen.only_stereo == 0 && g_seen.coarse == 1);
    CHECK((g_seen.kf1_has_mp == std::vector<uint8_t>{0, 0, 1, 0, 1, 0}));
    CHECK((g_seen.kf1_nodes == std::vector<uint32_t>{7, 12, 40}));
    CHECK((g_seen.kf1_offset == std::vector<int32_t>{0, 3, 4, 6}));
    CHECK((g_seen.kf1_index == std::vector<int32_t>{0, 5, 2, 4, 3, 1}));
    CHECK(g_seen.kf1.n == 6 && g_seen.kf1.nlevels == 3 && g_seen.kf1.fx == k1.K[0] && g_seen.kf1.cy == k1.K[3]);
    CHECK(g_seen.kf1.kps_un == k1.kps.data() && g_seen.kf1.desc == k1.desc.data() && g_seen.kf1.u_right == k1.ur.data());
    CHECK(g_seen.kf1.level_sigma2 == k1.sigma2.data() && g_seen.kf1.scale_factors == k1.scale.data());
    CHECK(g_seen.geoms.size() == 1 && g_seen.geoms[0].ep[0] == 1.f && g_seen.geoms[0].ep[1] == 2.f);
    CHECK(g_seen.h && g_seen.h->nnratio == 0.6f && g_seen.h->check_ori == 0);
    // batch over two neighbours
    g_match = {-1, -1, -1, -1, -1, 2, /* row 2 */ 0, -1, -1, 1, -1, -1};
    g_counts = {1, 2};
    std::vector<std::vector<std::pair<size_t, size_t>>> all;
    const std::vector<int> ns = matcher.SearchForTriangulation(&k1, std::vector<MockKF*>{&k2, &k3}, all, true);
    CHECK((ns == std::vector<int>{1, 2}));
    CHECK(all.size() == 2 && (all[0] == std::vector<std::pair<size_t, size_t>>{{5, 2}}));
    CHECK((all[1] == std::vector<std::pair<size_t, size_t>>{{0, 0}, {3, 1}}));
    CHECK(g_seen.n_pairs == 2 && g_seen.only_stereo == 1 && g_seen.coarse == 0);
    CHECK((g_seen.kf2_n == std::vector<int>{5, 4}) && g_seen.geoms[1].ep[1] == 3.f);
    // supports(): a two-camera keyframe is left to the reference body
    k3.cam2 = true;
    CHECK(Matcher::Supports(&k1, &k2) && !Matcher::Supports(&k1, &k3));
}

static void test_search_by_projection_frame() {
    MockMP a, b, c;
    a.obs = 2;
    a.X[0] = 1.f; a.X[1] = 2.f; a.X[2] = 3.f;
    a.desc[0] = 0xAB;
    b.obs = 0;
    b.X[2] = 7.f;
    b.desc[31] = 0x11;
    c.obs = 5;
    MockFrame last, cur;
    last.kps.resize(4);
    last.desc.resize(4 * 32);
    last.ur.assign(4, -1.f);
    last.mps = {&a, nullptr, &b, &c};
    last.outlier = {false, false, false, true};  // c is an outlier: not projected
    cur.kps.resize(5);
    cur.desc.resize(5 * 32);
    cur.ur.assign(5, -1.f);
    cur.mps.assign(5, nullptr);
    cur.outlier.assign(5, false);
    Matcher matcher(0.9f, true);
    g_match = {-1, 2, -1, 0, -1};
    g_counts = {2};
    const int n = matcher.SearchByProjection(cur, last, 15.f, true);
    CHECK(n == 2);
    CHECK((g_seen.valid == std::vector<uint8_t>{1, 0, 1, 0}));
    CHECK((g_seen.observed == std::vector<uint8_t>{1, 0, 0, 0}));
    CHECK(g_seen.xyz[0] == 1.f && g_seen.xyz[2] == 3.f && g_seen.xyz[8] == 7.f && g_seen.xyz[11] == 0.f);
    CHECK(g_seen.desc[0] == 0xAB && g_seen.desc[2 * 32 + 31] == 0x11);
    CHECK(g_seen.th == 15.f && g_seen.mono == 1 && g_seen.cur.n == 5 && g_seen.cur.Tcw[3] == 0.5f);
    CHECK((cur.mps == std::vector<MockMP*>{nullptr, &b, nullptr, &a, nullptr}));
    CHECK(g_seen.h->nnratio == 0.9f && g_seen.h->check_ori == 1);
    CHECK(g_seen.cur.kps_un == cur.kps.data());  // a cleared frame is passed as it is
    // a frame that still holds map points (the reference has no precondition, src/ORBmatcher.cc:1951-2185):
    // keypoint 3 holds a (observations 2): hidden from the candidate search; keypoint 1 holds b
    // (no observations): still a candidate, and overwritten when matched
    for (int i = 0; i < 5; ++i) cur.kps[i].x = 10.f * i;
    MockMP d;
    d.obs = 0;  // keypoint 2 holds d, also without observations: a candidate, kept when not matched
    cur.mps = {nullptr, &b, &d, &a, nullptr};
    g_match = {2, -1, -1, -1, 0};
    g_counts = {2};
    CHECK(matcher.SearchByProjection(cur, last, 15.f, true) == 2);
    CHECK(g_seen.cur_x.size() == 5 && g_seen.cur_x[3] < -1e5f && g_seen.cur_x[1] == 10.f && g_seen.cur_x[2] == 20.f &&
          g_seen.cur_x[4] == 40.f);
    CHECK(g_seen.cur.kps_un != cur.kps.data() && cur.kps[3].x == 30.f);  // the frame's own keypoints untouched
    CHECK((cur.mps == std::vector<MockMP*>{&b, &b, &d, &a, &a}));       // matched entries written, others kept
    CHECK(orbgpu::LastShimError() == ORB_OK);
}

static void test_search_by_projection_local() {
    MockMP held_obs, held_new, p0, p1, p2;
    held_obs.obs = 3;
    held_new.obs = 0;
    p0.track.in_view = true;
    p0.track.proj[0] = 100.f; p0.track.proj[1] = 50.f; p0.track.proj[2] = 80.f;
    p0.track.level = 2;
    p0.desc[5] = 9;
    p1.track.in_view = false;
    p1.desc[5] = 7;  // not in view: descriptor not read
    p2.track.in_view = true;
    p2.bad = true;
    p2.obs = 0;
    MockFrame f;
    f.kps.resize(4);
    f.desc.resize(4 * 32);
    f.ur.assign(4, -1.f);
    f.mps = {&held_obs, nullptr, &held_new, nullptr};
    f.outlier.assign(4, false);
    Matcher matcher(0.8f, true);
    g_match = {-1, 0, 2, -1};  // the double says: keypoint 1 <- p0, keypoint 2 <- p2
    g_counts = {2};
    const std::vector<MockMP*> pts{&p0, &p1, &p2};
    const int n = matcher.SearchByProjection(f, pts, 5.f, true, 20.f);
    CHECK(n == 2);
    CHECK((g_seen.taken == std::vector<uint8_t>{1, 0, 0, 0}));
    CHECK((g_seen.in_view == std::vector<uint8_t>{1, 0, 1}) && (g_seen.bad == std::vector<uint8_t>{0, 0, 1}));
    CHECK((g_seen.observed == std::vector<uint8_t>{1, 1, 0}));
    CHECK(g_seen.proj[0] == 100.f && g_seen.proj[2] == 80.f && (g_seen.level == std::vector<int32_t>{2, 0, 0}));
    CHECK(g_seen.desc[5] == 9 && g_seen.desc[32 + 5] == 0);
    CHECK(g_seen.th == 5.f && g_seen.far == 1 && g_seen.th_far == 20.f);
    CHECK((f.mps == std::vector<MockMP*>{&held_obs, &p0, &p2, nullptr}));
}

static void test_errors_and_handles() {
    MockKF k1 = make_kf(3, 1), k2 = make_kf(3, 2);
    k1.fv[1] = {0, 1, 2};
    Matcher matcher(0.75f, true);
    std::vector<std::pair<size_t, size_t>> pairs{{7, 7}};
    // every entry point on a library failure: no throw, the reference's empty result, the code reported
    orbgpu::ClearShimError();
    const long fails0 = orbgpu::ShimFailureCount();
    for (int rc : {ORB_ERR_ARG, ORB_ERR_DEVICE, ORB_ERR_CAPACITY}) {
        g_rc = rc;
        bool threw = false;
        try {
            CHECK(matcher.SearchForTriangulation(&k1, &k2, pairs, false) == 0 && pairs.empty());
            CHECK(orbgpu::LastShimError() == rc);
            CHECK(orbgpu::LastShimMessage().find("fake failure") != std::string::npos);
            MockMP held, lp;
            lp.obs = 3;
            MockFrame cur, last;
            cur.kps.resize(3), cur.desc.resize(96), cur.ur.assign(3, -1.f), cur.outlier.assign(3, false);
            cur.mps = {nullptr, &held, nullptr};
            last.kps.resize(2), last.desc.resize(64), last.ur.assign(2, -1.f), last.outlier.assign(2, false);
            last.mps = {&lp, &lp};
            orbgpu::ClearShimError();
            CHECK(matcher.SearchByProjection(cur, last, 7.f, false) == 0);
            CHECK((cur.mps == std::vector<MockMP*>{nullptr, &held, nullptr}) && orbgpu::LastShimError() == rc);
            const std::vector<MockMP*> pts{&lp};
            orbgpu::ClearShimError();
            CHECK(matcher.SearchByProjection(cur, pts, 3.f) == 0);
            CHECK((cur.mps == std::vector<MockMP*>{nullptr, &held, nullptr}) && orbgpu::LastShimError() == rc);
            MockKF K = make_kf(2, 9);
            MockMP q;
            q.obsmap[&K] = std::make_tuple(1, -1);
            q.desc[0] = 0x5A;
            orbgpu::ClearShimError();
            orbgpu::ComputeDistinctiveDescriptors<Access>(std::vector<MockMP*>{&q});
            CHECK(!q.desc_set && q.desc[0] == 0x5A && orbgpu::LastShimError() == rc);
        } catch (...) {
            threw = true;
        }
        CHECK(!threw);
    }
    g_rc = 0;
    CHECK(orbgpu::ShimFailureCount() == fails0 + 12);
    // a handle that cannot be created: the search fails softly, and the next call creates it
    g_create_rc = ORB_ERR_DEVICE;
    orbgpu::ClearShimError();
    {
        MockFrame cur, last;
        cur.kps.resize(2), cur.desc.resize(64), cur.ur.assign(2, -1.f), cur.mps.assign(2, nullptr);
        last.kps.resize(1), last.desc.resize(32), last.ur.assign(1, -1.f), last.outlier.assign(1, false);
        last.mps = {nullptr};
        bool threw = false;
        try {
            CHECK(Matcher(0.31f, true).SearchByProjection(cur, last, 7.f, true) == 0);
        } catch (...) {
            threw = true;
        }
        CHECK(!threw && orbgpu::LastShimError() == ORB_ERR_ARG);  // the null handle, after the create failure
        g_create_rc = 0;
        const int c0 = g_creates;
        g_match = {-1, -1};
        g_counts = {0};
        orbgpu::ClearShimError();
        CHECK(Matcher(0.31f, true).SearchByProjection(cur, last, 7.f, true) == 0);
        CHECK(g_creates == c0 + 1 && orbgpu::LastShimError() == ORB_OK);
    }
    // handles: one per (thread, nnratio, checkOri), reused across ORBmatcher objects
    const int before = g_creates;
    g_match = {-1, -1, -1};
    g_counts = {0};
    Matcher(0.75f, true).SearchForTriangulation(&k1, &k2, pairs, false);
    Matcher(0.75f, true).SearchForTriangulation(&k1, &k2, pairs, false);
    CHECK(g_creates == before);
    Matcher(0.75f, false).SearchForTriangulation(&k1, &k2, pairs, false);
    CHECK(g_creates == before + 1);
    CHECK(Matcher::DescriptorDistance(k1.desc.data(), k2.desc.data()) == 0);
}

static void test_distinctive_batch() {
    // keyframes laid out in one array: std::map<MockKF*> order = index order
    MockKF K[3];
    for (int k = 0; k < 3; ++k) {
        K[k] = make_kf(4, k);
        for (int r = 0; r < 4; ++r) K[k].desc[32 * r] = (uint8_t)(10 * k + r);  // row tag in byte 0
    }
    K[1].bad = true;
    MockMP a, b, c, d, e;
    a.obsmap[&K[2]] = std::make_tuple(1, 3);   // left 1 then right 3
    a.obsmap[&K[0]] = std::make_tuple(2, -1);
    a.obsmap[&K[1]] = std::make_tuple(0, -1);  // bad keyframe: skipped
    b.bad = true;                               // bad point: skipped
    b.obsmap[&K[0]] = std::make_tuple(0, -1);
    // c: no observations -> skipped
    d.obsmap[&K[1]] = std::make_tuple(1, -1);   // only a bad keyframe -> no rows -> skipped
    e.obsmap[&K[0]] = std::make_tuple(-1, 0);   // right index only
    orbgpu::ComputeDistinctiveDescriptors<Access>(std::vector<MockMP*>{&a, &b, nullptr, &c, &d, &e});
    CHECK((g_dd_off == std::vector<int32_t>{0, 3, 4}));
    std::vector<int> tags;
    for (size_t r = 0; r < g_dd_rows.size() / 32; ++r) tags.push_back(g_dd_rows[32 * r]);
    CHECK((tags == std::vector<int>{2, 21, 23, 0}));  // a: K0 row 2, K2 rows 1 and 3; e: K0 row 0
    CHECK(a.desc_set && a.desc[0] == 23 && e.desc_set && e.desc[0] == 0);
    CHECK(!b.desc_set && !c.desc_set && !d.desc_set);
}

int main() {
    test_distinctive_batch();
    test_search_for_triangulation();
    test_search_by_projection_frame();
    test_search_by_projection_local();
    test_errors_and_handles();
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK matcher_shim_check\n");
    return 0;
}
