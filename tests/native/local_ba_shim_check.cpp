// CPU check of include/orbgpu_optimizer.hpp (the Optimizer::LocalBundleAdjustment drop-in) on a mock
// keyframe / map-point graph.  The solve is a test double of orb_ba_optimize defined below (records the
// flattened problem, returns chosen chi2 / depth flags), so this runs without a GPU; the real solve is
// compared with the oracle in tests/test_ba_gpu.py.  What is checked here is the host side the shim
// restates from src/Optimizer.cc:
//   * the window (:1744-1808): pKF + good same-map covisible KFs, local points in KF-then-slot order,
//     fixed KFs in first-observer order, bad / other-map KFs marked but not added, num_fixedKF (:1810),
//     the abort on 0 fixed KFs (:1851-1855);
//   * vertices (:1884-1975): local KFs (init KF fixed) then fixed KFs, point ids mnId + maxKFid + 1;
//   * edges (:1977-2091): per point in std::map<KeyFrame*> order, mono when mvuRight < 0 else stereo,
//     information = mvInvLevelSigma2[octave], left index -1 skipped;
//   * the stop flag checked before optimize (:2094-2096) and passed on as a bool*;
//   * the cull (:2107-2150): mono edges then stereo edges, bad map points skipped, chi2 > 5.991 /
//     7.815 or depth <= 0; erase under mMutexMapUpdate (:2153-2164); write-back of local KFs only and
//     every local point, then IncreaseChangeIndex (:2169-2187).
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "orbgpu_optimizer.hpp"

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

struct MockMap;
struct MockMP;

struct MockKF {
    unsigned long mnId = 0, local = 0, fixed = 0;
    bool bad = false, cam2 = false;
    MockMap* map = nullptr;
    std::vector<MockKF*> cov;
    std::vector<MockMP*> mps;  // GetMapPointMatches (slot i = keypoint i)
    std::vector<float> ur;
    std::vector<std::tuple<float, float, int>> kps;  // mvKeysUn: x, y, octave
    double q[4] = {0, 0, 0, 1}, t[3] = {0, 0, 0};
    bool pose_written = false;
};

struct MockMP {
    unsigned long mnId = 0, local = 0;
    bool bad = false;
    MockMap* map = nullptr;
    std::map<MockKF*, std::tuple<int, int>> obs;
    double X[3] = {0, 0, 0};
    bool pos_written = false;
};

struct MockMap {
    unsigned long init_kf = 0;
    bool inertial = false;
    std::mutex mtx;
    std::set<unsigned long> opt, fixed;
    int change = 0;
    std::vector<std::pair<unsigned long, unsigned long>> erased;  // (KF id, MP id) in erase order
    bool erased_under_lock = true;
};

struct Access {
    using KeyFrame = MockKF;
    using MapPoint = MockMP;
    using Map = MockMap;
    static unsigned long Id(KeyFrame* k) { return k->mnId; }
    static unsigned long Id(MapPoint* p) { return p->mnId; }
    static unsigned long& BALocalForKF(KeyFrame* k) { return k->local; }
    static unsigned long& BAFixedForKF(KeyFrame* k) { return k->fixed; }
    static unsigned long& BALocalForKF(MapPoint* p) { return p->local; }
    static bool IsBad(KeyFrame* k) { return k->bad; }
    static bool IsBad(MapPoint* p) { return p->bad; }
    static Map* GetMap(KeyFrame* k) { return k->map; }
    static Map* GetMap(MapPoint* p) { return p->map; }
    static std::vector<KeyFrame*> Covisible(KeyFrame* k) { return k->cov; }
    static std::vector<MapPoint*> MapPointMatches(KeyFrame* k) { return k->mps; }
    static std::map<KeyFrame*, std::tuple<int, int>> Observations(MapPoint* p) { return p->obs; }
    static unsigned long InitKFid(Map* m) { return m->init_kf; }
    static bool IsInertial(Map* m) { return m->inertial; }
    static bool HasCamera2(KeyFrame* k) { return k->cam2; }
    static void Pose(KeyFrame* k, double q[4], double t[3]) {
        std::memcpy(q, k->q, sizeof k->q);
        std::memcpy(t, k->t, sizeof k->t);
    }
    static orb_ba_camera_t Camera(KeyFrame* k) { return {400.f + k->mnId, 401.f, 320.f, 240.f, 40.f}; }
    static float URight(KeyFrame* k, int i) { return k->ur[i]; }
    static void KeyUn(KeyFrame* k, int i, double* x, double* y, int* octave) {
        *x = std::get<0>(k->kps[i]);
        *y = std::get<1>(k->kps[i]);
        *octave = std::get<2>(k->kps[i]);
    }
    static float InvLevelSigma2(KeyFrame*, int octave) {
        float s = 1.f;
        for (int l = 0; l < octave; ++l) s *= 1.44f;
        return 1.f / s;
    }
    static void WorldPos(MapPoint* p, double X[3]) { std::memcpy(X, p->X, sizeof p->X); }
    static void DebugWindow(Map* m, const std::set<unsigned long>& opt, const std::set<unsigned long>& fixed) {
        m->opt = opt;
        m->fixed = fixed;
    }
    static std::mutex& MapUpdateMutex(Map* m) { return m->mtx; }
    static void EraseObservation(KeyFrame* k, MapPoint* p) {
        MockMap* m = p->map;
        if (m->mtx.try_lock()) {  // the shim must hold mMutexMapUpdate here
            m->erased_under_lock = false;
            m->mtx.unlock();
        }
        for (auto& s : k->mps)
            if (s == p) s = nullptr;
        p->obs.erase(k);
        m->erased.emplace_back(k->mnId, p->mnId);
    }
    static void SetPose(KeyFrame* k, const double q[4], const double t[3]) {
        std::memcpy(k->q, q, sizeof k->q);
        std::memcpy(k->t, t, sizeof k->t);
        k->pose_written = true;
    }
    static void SetWorldPos(MapPoint* p, const double X[3]) {
        std::memcpy(p->X, X, sizeof p->X);
        p->pos_written = true;
    }
    static void IncreaseChangeIndex(Map* m) { ++m->change; }
};

// ---- test double of the GPU solve ---------------------------------------------------------------
struct SolveRecord {
    int calls = 0;
    int rc = ORB_OK;
    std::vector<int64_t> pose_id, point_id;
    std::vector<uint8_t> pose_fixed;
    std::vector<orb_ba_edge_t> edges;
    std::vector<double> chi2;       // returned per edge
    std::vector<uint8_t> depth;     // returned per edge
    orb_ba_options_t opt{};
    double pose_shift = 0.5;        // added to every non-fixed pose's tx, every point's x
} g_solve;

// REGISTER_TIMES doubles: the shim's "LBA" bracket (timers off here; the GPU shim test links the library)
extern "C" int orb_timers_enabled(void) { return 0; }
extern "C" int orb_timer_add(const char*, double) { return 0; }
extern "C" int orb_ba_optimize(orb_ba_t, orb_ba_problem_t* p, const orb_ba_options_t* o, double* chi2,
                               uint8_t* depth, orb_ba_result_t* res) {
    ++g_solve.calls;
    g_solve.opt = *o;
    g_solve.pose_id.assign(p->pose_id, p->pose_id + p->n_poses);
    g_solve.point_id.assign(p->point_id, p->point_id + p->n_points);
    g_solve.pose_fixed.assign(p->pose_fixed, p->pose_fixed + p->n_poses);
    g_solve.edges.assign(p->edges, p->edges + p->n_edges);
    if (g_solve.rc != ORB_OK) return g_solve.rc;
    for (int i = 0; i < p->n_poses; ++i)
        if (!p->pose_fixed[i]) p->pose[7 * i] += g_solve.pose_shift;
    for (int i = 0; i < p->n_points; ++i) p->point[3 * i] += g_solve.pose_shift;
    for (int e = 0; e < p->n_edges; ++e) {
        chi2[e] = e < (int)g_solve.chi2.size() ? g_solve.chi2[e] : 0.0;
        depth[e] = e < (int)g_solve.depth.size() ? g_solve.depth[e] : 1;
    }
    *res = orb_ba_result_t{};
    return ORB_OK;
}

// ---- the graph ------------------------------------------------------------------------------------
// Keyframes K0..K9 (mnId = index), one map M plus another map M2.  pKF = K5.
//   K5 covisible: K4, K3, K7 (bad), K8 (other map), K2.        -> local = K5 K4 K3 K2
//   init KF = K0 (not local) -> fixed via observation.
// Map points P100..P107 (mnId = 100 + i), P106 bad, P107 in M2.  Observers (map order = address order,
// and the KFs are laid out in one array so address order = index order):
struct Graph {
    MockMap M, M2;
    MockKF K[10];
    MockMP P[8];
    Graph() {
        for (int i = 0; i < 10; ++i) {
            K[i].mnId = i;
            K[i].map = &M;
            K[i].t[0] = i;
            K[i].ur.assign(8, -1.f);
            for (int s = 0; s < 8; ++s) K[i].kps.emplace_back(10.f * i + s, 20.f * i + s, s % 8);
            K[i].mps.assign(8, nullptr);
        }
        K[7].bad = true;
        K[8].map = &M2;
        K[9].bad = true;
        K[5].cov = {&K[4], &K[3], &K[7], &K[8], &K[2]};
        for (int i = 0; i < 8; ++i) {
            P[i].mnId = 100 + i;
            P[i].map = &M;
            P[i].X[0] = i;
            P[i].X[2] = 5;
        }
        P[6].bad = true;
        P[7].map = &M2;
        // observation (kf, slot); stereo slots get ur >= 0
        auto obs = [&](int kf, int mp, int slot, float ur = -1.f) {
            K[kf].mps[slot] = &P[mp];
            K[kf].ur[slot] = ur;
            P[mp].obs[&K[kf]] = std::make_tuple(slot, -1);
        };
        obs(5, 2, 0);           // K5 slot 0 -> P2
        obs(5, 0, 1, 12.f);     // K5 slot 1 -> P0 (stereo)
        obs(5, 6, 2);           // K5 slot 2 -> P6 (bad point: not local)
        obs(4, 1, 0);           // K4 slot 0 -> P1
        obs(4, 2, 3);           // K4 slot 3 -> P2 (already local)
        obs(3, 3, 1, 0.f);      // K3 slot 1 -> P3 (stereo, ur = 0)
        obs(3, 7, 2);           // K3 slot 2 -> P7 (other map: not local)
        obs(2, 4, 4);           // K2 slot 4 -> P4
        obs(1, 0, 5);           // K1 observes P0 -> fixed
        obs(0, 1, 6);           // K0 observes P1 -> fixed (init KF)
        obs(9, 3, 7);           // K9 (bad) observes P3 -> marked, not fixed, no edge
        obs(8, 4, 0);           // K8 (other map) observes P4 -> marked, not fixed, no edge
        obs(7, 2, 1);           // K7 (bad, covisible) observes P2 -> no edge
        P[4].obs[&K[6]] = std::make_tuple(-1, 3);  // K6 sees P4 in a right image only: fixed, no edge
        K[6].mps[3] = nullptr;
        P[5].obs[&K[1]] = std::make_tuple(2, -1);  // P5 is seen by no local KF: not a local point
        M.init_kf = 0;
    }
};

static void test_window_and_problem() {
    Graph g;
    orbgpu::LocalBAWindow<Access> w;
    CHECK(w.Gather(&g.K[5], &g.M) == orbgpu::LocalBAWindow<Access>::kOk);
    // local KFs and points
    CHECK((w.local_kfs == std::vector<MockKF*>{&g.K[5], &g.K[4], &g.K[3], &g.K[2]}));
    CHECK((w.local_mps == std::vector<MockMP*>{&g.P[2], &g.P[0], &g.P[1], &g.P[3], &g.P[4]}));
    // fixed: observers of P2 (K4,K5,K7 local/bad), P0 (K1), P1 (K0), P3 (K9 bad), P4 (K6, K8 other map)
    CHECK((w.fixed_kfs == std::vector<MockKF*>{&g.K[1], &g.K[0], &g.K[6]}));
    CHECK(w.num_fixed_kf == 3);
    CHECK(g.K[9].fixed == 5);  // marked even though not added (:1803)
    CHECK(g.K[8].fixed == 0);  // K8 carries the local mark of the covisible loop, so it is never marked fixed
    CHECK(g.K[7].local == 5 && g.K[8].local == 5);
    CHECK(w.max_kf_id == 6);
    CHECK((w.pose_id == std::vector<int64_t>{5, 4, 3, 2, 1, 0, 6}));
    CHECK((w.pose_fixed == std::vector<uint8_t>{0, 0, 0, 0, 1, 1, 1}));
    CHECK((w.point_id == std::vector<int64_t>{102 + 7, 100 + 7, 101 + 7, 103 + 7, 104 + 7}));
    CHECK(w.pose[7 * 1] == 4.0 && w.pose[7 * 1 + 6] == 1.0);  // (tx ty tz qx qy qz qw)
    CHECK(w.point[3 * 1] == 0.0 && w.point[3 * 4] == 4.0);
    // edges: per point, observers in map order; {point, pose, stereo, keypoint slot}
    // P2 observers in map order: K4, K5, K7(bad) -> pose 1 (slot 3), pose 0 (slot 0)
    // P0: K1, K5 -> pose 4 (slot 5, mono), pose 0 (slot 1, stereo ur 12)
    // P1: K0, K4 -> pose 5 (slot 6), pose 1 (slot 0)
    // P3: K3, K9(bad) -> pose 2 (slot 1, stereo ur 0)
    // P4: K2, K6 (left -1), K8 (other map) -> pose 3 (slot 4)
    const int exp[][4] = {{0, 1, 0, 3}, {0, 0, 0, 0}, {1, 4, 0, 5}, {1, 0, 1, 1}, {2, 5, 0, 6},
                          {2, 1, 0, 0}, {3, 2, 1, 1}, {4, 3, 0, 4}};
    CHECK(w.edges.size() == 8);
    for (size_t i = 0; i < w.edges.size() && i < 8; ++i) {
        const orb_ba_edge_t& e = w.edges[i];
        CHECK(e.point == exp[i][0] && e.pose == exp[i][1] && e.stereo == exp[i][2]);
        const MockKF* k = w.edge_kf[i];
        const int slot = exp[i][3];
        CHECK(e.obs[0] == (double)std::get<0>(k->kps[slot]) && e.obs[1] == (double)std::get<1>(k->kps[slot]));
        CHECK(e.obs[2] == (e.stereo ? (double)k->ur[slot] : 0.0));
        CHECK(e.inv_sigma2 == Access::InvLevelSigma2(nullptr, slot % 8));
        CHECK(w.edge_mp[i] == w.local_mps[e.point]);
    }
    orb_ba_problem_t p = w.Problem();
    CHECK(p.n_poses == 7 && p.n_points == 5 && p.n_edges == 8 && p.pose == w.pose.data());
}

static void test_init_kf_local_and_abort() {
    {   // the map's init KF inside the window: a fixed local vertex, num_fixedKF counts it
        Graph g;
        g.M.init_kf = 4;
        orbgpu::LocalBAWindow<Access> w;
        CHECK(w.Gather(&g.K[5], &g.M) == orbgpu::LocalBAWindow<Access>::kOk);
        CHECK(w.num_fixed_kf == 4);
        CHECK((w.pose_fixed == std::vector<uint8_t>{0, 1, 0, 0, 1, 1, 1}));
    }
    {   // no fixed KF at all: "LBA aborted", nothing written, num_fixedKF = 0
        Graph g;
        g.M.init_kf = 99;
        g.P[0].obs.erase(&g.K[1]);
        g.P[1].obs.erase(&g.K[0]);
        g.P[4].obs.erase(&g.K[6]);
        g_solve = SolveRecord();
        int nf = -1, no = -1, nmp = 77, ne = -1;
        bool stop = false;
        const int rc = orbgpu::LocalBundleAdjustment<Access>(nullptr, &g.K[5], &stop, &g.M, nf, no, nmp, ne);
        CHECK(rc == ORB_OK && nf == 0 && no == -1 && ne == -1 && nmp == 77);
        CHECK(g_solve.calls == 0 && g.M.change == 0 && g.M.opt.empty());
    }
    {   // a two-camera keyframe in the window: left to the reference optimiser, with every mark restored
        Graph g;
        g.K[3].cam2 = true;
        g.K[1].fixed = 3;  // marks left by an earlier window (pKF = K3) must come back as they were
        g.P[0].local = 3;
        g_solve = SolveRecord();
        int nf = -7, no = -7, nmp = -7, ne = -7;
        CHECK(orbgpu::LocalBundleAdjustment<Access>(nullptr, &g.K[5], nullptr, &g.M, nf, no, nmp, ne) ==
              orbgpu::kFallback);
        CHECK(g_solve.calls == 0 && nf == -7 && no == -7 && ne == -7 && g.M.opt.empty());
        for (int i = 0; i < 10; ++i) CHECK(g.K[i].local == 0 && g.K[i].fixed == (i == 1 ? 3u : 0u));
        for (int i = 0; i < 8; ++i) CHECK(g.P[i].local == (i == 0 ? 3u : 0u));
        // the reference body, run next on the same graph, builds the full window from the marks
        // (src/Optimizer.cc:1748-1803; Gather restates exactly that part)
        orbgpu::LocalBAWindow<Access> ref;
        ref.Gather(&g.K[5], &g.M);
        CHECK((ref.local_kfs == std::vector<MockKF*>{&g.K[5], &g.K[4], &g.K[3], &g.K[2]}));
        CHECK((ref.local_mps == std::vector<MockMP*>{&g.P[2], &g.P[0], &g.P[1], &g.P[3], &g.P[4]}));
        CHECK((ref.fixed_kfs == std::vector<MockKF*>{&g.K[1], &g.K[0], &g.K[6]}) && ref.num_fixed_kf == 3);
    }
    {   // the library cannot take the window (or the device fails): the same fallback, nothing written
        Graph g;
        g_solve = SolveRecord();
        g_solve.rc = ORB_ERR_DEVICE;
        bool stop = false;
        int nf, no, nmp, ne;
        CHECK(orbgpu::LocalBundleAdjustment<Access>(nullptr, &g.K[5], &stop, &g.M, nf, no, nmp, ne) ==
              orbgpu::kFallback);
        CHECK(g_solve.calls == 1 && g.M.change == 0 && g.M.erased.empty() && !g.K[5].pose_written);
        for (int i = 0; i < 10; ++i) CHECK(g.K[i].local == 0 && g.K[i].fixed == 0);
        for (int i = 0; i < 8; ++i) CHECK(g.P[i].local == 0 && !g.P[i].pos_written);
    }
}

static void test_stop_flag_before_optimize() {
    Graph g;
    g_solve = SolveRecord();
    int nf = -1, no = -1, nmp = -1, ne = -1;
    bool stop = true;
    CHECK(orbgpu::LocalBundleAdjustment<Access>(nullptr, &g.K[5], &stop, &g.M, nf, no, nmp, ne) == ORB_OK);
    // counters and the DEBUG LBA sets are written before the flag test (:1879-1898, 2092-2096)
    CHECK(nf == 3 && no == 4 && ne == 8 && nmp == -1);
    CHECK((g.M.opt == std::set<unsigned long>{2, 3, 4, 5}) && (g.M.fixed == std::set<unsigned long>{0, 1, 6}));
    CHECK(g_solve.calls == 0 && g.M.change == 0 && !g.K[5].pose_written);
}

static void test_solve_cull_write_back() {
    Graph g;
    g.M.inertial = true;
    g_solve = SolveRecord();
    // edge order (see test_window_and_problem): 0 P2-K4 m, 1 P2-K5 m, 2 P0-K1 m, 3 P0-K5 s, 4 P1-K0 m,
    // 5 P1-K4 m, 6 P3-K3 s, 7 P4-K2 m
    g_solve.chi2 = {6.0, 5.991, 1.0, 7.9, 0.1, 0.2, 7.8, 0.3};
    g_solve.depth = {1, 1, 1, 1, 1, 0, 0, 1};
    bool stop = false;
    int nf, no, nmp = 5, ne;
    CHECK(orbgpu::LocalBundleAdjustment<Access>(nullptr, &g.K[5], &stop, &g.M, nf, no, nmp, ne) == ORB_OK);
    CHECK(g_solve.calls == 1);
    CHECK(g_solve.opt.iterations == 10 && g_solve.opt.user_lambda_init == 100.0);
    CHECK(g_solve.opt.stop_flag == nullptr && (const void*)g_solve.opt.stop_flag_bool == (const void*)&stop);
    // erase: mono 0 (chi2 6 > 5.991), mono 5 (depth), then stereo 3 (7.9 > 7.815), stereo 6 (depth)
    const std::vector<std::pair<unsigned long, unsigned long>> want = {{4, 102}, {4, 101}, {5, 100}, {3, 103}};
    CHECK(g.M.erased == want);
    CHECK(g.M.erased_under_lock);
    CHECK(g.K[4].mps[3] == nullptr && g.P[2].obs.count(&g.K[4]) == 0);
    // write-back: local KFs only (the fixed K0, K1, K6 are untouched), every local point
    for (int k : {5, 4, 3, 2}) CHECK(g.K[k].pose_written && g.K[k].t[0] == k + 0.5);
    for (int k : {0, 1, 6}) CHECK(!g.K[k].pose_written);
    for (int p : {0, 1, 2, 3, 4}) CHECK(g.P[p].pos_written && g.P[p].X[0] == p + 0.5);
    CHECK(!g.P[5].pos_written && !g.P[6].pos_written);
    CHECK(g.M.change == 1 && nmp == 5);
}

static void test_cull_skips_bad_points() {
    Graph g;
    g_solve = SolveRecord();
    g_solve.chi2.assign(8, 100.0);  // every edge over threshold
    // a map point that turned bad while the solve ran (LocalMapping's culling runs concurrently)
    orbgpu::LocalBAWindow<Access> w;
    CHECK(w.Gather(&g.K[5], &g.M) == orbgpu::LocalBAWindow<Access>::kOk);
    g.P[0].bad = true;
    std::vector<double> chi2(w.edges.size(), 100.0);
    std::vector<uint8_t> depth(w.edges.size(), 1);
    w.CullAndWriteBack(&g.M, chi2.data(), depth.data());
    // P0's edges (2 mono, 3 stereo) skipped; the rest in mono-then-stereo order
    const std::vector<std::pair<unsigned long, unsigned long>> want = {
        {4, 102}, {5, 102}, {0, 101}, {4, 101}, {2, 104}, {3, 103}};
    CHECK(g.M.erased == want);
}

static void test_aborted_solve_uses_depth_only() {
    Graph g;
    g_solve = SolveRecord();
    g_solve.rc = ORB_ERR_ABORTED;  // the flag went up between the check at :2094 and the first iteration
    g.P[3].X[2] = -5;              // P3 behind every camera (identity rotations): its edge is culled
    bool stop = false;
    int nf, no, nmp, ne;
    CHECK(orbgpu::LocalBundleAdjustment<Access>(nullptr, &g.K[5], &stop, &g.M, nf, no, nmp, ne) == ORB_OK);
    const std::vector<std::pair<unsigned long, unsigned long>> want = {{3, 103}};
    CHECK(g.M.erased == want);
    CHECK(g.K[5].pose_written && g.K[5].t[0] == 5.0);  // unchanged estimates written back
    CHECK(g.M.change == 1);
}

int main() {
    test_window_and_problem();
    test_init_kf_local_and_abort();
    test_stop_flag_before_optimize();
    test_solve_cull_write_back();
    test_cull_skips_bad_points();
    test_aborted_solve_uses_depth_only();
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK local_ba_shim_check\n");
    return 0;
}
