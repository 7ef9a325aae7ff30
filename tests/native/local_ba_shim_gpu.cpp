// GPU check of include/orbgpu_optimizer.hpp (the Optimizer::LocalBundleAdjustment drop-in) linked to the
// real liborbgpu.so: the shim gathers a mock keyframe / map-point graph, solves it with orb_ba_optimize
// on the device, culls and writes back.  The expected result comes from the oracle (oracle/_build/
// liborb_oracle.so, test infrastructure) run on the problem the same window flattens to, and from a
// restatement of the cull (src/Optimizer.cc:2107-2150) over the oracle's chi2 and depth flags:
//   full      -- write-back within 1e-6 RMSE of the oracle, erase set = the oracle's, in order;
//   before    -- flag up at the call: counters set, nothing solved or written (:2094-2096);
//   aborted   -- flag up between that check and the first iteration (raised from the accessor call the
//                shim makes after the check): the library returns ORB_ERR_ABORTED and the shim culls on
//                isDepthPositive of the unchanged estimates alone;
//   during    -- flag up from another thread while the device runs: the write-back equals the oracle
//                stopped right after the same number of LM trials (g2o polls the flag after each trial);
//   fallback  -- a two-camera keyframe: kFallback with every mark restored.
// Input: a C5-shaped problem written by tests/test_shims_gpu.py (synth.local_ba_problem).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "orbgpu_optimizer.hpp"

extern "C" int oracle_local_ba(orb_ba_problem_t* prob, const orb_ba_options_t* opt, double* edge_chi2_out,
                               uint8_t* depth_ok_out, orb_ba_result_t* res);
extern "C" int oracle_local_ba_stop_after(orb_ba_problem_t* prob, const orb_ba_options_t* opt, int stop_after_trials,
                                          double* edge_chi2_out, uint8_t* depth_ok_out, orb_ba_result_t* res);

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

// ---- mock graph ----------------------------------------------------------------------------------
struct MockMap;
struct MockMP;
struct MockKF {
    unsigned long mnId = 0, local = 0, fixed = 0;
    bool bad = false, cam2 = false;
    MockMap* map = nullptr;
    std::vector<MockKF*> cov;
    std::vector<MockMP*> mps;
    std::vector<float> ur;
    std::vector<double> kx, ky;
    std::vector<int> oct;
    double q[4] = {0, 0, 0, 1}, t[3] = {0, 0, 0};
    orb_ba_camera_t cam{};
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
    std::vector<std::pair<unsigned long, unsigned long>> erased;
    bool* raise_on_inertial = nullptr;  // test hook: the flag goes up at IsInertial (after the :2094 check)
};

static float g_inv_sigma2[32];

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
    static bool IsInertial(Map* m) {
        if (m->raise_on_inertial) *m->raise_on_inertial = true;
        return m->inertial;
    }
    static bool HasCamera2(KeyFrame* k) { return k->cam2; }
    static void Pose(KeyFrame* k, double q[4], double t[3]) {
        std::memcpy(q, k->q, sizeof k->q);
        std::memcpy(t, k->t, sizeof k->t);
    }
    static orb_ba_camera_t Camera(KeyFrame* k) { return k->cam; }
    static float URight(KeyFrame* k, int i) { return k->ur[i]; }
    static void KeyUn(KeyFrame* k, int i, double* x, double* y, int* octave) {
        *x = k->kx[i];
        *y = k->ky[i];
        *octave = k->oct[i];
    }
    static float InvLevelSigma2(KeyFrame*, int octave) { return g_inv_sigma2[octave]; }
    static void WorldPos(MapPoint* p, double X[3]) { std::memcpy(X, p->X, sizeof p->X); }
    static void DebugWindow(Map* m, const std::set<unsigned long>& opt, const std::set<unsigned long>& fixed) {
        m->opt = opt;
        m->fixed = fixed;
    }
    static std::mutex& MapUpdateMutex(Map* m) { return m->mtx; }
    static void EraseObservation(KeyFrame* k, MapPoint* p) {
        for (auto& s : k->mps)
            if (s == p) s = nullptr;
        p->obs.erase(k);
        p->map->erased.emplace_back(k->mnId, p->mnId);
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
using Window = orbgpu::LocalBAWindow<Access>;

// ---- input: a flattened C5 problem (tests/test_shims_gpu.py) ------------------------------------------
struct Input {
    int n_kf = 0, n_pt = 0, n_edge = 0, n_fixed = 0, n_oct = 0;
    std::vector<double> pose, point;
    std::vector<orb_ba_camera_t> cam;
    std::vector<orb_ba_edge_t> edges;
};

static bool read_input(const char* path, Input& in) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    int32_t hdr[5];
    bool ok = std::fread(hdr, sizeof hdr, 1, f) == 1;
    if (ok) {
        in.n_kf = hdr[0]; in.n_pt = hdr[1]; in.n_edge = hdr[2]; in.n_fixed = hdr[3]; in.n_oct = hdr[4];
        in.pose.resize(7 * (size_t)in.n_kf);
        in.point.resize(3 * (size_t)in.n_pt);
        in.cam.resize(in.n_kf);
        in.edges.resize(in.n_edge);
        ok = in.n_oct > 0 && in.n_oct <= 32 && std::fread(g_inv_sigma2, 4, in.n_oct, f) == (size_t)in.n_oct &&
             std::fread(in.pose.data(), 8, in.pose.size(), f) == in.pose.size() &&
             std::fread(in.point.data(), 8, in.point.size(), f) == in.point.size() &&
             std::fread(in.cam.data(), sizeof(orb_ba_camera_t), in.cam.size(), f) == in.cam.size() &&
             std::fread(in.edges.data(), sizeof(orb_ba_edge_t), in.edges.size(), f) == in.edges.size();
    }
    std::fclose(f);
    return ok;
}

// The window: pKF = the last keyframe; its covisible keyframes = every other keyframe except the first
// n_fixed (the map's init KF is keyframe 0), which enter as fixed observers of the local points.  Each
// edge becomes a keypoint slot of its keyframe; map-point observations in std::map (address) order.
struct Graph {
    MockMap M;
    std::vector<MockKF> K;
    std::vector<MockMP> P;
    explicit Graph(const Input& in) : K(in.n_kf), P(in.n_pt) {
        for (int k = 0; k < in.n_kf; ++k) {
            K[k].mnId = (unsigned long)k;
            K[k].map = &M;
            const double* v = &in.pose[7 * (size_t)k];
            for (int i = 0; i < 3; ++i) K[k].t[i] = v[i];
            for (int i = 0; i < 4; ++i) K[k].q[i] = v[3 + i];
            K[k].cam = in.cam[k];
        }
        for (int p = 0; p < in.n_pt; ++p) {
            P[p].mnId = (unsigned long)(1000 + p);
            P[p].map = &M;
            for (int i = 0; i < 3; ++i) P[p].X[i] = in.point[3 * (size_t)p + i];
        }
        for (const orb_ba_edge_t& e : in.edges) {
            MockKF& kf = K[e.pose];
            int oct = 0;
            while (oct + 1 < in.n_oct && g_inv_sigma2[oct] != e.inv_sigma2) ++oct;
            const int slot = (int)kf.mps.size();
            kf.mps.push_back(&P[e.point]);
            kf.kx.push_back(e.obs[0]);
            kf.ky.push_back(e.obs[1]);
            kf.oct.push_back(oct);
            kf.ur.push_back(e.stereo ? (float)e.obs[2] : -1.f);
            P[e.point].obs[&kf] = std::make_tuple(slot, -1);
        }
        const int last = in.n_kf - 1;
        for (int k = last - 1; k >= in.n_fixed; --k) K[last].cov.push_back(&K[k]);
        M.init_kf = 0;
    }
    MockKF* pKF() { return &K.back(); }
};

struct Expected {
    std::vector<double> pose, point;  // the window's problem arrays after the oracle's solve
    std::vector<std::pair<unsigned long, unsigned long>> erased;
    orb_ba_result_t res{};
    int rc = 0;
};

// the oracle on the problem the window flattens to, then the cull restated over its chi2 / depth flags
static Expected expect(const Input& in, int stop_after, bool inertial, bool depth_only = false) {
    Graph g(in);
    Window w;
    Expected x;
    if (w.Gather(g.pKF(), &g.M) != Window::kOk) return x;
    orb_ba_problem_t prob = w.Problem();
    orb_ba_options_t opt{};
    opt.iterations = 10;
    opt.user_lambda_init = inertial ? 100.0 : 0.0;
    std::vector<double> chi2(w.edges.size(), 0.0);
    std::vector<uint8_t> depth(w.edges.size(), 1);
    x.rc = stop_after >= 0 ? oracle_local_ba_stop_after(&prob, &opt, stop_after, chi2.data(), depth.data(), &x.res)
                           : oracle_local_ba(&prob, &opt, chi2.data(), depth.data(), &x.res);
    if (depth_only || x.rc == ORB_ERR_ABORTED) {
        // no iteration ran: chi2 of the constructed edges is 0; depth z = (R X + t).z of the initial state
        std::fill(chi2.begin(), chi2.end(), 0.0);
        for (size_t e = 0; e < w.edges.size(); ++e) {
            const double* T = &w.pose[7 * (size_t)w.edges[e].pose];
            const double* X = &w.point[3 * (size_t)w.edges[e].point];
            double qx = T[3], qy = T[4], qz = T[5], qw = T[6];
            const double nn = std::sqrt(qx * qx + qy * qy + qz * qz + qw * qw);
            qx /= nn; qy /= nn; qz /= nn; qw /= nn;
            const double z = 2 * (qx * qz - qw * qy) * X[0] + 2 * (qy * qz + qw * qx) * X[1] +
                             (1 - 2 * (qx * qx + qy * qy)) * X[2] + T[2];
            depth[e] = z > 0 ? 1 : 0;
        }
    }
    for (int pass = 0; pass < 2; ++pass)
        for (size_t e = 0; e < w.edges.size(); ++e) {
            if (w.edges[e].stereo != pass) continue;
            const double th = pass ? 7.815 : 5.991;
            if (chi2[e] > th || !depth[e]) x.erased.emplace_back(w.edge_kf[e]->mnId, w.edge_mp[e]->mnId);
        }
    x.pose = w.pose;
    x.point = w.point;
    return x;
}

// The window's local point order (Gather on an untouched copy of the graph: the write-back's erasures
// change MapPointMatches, so it cannot be re-derived from the graph after the call), as point indices.
static std::vector<int> local_point_order(const Input& in) {
    Graph g(in);
    Window w;
    w.Gather(g.pKF(), &g.M);
    std::vector<int> idx;
    for (MockMP* p : w.local_mps) idx.push_back((int)(p - g.P.data()));
    return idx;
}

// RMSE of the written-back local keyframe poses (t, q) and points against the expectation's arrays
static void written_rmse(Graph& g, const Input& in, const Expected& x, double* pose_rmse, double* point_rmse) {
    double sp = 0, sq = 0;
    size_t np = 0, nq = 0;
    // local KFs: pKF then its covisible list, the vertex order of the expectation
    std::vector<MockKF*> locals{g.pKF()};
    for (MockKF* k : g.pKF()->cov) locals.push_back(k);
    for (size_t i = 0; i < locals.size(); ++i) {
        const double* e = &x.pose[7 * i];
        for (int k = 0; k < 3; ++k) sp += (locals[i]->t[k] - e[k]) * (locals[i]->t[k] - e[k]);
        for (int k = 0; k < 4; ++k) sp += (locals[i]->q[k] - e[3 + k]) * (locals[i]->q[k] - e[3 + k]);
        np += 7;
    }
    const std::vector<int> order = local_point_order(in);
    for (size_t i = 0; i < order.size() && 3 * i + 2 < x.point.size(); ++i)
        for (int k = 0; k < 3; ++k) {
            const double d = g.P[order[i]].X[k] - x.point[3 * i + k];
            sq += d * d;
            ++nq;
        }
    *pose_rmse = std::sqrt(sp / std::max<size_t>(np, 1));
    *point_rmse = std::sqrt(sq / std::max<size_t>(nq, 1));
}

static void test_full(orb_ba_t h, const Input& in, bool inertial) {
    const Expected x = expect(in, -1, inertial);
    CHECK(x.rc == ORB_OK && x.res.iterations > 0);
    Graph g(in);
    g.M.inertial = inertial;
    bool stop = false;
    int nf = -1, no = -1, nmp = -1, ne = -1;
    const int rc = orbgpu::LocalBundleAdjustment<Access>(h, g.pKF(), &stop, &g.M, nf, no, nmp, ne);
    CHECK(rc == ORB_OK);
    if (rc != ORB_OK) std::printf("  rc %d: %s\n", rc, orb_last_error());
    double pr, qr;
    written_rmse(g, in, x, &pr, &qr);
    std::printf("full(inertial=%d): %d it %d trials, pose rmse %.3g, point rmse %.3g, %zu erased (oracle %zu)\n",
                (int)inertial, x.res.iterations, x.res.trials, pr, qr, g.M.erased.size(), x.erased.size());
    CHECK(pr < 1e-6 && qr < 1e-6);
    CHECK(g.M.erased == x.erased);
    CHECK(g.M.change == 1 && nf == in.n_fixed && no == in.n_kf - in.n_fixed && nmp == -1);
    CHECK(ne == in.n_edge || ne > 0);
    for (int k = 0; k < in.n_fixed; ++k) CHECK(!g.K[k].pose_written);
    for (int k = in.n_fixed; k < in.n_kf; ++k) CHECK(g.K[k].pose_written);
}

static void test_stop_before(orb_ba_t h, const Input& in) {
    Graph g(in);
    bool stop = true;
    int nf = -1, no = -1, nmp = -1, ne = -1;
    CHECK(orbgpu::LocalBundleAdjustment<Access>(h, g.pKF(), &stop, &g.M, nf, no, nmp, ne) == ORB_OK);
    CHECK(nf == in.n_fixed && no == in.n_kf - in.n_fixed && ne > 0 && g.M.change == 0 && g.M.erased.empty());
    for (auto& k : g.K) CHECK(!k.pose_written);
}

static void test_aborted(orb_ba_t h, Input in) {
    // some points behind every camera in the initial state, so that the depth-only cull erases edges
    for (int p = 0; p < in.n_pt; p += 97) in.point[3 * (size_t)p + 2] = -4.0;
    const Expected x = expect(in, 0, false, true);
    CHECK(x.rc == ORB_ERR_ABORTED);
    Graph g(in);
    bool stop = false;
    g.M.raise_on_inertial = &stop;
    int nf, no, nmp, ne;
    CHECK(orbgpu::LocalBundleAdjustment<Access>(h, g.pKF(), &stop, &g.M, nf, no, nmp, ne) == ORB_OK);
    double pr, qr;
    written_rmse(g, in, x, &pr, &qr);
    std::printf("aborted: %zu erased (expected %zu), pose diff %.3g, point diff %.3g\n", g.M.erased.size(),
                x.erased.size(), pr, qr);
    CHECK(!x.erased.empty() && g.M.erased == x.erased);
    CHECK(pr == 0.0 && qr == 0.0 && g.M.change == 1);  // the unchanged estimates, written back
}

static void test_stop_during(orb_ba_t h, const Input& in) {
    const Expected full = expect(in, -1, false);
    const int tfull = full.res.trials;
    std::vector<Expected> at(tfull + 1);
    for (int t = 0; t <= tfull; ++t) at[t] = expect(in, t, false);
    bool stopped_early = false;
    // raise the flag from another thread after a delay; shorten the delay until the solve is cut short
    for (int delay_us : {900, 600, 400, 250, 150, 80}) {
        Graph g(in);
        bool stop = false;
        std::atomic<bool> go{false};
        std::thread th([&] {
            while (!go.load()) std::this_thread::yield();
            std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
            reinterpret_cast<volatile bool&>(stop) = true;
        });
        int nf, no, nmp, ne;
        go = true;
        const int rc = orbgpu::LocalBundleAdjustment<Access>(h, g.pKF(), &stop, &g.M, nf, no, nmp, ne);
        th.join();
        CHECK(rc == ORB_OK);
        if (!g.M.change) continue;  // the flag beat the check at :2094: nothing solved, try again
        int best = -1;
        double best_p = 1e30, best_q = 1e30;
        for (int t = 0; t <= tfull; ++t) {
            double pr, qr;
            written_rmse(g, in, at[t], &pr, &qr);
            if (pr + qr < best_p + best_q) { best = t; best_p = pr; best_q = qr; }
        }
        std::printf("during (flag after %d us): matches the oracle stopped after %d of %d trials (pose %.3g, point "
                    "%.3g), %zu erased (oracle %zu)\n",
                    delay_us, best, tfull, best_p, best_q, g.M.erased.size(), best >= 0 ? at[best].erased.size() : 0);
        CHECK(best >= 0 && best_p < 1e-6 && best_q < 1e-6);
        if (best >= 0) CHECK(g.M.erased == at[best].erased);
        if (best >= 0 && best < tfull) {
            stopped_early = true;
            break;
        }
    }
    CHECK(stopped_early);
}

static void test_fallback_camera2(orb_ba_t h, const Input& in) {
    Graph g(in);
    g.K[in.n_kf / 2].cam2 = true;
    int nf = -7, no = -7, nmp = -7, ne = -7;
    CHECK(orbgpu::LocalBundleAdjustment<Access>(h, g.pKF(), nullptr, &g.M, nf, no, nmp, ne) == orbgpu::kFallback);
    CHECK(nf == -7 && g.M.change == 0);
    for (auto& k : g.K) CHECK(k.local == 0 && k.fixed == 0 && !k.pose_written);
    for (auto& p : g.P) CHECK(p.local == 0 && !p.pos_written);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("usage: %s problem.bin [full|all]\n", argv[0]);
        return 2;
    }
    Input in;
    if (!read_input(argv[1], in)) {
        std::printf("cannot read %s\n", argv[1]);
        return 2;
    }
    const bool all = argc < 3 || std::string(argv[2]) == "all";
    orb_ba_t h = nullptr;
    if (orb_ba_create(&h) != ORB_OK) {
        std::printf("orb_ba_create: %s\n", orb_last_error());
        return 2;
    }
    test_full(h, in, false);
    if (all) {
        test_full(h, in, true);
        test_stop_before(h, in);
        test_aborted(h, in);
        test_stop_during(h, in);
        test_fallback_camera2(h, in);
    }
    orb_ba_destroy(h);
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK local_ba_shim_gpu\n");
    return 0;
}
