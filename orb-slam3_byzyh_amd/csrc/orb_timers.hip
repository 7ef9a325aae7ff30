// REGISTER_TIMES on the ABI path.  The reference brackets its stages with std::chrono::steady_clock
// when the compile-time macro is on (include/Settings.h:24): the ORB extraction of a Frame
// (src/Frame.cc:132-146, mTimeORB_Ext), stereo matching (:158-170) and LocalMapping's LBA
// (src/LocalMapping.cc:213-230, vdLBA_ms), and prints mean $\pm$ population std per stage to ExecMean.txt
// (src/Tracking.cc:189-208, 318-420).  Here the same wall-clock brackets sit inside the synchronous
// entry points (orb_extract -> "ORB Extraction", orb_compute_stereo_matches -> "Stereo Matching",
// and the host side of Optimizer::LocalBundleAdjustment -> "LBA": the shim include/orbgpu_optimizer.hpp and
// the Python mirror, gather to write-back, no sample when the reference body has to take over),
// switched on at run time (orb_timers_enable, or ORBGPU_REGISTER_TIMES in the environment) instead of at
// compile time; off, a bracket costs one relaxed atomic load.  Mode 2 leaves the per-call brackets off
// for a caller that times a whole Frame itself: the reference's "ORB Extraction" sample is one per
// Frame, covering a stereo pair's two extractions run in parallel (src/Frame.cc:132-146), which such a
// caller records with orb_timer_add.  ExecMean.txt's numbers are fixed with 5 decimals: the reference
// sets `f << fixed` (src/Tracking.cc:327) and then `setprecision(5)` (:335).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "orbgpu.h"
#include "orbgpu_internal.h"

namespace {
std::atomic<int> g_on{-1};  // -1: not read from the environment yet
std::mutex g_mu;
std::map<std::string, std::vector<double>>& stats() {
    static std::map<std::string, std::vector<double>> s;
    return s;
}
// the stage order of ExecMean.txt's sections this build fills
const char* const kOrder[] = {"ORB Extraction", "Stereo Matching", "LBA"};
}  // namespace

namespace orbgpu {
bool timers_on() {
    int v = g_on.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("ORBGPU_REGISTER_TIMES");
        v = (e && *e && *e != '0') ? (*e == '2' ? 2 : 1) : 0;
        int expect = -1;
        g_on.compare_exchange_strong(expect, v);
        v = g_on.load(std::memory_order_relaxed);
    }
    return v == 1;  // mode 2: the caller brackets its own stages (orb_timer_add); no per-call brackets
}
void timer_add(const char* name, double ms) {
    std::lock_guard<std::mutex> lk(g_mu);
    stats()[name].push_back(ms);
}
}  // namespace orbgpu

extern "C" {

int orb_timers_enable(int on) {
    if (on < 0 || on > 2) return orbgpu_fail(ORB_ERR_ARG, "timer mode must be 0, 1 or 2");
    g_on.store(on, std::memory_order_relaxed);
    return ORB_OK;
}

int orb_timers_enabled(void) {
    (void)orbgpu::timers_on();  // (reads ORBGPU_REGISTER_TIMES on first use)
    return g_on.load(std::memory_order_relaxed);
}

int orb_timers_reset(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    stats().clear();
    return ORB_OK;
}

int orb_timer_add(const char* name, double ms) {
    if (!name) return orbgpu_fail(ORB_ERR_ARG, "null timer name");
    orbgpu::timer_add(name, ms);
    return ORB_OK;
}

int orb_timer_stats(const char* name, double* mean_ms, double* std_ms, long long* count) {
    if (!name) return orbgpu_fail(ORB_ERR_ARG, "null timer name");
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = stats().find(name);
    const size_t n = it == stats().end() ? 0 : it->second.size();
    double mean = 0, dev = 0;
    if (n) {  // calcAverage / calcDeviation (src/Tracking.cc:189-208): population std
        for (double v : it->second) mean += v;
        mean /= (double)n;
        for (double v : it->second) dev += (v - mean) * (v - mean);
        dev = std::sqrt(dev / (double)n);
    }
    if (mean_ms) *mean_ms = mean;
    if (std_ms) *std_ms = dev;
    if (count) *count = (long long)n;
    return ORB_OK;
}

int orb_timers_write(const char* path) {
    if (!path) return orbgpu_fail(ORB_ERR_ARG, "null path");
    FILE* f = fopen(path, "w");
    if (!f) return orbgpu_fail(ORB_ERR_ARG, "cannot open the timing file");
    fprintf(f, " TIME STATS in ms (mean$\\pm$std)\n");
    std::vector<std::string> names(std::begin(kOrder), std::end(kOrder));
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (const auto& kv : stats())
            if (std::find(names.begin(), names.end(), kv.first) == names.end()) names.push_back(kv.first);
    }
    for (const std::string& nm : names) {
        double mean, dev;
        long long n;
        orb_timer_stats(nm.c_str(), &mean, &dev, &n);
        if (n) fprintf(f, "%s: %.5f$\\pm$%.5f\n", nm.c_str(), mean, dev);
    }
    fclose(f);
    return ORB_OK;
}

}  // extern "C"
