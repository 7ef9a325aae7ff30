// Exhaustive check of the threshold form of MapPoint::PredictScale (orb-slam3_byzyh_amd/csrc/
// orb_predict_scale.h) against the reference's float expression (int)ceilf(logf(r) / lsf), clamped
// to [0, n_levels) (src/MapPoint.cc:715-731), with this libm's logf.  Covers every float ratio in
// [2^-12, 2^12) for the EuRoC scale factor and the whole positive range coarsely for others.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <initializer_list>

#include "../../orb-slam3_byzyh_amd/csrc/orb_predict_scale.h"

static int reference_level(float r, float lsf, int n) {
    const float q = std::ceil(std::log(r) / lsf);
    int s = std::isfinite(q) ? (int)q : INT32_MIN;  // x86 cvttss2si of +-inf / NaN
    return s < 0 ? 0 : (s >= n ? n - 1 : s);
}

static long long check(float scale, int n, uint32_t lo_bits, uint32_t hi_bits, uint32_t stride) {
    const float lsf = std::log(scale);
    float T[orbgpu::kPredictMaxLevels];
    if (!orbgpu::predict_scale_thresholds(lsf, n, T)) return -1;
    long long bad = 0;
    for (uint64_t b = lo_bits; b < hi_bits; b += stride) {
        float r;
        const uint32_t u = (uint32_t)b;
        std::memcpy(&r, &u, 4);
        if (orbgpu::predict_scale_level(r, T, n) != reference_level(r, lsf, n)) {
            if (bad < 5) printf("mismatch scale %g n %d r %.9g: %d vs %d\n", scale, n, r,
                                orbgpu::predict_scale_level(r, T, n), reference_level(r, lsf, n));
            ++bad;
        }
    }
    return bad;
}

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main() {
    long long bad = 0, cases = 0;
    // every float ratio in [2^-12, 2^12): the EuRoC / TUM scale factor, 8 and 12 levels
    for (int n : {8, 12}) { bad += check(1.2f, n, bits(0x1p-12f), bits(0x1p12f), 1); ++cases; }
    // other scale factors: [1/8, 64) exhaustively, the positive floats with a stride
    for (float s : {1.1f, 1.25f, 1.5f, 2.0f, 1.05f}) {
        bad += check(s, 8, bits(0.125f), bits(64.0f), 1);
        bad += check(s, 8, 1u, 0x7f800001u, 4099u);
        cases += 2;
    }
    // the non-finite ratios
    for (float r : {INFINITY, NAN, 0.0f}) {
        float T[orbgpu::kPredictMaxLevels];
        orbgpu::predict_scale_thresholds(std::log(1.2f), 8, T);
        if (orbgpu::predict_scale_level(r, T, 8) != reference_level(r, std::log(1.2f), 8)) ++bad;
    }
    if (bad) { printf("FAIL %lld mismatches\n", bad); return 1; }
    printf("OK %lld ranges\n", cases);
    return 0;
}
