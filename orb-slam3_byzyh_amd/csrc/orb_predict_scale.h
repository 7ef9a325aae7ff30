// MapPoint::PredictScale (reference src/MapPoint.cc:715-731) as level thresholds.
//
// The reference computes   nScale = ceil(log(ratio) / mfLogScaleFactor)   with ratio and
// mfLogScaleFactor both float.  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:36 puts a global
// `using namespace std` in front of MapPoint.cc (MapPoint.h -> Frame.h -> ORBVocabulary.h ->
// TemplatedVocabulary.h), so the unqualified log and ceil resolve to the float overloads: glibc's
// logf, a float division and ceilf.  mfLogScaleFactor is logf(mfScaleFactor) by the same rule
// (src/Frame.cc:121).
//
// A GPU cannot call glibc's logf, and ocml's differs from it in the last place, which decides the
// level exactly on the scale steps (ratio == mvScaleFactors[k]: a frame at its reference keyframe's
// distance, the common tracking case).  For a fixed mfLogScaleFactor the level is a step function
// of the ratio, so the host evaluates glibc's logf to find the steps once per call:
//   T[k] = the largest float r with ceilf(logf(r) / lsf) <= k,   k = 0 .. n_levels - 2
// and the kernel counts the thresholds the ratio exceeds.  That equals the reference's clamped
// level for every float ratio as long as glibc's logf is monotone (tests/native/predict_scale_check.cpp
// checks it exhaustively over the ratios a map point can produce).  The reference's (int) cast of
// the float is kept for the two non-finite cases: NaN compares false everywhere (level 0) and +inf
// converts to INT_MIN on x86, clamped to level 0.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace orbgpu {

constexpr int kPredictMaxLevels = 32;

// the reference's test ceilf(logf(r) / lsf) <= k, with the caller's libm (float overloads)
inline bool predict_scale_le(float r, float lsf, int k) { return std::ceil(std::log(r) / lsf) <= (float)k; }

// T[0 .. n_levels - 2]; false on lsf <= 0 / not finite or a level count out of range
inline bool predict_scale_thresholds(float lsf, int n_levels, float* T) {
    if (!(lsf > 0.0f) || !std::isfinite(lsf) || n_levels < 1 || n_levels > kPredictMaxLevels) return false;
    for (int k = 0; k + 1 < n_levels; ++k) {
        // binary search over the bit patterns of the non-negative floats [0, +inf):
        // f(0) = -inf <= k, f(+inf) = +inf > k
        uint32_t lo = 0u, hi = 0x7f800000u;
        while (hi - lo > 1u) {
            const uint32_t mid = lo + (hi - lo) / 2u;
            float r;
            std::memcpy(&r, &mid, 4);
            if (predict_scale_le(r, lsf, k)) lo = mid;
            else hi = mid;
        }
        std::memcpy(&T[k], &lo, 4);
    }
    return true;
}

// the level from the thresholds (the kernel's computation; also usable on the host)
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int predict_scale_level(float ratio, const float* T, int n_levels) {
    if (ratio == INFINITY) return 0;  // (int)ceilf(+inf) is INT_MIN on x86, clamped to level 0
    int n = 0;
    for (int k = 0; k + 1 < n_levels; ++k) n += ratio > T[k] ? 1 : 0;
    return n;
}

}  // namespace orbgpu
