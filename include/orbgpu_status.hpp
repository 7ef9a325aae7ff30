/*
 * orbgpu_status.hpp -- the failure contract of the C++ drop-in shims (orbgpu_cv.hpp, orbgpu_matcher.hpp),
 * the same one orbgpu_optimizer.hpp's LocalBundleAdjustment keeps with kFallback.
 *
 * The reference calls ORBextractor / ORBmatcher from the Tracking and LocalMapping threads
 * (src/System.cc:223, src/Frame.cc:136-141); an exception escaping there would std::terminate the
 * process where the reference keeps running.  So no shim entry point throws on a library failure
 * (a device error, an invalid argument, a handle that could not be created).  It returns the result the
 * reference returns when it finds nothing -- no keypoints and monoIndex 0, 0 matches with the output
 * containers untouched as the reference leaves them on a search that matches nothing, descriptors left
 * as they were -- and records the failure here, where the caller can test for it:
 *
 *     int n = matcher.SearchByProjection(F, LastFrame, th, bMono);
 *     if (orbgpu::LastShimError() != ORB_OK) { ... run the reference body, or treat the frame as lost ... }
 *
 * LastShimError() is per thread (the reference's callers run on their own threads), cleared by
 * ClearShimError(); ShimFailureCount() counts every failure in the process; LastShimMessage() keeps
 * orb_last_error()'s text of the last failure on this thread.
 */
#ifndef ORBGPU_STATUS_HPP
#define ORBGPU_STATUS_HPP

#include <atomic>
#include <string>

#include "orbgpu.h"

namespace orbgpu {
namespace detail {
inline int& last_code() {
    thread_local int code = ORB_OK;
    return code;
}
inline std::string& last_message() {
    thread_local std::string msg;
    return msg;
}
inline std::atomic<long>& failure_count() {
    static std::atomic<long> n{0};
    return n;
}

// rc < 0: record the failure (code, "what: orb_last_error()") and return true.  Never throws.
inline bool Failed(int rc, const char* what) noexcept {
    if (rc >= 0) return false;
    last_code() = rc;
    failure_count().fetch_add(1, std::memory_order_relaxed);
    try {
        const char* e = orb_last_error();
        last_message() = std::string(what) + ": " + (e ? e : "");
    } catch (...) {  // allocation failure: the code is kept, the text is not
    }
    return true;
}
}  // namespace detail

// This thread's last shim failure (an ORB_ERR_* code), ORB_OK when none since ClearShimError().
inline int LastShimError() noexcept { return detail::last_code(); }
inline const std::string& LastShimMessage() noexcept { return detail::last_message(); }
inline void ClearShimError() noexcept {
    detail::last_code() = ORB_OK;
    detail::last_message().clear();
}
// Library failures seen by every shim in this process.
inline long ShimFailureCount() noexcept { return detail::failure_count().load(std::memory_order_relaxed); }

}  // namespace orbgpu

#endif  // ORBGPU_STATUS_HPP
