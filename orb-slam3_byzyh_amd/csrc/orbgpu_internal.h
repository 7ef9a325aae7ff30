// Internal helpers shared by the liborbgpu.so translation units (not part of the C ABI).
#pragma once
#include <chrono>
#include <cstdint>

#include "orbgpu.h"

// Record `msg` as this thread's last error (orb_last_error) and return `code`.
int orbgpu_fail(int code, const char* msg);

// Device view of an extractor handle's image pyramids (the padded planes of its last batch), for
// kernels that read mvImagePyramid (Frame::ComputeStereoMatches).
struct OrbPyramidView {
    const uint8_t* base;    // frame 0's padded pyramid block (device)
    long long frame_bytes;  // stride between frames' blocks
    int nframes;            // frames extracted by the last launch
    int nlevels;
    long long plane_off[12];
    int pitch[12], w[12], h[12];  // padded-plane pitch, level (view) size
    float scale[12], inv_scale[12];
    void* stream;           // the handle's stream (orb_extract's synchronous path runs on it)
};
extern "C" int orbgpu_extractor_pyramid(orb_extractor_t h, OrbPyramidView* out);

// The device SearchByProjection forms and PoseOptimization with the caller's scratch (the tracking
// chain's, reused stage after stage on its stream): `scratch` of at least the _bytes size, or NULL
// for the public functions' stream-ordered allocation.
size_t orbgpu_sbp_frame_scratch_bytes(int cap, int last_cap);
size_t orbgpu_sbp_local_scratch_bytes(int cap, int n_points);
int orbgpu_sbp_frame_device_scratch(orb_matcher_t m, const orb_frame_device_t* cur, const orb_last_points_device_t* last,
                                    float th, int mono, int32_t* d_match, int32_t* d_n_matches, void* stream,
                                    void* scratch);
int orbgpu_sbp_local_device_scratch(orb_matcher_t m, const orb_frame_device_t* F, const uint8_t* d_frame_taken,
                                    const orb_local_points_device_t* pts, float th, int far_points, float th_far_points,
                                    int32_t* d_match, int32_t* d_n_matches, void* stream, void* scratch);
int orbgpu_pose_optimization_device_scratch(int n_frames, const orb_pose_frame_t* d_frames, int n_edges,
                                            const orb_pose_edge_t* d_edges, double* d_pose_out, uint8_t* d_outlier,
                                            int32_t* d_inliers, void* stream, double* d_chi);

// The tracking chain's batch (orb_tracking_chain_batch_device): frame b's SearchByProjection scratch at
// scratch + b stride; each call writes its frames' argument blocks into the pinned h_args and copies
// them into d_args (args_cap bytes each) on the stream.
int orbgpu_sbp_frame_batch(orb_matcher_t m, int B, const orb_frame_device_t* const* cur,
                           const orb_last_points_device_t* const* last, float th, int mono, int32_t* const* d_match,
                           int32_t* const* d_n_matches, char* scratch, size_t stride, void* d_args, void* h_args,
                           size_t args_cap, void* stream);
int orbgpu_sbp_local_batch(orb_matcher_t m, int B, const orb_frame_device_t* const* F, const uint8_t* const* d_frame_taken,
                           const orb_local_points_device_t* const* pts, float th, int far_points, float th_far_points,
                           int32_t* const* d_match, int32_t* const* d_n_matches, char* scratch, size_t stride,
                           void* d_args, void* h_args, size_t args_cap, void* stream);
int orbgpu_frustum_chain_batch(int B, const orb_tracking_chain_frame_t* fr, const double* d_poses, float viewing_cos_limit,
                               void* d_args, void* h_args, size_t args_cap, void* stream);

// REGISTER_TIMES brackets (csrc/orb_timers.hip): StageTimer t("LBA") records the scope's wall time
// under that name when the timers are on.
namespace orbgpu {
bool timers_on();
void timer_add(const char* name, double ms);
struct StageTimer {
    const char* name;
    bool on;
    std::chrono::steady_clock::time_point t0;
    explicit StageTimer(const char* n) : name(n), on(timers_on()) {
        if (on) t0 = std::chrono::steady_clock::now();
    }
    ~StageTimer() {
        if (on) timer_add(name, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};
}  // namespace orbgpu
