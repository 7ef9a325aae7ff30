// ORACLE (test infrastructure only): Frame::SetPose after PoseOptimization (src/Optimizer.cc:390-395,
// src/Frame.cc:533-599) -- the float frame matrices the tracking chain's isInFrustum reads -- through the
// restatement the device chain shares (orb-slam3_byzyh_amd/csrc/orb_pose_frame.h: Sophus's quaternion
// normalisation, Eigen's toRotationMatrix and quaternion vector rotation in float, in the written
// order).  Parity with a real Eigen / Sophus build is unpinned (no Eigen in this image).
#include "../orb-slam3_byzyh_amd/csrc/orb_pose_frame.h"

extern "C" void oracle_pose7_to_frame(const double* pose7, float* Tcw, float* Ow) { orb_pose7_to_frame(pose7, Tcw, Ow); }
extern "C" void oracle_pose7_float_roundtrip(const double* pose7, double* out) { orb_pose7_float_roundtrip(pose7, out); }
