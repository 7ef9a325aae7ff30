"""MI355X-native ORB-SLAM3 front-end + local BA hot path (import name: ``orbslam3_amd``).

The package directory is ``orb-slam3_byzyh_amd/`` (not a valid identifier); load it with
``orbslam3_amd = load_package()`` from the repo root helpers (tests/conftest.py, bench.py,
__graft_entry__.py), which register it under the import name ``orbslam3_amd``.
"""
from . import _lib
from ._lib import KEYPOINT_DTYPE, POSE_EDGE_DTYPE, POSE_FRAME_DTYPE, OrbGpuError
from .extractor import ORBextractor, keypoints_to_structured, undistort_keypoints_device
from .keyframe import DeviceKeyFrame, Frame, KeyFrame, LocalMapPoints, frustum_frame, is_in_frustum
from .matcher import ORBmatcher
from .optimizer import LocalBA, local_bundle_adjustment, pose_optimization
from . import distributed, timers
from .stereo import compute_stereo_matches, compute_stereo_matches_batch_device
from .tracking import DeviceFrame, DeviceLastPoints, DeviceLocalMap, TrackingChain, TrackingChainBatch
from .vocabulary import ORBVocabulary

__all__ = ["ORBextractor", "ORBmatcher", "KeyFrame", "Frame", "LocalMapPoints", "LocalBA", "local_bundle_adjustment", "pose_optimization", "compute_stereo_matches", "compute_stereo_matches_batch_device", "ORBVocabulary", "frustum_frame", "is_in_frustum", "KEYPOINT_DTYPE", "OrbGpuError", "keypoints_to_structured", "undistort_keypoints_device", "DeviceFrame", "DeviceLastPoints", "DeviceLocalMap", "TrackingChain", "TrackingChainBatch", "_lib"]
