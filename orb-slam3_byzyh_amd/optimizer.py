"""Optimizer::LocalBundleAdjustment's solve on the MI355X (reference src/Optimizer.cc:1740-2188).

The reference gathers the local window from its map (B1, :1744-1855), builds a g2o graph, runs
optimizer.optimize(10) (:2101), then culls edges by chi2 / depth and writes the estimates back
(B10, :2107-2185).  This module takes the flattened graph (poses as g2o::SE3Quat vectors, points,
edges with their measurements, information and camera) and runs the g2o Levenberg-Marquardt /
Schur solve on the GPU through orb_ba_optimize (include/orbgpu.h).  `local_bundle_adjustment`
then applies the reference's culling thresholds (5.991 mono, 7.815 stereo) and reports the
observations LocalBundleAdjustment would erase.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check

CHI2_MONO = 5.991    # src/Optimizer.cc:2115
CHI2_STEREO = 7.815  # src/Optimizer.cc:2145

_p = ctypes.c_void_p


class BaProblem(ctypes.Structure):
    _fields_ = [("n_poses", ctypes.c_int32), ("n_points", ctypes.c_int32), ("n_edges", ctypes.c_int32),
                ("pose", _p), ("pose_id", _p), ("pose_fixed", _p), ("pose_camera", _p), ("point", _p),
                ("point_id", _p), ("edges", _p)]


class BaOptions(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("user_lambda_init", ctypes.c_double), ("stop_flag", _p), ("stop_flag_bool", _p)]


class BaResult(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("trials", ctypes.c_int32), ("terminated", ctypes.c_int32),
                ("stopped", ctypes.c_int32), ("initial_chi2", ctypes.c_double), ("final_chi2", ctypes.c_double),
                ("lambda_", ctypes.c_double)]

    def as_dict(self):
        return {"iterations": self.iterations, "trials": self.trials, "terminated": self.terminated,
                "stopped": self.stopped, "initial_chi2": self.initial_chi2, "final_chi2": self.final_chi2,
                "lambda": self.lambda_}


def make_problem_struct(prob: dict) -> tuple[BaProblem, dict]:
    """Contiguous copies of the problem arrays (pose and point are optimised in place) + the struct."""
    from .synth import BA_CAMERA_DTYPE, BA_EDGE_DTYPE
    arrs = {
        "pose": np.ascontiguousarray(prob["pose"], dtype=np.float64).copy(),
        "pose_id": np.ascontiguousarray(prob["pose_id"], dtype=np.int64),
        "pose_fixed": np.ascontiguousarray(prob["pose_fixed"], dtype=np.uint8),
        "pose_camera": np.ascontiguousarray(prob["pose_camera"], dtype=BA_CAMERA_DTYPE),
        "point": np.ascontiguousarray(prob["point"], dtype=np.float64).copy(),
        "point_id": np.ascontiguousarray(prob["point_id"], dtype=np.int64),
        "edges": np.ascontiguousarray(prob["edges"], dtype=BA_EDGE_DTYPE),
    }
    s = BaProblem(len(arrs["pose"]), len(arrs["point"]), len(arrs["edges"]), arrs["pose"].ctypes.data,
                  arrs["pose_id"].ctypes.data, arrs["pose_fixed"].ctypes.data, arrs["pose_camera"].ctypes.data,
                  arrs["point"].ctypes.data, arrs["point_id"].ctypes.data, arrs["edges"].ctypes.data)
    return s, arrs


def stop_flag_address(stop_flag):
    """Address the library polls for pbStopFlag, or None.  The flag must be memory the caller's
    other thread writes: a silent converting copy would never see the request, so anything other
    than a C-contiguous np.int32 array or a ctypes.c_int32 is rejected."""
    if stop_flag is None:
        return None
    if isinstance(stop_flag, ctypes.c_int32):
        return ctypes.addressof(stop_flag)
    if isinstance(stop_flag, np.ndarray):
        if stop_flag.dtype != np.int32 or not stop_flag.flags["C_CONTIGUOUS"] or stop_flag.size < 1:
            raise TypeError("stop_flag must be a non-empty C-contiguous np.int32 array")
        return stop_flag.ctypes.data
    raise TypeError(f"stop_flag must be an np.int32 array or ctypes.c_int32, not {type(stop_flag).__name__}")


# orb_ba_host_reduce_fn (include/orbgpu.h): in-place all-reduce of n doubles, op 0 = SUM, 1 = MAX
HOST_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                  ctypes.c_int)
BA_SUM, BA_MAX = 0, 1


def make_host_reducer(group=None):
    """An orb_ba_host_reduce_fn that all-reduces the library's host buffer with the group's own
    all_reduce (in place, float64).  Returns nonzero to the library when the collective raises."""
    import torch
    import torch.distributed as dist
    ops = {BA_SUM: dist.ReduceOp.SUM, BA_MAX: dist.ReduceOp.MAX}

    def reduce_cb(_ctx, buf, n, op):
        try:
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(n,)))
            dist.all_reduce(t, op=ops[op], group=group)
            return 0
        except Exception:  # noqa: BLE001 -- reported to the library as a failed collective
            return -1

    return HOST_REDUCE_FN(reduce_cb)


class LocalBA:
    """A device handle for repeated local BA solves (one per LocalMapping thread).

    attach() shards each solve's landmarks over the ranks of a torch.distributed group (DESIGN.md
    sec. 5): every rank passes the SAME problem; each builds the Schur complement of its landmark
    range and the partial systems are all-reduced (RCCL for an nccl group, the group's own
    all_reduce on host buffers for gloo).  Results are identical on every rank.
    """

    def __init__(self):
        lib = _lib.load()
        _lib.require_device()
        h = ctypes.c_void_p()
        check(lib.orb_ba_create(ctypes.byref(h)), "orb_ba_create")
        self._h = h
        self._lib = lib

    def attach(self, group=None, transport: str | None = None):
        """Join the ranks of `group` (default: the world group) for sharded solves.

        transport: "rccl" (device all-reduce inside the library, needs one GPU per rank) or "host"
        (the group's all_reduce on CPU tensors through a callback).  Default: "rccl" when the
        group's backend is nccl, else "host"."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        if transport is None:
            transport = "rccl" if dist.get_backend(group) == "nccl" else "host"
        if transport == "rccl":
            uid = (ctypes.c_uint8 * 128)()
            if rank == 0:
                check(self._lib.orb_ba_dist_unique_id(uid), "orb_ba_dist_unique_id")
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
            check(self._lib.orb_ba_dist_init_rccl(self._h, uid, world, rank), "orb_ba_dist_init_rccl")
            self._reduce_cb = None
        elif transport == "host":
            self._reduce_cb = make_host_reducer(group)  # kept alive with the handle
            check(self._lib.orb_ba_dist_init_host(self._h, self._reduce_cb, None, world, rank),
                  "orb_ba_dist_init_host")
        else:
            raise ValueError(f"unknown transport {transport!r}")
        self.world, self.rank, self.transport = world, rank, transport
        return self

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.orb_ba_destroy(h)
            except Exception:
                pass
            self._h = None

    def optimize(self, prob: dict, iterations: int = 10, user_lambda_init: float = 0.0, stop_flag=None):
        """Run optimize(iterations) on a copy of `prob`.  Returns (pose, point, edge_chi2, depth_ok, result).

        stop_flag is the reference's pbStopFlag (sparse_optimizer.h:188): a C-contiguous np.int32
        array (element 0 is polled) or a ctypes.c_int32, shared with the thread that sets it."""
        s, arrs = make_problem_struct(prob)
        opt = BaOptions(int(iterations), float(user_lambda_init), stop_flag_address(stop_flag))
        ne = len(arrs["edges"])
        chi2 = np.zeros(ne, np.float64)
        depth = np.zeros(ne, np.uint8)
        res = BaResult()
        rc = self._lib.orb_ba_optimize(self._h, ctypes.byref(s), ctypes.byref(opt), chi2.ctypes.data,
                                       depth.ctypes.data, ctypes.byref(res))
        if rc != _lib.ORB_ERR_ABORTED:
            check(rc, "orb_ba_optimize")
        return arrs["pose"], arrs["point"], chi2, depth.astype(bool), res.as_dict()


def local_bundle_adjustment(prob: dict, iterations: int = 10, solver: LocalBA | None = None):
    """optimize(10) and the reference's culling pass (src/Optimizer.cc:2107-2160): returns
    (pose, point, erase_mask over edges, result)."""
    import time
    lib = _lib.load()
    timed = lib.orb_timers_enabled() != 0  # REGISTER_TIMES "LBA": the whole call (src/LocalMapping.cc:208-219)
    t0 = time.perf_counter()
    solver = solver or LocalBA()
    pose, point, chi2, depth, res = solver.optimize(prob, iterations)
    stereo = np.asarray(prob["edges"]["stereo"]) != 0
    erase = np.where(stereo, chi2 > CHI2_STEREO, chi2 > CHI2_MONO) | ~depth
    if timed:
        check(lib.orb_timer_add(b"LBA", (time.perf_counter() - t0) * 1e3), "orb_timer_add")
    return pose, point, erase, res


def pose_optimization(frames, edges):
    """Optimizer::PoseOptimization (src/Optimizer.cc:55-415) on a batch of frames, on the GPU.

    frames: POSE_FRAME_DTYPE records (Tcw as SE3Quat vector, camera, the frame's edge range);
    edges: POSE_EDGE_DTYPE records (MapPoint position, observation, information, stereo flag).
    Returns (poses [n, 7], mvbOutlier per edge (bool), inliers per frame = the reference's return
    value).  The reference's Frame writes (SetPose, mvbOutlier) are the caller's."""
    from ._lib import POSE_EDGE_DTYPE, POSE_FRAME_DTYPE
    fr = np.ascontiguousarray(frames, POSE_FRAME_DTYPE)
    ed = np.ascontiguousarray(edges, POSE_EDGE_DTYPE)
    poses = np.zeros((len(fr), 7), np.float64)
    outl = np.zeros(max(len(ed), 1), np.uint8)
    inl = np.zeros(max(len(fr), 1), np.int32)
    check(_lib.load().orb_pose_optimization(len(fr), fr.ctypes.data, len(ed), ed.ctypes.data, poses.ctypes.data,
                                            outl.ctypes.data, inl.ctypes.data), "orb_pose_optimization")
    return poses, outl[:len(ed)].astype(bool), inl[:len(fr)]
