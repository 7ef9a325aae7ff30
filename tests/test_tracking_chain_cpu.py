"""TrackingChainBatch's host side without a GPU: the frame records it packs column-wise (numpy) are,
byte for byte, the orb_tracking_chain_frame_t structs a per-frame ctypes construction gives
(include/orbgpu.h), for frames with and without a last-frame link table and an empty local map."""
from __future__ import annotations

import ctypes
import types

import numpy as np


def _items(pkg, synth):
    import torch
    cpu = torch.device("cpu")
    out = []
    specs = ((81, True, None), (82, False, 600), (84, True, 0))
    scenes = [synth.tracking_chain_scene(seed=seed) for seed, _, _ in specs]
    frames = [(pkg.Frame(**sc["cur"]), pkg.Frame(**sc["last"])) for sc in scenes]
    cap = max(max(C.N, L.N) for C, L in frames) + 5  # one capacity for the batch, as the ABI requires
    for (seed, links, nloc), sc, (C, L) in zip(specs, scenes, frames):

        def dframe(F):
            t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt))  # noqa: E731
            pad = cap - F.N
            kps = np.concatenate([F.mvKeysUn.view(np.float32).reshape(F.N, 7), np.zeros((pad, 7), np.float32)])
            desc = np.concatenate([F.mDescriptors.reshape(F.N, 32), np.zeros((pad, 32), np.uint8)])
            ur = None if F.mvuRight is None else t(np.concatenate([F.mvuRight, np.zeros(pad, np.float32)])[None],
                                                   np.float32)
            return pkg.DeviceFrame(t(kps[None], np.float32), t(desc[None], np.uint8),
                                   t(np.array([[F.N, 0]]), np.int32), 0, F.Tcw, sc["cur"]["camera"],
                                   F.mvScaleFactors, sc["level_sigma2"], int(F.mnMaxX), int(F.mnMaxY), F.mbf, ur)
        cur, lastf = dframe(C), dframe(L)
        pad = cap - L.N
        mp = L.map_points
        padded = lambda a, dt: torch.from_numpy(np.ascontiguousarray(  # noqa: E731
            np.concatenate([np.asarray(a, dt), np.zeros((pad,) + np.shape(a)[1:], dt)])))
        last = pkg.DeviceLastPoints(lastf, padded(mp["valid"], np.uint8), padded(mp["observed"], np.uint8),
                                    padded(mp["xyz"], np.float32), padded(mp["desc"], np.uint8))
        loc = {k: (v if nloc is None else v[:nloc]) for k, v in sc["local"].items() if links or k != "last_row"}
        local = pkg.DeviceLocalMap.from_host(cpu, **loc)
        out.append((cur, last, local, sc["pose7_pred"]))
    return out


def test_batch_records_match_ctypes(pkg, synth):
    from orbslam3_amd import tracking
    items = _items(pkg, synth)
    assert len({it[0].cap for it in items}) == 1
    host = types.SimpleNamespace(cap=items[0][0].cap, scale_factor=1.2)
    arr, keep, last_cap, n_local = tracking.TrackingChainBatch._records(host, items)
    assert len(arr) == 3 and n_local > 0 and any(it[2].last_row is None for it in items)
    assert arr.dtype.itemsize == ctypes.sizeof(tracking.TrackingChainFrame) and len(keep) == len(items)
    for b, (cur, last, local, pose7) in enumerate(items):
        lr = local.last_row
        ref = tracking.TrackingChainFrame(
            ctypes.addressof(cur.view()), ctypes.addressof(last.view()), ctypes.addressof(local.view()),
            local.pos.data_ptr(), local.normal.data_ptr(), local.min_dist.data_ptr(), local.max_dist.data_ptr(),
            None if lr is None else lr.data_ptr(), ctypes.addressof(cur.frustum_frame(1.2)),
            cur.mvInvLevelSigma2.ctypes.data, (ctypes.c_double * 7)(*np.asarray(pose7, np.float64).reshape(7)))
        assert bytes(ref) == arr[b].tobytes(), b
    assert last_cap == max(it[1].cap for it in items) and n_local == max(it[2].n for it in items)
