#!/usr/bin/env python3
"""Benchmark of the MI355X ORB front-end hot path (BASELINE.json metric, config C2 at N=1).

  python bench.py [--gpus N] [--steps K] [--warmup W]

One "step" = ORBextractor::operator() on one batch of 64 synthetic 640x480 frames (nFeatures 1000,
8 levels, scale 1.2, FAST 20/7), device-resident inputs and outputs, on each rank's GPU.  Frames are
independent units: each rank extracts its own batch (weak scaling, no data-path collective).
`value` = keypoints extracted+described by all ranks per ms of the max-over-ranks timed region.

Extra fields: `roofline` for the dominant kernel (HIP-event time on the launch stream, algorithmic
bytes per DESIGN.md), `cpu_baseline` (the CPU oracle -- a restatement of the reference -- timed on
this host's cores on a bounded sample), `stages_ms` (per-stage HIP-event ms per step).
"""
from __future__ import annotations

import argparse
import ctypes
import concurrent.futures as cf
import importlib.util
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FRAMES, WIDTH, HEIGHT, NFEAT, NLEVELS = 64, 640, 480, 1000, 8


def load_package():
    if "orbslam3_amd" in sys.modules:
        return sys.modules["orbslam3_amd"]
    pkg_dir = ROOT / "orb-slam3_byzyh_amd"
    spec = importlib.util.spec_from_file_location("orbslam3_amd", pkg_dir / "__init__.py",
                                                  submodule_search_locations=[str(pkg_dir)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["orbslam3_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def level_sizes(w, h, n=NLEVELS, s=1.2):
    import numpy as np
    out, f = [], np.float32(1.0)
    for l in range(n):
        if l:
            f = np.float32(float(f) * float(np.float32(s)))
        inv = np.float32(1.0) / f
        out.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return out


def survey_bytes_per_frame(w, h, nkp):
    """SURVEY.md sec. 8(d)'s algorithmic bytes per frame of the whole extraction path: read L0,
    write + read levels 1..7 (mvImagePyramid must be materialised), keypoints + descriptors out
    (28 + 32 B each).  640x480 with N = 1000 keypoints: 1,653,864 B."""
    sizes = level_sizes(w, h)
    return w * h + 2 * sum(a * b for a, b in sizes[1:]) + nkp * 60


def algorithmic_bytes_per_frame(w, h, nkp, pairs=False):
    """Per-frame bytes each stage of THIS implementation moves (a traffic model, not the roofline's
    algorithmic figure, which is survey_bytes_per_frame)."""
    sizes = level_sizes(w, h)
    px = [a * b for a, b in sizes]
    written = [(a + 6) * (b + 6) for a, b in sizes]  # each view + its 3-px REFLECT_101 border
    # level passes read the input and levels 0..6; two-level passes (k_pyramid_pair) the input and
    # levels 1, 3, 5 (level l + 1 is resized from level l while it is in LDS)
    reads = sum(px[1:-1:2]) if pairs else sum(px[:-1])
    return {
        # write every level's view + border (no blurred levels: k_describe blurs its own samples)
        "pyramid": w * h + reads + sum(written),
        # read every level once; candidates are ~1% of pixels (not counted)
        "fast": sum(px),
        # candidates in, selected keys out (small); counted as one level read equivalent of 4 B/cand
        "quadtree": 0,
        "place": 0,
        # per keypoint: the 43x43 patch (disc + Gaussian taps of the 512 samples) in, 28 + 32 B out
        "describe": nkp * (43 * 43 + 60),
        # SURVEY.md sec. 8(d) whole-path figure: L0 read + levels 1..7 written and read + kps/descs out
        "path": w * h + 2 * sum(px[1:]) + nkp * 60,
    }


def host_cores():
    """(threads, description): every core this process may run on (sched_getaffinity), limited by
    a cgroup CPU quota when one is set (a quota of Q CPUs runs at most Q threads at a time)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    try:
        q, period = pathlib.Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except Exception:  # noqa: BLE001 -- no cgroup v2 quota
        quota = None
    threads = min(affinity, quota) if quota else affinity
    model = ""
    try:
        for line in pathlib.Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:  # noqa: BLE001
        pass
    desc = f"{affinity} cores in the affinity mask" + (f", cgroup quota {quota} CPUs" if quota else ", no cgroup quota")
    return max(1, threads), desc + (f", {model}" if model else "")


ORACLE_FLAGS = "g++ -O3 -march=x86-64-v3 -ffp-contract=off (oracle/Makefile)"


def cpu_baseline(oracle_mod, frames, budget_s=10.0):
    """Oracle (CPU restatement of ORBextractor) on a thread pool over every available host core,
    one frame per thread at a time (C2 thread pool, one frame per core)."""
    cores, cores_desc = host_cores()
    ex = [oracle_mod.OracleExtractor(NFEAT, 1.2, NLEVELS, 20, 7) for _ in range(cores)]
    t0 = time.perf_counter()
    done = [0] * cores
    feats = [0] * cores

    def worker(i):
        j = i
        while time.perf_counter() - t0 < budget_s:
            k, _, _ = ex[i](frames[j % len(frames)], (0, 1000))
            feats[i] += len(k)
            done[i] += 1
            j += cores

    with cf.ThreadPoolExecutor(cores) as pool:
        list(pool.map(worker, range(cores)))
    dt = time.perf_counter() - t0
    nf = sum(done)
    return {"value": round(sum(feats) / (dt * 1e3), 3), "unit": "features/ms", "cores": cores, "kind": "port",
            "sample": f"{nf} frames of the C2 set (640x480, nFeatures 1000) in {dt:.1f} s on {cores} threads "
                      f"({cores_desc}), oracle/orb_extractor_oracle.cpp, {ORACLE_FLAGS}"}


FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (= FP64 matrix) peak, AMD spec; not listed in MI355X_MICROARCH.md


def ba_flops_per_iteration(prob):
    """Algorithmic FP64 FLOPs of one LM iteration with one trial."""
    import numpy as np
    e = prob["edges"]
    ne = len(e)
    free = np.asarray(prob["pose_fixed"]) == 0
    nfree = int(free.sum())
    fe = free[e["pose"]]
    per_point = np.bincount(e["point"][fe], minlength=len(prob["point"]))
    pairs = int((per_point * (per_point + 1) // 2).sum())
    n = 6 * nfree
    return (ne * 450            # error, Jacobians, Huber weight, quadratic-form parts
            + 2 * ne * 30       # the trial's error re-evaluation + chi2
            + int(fe.sum()) * (150 + 36)   # Z = Hpl Dinv, Hpl db, back-substitution
            + pairs * 216       # Schur block products
            + n ** 3 // 3 + 4 * n * n)     # Cholesky + two triangular solves


def bench_local_ba(pkg, synth, world, dev, steps, cpu_baseline_on):
    """C5: LocalBundleAdjustment's optimize(10) on 50 KF / 2000 MP / ~12k edges.  For N > 1 the same
    problem is solved once by all ranks, landmarks sharded and the Schur system all-reduced over
    RCCL (LocalBA.attach).  Returns the localba object of the JSON line (rank 0)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    prob = synth.local_ba_problem(n_kf=50, n_points=2000, obs_per_point=6, stereo_frac=0.0, seed=7)
    ba = pkg.LocalBA()
    transport = None
    if world > 1:
        ba.attach()
        transport = ba.transport
    for _ in range(2):
        ba.optimize(prob, 10)
    reps = max(3, min(steps, 20))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    iters = 0
    res = None
    for _ in range(reps):
        _, _, _, _, res = ba.optimize(prob, 10)
        iters += res["iterations"]
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    iter_ms = dt / iters
    flops = ba_flops_per_iteration(prob)
    achieved = flops / (iter_ms * 1e-3) / 1e12
    out = {"config": "C5: 50 keyframes (2 fixed) / 2000 map points / %d mono edges, optimize(10)" % len(prob["edges"])
                     + (f", landmarks sharded over {world} GPUs, Schur system all-reduced ({transport})"
                        if world > 1 else ", one GPU"),
           "iter_ms": round(iter_ms, 4), "solve_ms": round(dt / reps, 4), "iterations": res["iterations"],
           "trials": res["trials"], "dtype": "f64",
           "roofline": {"bound": "fp64", "achieved": round(achieved, 5), "peak": FP64_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 7),
                        "flops_per_iteration": int(flops)}}
    if cpu_baseline_on:
        from oracle import oracle as oracle_mod
        t0 = time.perf_counter()
        nrep = 0
        it_cpu = 0
        while time.perf_counter() - t0 < 3.0 or nrep < 2:
            _, _, _, _, r = oracle_mod.local_ba(prob, 10)
            it_cpu += r["iterations"]
            nrep += 1
        cdt = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"value": round(cdt / it_cpu, 4), "unit": "ms/iteration", "cores": 1, "kind": "port",
                               "sample": f"{nrep} solves of the same C5 problem, oracle/orb_ba_oracle.cpp, " + ORACLE_FLAGS + ", "
                                         "one thread (g2o is built without OpenMP)"}
    return out


def bench_stereo(pkg, synth, dev, steps, cpu_baseline_on, n_pairs=32, n_sets=2):
    """C3 stereo stream (752x480, nFeatures 1200, EuRoC bf/b): one step = extract the left and the
    right batch of n_pairs frames + Frame::ComputeStereoMatches on the device pyramids.  Reports
    stereo frames per ms, the matching kernels' share, and the CPU oracle on a bounded sample.
    `n_sets` (left, right) extractor pairs take the steps in turn, each with its own left, right and
    matching streams, so one step's matching and quad-tree tail overlap the next step's pyramids (as
    the main line's batches in flight)."""
    import numpy as np
    import torch
    bf, b = 47.90639384423901, 0.110074
    pairs = [synth.stereo_pair(752, 480, seed=2000 + i) for i in range(n_pairs)]
    L = torch.from_numpy(np.stack([p[0] for p in pairs])).to(dev)
    R = torch.from_numpy(np.stack([p[1] for p in pairs])).to(dev)
    cap = 1200 + 16 * 8
    mk = lambda: (torch.empty((n_pairs, cap, 7), dtype=torch.float32, device=dev),  # noqa: E731
                  torch.empty((n_pairs, cap, 32), dtype=torch.uint8, device=dev),
                  torch.empty((n_pairs, 2), dtype=torch.int32, device=dev))
    sets = []
    for _ in range(max(1, n_sets)):
        sets.append({"exl": pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=n_pairs),
                     "exr": pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=n_pairs),
                     "out_l": mk(), "out_r": mk(), "s_l": torch.cuda.Stream(dev), "s_r": torch.cuda.Stream(dev),
                     "s_m": torch.cuda.Stream(dev)})
        throughput_mode([sets[-1]["exl"], sets[-1]["exr"]])

    # left and right extractions run concurrently on their own streams, as Frame.cc:136-141 runs the
    # two extractors on two threads; the matching waits for both
    def step(i, ev=None):
        S = sets[i % len(sets)]
        S["s_l"].wait_stream(S["s_m"])  # this set's previous matching has read the pyramids
        S["s_r"].wait_stream(S["s_m"])
        S["exl"].extract_batch_device(L, (0, 0), cap=cap, out=S["out_l"], stream=S["s_l"])
        S["exr"].extract_batch_device(R, (0, 0), cap=cap, out=S["out_r"], stream=S["s_r"])
        S["s_m"].wait_stream(S["s_l"])
        S["s_m"].wait_stream(S["s_r"])
        if ev is not None:
            ev[0].record(S["s_m"])
        with torch.cuda.stream(S["s_m"]):
            r = pkg.compute_stereo_matches_batch_device(S["exl"], S["exr"], S["out_l"], S["out_r"], bf, b, stream=S["s_m"])
        if ev is not None:
            ev[1].record(S["s_m"])
        return r

    for i in range(3 * len(sets)):
        step(i)
    torch.cuda.synchronize(dev)
    reps = max(6, min(steps, 20))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    t0 = time.perf_counter()
    for i in range(reps):
        _, _, kept = step(i, ev[i])
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    match_ms = sum(a.elapsed_time(z) for a, z in ev)
    kept = kept.cpu().numpy()
    out = {"config": f"C3: {n_pairs} stereo pairs 752x480 per step (synthetic EuRoC-shaped, disparity 4-48 px), "
                     "nFeatures 1200, extract left || right (two streams) + Frame::ComputeStereoMatches, one GPU, "
                     f"{len(sets)} steps in flight",
           "stereo_frames_per_ms": round(n_pairs * reps / dt, 4), "ms_per_step": round(dt / reps, 4),
           "match_ms_per_step": round(match_ms / reps, 4),
           "matches_per_frame": round(float(kept.mean()), 1)}
    if cpu_baseline_on:
        from oracle import oracle as oracle_mod
        import concurrent.futures as cf
        exo = [oracle_mod.OracleExtractor(1200, 1.2, 8, 20, 7) for _ in range(2)]
        sc = exo[0].params()
        t0 = time.perf_counter()
        nfr = 0
        with cf.ThreadPoolExecutor(2) as pool:  # left || right, as Frame.cc:136-141
            while time.perf_counter() - t0 < 3.0 or nfr < 2:
                lft, rgt, _ = pairs[nfr % n_pairs]
                (kl, dl, _), (kr, dr, _) = pool.map(lambda a: a[0](a[1], (0, 0)), [(exo[0], lft), (exo[1], rgt)])
                oracle_mod.compute_stereo_matches(kl, dl, kr, dr, [exo[0].level_padded(l) for l in range(8)],
                                                  [exo[1].level_padded(l) for l in range(8)], sc["scale"],
                                                  sc["inv_scale"], bf, b)
                nfr += 1
        cdt = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"value": round(nfr / cdt, 5), "unit": "stereo frames/ms", "cores": 2, "kind": "port",
                               "sample": f"{nfr} stereo frames of the C3 set in {cdt / 1e3:.1f} s, left and right "
                                         "extraction on 2 threads + the stereo oracle"}
    return out


def bench_c3_chain(pkg, synth, dev, steps, cpu_baseline_on, n_kf=32, n_nb=10):
    """C3 as LocalMapping consumes it, device-resident end to end: one step = n_kf new stereo keyframes
    (752x480, nFeatures 1200) extracted left || right, Frame::ComputeStereoMatches, KeyFrame::ComputeBoW
    (levelsup 4, k=10 L=6 vocabulary) and SearchForTriangulation of every new keyframe against its n_nb
    predecessors in the stream (LocalMapping::CreateNewMapPoints, src/LocalMapping.cc:506-610), the
    predecessors of the first keyframes coming from the previous step's buffers.  No host hop between the
    stages.  Also one keyframe alone through the same chain (the latency LocalMapping sees)."""
    import numpy as np
    import torch
    bf, b = 47.90639384423901, 0.110074
    n_img = n_kf + n_nb
    L_all, R_all, Tcw, _ = synth.stereo_sequence(n_img, seed=2100)
    # step images: frames n_nb .. n_nb + n_kf - 1 of the stream; the previous step's buffers hold the
    # same images, standing for frames 0 .. n_kf - 1 (their poses give the true relative geometry)
    L = torch.from_numpy(L_all[n_nb:]).to(dev)
    R = torch.from_numpy(R_all[n_nb:]).to(dev)
    voc = synth.dbow_vocabulary(10, 6, seed=5, kmin=10, leaf_early=0.0)
    vocab = pkg.ORBVocabulary(voc)
    scale, sigma2 = synth.scale_tables()
    cap = 1200 + 16 * 8
    # n_new buffer sets of new keyframes take the steps in turn (a step's extraction overlaps the
    # previous step's matching), plus one set of predecessors (the previous step's keyframes)
    n_new = max(1, int(os.environ.get("ORB_C3_INFLIGHT", "3")))
    sets = []
    for _ in range(n_new + 1):
        S = {"exl": pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=n_kf),
             "exr": pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=n_kf),
             "s_l": torch.cuda.Stream(dev), "s_r": torch.cuda.Stream(dev), "s_m": torch.cuda.Stream(dev)}
        mk = lambda: (torch.empty((n_kf, cap, 7), dtype=torch.float32, device=dev),  # noqa: E731
                      torch.empty((n_kf, cap, 32), dtype=torch.uint8, device=dev),
                      torch.empty((n_kf, 2), dtype=torch.int32, device=dev))
        S["out_l"], S["out_r"] = mk(), mk()
        throughput_mode([S["exl"], S["exr"]])
        S["u"] = torch.empty((n_kf, cap), dtype=torch.float32, device=dev)
        S["st_out"] = (S["u"], torch.empty((n_kf, cap), dtype=torch.float32, device=dev),
                       torch.empty(n_kf, dtype=torch.int32, device=dev))
        S["bow"] = (torch.empty((n_kf, cap), dtype=torch.int32, device=dev),
                    torch.empty((n_kf, cap), dtype=torch.float64, device=dev),
                    torch.empty((n_kf, cap), dtype=torch.int32, device=dev),
                    torch.empty((n_kf, cap + 1), dtype=torch.int32, device=dev),
                    torch.empty((n_kf, cap), dtype=torch.int32, device=dev),
                    torch.empty((n_kf, 2), dtype=torch.int32, device=dev))
        sets.append(S)
    # kfs[set][f]: frame f of that set's buffers, at stream index n_nb + f (new sets) or f (predecessors)
    kfs = []
    for si, S in enumerate(sets):
        base = n_nb if si < n_new else 0
        kfs.append([pkg.DeviceKeyFrame(S["out_l"], S["bow"], f, Tcw[base + f], synth.EUROC_K, scale, sigma2,
                                       u_right=S["u"]) for f in range(n_kf)])
    matcher = pkg.ORBmatcher(0.6, False)  # LocalMapping's ORBmatcher(0.6, false) (src/LocalMapping.cc:536)
    # the new keyframes of a set against their predecessors: in that set before them, then the end of
    # the predecessor set
    for k in range(n_new):
        groups = []
        for f in range(n_kf):
            nb = [kfs[k][f - j] if f - j >= 0 else kfs[n_new][n_kf + f - j] for j in range(1, n_nb + 1)]
            groups.append((kfs[k][f], nb))
        sets[k]["groups"] = groups
        sets[k]["prepared"] = matcher.prepare_device_batch(groups)
        sets[k]["m_out"] = (torch.empty((n_kf * n_nb, cap), dtype=torch.int32, device=dev),
                            torch.empty(n_kf * n_nb, dtype=torch.int32, device=dev))
    m_out = sets[0]["m_out"]

    def extract(S, stream_done=None):
        S["s_l"].wait_stream(S["s_m"])
        S["s_r"].wait_stream(S["s_m"])
        S["exl"].extract_batch_device(L, (0, 0), cap=cap, out=S["out_l"], stream=S["s_l"])
        S["exr"].extract_batch_device(R, (0, 0), cap=cap, out=S["out_r"], stream=S["s_r"])
        S["s_m"].wait_stream(S["s_l"])
        S["s_m"].wait_stream(S["s_r"])
        pkg.compute_stereo_matches_batch_device(S["exl"], S["exr"], S["out_l"], S["out_r"], bf, b, stream=S["s_m"],
                                                out=S["st_out"])
        vocab.transform_frames_device(S["out_l"][1], S["out_l"][2], 4, stream=S["s_m"], out=S["bow"])

    # the predecessor set holds the previous step once; every timed step rebuilds one new set and
    # matches it
    extract(sets[n_new])

    def step(i, ev=None):
        S = sets[i % n_new]
        extract(S)
        if ev is not None:
            ev[0].record(S["s_m"])
        matcher.SearchForTriangulationDeviceBatch(S["groups"], False, False, stream=S["s_m"], out=S["m_out"],
                                                  prepared=S["prepared"])
        if ev is not None:
            ev[1].record(S["s_m"])

    for i in range(3 * n_new):
        step(i)
    torch.cuda.synchronize(dev)
    reps = max(6, min(steps, 20))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    t0 = time.perf_counter()
    for i in range(reps):
        step(i, ev[i])
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    sft_ms = sum(a.elapsed_time(z) for a, z in ev) / reps
    cnt = m_out[1].cpu().numpy()
    # one keyframe alone (LocalMapping's latency): batch of 1 through the same chain, host sync at the end
    one = {"exl": pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=1),
           "exr": pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=1)}
    st = torch.cuda.Stream(dev)
    L1, R1 = L[n_kf - 1:n_kf].contiguous(), R[n_kf - 1:n_kf].contiguous()
    o_l = (torch.empty((1, cap, 7), dtype=torch.float32, device=dev), torch.empty((1, cap, 32), dtype=torch.uint8, device=dev),
           torch.empty((1, 2), dtype=torch.int32, device=dev))
    o_r = tuple(torch.empty_like(t) for t in o_l)
    nb1 = [kfs[0][n_kf - 1 - j] for j in range(1, n_nb + 1)]
    o_st = (torch.empty((1, cap), dtype=torch.float32, device=dev), torch.empty((1, cap), dtype=torch.float32, device=dev),
            torch.empty(1, dtype=torch.int32, device=dev))
    o_bow = tuple(t[:1].clone() for t in sets[0]["bow"])
    k1 = pkg.DeviceKeyFrame(o_l, o_bow, 0, Tcw[n_nb + n_kf - 1], synth.EUROC_K, scale, sigma2, u_right=o_st[0])
    prep1 = matcher.prepare_device_batch([(k1, nb1)])
    o_m = (torch.empty((n_nb, cap), dtype=torch.int32, device=dev), torch.empty(n_nb, dtype=torch.int32, device=dev))

    def single():
        one["exl"].extract_batch_device(L1, (0, 0), cap=cap, out=o_l, stream=st)
        one["exr"].extract_batch_device(R1, (0, 0), cap=cap, out=o_r, stream=st)
        pkg.compute_stereo_matches_batch_device(one["exl"], one["exr"], o_l, o_r, bf, b, stream=st, out=o_st)
        vocab.transform_frames_device(o_l[1], o_l[2], 4, stream=st, out=o_bow)
        r = matcher.SearchForTriangulationDeviceBatch(None, False, False, stream=st, out=o_m, prepared=prep1)
        st.synchronize()
        return r

    for _ in range(3):
        single()
    lat = _median_ms(single, 30)
    out = {"config": f"C3 keyframe stream: {n_kf} new stereo keyframes 752x480 per step (synthetic plane, camera "
                     "translating along x), nFeatures 1200, extract left || right + ComputeStereoMatches + ComputeBoW "
                     f"(k=10 L=6) + SearchForTriangulation of each against its {n_nb} predecessors, device-resident, "
                     "one GPU",
           "keyframes_per_ms": round(n_kf * reps / dt, 4), "ms_per_step": round(dt / reps, 4), "step_buffers": n_new,
           "sft_ms_per_step": round(sft_ms, 4), "sft_pairs_per_step": n_kf * n_nb,
           "matches_per_pair": round(float(cnt.mean()), 1), "single_keyframe_ms": round(lat, 4)}
    if cpu_baseline_on:
        from oracle import oracle as oracle_mod
        import concurrent.futures as cf
        exo = [oracle_mod.OracleExtractor(1200, 1.2, 8, 20, 7) for _ in range(2)]
        sc = exo[0].params()
        hist = []
        t0 = time.perf_counter()
        nfr = 0
        with cf.ThreadPoolExecutor(2) as pool:  # left || right, as Frame.cc:136-141; the rest on one thread
            while time.perf_counter() - t0 < 4.0 or nfr < n_nb + 2:
                g = nfr % n_img
                (kl, dl, _), (kr, dr, _) = pool.map(lambda a: a[0](a[1], (0, 0)), [(exo[0], L_all[g]), (exo[1], R_all[g])])
                ur, _, _ = oracle_mod.compute_stereo_matches(kl, dl, kr, dr, [exo[0].level_padded(l) for l in range(8)],
                                                             [exo[1].level_padded(l) for l in range(8)], sc["scale"],
                                                             sc["inv_scale"], bf, b)
                _, fv = oracle_mod.bow_transform(voc, dl, 4)
                k = pkg.KeyFrame(keys_un=kl, descriptors=dl, Tcw=Tcw[g], camera=synth.EUROC_K, scale_factors=scale,
                                 level_sigma2=sigma2, u_right=ur, feat_vec=fv)
                for k2 in hist[-n_nb:]:
                    oracle_mod.search_for_triangulation(k, k2, matcher.pair_geometry(k, k2), False, False, False)
                hist.append(k)
                nfr += 1
        cdt = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"value": round(nfr / cdt, 5), "unit": "keyframes/ms", "cores": 2, "kind": "port",
                               "sample": f"{nfr} keyframes of the stream in {cdt / 1e3:.1f} s: left and right extraction "
                                         "on 2 threads, then stereo, BoW and SearchForTriangulation against up to "
                                         f"{n_nb} predecessors on one (oracle)"}
    return out


def bench_pose(pkg, synth, dev, steps, cpu_baseline_on, n_frames=256, n_points=500):
    """Optimizer::PoseOptimization (tracking's motion-only BA), batched: one step = n_frames frames of
    ~n_points matched map points (50 % stereo, 8 % gross outliers), device-resident inputs."""
    import numpy as np
    import torch
    frames, edges, _ = synth.pose_opt_batch(n_frames, n_points, stereo_frac=0.5, seed=4242)
    lib = pkg._lib.load()
    d_fr = torch.from_numpy(frames.view(np.uint8).reshape(-1)).to(dev)
    d_ed = torch.from_numpy(edges.view(np.uint8).reshape(-1)).to(dev)
    d_pose = torch.empty((n_frames, 7), dtype=torch.float64, device=dev)
    d_out = torch.empty(len(edges), dtype=torch.uint8, device=dev)
    d_inl = torch.empty(n_frames, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)

    def step():
        pkg._lib.check(lib.orb_pose_optimization_device(n_frames, d_fr.data_ptr(), len(edges), d_ed.data_ptr(),
                                                        d_pose.data_ptr(), d_out.data_ptr(), d_inl.data_ptr(),
                                                        ctypes.c_void_p(st.cuda_stream)), "orb_pose_optimization_device")

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    reps = max(5, min(steps, 20))
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    # tracking's own call: one frame, device-resident, back to back (the frame's kernel time)
    n1 = int(frames["n_edges"][0])

    def step1():
        pkg._lib.check(lib.orb_pose_optimization_device(1, d_fr.data_ptr(), n1, d_ed.data_ptr(), d_pose.data_ptr(),
                                                        d_out.data_ptr(), d_inl.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
                       "orb_pose_optimization_device")
    for _ in range(3):
        step1()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        step1()
    torch.cuda.synchronize(dev)
    dt1 = (time.perf_counter() - t0) * 1e3
    out = {"config": f"PoseOptimization: {n_frames} frames x {n_points} edges (50 % stereo, 8 % outliers) per step, "
                     "4 rounds x optimize(10), one GPU", "frames_per_ms": round(n_frames * reps / dt, 3),
           "ms_per_step": round(dt / reps, 4), "single_frame_ms": round(dt1 / reps, 4), "dtype": "f64"}
    if cpu_baseline_on:
        from oracle import oracle as oracle_mod
        t0 = time.perf_counter()
        nfr = 0
        while time.perf_counter() - t0 < 2.0 or nfr < 8:
            oracle_mod.pose_optimization(frames[nfr % n_frames:nfr % n_frames + 1], edges)
            nfr += 1
        cdt = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"value": round(nfr / cdt, 4), "unit": "frames/ms", "cores": 1, "kind": "port",
                               "sample": f"{nfr} frames of the same set in {cdt / 1e3:.1f} s, "
                                         "oracle/orb_pose_oracle.cpp, " + ORACLE_FLAGS + ", one thread (as Tracking runs it)"}
    return out


def bench_bow(pkg, synth, dev, steps, cpu_baseline_on, n_frames=64, n_feat=1000):
    """KeyFrame::ComputeBoW: DBoW2 transform(descriptors, BowVector, FeatureVector, 4) of n_frames
    frames x n_feat descriptors against an ORBvoc-shaped synthetic vocabulary (k=10, L=6, about a
    million words), device-resident descriptors."""
    import numpy as np
    import torch
    voc = synth.dbow_vocabulary(10, 6, seed=5, kmin=10, leaf_early=0.0)
    v = pkg.ORBVocabulary(voc)
    desc = synth.bow_descriptors(voc, n_frames * n_feat, seed=77)
    d_desc = torch.from_numpy(desc).to(dev)
    d_fb = torch.from_numpy(np.arange(n_frames + 1, dtype=np.int32) * n_feat).to(dev)
    st = torch.cuda.current_stream(dev)
    for _ in range(3):
        v.transform_batch_device(d_desc, d_fb, 4, stream=st)
    torch.cuda.synchronize(dev)
    reps = max(5, min(steps, 20))
    t0 = time.perf_counter()
    for _ in range(reps):
        v.transform_batch_device(d_desc, d_fb, 4, stream=st)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    out = {"config": f"DBoW2 transform (KeyFrame::ComputeBoW, levelsup 4): {n_frames} frames x {n_feat} descriptors "
                     f"per step, synthetic k=10 L=6 vocabulary ({len(voc['leaves'])} words), one GPU",
           "frames_per_ms": round(n_frames * reps / dt, 3), "ms_per_step": round(dt / reps, 4)}
    if cpu_baseline_on:
        from oracle import oracle as oracle_mod
        t0 = time.perf_counter()
        nfr = 0
        while time.perf_counter() - t0 < 2.0 or nfr < 4:
            oracle_mod.bow_transform(voc, desc[(nfr % n_frames) * n_feat:(nfr % n_frames + 1) * n_feat], 4)
            nfr += 1
        cdt = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"value": round(nfr / cdt, 4), "unit": "frames/ms", "cores": 1, "kind": "port",
                               "sample": f"{nfr} frames in {cdt / 1e3:.1f} s, oracle/orb_bow_oracle.cpp, " + ORACLE_FLAGS + ", one thread"}
    return out


def _median_ms(fn, reps):
    import numpy as np
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(t))


def bench_matchers(pkg, synth, dev, steps, cpu_baseline_on):
    """The ORBmatcher calls of C3's workload, each as its caller issues it (host memory in and out,
    synchronous, PCIe included), next to the oracle on one core (LocalMapping and Tracking are single
    threads):
      * SearchForTriangulation: a new keyframe against its 10 best covisible keyframes (stereo,
        src/LocalMapping.cc:511-515,536,610; ORBmatcher(0.6, false), bOnlyStereo false), batched in
        one launch;
      * SearchByProjection(CurrentFrame, LastFrame, th = 7, stereo) (src/Tracking.cc:4149, ORBmatcher(0.9, true));
      * SearchByProjection(F, local map points, th = 3) (src/Tracking.cc:4825, ORBmatcher(0.8));
      * knn2 (best / second-best Hamming) of a 1000-descriptor frame against another, device-resident."""
    import numpy as np
    import torch
    from oracle import oracle as oracle_mod
    reps = max(10, min(steps, 50))
    out = {}
    # ---- SearchForTriangulation, 1 + 10 keyframes (752x480, ~1000 keypoints each)
    kfs = [pkg.KeyFrame(**k) for k in synth.keyframe_scene(n_kf=11, n_points=1500, seed=201)]
    k1, nbrs = kfs[0], kfs[1:]
    m = pkg.ORBmatcher(0.6, False)
    geoms = [m.pair_geometry(k1, k) for k in nbrs]
    got = m.SearchForTriangulationMany(k1, nbrs, False, False, geoms=geoms)
    for _ in range(3):
        m.SearchForTriangulationMany(k1, nbrs, False, False, geoms=geoms)
    ms = _median_ms(lambda: m.SearchForTriangulationMany(k1, nbrs, False, False, geoms=geoms), reps)
    sft = {"config": f"C3 keyframe ({k1.N} keypoints) vs its 10 covisible keyframes ({int(np.mean([k.N for k in nbrs]))} "
                     "keypoints avg), one batched call, host arrays in/out",
           "ms_per_keyframe": round(ms, 4), "matches": int(sum(n for n, _ in got))}
    if cpu_baseline_on:
        t0 = time.perf_counter()
        nrep = 0
        while time.perf_counter() - t0 < 2.0 or nrep < 2:
            for k, g in zip(nbrs, geoms):
                oracle_mod.search_for_triangulation(k1, k, g, False, False, False)
            nrep += 1
        cms = (time.perf_counter() - t0) * 1e3 / nrep
        sft["cpu_baseline"] = {"value": round(cms, 4), "unit": "ms/keyframe", "cores": 1, "kind": "port",
                               "sample": f"{nrep} x 10 neighbour calls, oracle/orb_matcher_oracle.cpp, {ORACLE_FLAGS}"}
    out["search_for_triangulation"] = sft
    # ---- SearchByProjection(Frame, Frame)
    cur, last = synth.tracking_pair(seed=31, stereo=True, forward=0.02, dup_frac=0.08)
    C, L = pkg.Frame(**cur), pkg.Frame(**last)
    mp = pkg.ORBmatcher(0.9, True)
    n_ff, _ = mp.SearchByProjectionFrame(C, L, 7, False)
    ms = _median_ms(lambda: mp.SearchByProjectionFrame(C, L, 7, False), reps)
    sbf = {"config": f"current frame {C.N} keypoints, last frame {L.N} keypoints with map points, th 7, stereo",
           "ms_per_call": round(ms, 4), "matches": int(n_ff)}
    # ---- SearchByProjection(Frame, local map points)
    P = pkg.LocalMapPoints(**synth.local_map_points(cur, n_points=3000, seed=151))
    ml = pkg.ORBmatcher(0.8, True)
    n_lm, _ = ml.SearchByProjection(C, P, 3, False, 50.0)
    ms = _median_ms(lambda: ml.SearchByProjection(C, P, 3, False, 50.0), reps)
    sbl = {"config": f"frame {C.N} keypoints, 3000 local map points, th 3", "ms_per_call": round(ms, 4),
           "matches": int(n_lm)}
    if cpu_baseline_on:
        for d, fn, what in ((sbf, lambda: oracle_mod.search_by_projection_frame(C, L, 7, False, True), "frame"),
                            (sbl, lambda: oracle_mod.search_by_projection_local(C, P, 3, False, 50.0, 0.8), "local")):
            cms = _median_ms(fn, 20)
            d["cpu_baseline"] = {"value": round(cms, 4), "unit": "ms/call", "cores": 1, "kind": "port",
                                 "sample": f"20 calls, oracle/orb_projection_oracle.cpp ({what}), {ORACLE_FLAGS}"}
    out["search_by_projection_frame"] = sbf
    out["search_by_projection_local"] = sbl
    # ---- knn2, 1000 x 1000, device-resident
    rng = np.random.default_rng(5)
    q = torch.from_numpy(rng.integers(0, 256, (1000, 32), dtype=np.uint8)).to(dev)
    t = torch.from_numpy(rng.integers(0, 256, (1000, 32), dtype=np.uint8)).to(dev)
    st = torch.cuda.current_stream(dev)
    for _ in range(5):
        pkg.ORBmatcher.knn2_device(q, t, stream=st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        pkg.ORBmatcher.knn2_device(q, t, stream=st)
    e1.record(st)
    torch.cuda.synchronize(dev)
    kms = e0.elapsed_time(e1) / reps
    knn = {"config": "1000 query x 1000 train descriptors, device-resident, async on one stream",
           "us_per_call": round(kms * 1e3, 2), "pairs_per_us": round(1e6 / (kms * 1e3), 1)}
    if cpu_baseline_on:
        qa, ta = q.cpu().numpy(), t.cpu().numpy()
        cms = _median_ms(lambda: oracle_mod.hamming_knn2(qa, ta), 10)
        knn["cpu_baseline"] = {"value": round(cms * 1e3, 1), "unit": "us/call", "cores": 1, "kind": "port",
                               "sample": f"10 scans of the same 1000 x 1000 set, oracle_hamming_knn2 "
                                         f"(oracle/orb_matcher_oracle.cpp, popcount scan), {ORACLE_FLAGS}"}
    out["knn2"] = knn
    # ---- MapPoint::ComputeDistinctiveDescriptors batched over the map points LocalMapping updates after
    # a keyframe (new and fused points, src/LocalMapping.cc:416,901,1054): 2000 points of 2-12 observations
    rng = np.random.default_rng(7)
    nobs = rng.integers(2, 13, 2000).astype(np.int32)
    offs = np.concatenate([[0], np.cumsum(nobs)]).astype(np.int32)
    dd = rng.integers(0, 256, (int(offs[-1]), 32), dtype=np.uint8)
    best_h, _ = ml.ComputeDistinctiveDescriptors(dd, offs)
    ms = _median_ms(lambda: ml.ComputeDistinctiveDescriptors(dd, offs), reps)
    d_dd, d_offs = torch.from_numpy(dd).to(dev), torch.from_numpy(offs).to(dev)
    d_out = torch.zeros((2000, 32), dtype=torch.uint8, device=dev)
    with torch.cuda.stream(st):
        for _ in range(3):
            pkg.ORBmatcher.compute_distinctive_descriptors_device(d_dd, d_offs, out=d_out, stream=st)
        e0.record(st)
        for _ in range(reps):
            pkg.ORBmatcher.compute_distinctive_descriptors_device(d_dd, d_offs, out=d_out, stream=st)
        e1.record(st)
    torch.cuda.synchronize(dev)
    dist = {"config": f"2000 map points, 2-12 observations each ({int(offs[-1])} descriptors), host arrays in/out "
                      f"(synchronous, as LocalMapping calls it); device_us_per_batch: the same batch device-resident, async",
            "ms_per_batch": round(ms, 4), "device_us_per_batch": round(e0.elapsed_time(e1) / reps * 1e3, 1)}
    if cpu_baseline_on:
        ob = oracle_mod.compute_distinctive_descriptors(dd, offs)
        assert np.array_equal(ob, best_h), "ComputeDistinctiveDescriptors differs from the oracle"
        cms = _median_ms(lambda: oracle_mod.compute_distinctive_descriptors(dd, offs), 10)
        dist["cpu_baseline"] = {"value": round(cms, 4), "unit": "ms/batch", "cores": 1, "kind": "port",
                                "sample": f"10 batches of the same 2000 points, oracle_compute_distinctive_descriptors "
                                          f"(oracle/orb_matcher_oracle.cpp), {ORACLE_FLAGS}"}
    out["compute_distinctive_descriptors"] = dist
    return out


def _chain_inputs(pkg, synth, dev, seed, cap=None):
    """One tracking-chain frame (synth.tracking_chain_scene) as device tables: the current frame, the
    last frame's map points and the local map; plus the host Frames for the oracle.  cap: the frames'
    capacity (rows past N zero, never read), default N."""
    import numpy as np
    import torch
    sc = synth.tracking_chain_scene(seed=seed)
    C, L = pkg.Frame(**sc["cur"]), pkg.Frame(**sc["last"])

    def up(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)

    def pad(a, c):
        return np.concatenate([a, np.zeros((c - len(a),) + a.shape[1:], a.dtype)])

    def dframe(F):
        c = F.N if cap is None else cap
        ur = None if F.mvuRight is None else up(pad(F.mvuRight, c).reshape(1, c), np.float32)
        return pkg.DeviceFrame(up(pad(F.mvKeysUn, c).view(np.float32).reshape(1, c, 7), np.float32),
                               up(pad(F.mDescriptors, c).reshape(1, c, 32), np.uint8), up(np.array([[F.N, 0]]), np.int32), 0,
                               F.Tcw, sc["cur"]["camera"], F.mvScaleFactors, sc["level_sigma2"], int(F.mnMaxX),
                               int(F.mnMaxY), F.mbf, ur)
    cur, lastf = dframe(C), dframe(L)
    mp = L.map_points
    cl = L.N if cap is None else cap
    last = pkg.DeviceLastPoints(lastf, up(pad(mp["valid"], cl), np.uint8), up(pad(mp["observed"], cl), np.uint8),
                                up(pad(mp["xyz"], cl), np.float32), up(pad(mp["desc"], cl), np.uint8))
    local = pkg.DeviceLocalMap.from_host(dev, **sc["local"])
    return sc, C, L, cur, last, local


def bench_tracking_chain(pkg, synth, dev, steps, cpu_baseline_on, n_scenes=8, batch=32, n_streams=4):
    """One frame of Tracking::TrackWithMotionModel -> TrackLocalMap, device-resident (tracking.TrackingChain:
    SearchByProjection(LastFrame) -> PoseOptimization -> discard -> isInFrustum -> SearchByProjection(local
    map) -> PoseOptimization, no host hop): single-frame latency (host launch to result, one stream) and
    batched throughput (`batch` frames' chains over `n_streams` streams), next to the oracle chain on one
    core.  Scenes: synth.tracking_chain_scene, EuRoC stereo geometry, ~1850 keypoints, 1800 local points."""
    import numpy as np
    import torch
    scenes = [_chain_inputs(pkg, synth, dev, 4400 + s) for s in range(n_scenes)]
    cap = max(s[3].cap for s in scenes)
    chains = [pkg.TrackingChain(cap, device=dev, th_motion=7, th_local=1) for _ in range(batch)]
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    reps = max(10, min(steps, 50))
    # single frame: launch on one stream, wait for it
    sc, C, L, cur, last, local = scenes[0]
    st = streams[0]
    ch = chains[0]
    for _ in range(3):
        ch.track(cur, last, local, sc["pose7_pred"], stream=st)
        st.synchronize()
    lat, gpu, enq = [], [], []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(reps):
        t0 = time.perf_counter()
        e0.record(st)
        ch.track(cur, last, local, sc["pose7_pred"], stream=st)
        enq.append((time.perf_counter() - t0) * 1e3)
        e1.record(st)
        st.synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
        gpu.append(e0.elapsed_time(e1))
    n1 = int(ch.n_match[0])
    n2 = int(ch.n_match[1])

    def batched():
        for b, chn in enumerate(chains):
            s = scenes[b % n_scenes]
            chn.track(s[3], s[4], s[5], s[0]["pose7_pred"], stream=streams[b % n_streams])

    for _ in range(2):
        batched()
    torch.cuda.synchronize(dev)
    brep = max(3, min(steps, 10))
    t0 = time.perf_counter()
    for _ in range(brep):
        batched()
    torch.cuda.synchronize(dev)
    bdt = (time.perf_counter() - t0) * 1e3
    # the batch API (orb_tracking_chain_batch_device): nb frames per call, one launch per stage for the
    # whole batch; every slot its own local map (the chain writes its tracking fields), frames shared
    nb, capb = int(os.environ.get("ORB_CHAIN_NB", "512")), 2048  # 256: 171, 512: 183, 1024: 173-179 frames/ms
    sb = [_chain_inputs(pkg, synth, dev, 4400 + s, cap=capb) for s in range(n_scenes)]
    locs = [pkg.DeviceLocalMap.from_host(dev, **sb[b % n_scenes][0]["local"]) for b in range(nb)]
    items = [(sb[b % n_scenes][3], sb[b % n_scenes][4], locs[b], sb[b % n_scenes][0]["pose7_pred"]) for b in range(nb)]
    # ORB_CHAIN_NBUF batch objects (scratch + pinned argument staging each) take the calls in turn: a
    # call waits on the host until the previous call on its scratch has copied its arguments up
    nbuf = max(1, int(os.environ.get("ORB_CHAIN_NBUF", "1")))
    chbs = [pkg.TrackingChainBatch(capb, nb, device=dev, th_motion=7, th_local=1) for _ in range(nbuf)]
    chb = chbs[0]
    for i in range(2 * nbuf):
        chbs[i % nbuf].track(items, stream=st)
    st.synchronize()
    t0 = time.perf_counter()
    enq_b = []
    for i in range(brep):
        t1 = time.perf_counter()
        chbs[i % nbuf].track(items, stream=st)
        enq_b.append((time.perf_counter() - t1) * 1e3)
    st.synchronize()
    bat_ms = (time.perf_counter() - t0) * 1e3 / brep
    res0 = chb.track(items[:1], stream=st).sync()[0]  # slot 0 is scene 0: the single chain's answer
    assert res0["n1"] == n1 and res0["n2"] == n2, "batch API disagrees with the single chain"
    out = {"config": f"TrackWithMotionModel -> TrackLocalMap on one frame: {C.N} keypoints (stereo), last frame "
                     f"{L.N} keypoints / {int(L.map_points['valid'].sum())} map points, {len(sc['local']['pos'])} local "
                     f"map points; th 7 / 1, ORBmatcher(0.9, true) / (0.8); device-resident, one GPU",
           "single_frame_ms": round(float(np.median(lat)), 4), "single_frame_gpu_ms": round(float(np.median(gpu)), 4),
           "single_frame_enqueue_ms": round(float(np.median(enq)), 4),
           "batched_frames_per_ms": round(batch * brep / bdt, 4), "batch": batch, "streams": n_streams,
           "batch_api": {"frames_per_call": nb, "batch_objects": nbuf, "ms_per_call": round(bat_ms, 4),
                         "frames_per_ms": round(nb / bat_ms, 3),
                         "host_enqueue_ms": {"median": round(float(np.median(enq_b)), 4),
                                             "max": round(float(np.max(enq_b)), 4)},
                         "note": "orb_tracking_chain_batch_device: one launch per stage for the whole batch, one "
                                 "stream; frames padded to cap 2048; 8 scenes repeated, a local map per slot"},
           "matches_last_frame": n1, "matches_local_map": n2, "dtype": "u8 / f32 / f64"}
    if cpu_baseline_on:
        from oracle import tracking_chain as oracle_chain
        t0 = time.perf_counter()
        nfr = 0
        while time.perf_counter() - t0 < 3.0 or nfr < 4:
            s = scenes[nfr % n_scenes]
            oracle_chain.track(pkg, s[1], s[2], s[0]["local"], s[0]["pose7_pred"], s[0]["level_sigma2"], 7, 1)
            nfr += 1
        cdt = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"] = {"value": round(cdt / nfr, 4), "unit": "ms/frame", "cores": 1, "kind": "port",
                               "sample": f"{nfr} frames of the {n_scenes} scenes in {cdt / 1e3:.1f} s, the oracle chain "
                                         "(oracle/tracking_chain.py over oracle/orb_projection_oracle.cpp, "
                                         "orb_pose_oracle.cpp, orb_frustum_oracle.cpp), " + ORACLE_FLAGS + ", one thread"}
    return out


def bench_single_frame(pkg, synth, cpu_baseline_on, reps=50):
    """Tracking's own call pattern: ORBextractor::operator() on ONE host frame (PCIe-inclusive:
    upload, extraction, download of keypoints and descriptors), 640x480 and EuRoC 752x480; the
    latency the tracking thread sees, next to the oracle on one core."""
    import numpy as np
    out = {}
    for (w, h, nf) in ((640, 480, 1000), (752, 480, 1200)):
        img = synth.polygon_frame(w, h, seed=7)
        ex = pkg.ORBextractor(nf, 1.2, 8, 20, 7, max_width=w, max_height=h)
        for _ in range(5):
            ex(img, None, (0, 0))
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ex(img, None, (0, 0))
            t.append((time.perf_counter() - t0) * 1e3)
        key = f"{w}x{h}"
        out[key] = {"median_ms": round(float(np.median(t)), 4), "p90_ms": round(float(np.percentile(t, 90)), 4)}
        if cpu_baseline_on:
            from oracle import oracle as oracle_mod
            o = oracle_mod.OracleExtractor(nf, 1.2, 8, 20, 7)
            tc = []
            for _ in range(10):
                t0 = time.perf_counter()
                o(img, (0, 0))
                tc.append((time.perf_counter() - t0) * 1e3)
            out[key]["cpu_port_median_ms"] = round(float(np.median(tc)), 4)
    out["note"] = "host image in, host keypoints/descriptors out (orb_extract, synchronous); cpu: the oracle, 1 thread"
    return out


def bench_c2_pcie(pkg, synth, dev, steps, n_frames=64, in_flight=16):
    """SURVEY.md 8(d)'s wording of the metric, H2D -> extract -> D2H: the C2 batch starts in pinned
    host memory and the keypoints, descriptors and counts end there, every step.  `in_flight` handles
    take the steps in turn.  The uploads run by DMA on one upload stream; each handle's extraction
    waits for its batch's upload on the handle's stream and its kernels write the outputs straight into
    the pinned host buffers (the D2H leg is the describe kernel's own stores over the link), so the next
    batch's upload overlaps this batch's kernels.  The handles run without their side streams
    (set_overlap(False)).  The link's own rates are measured here too (each direction alone, both at
    once) and the step is compared with its bound, max(upload, extraction).  Never `value` (the task's
    value is device-resident); reported beside it."""
    import numpy as np
    import torch
    frames = np.stack([synth.polygon_frame(640, 480, seed=100 + i) for i in range(n_frames)])
    host = torch.from_numpy(frames).pin_memory()
    # 16 handles: the upload of batch i + H waits for batch i's extraction to have read its buffer, so
    # the handle count is how far the upload stream runs ahead (tools/pcie_h_sweep.sh, round 5: H = 3
    # 129k, 4 135-139k, 8 142k, 12 145-148k, 16 150-151k features/ms; 0.83 of the link bound)
    H = int(os.environ.get("ORB_PCIE_H", max(1, in_flight)))
    exs = [pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=n_frames)
           for _ in range(H)]
    for e in exs:
        e.set_overlap(False)  # one chain per batch on its handle's stream (no side streams)
    cap = 1000 + 16 * 8
    dimg = [torch.empty_like(host, device=dev) for _ in range(H)]
    outs = [(torch.empty((n_frames, cap, 7), dtype=torch.float32, device=dev),
             torch.empty((n_frames, cap, 32), dtype=torch.uint8, device=dev),
             torch.empty((n_frames, 2), dtype=torch.int32, device=dev)) for _ in range(H)]
    houts = [tuple(torch.empty(o.shape, dtype=o.dtype).pin_memory() for o in outs[h]) for h in range(H)]
    sts = [torch.cuda.Stream(dev) for _ in range(H)]
    up, down = sts[0], sts[0]  # (the link measurements below)

    # ORB_PCIE_MODE (A/B, tools: one box, two passes each, ms per step at H = 2 / 3):
    #   "up_zc_out" (default): uploads by DMA on one upload stream, event-ordered with each handle's
    #       extraction, which writes keypoints, descriptors and counts straight into the pinned host
    #       buffers (no download copy): 0.456-0.519 / 0.508-0.524;
    #   "copy": upload, extraction and download copy on each handle's stream: 0.494-0.497 / 0.733-0.742;
    #   "zc_out": upload on the handle's stream, outputs written to host: 0.596-0.748 / 0.783-0.793;
    #   "zc_in": the level-0 pyramid kernel reads the pinned frames itself: 1.01-1.06;
    #   "zc_all": zc_in + outputs written to host: 0.707-0.733.
    mode = os.environ.get("ORB_PCIE_MODE", "up_zc_out")

    def abi_extract(h, img_ptr, o):
        e = exs[h]
        rc = e._lib.orb_extract_batch_device(e._h, img_ptr, n_frames, 640, 480, 640, 640 * 480, 0, 1000,
                                             o[0].data_ptr(), o[1].data_ptr(), cap, o[2].data_ptr(),
                                             ctypes.c_void_p(sts[h].cuda_stream))
        if rc < 0:
            raise RuntimeError(f"orb_extract_batch_device failed ({rc})")

    # "zc_out": upload by DMA on the handle's stream, outputs written by the kernels into the pinned host
    # buffers; "up_zc_out": the same with the uploads on one upload stream, event-ordered
    upl = torch.cuda.Stream(dev) if mode == "up_zc_out" else None
    up_done = [torch.cuda.Event() for _ in range(H)]
    ext_done = [torch.cuda.Event() for _ in range(H)]
    started = [False] * H

    def step(i):
        h = i % H
        if mode == "up_zc_out":
            with torch.cuda.stream(upl):
                if started[h]:
                    upl.wait_event(ext_done[h])  # the handle's previous extraction has read dimg[h]
                dimg[h].copy_(host, non_blocking=True)
                up_done[h].record(upl)
            sts[h].wait_event(up_done[h])
            abi_extract(h, dimg[h].data_ptr(), houts[h])
            ext_done[h].record(sts[h])
            started[h] = True
            return
        with torch.cuda.stream(sts[h]):
            if mode in ("copy", "zc_out"):
                dimg[h].copy_(host, non_blocking=True)
                if mode == "copy":
                    exs[h].extract_batch_device(dimg[h], (0, 1000), cap=cap, out=outs[h], stream=sts[h])
                else:
                    abi_extract(h, dimg[h].data_ptr(), houts[h])
            else:  # the level-0 pyramid kernel reads the pinned host frames itself
                abi_extract(h, host.data_ptr(), outs[h] if mode == "zc_in" else houts[h])
            if mode in ("copy", "zc_in"):
                for d, o in zip(houts[h], outs[h]):
                    d.copy_(o, non_blocking=True)

    for i in range(3 * H):
        step(i)
    torch.cuda.synchronize(dev)
    nfeat = int(houts[0][2][:, 0].sum().item())
    reps = max(6, min(steps, 21))
    t0 = time.perf_counter()
    for i in range(reps):
        step(i)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    h2d = host.numel()
    d2h = sum(o.numel() * o.element_size() for o in outs[0])

    # the link alone: each direction, then both at once (the same buffers and sizes as the step)
    def timed(fn, n=10):
        fn()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) * 1e3 / n

    def upload():
        with torch.cuda.stream(up):
            dimg[0].copy_(host, non_blocking=True)

    def download():
        with torch.cuda.stream(down):
            for d, o in zip(houts[0], outs[0]):
                d.copy_(o, non_blocking=True)

    def both():
        with torch.cuda.stream(sts[0]):
            dimg[0].copy_(host, non_blocking=True)
        with torch.cuda.stream(sts[1 % H]):
            for d, o in zip(houts[1 % H], outs[1 % H]):
                d.copy_(o, non_blocking=True)

    def extract():
        exs[0].extract_batch_device(dimg[0], (0, 1000), cap=cap, out=outs[0], stream=sts[0])
    up_ms, down_ms, both_ms, ext_ms = timed(upload), timed(download), timed(both), timed(extract)
    bound = max(up_ms, ext_ms) if mode in ("up_zc_out", "zc_out", "zc_all") else max(up_ms, down_ms, ext_ms)
    return {"config": f"C2 ({n_frames} x 640x480) from pinned host memory to pinned host outputs, {H} handles taking the batches in turn "
                      f"(mode {mode}: uploads on one upload stream, each extraction on its handle's stream writing "
                      f"its outputs into pinned host memory)",
            "features_per_ms": round(nfeat * reps / dt, 3), "ms_per_step": round(dt / reps, 4),
            "h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
            "pcie_gb_per_s": round((h2d + d2h) * reps / dt / 1e6, 2),
            "link": {"h2d_gb_per_s": round(h2d / up_ms / 1e6, 2), "d2h_gb_per_s": round(d2h / down_ms / 1e6, 2),
                     "both_directions_gb_per_s": round((h2d + d2h) / both_ms / 1e6, 2),
                     "upload_ms": round(up_ms, 4), "download_ms": round(down_ms, 4), "extract_ms": round(ext_ms, 4)},
            "bound_ms_per_step": round(bound, 4), "frac_of_bound": round(bound / (dt / reps), 3)}


def throughput_mode(exs):
    """Handles that keep several batches in flight run each batch as one chain on its own stream
    (ORBextractor.set_overlap(False)); ORB_BENCH_OVERLAP=1 keeps the side streams (A/B)."""
    if len(exs) > 1:
        on = os.environ.get("ORB_BENCH_OVERLAP", "0") == "1"
        for e in exs:
            e.set_overlap(on)
    return exs


def run_pcie_child(steps):
    """bench_c2_pcie in a process of its own.  HIP maps a process's streams onto 4 hardware queues
    by use count; after the other measurements have created their handles' streams, the PCIe
    handles' streams can share a queue and serialise (0.73 ms per step in-process vs 0.41 in a
    fresh process, tools/pcie_probe.py).  The child is started as a child (no exec of this process)."""
    import subprocess
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--pcie-only", "--steps", str(steps)],
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"child exited {r.returncode}: {r.stderr.strip()[-400:]}"}
    out = json.loads(lines[-1])
    out["process"] = "a child process of its own (fresh HIP queues)"
    return out


def bench_c4(pkg, synth, dev, steps, n_frames=32, in_flight=3):
    """C4's per-GPU shard: 32 frames of 1280x720 (nFeatures 1000) per step, device-resident (the
    8-GPU run all-gathers the features of every shard; see the main line's N > 1 path), with
    `in_flight` extractor handles taking the steps in turn on their own streams (as the main line)."""
    import numpy as np
    import torch
    frames = np.stack([synth.polygon_frame(1280, 720, seed=1000 + i) for i in range(n_frames)])
    imgs = torch.from_numpy(frames).to(dev)
    H = max(1, in_flight)
    exs = throughput_mode([pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=1280, max_height=720, max_batch=n_frames)
                           for _ in range(H)])
    cap = 1000 + 16 * 8
    outs = [(torch.empty((n_frames, cap, 7), dtype=torch.float32, device=dev),
             torch.empty((n_frames, cap, 32), dtype=torch.uint8, device=dev),
             torch.empty((n_frames, 2), dtype=torch.int32, device=dev)) for _ in range(H)]
    sts = [torch.cuda.current_stream(dev)] if H == 1 else [torch.cuda.Stream(dev) for _ in range(H)]
    for i in range(3 * H):
        exs[i % H].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[i % H], stream=sts[i % H])
    torch.cuda.synchronize(dev)
    nfeat = int(outs[0][2][:, 0].sum().item())
    reps = max(5, min(steps, 20))
    t0 = time.perf_counter()
    for i in range(reps):
        exs[i % H].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[i % H], stream=sts[i % H])
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) * 1e3
    return {"config": f"C4 shard: {n_frames} synthetic 1280x720 frames per GPU per step, nFeatures 1000, 8 levels, "
                      f"{H} batches in flight",
            "features_per_ms": round(nfeat * reps / dt, 3), "frames_per_ms": round(n_frames * reps / dt, 3),
            "ms_per_step": round(dt / reps, 4)}


def bench_c4_strong(pkg, synth, world, rank, dev, steps, in_flight=3, n_global=256, n_distinct=32):
    """C4 as strong scaling (BASELINE.json configs[3]): a fixed global batch of 256 1280x720 frames,
    256/N per rank; every step extracts each rank's shard and all-gathers all ranks' features
    (keypoints + descriptors + counts, RCCL over xGMI), overlapped with the next step's extraction
    (distributed.ShardedExtractor).  N = 1 extracts the 256 frames on one GPU with no collective.  At
    N > 1, rank 0 also times the same 256 frames alone on its GPU (while the others wait), so the line
    carries the N = 1 reference and the strong-scaling efficiency.  Every step also matches each frame
    against its predecessor in the global batch (knn2 over the gathered blocks, one
    orb_hamming_knn2_frames_device launch per rank for its frames; at N = 1 over the local blocks).
    Frames: n_distinct synthetic 1280x720 frames (seeds 1000..) repeated over the batch (generating 256
    distinct ones takes ~25 s)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from orbslam3_amd.distributed import ShardedExtractor, frame_pairs, match_gathered, shard_range
    b, e = shard_range(n_global, world, rank)
    per = e - b
    if world > 1 and n_global % world:
        raise ValueError("the global batch must divide evenly over the ranks")
    distinct = {}

    def frame(f):
        k = f % n_distinct
        if k not in distinct:
            distinct[k] = synth.polygon_frame(1280, 720, seed=1000 + k)
        return distinct[k]
    H = max(1, in_flight)
    cap = 1000 + 16 * 8

    def run(first, count, collective):
        imgs = torch.from_numpy(np.stack([frame(f) for f in range(first, first + count)])).to(dev)
        # (batches of 256 frames fill the chip alone: the side-stream overlap stays on, 131k vs 123k
        # features/ms without it)
        exs = [pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=1280, max_height=720, max_batch=count)
               for _ in range(H)]
        sts = [torch.cuda.Stream(dev) for _ in range(H)]
        if collective:
            sh = ShardedExtractor(exs, count, cap, match=True)
            step = lambda i: sh.step(imgs, (0, 1000), stream=sts[i % H])  # noqa: E731

            def fin():
                sh.finish()  # the last step's gather, matched like the others (inside finish)
            counts = lambda: sh.local.counts[0]  # noqa: E731
            match_once = lambda: match_gathered(sh.local.desc[0], sh.local.counts[0],  # noqa: E731
                                                frame_pairs(0, count, count).to(dev))
        else:
            outs = [(torch.empty((count, cap, 7), dtype=torch.float32, device=dev),
                     torch.empty((count, cap, 32), dtype=torch.uint8, device=dev),
                     torch.empty((count, 2), dtype=torch.int32, device=dev)) for _ in range(H)]
            pairs = frame_pairs(0, count, count).to(dev)
            mouts = [tuple(torch.empty((count, cap), dtype=torch.int32, device=dev) for _ in range(3)) for _ in range(H)]

            def step(i):
                o = exs[i % H].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[i % H], stream=sts[i % H])
                match_gathered(o[1], o[2], pairs, stream=sts[i % H], out=mouts[i % H])
            fin = lambda: None  # noqa: E731
            counts = lambda: outs[0][2]  # noqa: E731
            match_once = lambda: match_gathered(outs[0][1], outs[0][2], pairs, out=mouts[0])  # noqa: E731
        for i in range(2 * H):
            step(i)
        fin()
        torch.cuda.synchronize(dev)
        feats = int(counts()[:, 0].sum().item())
        reps = max(5, min(steps, 20))
        if collective:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(reps):
            step(i)
        fin()
        torch.cuda.synchronize(dev)
        if collective:
            dist.barrier()
        ms_step = (time.perf_counter() - t0) * 1e3 / reps
        # the matching launch alone (its share of the step), timed on the current stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        match_once()
        e0.record()
        for _ in range(10):
            match_once()
        e1.record()
        torch.cuda.synchronize(dev)
        run.match_ms = e0.elapsed_time(e1) / 10
        return ms_step, feats

    ms, feats = run(b, per, world > 1)
    match_ms = run.match_ms
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        f = torch.tensor([feats], dtype=torch.int64, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.SUM)
        feats = int(f.item())
    out = {"config": f"C4 strong scaling: {n_global} synthetic 1280x720 frames per step in total ({n_distinct} distinct, "
                     f"repeated), {per} per GPU x {world} GPU(s), nFeatures 1000, 8 levels"
                     + (", all-gather of keypoints + descriptors + counts per step (" + {"nccl": "RCCL"}.get(dist.get_backend(), dist.get_backend()) + ")" if world > 1 else ""),
           "n_gpus": world, "frames_per_gpu": per, "ms_per_step": round(ms, 4),
           "frames_per_ms": round(n_global / ms, 3), "features_per_ms": round(feats / ms, 3),
           "cross_frame_match": {"pairs_per_gpu": per, "ms_per_launch": round(match_ms, 4),
                                 "what": "each frame's descriptors vs its predecessor's (knn2, best / second "
                                         "best, DescriptorDistance), one orb_hamming_knn2_frames_device launch "
                                         "per rank after the all-gather, inside the timed step"}}
    if world > 1:
        ref = torch.zeros(1, dtype=torch.float64, device=dev)
        if rank == 0:
            ms1, _ = run(0, n_global, False)
            ref[0] = ms1
        dist.broadcast(ref, 0)
        ms1 = float(ref.item())
        out["single_gpu_ms_per_step"] = round(ms1, 4)
        out["speedup"] = round(ms1 / ms, 3)
        out["efficiency"] = round(ms1 / (world * ms), 3)
    return out


def pmc_traffic():
    p = ROOT / "profiles" / "pmc_latest.json"
    if p.exists():
        try:
            return json.loads(p.read_text())
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=FRAMES)
    ap.add_argument("--in-flight", type=int, default=4,
                    help="extractor handles with a batch in flight, each on its own stream (consecutive steps "
                         "overlap: one batch's latency-bound quad-tree/describe tail runs beside the next "
                         "batch's pyramid/FAST); 1 = one batch at a time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-ba", action="store_true", help="skip the LocalBA (C5) measurement")
    ap.add_argument("--no-stereo", action="store_true", help="skip the stereo stream (C3) measurement")
    ap.add_argument("--no-pose", action="store_true", help="skip the PoseOptimization measurement")
    ap.add_argument("--no-bow", action="store_true", help="skip the DBoW2 transform measurement")
    ap.add_argument("--no-single", action="store_true", help="skip the single-frame latency measurement")
    ap.add_argument("--no-c4", action="store_true", help="skip the 1280x720 (C4 shard) measurement")
    ap.add_argument("--no-matchers", action="store_true", help="skip the ORBmatcher measurements")
    ap.add_argument("--no-chain", action="store_true", help="skip the device tracking-chain measurement")
    ap.add_argument("--pcie-only", action="store_true",
                    help="internal: run only the PCIe-inclusive C2 measurement and print its JSON (bench.py runs "
                         "it in a child process of its own)")
    ap.add_argument("--launch-dump", default=None,
                    help="write the timed region's per-launch kernel durations (JSON) to this path")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")  # "gloo": multi-rank rehearsal on one GPU
    if world > 1:
        dist.init_process_group(backend, init_method="env://")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    pkg = load_package()
    from orbslam3_amd import synth
    if args.pcie_only:
        print(json.dumps(bench_c2_pcie(pkg, synth, dev, args.steps)), flush=True)
        return

    nfr = args.frames
    frames = np.stack([synth.polygon_frame(WIDTH, HEIGHT, seed=100 + i) for i in range(nfr)])
    imgs = torch.from_numpy(frames).to(dev)
    H = max(1, args.in_flight)
    exs = [pkg.ORBextractor(NFEAT, 1.2, NLEVELS, 20, 7, max_width=WIDTH, max_height=HEIGHT, max_batch=nfr)
           for _ in range(H)]
    # several batches in flight: each batch as one chain on its handle's stream.  The side streams
    # (intra-batch overlap, the default) shorten one batch alone but share the process's 4 hardware
    # queues with the other handles' streams: 297k -> 320k features/ms without them at H = 3.
    throughput_mode(exs)
    ex = exs[0]
    cap = NFEAT + 16 * NLEVELS
    outs = [(torch.empty((nfr, cap, 7), dtype=torch.float32, device=dev),
             torch.empty((nfr, cap, 32), dtype=torch.uint8, device=dev),
             torch.empty((nfr, 2), dtype=torch.int32, device=dev)) for _ in range(H)]
    out = outs[0]
    # H > 1: every handle on a stream of its own (not the legacy default stream, which would
    # serialise with the others)
    streams = [torch.cuda.current_stream(dev)] if H == 1 else [torch.cuda.Stream(dev) for _ in range(H)]
    sharded = None
    if world > 1:
        # C4 data path: every step all-gathers the features of all ranks' frames (RCCL over xGMI),
        # asynchronously and multi-buffered so it overlaps the next steps' extraction
        from orbslam3_amd.distributed import ShardedExtractor
        sharded = ShardedExtractor(exs, nfr, cap)
    it = [0]

    def step():
        h = it[0] % H
        it[0] += 1
        if sharded is None:
            exs[h].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[h], stream=streams[h])
        else:
            sharded.step(imgs, (0, 1000), stream=streams[h])

    for _ in range(args.warmup):
        step()
    if sharded is not None:
        sharded.finish()
    torch.cuda.synchronize(dev)
    for h in range(min(H, args.warmup)):
        c = outs[h][2] if sharded is None else sharded.local.counts[h]
        if not torch.equal(c, outs[0][2] if sharded is None else sharded.local.counts[0]):
            raise RuntimeError("extractor handles disagree")
    counts = (out[2] if sharded is None else sharded.local.counts[0]).cpu().numpy()
    feats_per_step = int(counts[:, 0].sum())
    if (counts[:, 1] < 0).any():
        raise RuntimeError("a frame exceeded the keypoint capacity")

    # per-stage breakdown (HIP events at every stage boundary) in an untimed pass: one batch at a
    # time on handle 0, so the stage times are those of a single batch
    ex.profile(True)
    for _ in range(min(10, args.steps)):
        ex.extract_batch_device(imgs, (0, 1000), cap=cap, out=out, stream=streams[0])
    torch.cuda.synchronize(dev)
    stage_ms, launches, _ = ex.stage_ms()
    ex.profile(False)
    # latency of one batch alone (no batch in flight beside it), untimed for `value`
    t1 = time.perf_counter()
    for _ in range(min(10, args.steps)):
        ex.extract_batch_device(imgs, (0, 1000), cap=cap, out=out, stream=streams[0])
        torch.cuda.synchronize(dev)
    single_ms = (time.perf_counter() - t1) * 1e3 / min(10, args.steps)
    # untimed steps for at least ORB_BENCH_SETTLE_MS (default 300 ms) so the GPU clocks have left
    # their idle state: the timed region of the default 20 steps lasts only ~5 ms
    settle_s = float(os.environ.get("ORB_BENCH_SETTLE_MS", "300")) * 1e-3
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < settle_s:
        for _ in range(8 * H):  # batches stay in flight; a sync every 8 rounds bounds the queue
            step()
        torch.cuda.synchronize(dev)
    if sharded is not None:
        sharded.finish()
    # timed region (value), uninstrumented
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if sharded is not None:
        sharded.finish()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed_ms = (time.perf_counter() - t0) * 1e3
    # the same steps again, every handle recording an HIP event pair on each stage kernel's dispatch
    # (hipExtLaunchKernel: the dispatch's own begin / end, on its stream): the roofline's launch
    # durations.  (A separate pass: the event pairs on every launch cost the timed region ~5 %.)
    for e_ in exs:
        e_.profile("pyramid_launches")
    for _ in range(args.steps):
        step()
    if sharded is not None:
        sharded.finish()
    torch.cuda.synchronize(dev)
    launch_ms = {k: [] for k in pkg.ORBextractor.LAUNCH_KERNELS}
    for e_ in exs:
        for k in launch_ms:
            launch_ms[k] += e_.launch_durations(k)
        e_.profile(False)
    # exclusive launch durations: the same batches once more, one at a time on
    # handle 0 with a synchronize after each, so no other batch's kernels share the chip while a
    # dispatch runs.  The shared-pass durations above overlap 3-4 batches and sum to ~3.6x the step;
    # the roofline's `achieved` / `frac` come from these exclusive ones.
    ex.profile("pyramid_launches")
    for _ in range(args.steps):
        ex.extract_batch_device(imgs, (0, 1000), cap=cap, out=out, stream=streams[0])
        torch.cuda.synchronize(dev)
    excl_ms = {k: ex.launch_durations(k) for k in pkg.ORBextractor.LAUNCH_KERNELS}
    ex.profile(False)
    if args.launch_dump and rank == 0:
        pathlib.Path(args.launch_dump).write_text(json.dumps(
            {"steps": args.steps, "frames_per_step": nfr, "features_per_step": feats_per_step,
             "note": "per-launch durations (ms), HIP event pair on each dispatch (hipExtLaunchKernel). "
                     "launch_ms: the timed region's steps again, all in-flight handles (shared chip); "
                     "exclusive_ms: the same steps one batch at a time on handle 0 (the roofline's)",
             "launch_ms": launch_ms, "exclusive_ms": excl_ms}))
    # pyramid launches per batch: 4 two-level passes (k_pyramid_pair), or 8 level passes
    # (k_pyramid_level, ORBGPU_PYR_PAIR=0 or a geometry outside the pair kernel's boxes); both are
    # recorded under the pyramid tag
    launches_per_step = max(1, round(len(excl_ms["k_pyramid_level"]) / max(1, args.steps)))
    pyr_kernel = "k_pyramid_pair" if launches_per_step < NLEVELS else "k_pyramid_level"
    excl_ms = {(pyr_kernel if k == "k_pyramid_level" else k): v for k, v in excl_ms.items()}
    launch_ms = {(pyr_kernel if k == "k_pyramid_level" else k): v for k, v in launch_ms.items()}
    pyr_launch_avg_ms = sum(excl_ms[pyr_kernel]) / max(1, len(excl_ms[pyr_kernel]))

    total_feats = feats_per_step * args.steps
    if world > 1:
        t = torch.tensor([elapsed_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed_ms = float(t.item())
        f = torch.tensor([total_feats], dtype=torch.int64, device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.SUM)
        total_feats = int(f.item())

    if rank == 0:
        per_step = {k: v / max(1, launches) for k, v in stage_ms.items()}
        # roofline kernel: k_pyramid_level, the HBM-facing stage (it reads every input frame and
        # writes every level), launches_per_step launches per step, each one level of all nfr frames.
        # achieved = SURVEY.md 8(d)'s algorithmic bytes per frame x nfr / launches_per_step, divided
        # by the mean launch duration measured in the timed region with HIP events around each launch
        # on its stream (the interval rocprofv3's kernel trace reports for the dispatch).
        # The stage with the most time is reported next to it (`dominant_stage`).
        dom = "pyramid"
        nkp_frame = feats_per_step / nfr
        dom_bytes = survey_bytes_per_frame(WIDTH, HEIGHT, nkp_frame) * nfr / launches_per_step
        model_bytes = algorithmic_bytes_per_frame(WIDTH, HEIGHT, nkp_frame, pairs=pyr_kernel == "k_pyramid_pair")[dom] * nfr / launches_per_step
        achieved = dom_bytes / (pyr_launch_avg_ms * 1e-3) / 1e9 if pyr_launch_avg_ms > 0 else 0.0
        pmc = pmc_traffic()
        traffic = None
        if pmc and pmc.get("kernel_stage") == dom and pmc.get("frames_per_launch") == nfr:
            traffic = pmc.get("hbm_bytes_per_launch")
        dominant_stage = max(per_step, key=per_step.get) if per_step else dom
        # every stage kernel against HBM: its algorithmic bytes per step / its EXCLUSIVE launch time per
        # step (one batch alone on the chip), and against the integer-VALU bound (PMC counters,
        # profiles/pmc_latest.json).  Beside it the step-level attribution: the kernel's share of the
        # summed shared-pass launch time x ms_per_step (what the kernel costs the overlapped step).
        alg = algorithmic_bytes_per_frame(WIDTH, HEIGHT, nkp_frame, pairs=pyr_kernel == "k_pyramid_pair")
        stage_of = {"k_pyramid_level": "pyramid", "k_pyramid_pair": "pyramid", "k_fast_cells": "fast",
                    "k_quadtree_kp": "quadtree", "k_describe": "describe"}
        step_ms = elapsed_ms / args.steps
        shared_total = sum(sum(v) for v in launch_ms.values()) / args.steps
        kern = {}
        for k, v in excl_ms.items():
            if not v:
                continue
            per_step_ms = sum(v) / args.steps
            shared_step_ms = sum(launch_ms.get(k, [])) / args.steps
            st = stage_of[k]
            bytes_step = (survey_bytes_per_frame(WIDTH, HEIGHT, nkp_frame) if st == "pyramid" else alg[st]) * nfr
            attributed = step_ms * shared_step_ms / shared_total if shared_total > 0 else 0.0
            ent = {"launches_per_step": round(len(v) / args.steps, 2), "launch_avg_us": round(1e3 * sum(v) / len(v), 2),
                   "ms_per_step": round(per_step_ms, 4), "algorithmic_bytes_per_step": int(bytes_step),
                   "hbm_frac": round(bytes_step / (per_step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if bytes_step else 0.0,
                   "shared_launch_avg_us": round(1e3 * shared_step_ms * args.steps / max(1, len(launch_ms.get(k, []))), 2),
                   "shared_ms_per_step": round(shared_step_ms, 4),
                   "attributed_ms_per_step": round(attributed, 4),
                   "attributed_hbm_frac": round(bytes_step / (attributed * 1e-3) / 1e9 / HBM_PEAK_GBS, 5) if attributed > 0 else None}
            ps = (pmc or {}).get("stages", {}).get(st, {})
            if ps.get("valu_frac") is not None:
                ent["valu_frac"] = round(ps["valu_frac"], 4)
                ent["valu_insts_per_launch"] = int(ps["valu_insts_per_launch"])
            if ps.get("hbm_bytes"):
                ent["traffic_bytes_per_step"] = int(ps["hbm_bytes"])
            if ps.get("lds_conflict_cycles_per_lds_inst") is not None:
                ent["lds_conflict_cycles_per_lds_inst"] = round(ps["lds_conflict_cycles_per_lds_inst"], 3)
            kern[k] = ent
        dom_k = max(kern, key=lambda k: kern[k]["ms_per_step"]) if kern else pyr_kernel
        dk = kern.get(dom_k, {})
        dom_ach = dk.get("algorithmic_bytes_per_step", 0) / (dk.get("ms_per_step", 1) * 1e-3) / 1e9 if dk else 0.0
        # cross-check: the dominant kernel's exclusive time per step fits inside the step,
        # and the whole path's algorithmic bytes / step stay under the HBM peak
        path_bytes = sum(kern[k]["algorithmic_bytes_per_step"] for k in kern)
        path_gbs = path_bytes / (step_ms * 1e-3) / 1e9
        checks = {"dominant_kernel_ms_per_step_le_step": bool(dk.get("ms_per_step", 0) <= step_ms),
                  "path_bytes_per_step": int(path_bytes), "path_achieved_gbs": round(path_gbs, 2),
                  "path_frac": round(path_gbs / HBM_PEAK_GBS, 5),
                  "path_bytes_over_step_le_peak": bool(path_gbs <= HBM_PEAK_GBS)}
        if not (checks["dominant_kernel_ms_per_step_le_step"] and checks["path_bytes_over_step_le_peak"]):
            raise RuntimeError(f"roofline cross-check failed: {checks}, {dom_k} {dk}")
        result = {
            "metric": "ORB features/ms (640x480, 8-level) + LocalBA iter ms @1/2/4/8 GPU",
            "value": round(total_feats / elapsed_ms, 3),
            "unit": "features/ms",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_ms / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (polygon frames, seeds 100..163; no EuRoC images ship with the reference)",
            "config": {"workload": "C2: batch of 64 synthetic 640x480 frames per GPU, nFeatures=1000, 8 levels, "
                                   "extraction+description (ORBextractor::operator())",
                       "frames_per_gpu": nfr, "width": WIDTH, "height": HEIGHT, "nfeatures": NFEAT,
                       "nlevels": NLEVELS, "features_per_step_per_gpu": feats_per_step,
                       "batches_in_flight": H, "single_batch_ms": round(single_ms, 4),
                       "parallelism": f"frame-sharded x{world}" + (
                           f", all-gather of descriptors+keypoints ({backend})" if world > 1 else "")},
            "stages_ms": {k: round(v, 4) for k, v in per_step.items()},
            "roofline": {"bound": "hbm", "kernel": dom_k, "achieved": round(dom_ach, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(dom_ach / HBM_PEAK_GBS, 5),
                         "traffic": (round(dk["traffic_bytes_per_step"] / dk["launches_per_step"])
                                     if dk.get("traffic_bytes_per_step") and dk.get("launches_per_step") else None),
                         "algorithmic_bytes_per_launch": (int(dk["algorithmic_bytes_per_step"] / dk["launches_per_step"])
                                                          if dk.get("launches_per_step") else None),
                         "launches_per_step": dk.get("launches_per_step"), "launch_avg_us": dk.get("launch_avg_us"),
                         "valu": {"bound": "integer VALU", "frac": dk.get("valu_frac"),
                                  "formula": "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), "
                                             "profiles/pmc_latest.json (rocprofv3 --pmc pass of this bench)"},
                         "kernels": kern, "dominant_stage": dominant_stage, "checks": checks,
                         "durations": "exclusive: one batch alone on the chip (handle 0, synchronize after each batch); "
                                      "shared_*: the timed region's steps with every in-flight handle; attributed = "
                                      "share of the summed shared launch time x ms_per_step",
                         "pyramid": {"kernel": pyr_kernel, "achieved": round(achieved, 2),
                                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                                     "algorithmic_bytes_per_launch": int(dom_bytes),
                                     "traffic_over_algorithmic": round(traffic / dom_bytes, 3) if traffic else None,
                                     "traffic_model_bytes_per_launch": int(model_bytes),
                                     "launches_per_step": launches_per_step,
                                     "launch_avg_us": round(pyr_launch_avg_ms * 1e3, 2)},
                         "note": "kernel = the stage kernel with the most launch time in the timed region; achieved = its "
                                 "algorithmic bytes per step (bench.algorithmic_bytes_per_frame: FAST reads every level "
                                 "once; describe 43x43 patch + 60 B per keypoint; pyramid: SURVEY.md 8(d) 1,653,864 B "
                                 "per 640x480 frame) / its summed EXCLUSIVE launch time per step; launch times from an HIP event "
                                 "pair on every dispatch in a pass of the timed region's batches one at a time (bench.py --launch-dump writes them; "
                                 "profiles/r06/launch_durations_*.json); traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per "
                                 "launch (profiles/pmc_latest.json)"},
        }
        if not args.no_cpu_baseline and world == 1:
            from oracle import oracle as oracle_mod
            result["cpu_baseline"] = cpu_baseline(oracle_mod, frames[: min(nfr, 32)], args.cpu_budget)
    localba = None
    if not args.no_ba:
        try:
            localba = bench_local_ba(pkg, synth, world, dev, args.steps,
                                     rank == 0 and world == 1 and not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001 -- the extraction line is still reported
            localba = {"error": repr(e)}
    stereo = None
    if not args.no_stereo and world == 1:
        try:
            stereo = bench_stereo(pkg, synth, dev, args.steps, not args.no_cpu_baseline,
                                  n_sets=int(os.environ.get("ORB_STEREO_SETS", "2")))
        except Exception as e:  # noqa: BLE001
            stereo = {"error": repr(e)}
    pose = None
    if not args.no_pose and world == 1:
        try:
            pose = bench_pose(pkg, synth, dev, args.steps, not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            pose = {"error": repr(e)}
    c3_chain = None
    if not args.no_stereo and world == 1:
        try:
            c3_chain = bench_c3_chain(pkg, synth, dev, args.steps, not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            c3_chain = {"error": repr(e)}
    bow = None
    if not args.no_bow and world == 1:
        try:
            bow = bench_bow(pkg, synth, dev, args.steps, not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            bow = {"error": repr(e)}
    single = None
    if not args.no_single and world == 1:
        try:
            single = bench_single_frame(pkg, synth, not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            single = {"error": repr(e)}
    c4_strong = None
    if not args.no_c4:
        try:
            c4_strong = bench_c4_strong(pkg, synth, world, rank, dev, args.steps, in_flight=H)
        except Exception as e:  # noqa: BLE001
            c4_strong = {"error": repr(e)}
    matchers = None
    if not args.no_matchers and world == 1:
        try:
            matchers = bench_matchers(pkg, synth, dev, args.steps, not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            matchers = {"error": repr(e)}
    chain = None
    if not args.no_chain and world == 1:
        try:
            chain = bench_tracking_chain(pkg, synth, dev, args.steps, not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001
            chain = {"error": repr(e)}
    pcie = None
    if not args.no_single and world == 1:
        try:
            pcie = run_pcie_child(args.steps)
        except Exception as e:  # noqa: BLE001
            pcie = {"error": repr(e)}
    c4 = None
    if not args.no_c4 and world == 1:
        try:
            c4 = bench_c4(pkg, synth, dev, args.steps, in_flight=H)
        except Exception as e:  # noqa: BLE001
            c4 = {"error": repr(e)}
    if rank == 0:
        if pcie is not None:
            result["pcie_inclusive"] = pcie
        if c4 is not None:
            result["c4_shard"] = c4
        if c4_strong is not None:
            result["c4_strong"] = c4_strong
        if matchers is not None:
            result["matchers"] = matchers
        if chain is not None:
            result["tracking_chain"] = chain
        if single is not None:
            result["single_frame_latency"] = single
        if pose is not None:
            result["pose_optimization"] = pose
        if bow is not None:
            result["bow"] = bow
        result["localba_iter_ms"] = localba.get("iter_ms") if localba else None
        result["localba"] = localba
        if stereo is not None:
            result["stereo"] = stereo
        if c3_chain is not None:
            result["c3_chain"] = c3_chain
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
