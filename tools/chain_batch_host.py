"""Host cost of TrackingChainBatch.track for a 512-frame batch (the bench's items): the enqueue time per
call without a sync, and a cProfile of the Python side (profiles/r05/chain_batch_host_r05.txt)."""
import cProfile
import io
import pstats
import sys
import time

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import torch  # noqa: E402
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402
import test_tracking_chain_gpu as T  # noqa: E402

nb, n_scenes = 512, 4
scenes = [synth.tracking_chain_scene(seed=81 + s) for s in range(n_scenes)]
fr = [T._frames(pkg, sc) for sc in scenes]
cap = 2048
devs = [T._device(pkg, sc, C, L, cap=cap) for sc, (C, L) in zip(scenes, fr)]
locs = [pkg.DeviceLocalMap.from_host(torch.device("cuda"), **scenes[b % n_scenes]["local"]) for b in range(nb)]
items = [(devs[b % n_scenes][0], devs[b % n_scenes][1], locs[b], scenes[b % n_scenes]["pose7_pred"]) for b in range(nb)]
chb = pkg.TrackingChainBatch(cap, nb)
st = torch.cuda.Stream()
for _ in range(2):
    chb.track(items, stream=st)
st.synchronize()
enq = []
t0 = time.perf_counter()
for _ in range(10):
    a = time.perf_counter()
    chb.track(items, stream=st)
    enq.append((time.perf_counter() - a) * 1e3)
st.synchronize()
tot = (time.perf_counter() - t0) * 1e3 / 10
print(f"per call: {tot:.3f} ms wall, enqueue (host) median {sorted(enq)[5]:.3f} ms")
# device time of one call alone (events on the stream around it), and the host time of the same call
# with the stream idle (no wait on a previous call's staging)
for _ in range(3):
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    a = time.perf_counter()
    chb.track(items, stream=st)
    h = (time.perf_counter() - a) * 1e3
    e1.record(st)
    st.synchronize()
    print(f"one call: device {e0.elapsed_time(e1):.3f} ms (from its first enqueue), host enqueue {h:.3f} ms")
# device time alone: the stream held by a sleep kernel while the whole call is enqueued behind it
for _ in range(3):
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        torch.cuda._sleep(20_000_000)
    e0.record(st)
    chb.track(items, stream=st)
    e1.record(st)
    st.synchronize()
    print(f"one call, enqueued behind a sleep: device {e0.elapsed_time(e1):.3f} ms")
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    chb.track(items, stream=st)
pr.disable()
st.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(15)
print(s.getvalue())
