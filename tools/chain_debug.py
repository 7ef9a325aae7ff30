"""Debug helper: SearchByProjection(LastFrame) on the device form vs the host form vs the oracle for the
tracking-chain scene (prints counts and the first differing keypoints)."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import load_package  # noqa: E402

pkg = load_package()
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from orbslam3_amd import synth  # noqa: E402
import test_tracking_chain_gpu as T  # noqa: E402

for seed in (81, 83):
    sc = synth.tracking_chain_scene(seed=seed, stereo=seed != 83)
    C, L = T._frames(pkg, sc)
    th = 7
    m = pkg.ORBmatcher(0.9, True)
    nh, mh = m.SearchByProjectionFrame(C, L, th, False)
    no, mo = oracle.search_by_projection_frame(C, L, th, False, True)
    cur, last, local = T._device(pkg, sc, C, L)
    chain = pkg.TrackingChain(cur.cap, th_motion=th)
    r = chain.track(cur, last, local, sc["pose7_pred"]).sync()
    md = r["m1"][:C.N].copy()
    # undo the discard for the comparison
    md_raw = md.copy()
    print("seed", seed, "host", nh, "oracle", no, "device n1", r["n1"], "host==oracle", np.array_equal(mh, mo))
    # rerun only the search on the device
    lib = pkg._lib.load()
    import ctypes
    d_m = torch.empty(cur.cap, dtype=torch.int32, device="cuda")
    d_n = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    pkg._lib.check(lib.orb_search_by_projection_frame_device(m._handle(), ctypes.byref(cur.view()),
                                                             ctypes.byref(last.view()), float(th), 0, d_m.data_ptr(),
                                                             d_n.data_ptr(), ctypes.c_void_p(st.cuda_stream)), "sbp")
    torch.cuda.synchronize()
    dm = d_m.cpu().numpy()[:C.N]
    diff = np.flatnonzero(dm != mo)
    print("  device-only n", int(d_n.item()), "diffs", len(diff), diff[:10], dm[diff[:10]], mo[diff[:10]])
    for i in diff[:5]:
        k = C.mvKeysUn[i]
        print("   kp", i, k["x"], k["y"], k["octave"], k["angle"], "ur", None if C.mvuRight is None else C.mvuRight[i])
