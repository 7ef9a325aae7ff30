"""Debug probe: the one-rank RCCL communicator of LocalBA (orb_ba_dist_init_rccl) and the sharded device
loop, step by step with progress on stderr (run under `timeout`)."""
import os
import sys
import time

sys.path.insert(0, ".")
sys.path.insert(0, "tests")


def say(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ["ORBGPU_BA_DIST_FORCE"] = "1"
    torch.cuda.set_device(0)
    say("init_process_group nccl")
    dist.init_process_group("nccl", rank=0, world_size=1)
    t = torch.ones(4, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    say("torch all_reduce ok", t.tolist())
    from conftest import load_package
    pkg = load_package()
    from orbslam3_amd import synth
    ba = pkg.LocalBA()
    say("attach rccl")
    ba.attach(transport="rccl")
    say("attached")
    prob = synth.local_ba_problem(n_kf=20, n_points=800, obs_per_point=5, stereo_frac=0.3, seed=12)
    say("optimize")
    _, _, _, _, res = ba.optimize(prob, 10)
    say("optimize done", res)
    dist.destroy_process_group()


if __name__ == "__main__" and "--timing" not in sys.argv:
    main()


def timing():
    """C5 solve time: one-rank RCCL sharded device loop vs the plain single-GPU handle."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29562")
    os.environ["ORBGPU_BA_DIST_FORCE"] = "1"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    from conftest import load_package
    pkg = load_package()
    from orbslam3_amd import synth
    prob = synth.local_ba_problem(n_kf=50, n_points=2000, obs_per_point=6, stereo_frac=0.0, seed=7)
    for name, ba in (("single", pkg.LocalBA()), ("sharded-1rank-rccl", pkg.LocalBA().attach(transport="rccl"))):
        for _ in range(3):
            ba.optimize(prob, 10)
        t0 = time.perf_counter()
        it = tr = 0
        for _ in range(10):
            _, _, _, _, r = ba.optimize(prob, 10)
            it += r["iterations"]
            tr += r["trials"]
        dt = (time.perf_counter() - t0) * 1e3
        say(f"{name}: {dt / 10:.3f} ms/solve, {dt / it:.4f} ms/iteration, {dt / tr:.4f} ms/trial")
    dist.destroy_process_group()


if __name__ == "__main__" and "--timing" in sys.argv:
    timing()
