"""Host-side (Python) cost of eager bounded steps: cProfile over `steps` eager steps of a
config's workload on one GPU, the GPU kept ahead by a spin before each step so the host never
waits on it (the profile is then the host's own enqueue work).  On the GPU box:
    python3 tools/host_profile.py CONFIG [RANKS RANK]   (RANKS > 1: that rank's strong share)"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = [sys.argv[0]] + sys.argv[1:]
import bench  # noqa: E402


def main():
    from gsr import render as R
    from gsr.scenes import CONFIGS
    cfg = CONFIGS[int(sys.argv[1])]
    R.set_capacity_mode("bounded")   # bench.py's default: the sync-free step
    n, r = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1, 0)
    dev = torch.device("cuda:0")
    w = bench.Workload(cfg, dev, n, r, "units", 4, "none", comm=False, view_cost=0.3, exchange="dense")
    for _ in range(5):
        w.step()
    torch.cuda.synchronize()
    steps = 30
    t0 = time.perf_counter()
    for _ in range(steps):
        w.step()
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / steps
    torch.autograd.set_multithreading_enabled(False)   # the backward on this thread: profiled too
    pr = cProfile.Profile()
    torch.cuda._sleep(200_000_000)   # the GPU busy while the host enqueues every profiled step
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(steps):
        w.step()
    pr.disable()
    t_host = (time.perf_counter() - t0) / steps
    torch.cuda.synchronize()
    print(f"config {sys.argv[1]} share {r}/{n}: eager step {1e3 * t_eager:.3f} ms, host enqueue (profiled) "
          f"{1e3 * t_host:.3f} ms per step", flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(40)
    pstats.Stats(pr).sort_stats("cumtime").print_stats(40)


if __name__ == "__main__":
    main()
