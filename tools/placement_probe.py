"""Does a kernel's time depend on where its buffers land?  One process, config C's eager step
timed per kernel (HIP events) in several trials; between trials a spacer allocation of a
different size shifts every later allocation of the caching allocator.
Usage (GPU box): python tools/placement_probe.py [CONFIG] [TRIALS]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))

import bench  # noqa: E402
from gsr.scenes import CONFIGS  # noqa: E402


def main():
    c = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda:0")
    w = bench.Workload(CONFIGS[c], dev, 1, 0, "views", 0, "none", False)
    R = w.R
    spacers = []
    for t in range(trials):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        mb = 7 + 13 * t
        spacers.append(torch.empty(mb * 2**20 // 4, device=dev))
        for _ in range(3):
            w.step()
        torch.cuda.synchronize()
        R.enable_kernel_timing(True)
        for _ in range(10):
            w.step()
        k = R.kernel_times_ms()
        R.enable_kernel_timing(False)
        print(f"trial {t} spacer {mb} MB:", {n: round(v[0] * 1000, 1) for n, v in sorted(k.items())}, flush=True)


if __name__ == "__main__":
    main()
