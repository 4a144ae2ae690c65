"""Do independent branches of a captured HIP graph run concurrently on this ROCm stack?

Captures two spin kernels (torch.cuda._sleep, one thread each) either on one stream or
forked onto two streams (event fork/join inside the capture), replays each graph and
prints the replay times.  Concurrent branches replay in ~1x the spin, serial ones in ~2x.
Usage (GPU box): python tools/graph_branch_probe.py
"""
import time

import torch


def replay_ms(g, reps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / reps


def main():
    cyc = 20_000_000   # ~8 ms at ~2.4 GHz
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    # one spin, eager
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(cyc)
    e1.record()
    torch.cuda.synchronize()
    one = e0.elapsed_time(e1)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # serial graph: two spins on the capture stream
    g_ser = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_ser, stream=s1):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    # branched graph: fork onto s2 and join
    g_br = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_br, stream=s1):
        s2.wait_stream(s1)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        s1.wait_stream(s2)
    # eager on two streams
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(cyc)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    eager2 = (time.perf_counter() - t0) * 1e3
    print(f"one spin {one:.2f} ms; graph serial {replay_ms(g_ser):.2f} ms; graph two branches "
          f"{replay_ms(g_br):.2f} ms; eager two streams {eager2:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
