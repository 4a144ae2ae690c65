"""Graph replay of projection + tile scan only (no emission, nothing indexes by the counts):
does the tile-count buffer survive a second replay, depending on where it was allocated and
how it is zeroed?  Finding (ROCm 7.2, MI355X): with the zeroing done by hipMemsetAsync (a
memset node) every replay after the first saw garbage counts; a kernel node (torch's fill, or
libgsr's k_zero_i32 now used by the projection) replays correctly."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pose-splatter_amd")]
import ctypes
import torch
from gsr import render as R, _lib
from gsr.scenes import gaussians3d, ring_cameras
dev = torch.device("cuda:0")
W, H, C, N = 192, 170, 3, 20000
params = gaussians3d(N, 11).to(dev)
V, K = [t.to(dev) for t in ring_cameras(C, W, H)]
L = _lib.lib()
CT = C * 12 * 11
pre = R._Arena(dev, {"rec": C * N * 48, "depth": C * N * 4, "rect": C * N * 8, "cnt": C * N * 4,
                     "isect_off": C * N * 4, "tile_off": (CT + 1) * 4, "busy": CT * 4, "chunk_base": (CT + 1) * 4,
                     "tile_end": CT * 4, "tile_cut": CT * 8, "stats_dev": 128})
q = pre.ptr
caps = _lib.BinCaps(0, 0, None, 128, 0)

def stage1(tc, zeroed):
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(L.gsr3d_project_fwd(params.data_ptr(), N, 14, V.data_ptr(), K.data_ptr(), C, W, H, 0.01, 1e10, 0.0, 0.3,
                                   0, 0, 0, -1, q["rec"], q["depth"], q["rect"], q["cnt"], q["isect_off"], tc.data_ptr(),
                                   zeroed, stream), "proj")
    _lib.check(L.gsr_bin_offsets(tc.data_ptr(), CT, q["tile_off"], q["chunk_base"], q["busy"], q["tile_end"],
                                 q["tile_cut"], ctypes.byref(caps), q["stats_dev"], stream), "scan")

def run(name, make_tc, zeroed, in_capture):
    tc = None if in_capture else make_tc()
    g = torch.cuda.CUDAGraph()
    holder = {}
    with torch.cuda.graph(g):
        t = make_tc() if in_capture else tc
        holder["tc"] = t
        stage1(t, zeroed)
    t = holder["tc"]
    for k in range(3):
        g.replay()
        torch.cuda.synchronize()
        st = pre.view("stats_dev", torch.int32).tolist()
        print(f"{name}: replay {k} I={st[0]} busy={st[3]} tc sum={int(t[:-1].sum())}", flush=True)

run("outside+memset", lambda: torch.zeros(CT + 1, device=dev, dtype=torch.int32), 0, False)
run("inside-empty+memset", lambda: torch.empty(CT + 1, device=dev, dtype=torch.int32), 0, True)
run("inside-empty+zero kernel", lambda: torch.empty(CT + 1, device=dev, dtype=torch.int32), 0, True)
run("inside-zeros(torch fill)", lambda: torch.zeros(CT + 1, device=dev, dtype=torch.int32), 1, True)
