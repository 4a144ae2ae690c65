"""CPU, world_size 2 (gloo): view-sharded rendering + all-reduce of the parameter gradient
equals the single-process multi-view gradient (the multi-GPU path of bench.py / §8(e)).

The renderer inside the ranks is the CPU oracle (test infrastructure); on the GPU box the
same gsr.multiview code runs with libgsr and backend "nccl" (RCCL).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _scene():
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(300, 5, extent=0.05)
    p[:, 3:6] += 1.0
    V, K = ring_cameras(5, 40, 32)
    g = torch.Generator().manual_seed(9)
    vr = torch.randn(5, 32, 40, 3, generator=g)
    va = torch.randn(5, 32, 40, generator=g)
    return p, V, K, vr, va


def _render(p, V, K):
    from oracle.oracle3d import render3d
    return render3d(p, V, K, 40, 32, torch.ones(3))


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "pose-splatter_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gsr.multiview import sharded_backward
    p, V, K, vr, va = _scene()
    grad = sharded_backward(_render, p, V, K, vr, va)
    out[rank] = grad
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_view_sharded_allreduce_matches_single_process(world):
    from gsr.multiview import sharded_backward
    p, V, K, vr, va = _scene()
    ref = sharded_backward(_render, p, V, K, vr, va)     # world 1: all views locally
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        assert torch.allclose(out[r], ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max())), r
    assert torch.equal(out[0], out[1])
