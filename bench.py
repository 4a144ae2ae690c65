#!/usr/bin/env python3
"""Benchmark: rendered frames/s (fwd+bwd) of the MI355X rasterizer on BASELINE config 3.

A "step" = one full pass of the hot path over one batch of synthetic input: projection →
tile binning (incl. its one 16-byte host read) → raster fwd → raster bwd (fixed random
cotangents) → projection bwd, for the 6 cameras of config 3 (3D, 200k Gaussians, 576x512)
— the shape BASELINE.json's north-star target is quoted on.  Inputs are resident in HBM
before the timed region.  value = views (frames) rendered fwd+bwd per second, summed over
ranks.

Multi-GPU (torchrun, one process per GPU, RCCL): every rank renders 6 cameras of its own
(ring azimuths offset per rank) of the SAME Gaussian set and the per-rank parameter
gradients are all-reduced (SUM) — the one real exchange of multi-view training.  Per-GPU
work is fixed as N grows → "scaling": "weak".

Also reported: the dominant kernel's roofline (algorithmic bytes per launch, SURVEY.md
§8(d), over its HIP-event-timed average duration) and the CPU baseline (the oracle, a
restatement of the reference semantics, timed on a bounded sample on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# PMC counter run of the same bench command (FETCH_SIZE and WRITE_SIZE passes), committed
DEFAULT_TRAFFIC_CSV = os.path.join(ROOT, "profiles", "r01_pmc_counters.csv")
# SQ counter passes (tools/pmc_sq.sh) for the dominant kernel's VALU occupancy
DEFAULT_SQ_CSVS = [os.path.join(ROOT, "profiles", f"r01_v16_pmc_sq_p{i}.csv") for i in (1, 2)]
N_SIMDS = 256 * 4   # MI355X: 256 CUs x 4 SIMDs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU oracle timing")
    ap.add_argument("--cpu-views", type=int, default=1, help="views in the bounded CPU sample")
    ap.add_argument("--shard", default="views", choices=["views", "bands"],
                    help="N>1, 3D: 'views' = every rank renders its own 6 views (weak scaling); "
                         "'bands' = the ranks split the tile rows of ONE 6-view job (strong scaling, "
                         "bands balanced by the per-row list lengths of a warm-up render)")
    ap.add_argument("--loss", default="none", choices=["none", "fused", "torch"],
                    help="3D, 1 GPU: time render + the reference IoU/L1 training loss "
                         "(train_script.py:128-133) fused into the kernels, or as plain torch ops")
    ap.add_argument("--traffic-csv", default=DEFAULT_TRAFFIC_CSV,
                    help="rocprofv3 --pmc counter_collection.csv to fill roofline.traffic "
                         "(default: the committed profiles/ counter run, if present)")
    return ap.parse_args()


def algorithmic_bytes(kernel: str, C: int, N: int, P: int, I: int, I_eff: int, p: int) -> float:
    """Per-launch algorithmic bytes, SURVEY.md §8(d) per-unit figures × units per launch."""
    if kernel.startswith("raster") and kernel.endswith("_fwd"):
        return 40.0 * I_eff + 20.0 * P                 # read id+xy+conic+opac+colour; write rgb+alpha+last
    if kernel.startswith("raster") and kernel.endswith("_bwd"):
        return 24.0 * P + 40.0 * I_eff + 36.0 * C * N  # cotangents+alpha+last; list; reduced grads
    if kernel.startswith("project") and kernel.endswith("_fwd"):
        return C * N * (4.0 * p + 32.0)
    if kernel.startswith("project") and kernel.endswith("_bwd"):
        return N * (36.0 + 32.0 + 8.0 * p) * C
    if kernel == "bin_sort":
        return 36.0 * I
    return 0.0


def step_bytes(C: int, N: int, P_view: int, I: int, I_eff: int, p: int, backward: bool = True) -> float:
    """Whole step, SURVEY.md §8(d): fwd+bwd C·N·(12p+136) + 36·I + 80·I_eff + 44·C·P;
    fwd-only C·N·(4p+32) + 36·I + 40·I_eff + 20·C·P."""
    if not backward:
        return C * N * (4.0 * p + 32.0) + 36.0 * I + 40.0 * I_eff + 20.0 * C * P_view
    return C * N * (12.0 * p + 136.0) + 36.0 * I + 80.0 * I_eff + 44.0 * C * P_view


# libgsr call name (render.py timing brackets) -> substring of its dominant kernel's symbol
KERNEL_SYMBOL = {"raster3d_bwd": "k_raster_bwd<false, false>", "raster3d_fwd": "k_raster_fwd<false>",
                 "raster2d_bwd": "k_raster_bwd<false, true>", "raster2d_fwd": "k_raster_fwd<true>",
                 "bin_sort": "k_segsort"}


def traffic_from_csv(path: str, kernel_substr: str):
    """HBM bytes per launch from a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass (KB units;
    FETCH_SIZE doubled per the gfx950 correction in MI355X_MICROARCH.md §HBM)."""
    import csv
    fetch, write = [], []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_substr not in row.get("Kernel_Name", ""):
                continue
            name, val = row.get("Counter_Name"), float(row.get("Counter_Value", 0))
            if name == "FETCH_SIZE":
                fetch.append(val)
            elif name == "WRITE_SIZE":
                write.append(val)
    if not fetch and not write:
        return None
    f = 2.0 * 1024.0 * (sum(fetch) / max(len(fetch), 1))
    w = 1024.0 * (sum(write) / max(len(write), 1))
    return f + w


def valu_from_csv(paths, kernel_substr: str):
    """VALU occupancy of one kernel from rocprofv3 SQ passes: SQ_ACTIVE_INST_VALU (quad-cycles,
    summed over SIMDs) x 4 over N_SIMDS x the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs), and
    the issue-slot fraction SQ_INSTS_VALU x 4 cycles (a full-rate wave64 fp32 op on a 16-lane
    SIMD) over the same SIMD-cycles.  None when the passes are missing."""
    import csv
    acc = {}
    for path in paths:
        if not os.path.exists(path):
            return None
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_substr in row.get("Kernel_Name", ""):
                    acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    need = ("SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")
    if not all(k in acc for k in need):
        return None
    mean = {k: sum(v) / len(v) for k, v in acc.items()}
    simd_cycles = N_SIMDS * mean["GRBM_GUI_ACTIVE"] / 8.0
    return {"active_frac": 4.0 * mean["SQ_ACTIVE_INST_VALU"] / simd_cycles,
            "issue_frac": 4.0 * mean["SQ_INSTS_VALU"] / simd_cycles,
            "insts_per_launch": mean["SQ_INSTS_VALU"], "source": "profiles/r01_v16_pmc_sq_p{1,2}.csv"}


def cpu_baseline(cfg, params, V, K, views: int):
    """The oracle (CPU restatement of the reference semantics) on `views` of the workload."""
    from oracle.oracle3d import render3d as oracle_render3d
    from oracle.oracle2d import render2d_dense
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(cfg.seed + 1)
    t0 = time.perf_counter()
    if cfg.mode == "3d":
        p = params.detach().cpu().clone().requires_grad_(cfg.backward)
        rgb, alpha = oracle_render3d(p, V[:views].cpu(), K[:views].cpu(), cfg.width, cfg.height, torch.ones(3))
        if cfg.backward:
            vr = torch.randn(rgb.shape, generator=g)
            va = torch.randn(alpha.shape, generator=g)
            ((rgb * vr).sum() + (alpha * va).sum()).backward()
        sample = (f"{views} of {cfg.views} views of {cfg.name}, "
                  f"{'fwd+bwd' if cfg.backward else 'fwd'}, oracle/oracle3d.py")
    else:
        n = 2000
        p = params[:n].detach().cpu().clone().requires_grad_(True)
        rgb, alpha = render2d_dense(p, cfg.width, cfg.height, torch.ones(3))
        ((rgb * torch.randn(rgb.shape, generator=g)).sum()).backward()
        sample = f"first {n} of {cfg.N} Gaussians, 1 view, dense reference algorithm (linear in N)"
    dt = time.perf_counter() - t0
    value = views / dt if cfg.mode == "3d" else (n / cfg.N) / dt
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": value, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": sample, "seconds": round(dt, 2), "cpu": cpu}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GSR_DIST_BACKEND=gloo + GSR_SAME_DEVICE=1 rehearse N ranks on a single GPU (box tests);
    # the driver's scaling runs use the defaults: backend "nccl" (RCCL), one GPU per rank.
    if os.environ.get("GSR_SAME_DEVICE") == "1":
        local = 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("GSR_DIST_BACKEND", "nccl"))
    dev = torch.device("cuda", local)

    from gsr import render as R
    from gsr.scenes import CONFIGS, gaussians2d, gaussians3d, ring_cameras
    cfg = CONFIGS[args.config]
    C = cfg.views
    P = C * cfg.width * cfg.height
    if cfg.mode == "3d":
        params_cpu = gaussians3d(cfg.N, cfg.seed)
        V, K = ring_cameras(C, cfg.width, cfg.height)
        p_dim = 14
    else:
        params_cpu = gaussians2d(cfg.N, cfg.width, cfg.height, cfg.seed + rank)
        V, K = ring_cameras(1, cfg.width, cfg.height)
        p_dim = 9
    params = params_cpu.to(dev).requires_grad_(True)
    Vd, Kd = V.to(dev), K.to(dev)
    bg = torch.ones(3, device=dev)
    g = torch.Generator().manual_seed(cfg.seed + 1)
    if cfg.mode == "3d":
        v_rgb = torch.randn(C, cfg.height, cfg.width, 3, generator=g).to(dev)
        v_alpha = torch.randn(C, cfg.height, cfg.width, generator=g).to(dev)
    else:
        v_rgb = torch.randn(cfg.height, cfg.width, 3, generator=g).to(dev)
        v_alpha = torch.randn(cfg.height, cfg.width, generator=g).to(dev)

    bands = args.shard == "bands" and cfg.mode == "3d" and world > 1
    if bands:
        # one 6-view job split by tile rows; bands balanced by a full warm-up render's row work
        from gsr.multiview import band_shard, row_work, sharded_backward_bands
        th, tw = (cfg.height + 15) // 16, (cfg.width + 15) // 16
        with torch.no_grad():
            R.render3d(params, Vd, Kd, cfg.width, cfg.height, bg)
        weights = row_work(R.tile_work(), C, th, tw)
        my_band = band_shard(th, world, rank, weights)

        def render_band(p, Vs, Ks, band):
            return R.render3d(p, Vs, Ks, cfg.width, cfg.height, bg, R.RenderOptions3D(band=band))
    elif cfg.mode == "3d" and world > 1:
        # all ranks hold the same Gaussians; this rank renders its shard of the 6*world views
        from gsr.multiview import sharded_backward, view_shard
        V_all, K_all = ring_cameras(C * world, cfg.width, cfg.height)
        V_all, K_all = V_all.to(dev), K_all.to(dev)
        assert view_shard(C * world, world, rank).stop - view_shard(C * world, world, rank).start == C
        g2 = torch.Generator().manual_seed(cfg.seed + 2)
        vr_all = torch.randn(C * world, cfg.height, cfg.width, 3, generator=g2).to(dev)
        va_all = torch.randn(C * world, cfg.height, cfg.width, generator=g2).to(dev)

        def render_views(p, Vs, Ks):
            return R.render3d(p, Vs, Ks, cfg.width, cfg.height, bg)

    if args.loss != "none":
        if cfg.mode != "3d" or world > 1:
            raise SystemExit("--loss: 3D configs on one GPU only")
        from gsr.loss import render3d_iou_l1
        g3 = torch.Generator().manual_seed(cfg.seed + 3)
        timg = torch.rand(C, 3, cfg.height, cfg.width, generator=g3).to(dev)
        tmask = (torch.rand(C, cfg.height, cfg.width, generator=g3) < 0.3).float().to(dev)

    def step():
        params.grad = None
        if args.loss == "fused":
            li, lm, rgb, alpha = render3d_iou_l1(params, Vd, Kd, cfg.width, cfg.height, bg, timg, tmask, 1.0)
            (li + lm).backward()
        elif args.loss == "torch":
            rgb, alpha = R.render3d(params, Vd, Kd, cfg.width, cfg.height, bg)
            inter = (alpha * tmask).sum(dim=(-2, -1))
            union = (alpha + tmask - alpha * tmask).sum(dim=(-2, -1))
            li = 1 - ((inter + 1e-6) / (union + 1e-6)).mean()
            lm = torch.abs(timg - rgb.permute(0, 3, 1, 2)).sum() / tmask.sum()
            (li + lm).backward()
        elif bands:
            params.grad = sharded_backward_bands(render_band, params, Vd, Kd, v_rgb, v_alpha, th, weights)
        elif cfg.mode == "3d" and world > 1:
            params.grad = sharded_backward(render_views, params, V_all, K_all, vr_all, va_all)
        elif cfg.mode == "3d" and not cfg.backward:
            with torch.no_grad():   # config 2 is forward-only
                R.render3d(params, Vd, Kd, cfg.width, cfg.height, bg)
        elif cfg.mode == "3d":
            rgb, alpha = R.render3d(params, Vd, Kd, cfg.width, cfg.height, bg)
            torch.autograd.backward([rgb, alpha], [v_rgb, v_alpha])
        else:
            # 2D: the reference ignores the camera, so every view of a frame is the same image
            for _ in range(C):
                rgb, alpha = R.render2d(params, cfg.width, cfg.height, bg)
                torch.autograd.backward([rgb, alpha], [v_rgb, v_alpha])
            if world > 1:
                import torch.distributed as dist
                dist.all_reduce(params.grad)

    for _ in range(args.warmup):
        step()
    # per-call breakdown from a separate profiled pass (every libgsr call bracketed by
    # events); it also names the dominant kernel
    torch.cuda.synchronize()
    R.enable_kernel_timing(True)
    for _ in range(max(2, min(args.steps, 5))):
        step()
    breakdown = R.kernel_times_ms()
    R.enable_kernel_timing(False)
    dom_name = max(breakdown.items(), key=lambda kv: kv[1][0] * kv[1][1])[0] if breakdown else None
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    # timed region: events only around the dominant kernel (its live average duration)
    R.enable_kernel_timing(True, only={dom_name} if dom_name else None)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ktimes = R.kernel_times_ms()
    R.enable_kernel_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)

    allreduce_ms = None
    if world > 1:
        # the step's one collective, timed on its own: all_reduce(SUM) of the fp32 v_params
        buf = torch.zeros(cfg.N, p_dim, device=dev)
        for _ in range(3):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            dist.all_reduce(buf)
        e1.record()
        torch.cuda.synchronize()
        t = torch.tensor([e0.elapsed_time(e1) / 10], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        allreduce_ms = float(t)

    st = R.last_stats()
    I = st.get("n_isect", 0)
    I_eff = R.effective_isect()
    views_per_step = C if bands else C * world
    value = views_per_step * args.steps / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    # dominant kernel (largest total time in the profiled pass), timed live in the region
    dom_ms, dom_n = ktimes.get(dom_name, (0.0, 0)) if dom_name else (0.0, 0)
    Pd = P if cfg.mode == "3d" else cfg.width * cfg.height
    Cd = C if cfg.mode == "3d" else 1
    alg = algorithmic_bytes(dom_name or "", Cd, cfg.N, Pd, I, I_eff, p_dim)
    achieved = alg / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic = None
    if args.traffic_csv and dom_name and os.path.exists(args.traffic_csv):
        traffic = traffic_from_csv(args.traffic_csv, KERNEL_SYMBOL.get(dom_name, "k_" + dom_name))
    valu = valu_from_csv(DEFAULT_SQ_CSVS, KERNEL_SYMBOL.get(dom_name, "k_" + dom_name)) if dom_name else None
    sb = step_bytes(Cd, cfg.N, cfg.width * cfg.height, I, I_eff, p_dim, cfg.backward) * (1 if cfg.mode == "3d" else C)

    out = {
        "metric": "rendered frames/sec (%s) at N_gauss x H x W" % ("fwd+bwd" if cfg.backward else "fwd"),
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if bands else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md §8(d) distribution A, seed 1000+config)",
        "config": {"workload": cfg.name, "N_gauss": cfg.N, "width": cfg.width, "height": cfg.height,
                   "views_per_gpu": C, "background": "white", "loss": args.loss,
                   "parallelism": (f"tile-row bands x{world} (band {my_band[0]}-{my_band[1]} on rank 0) + RCCL "
                                   f"all-reduce of v_params" if bands else
                                   f"view-sharded x{world} + RCCL all-reduce of v_params" if world > 1 else "single GPU")},
        "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes": alg, "avg_ms": dom_ms, "launches": dom_n, "valu": valu},
        "kernels_ms": {k: round(v[0], 4) for k, v in sorted(breakdown.items())},
        "allreduce_ms": allreduce_ms,
        "sets_per_s": value / C,
        "pair_evals_per_s": 2.0 * 256.0 * I_eff * (1 if cfg.mode == "3d" else C) * world / (ms_per_step * 1e-3),
        "step_roofline": {"algorithmic_bytes": sb, "achieved": sb / (ms_per_step * 1e-3) / 1e9,
                          "unit": "GB/s", "frac": sb / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "formula": ("SURVEY.md 8(d): C*N*(12p+136) + 36*I + 80*I_eff + 44*C*P per rank" if cfg.backward
                                      else "SURVEY.md 8(d) fwd-only: C*N*(4p+32) + 36*I + 40*I_eff + 20*C*P per rank")},
        "binning": {"I": I, "I_eff": I_eff, "max_list": st.get("max_seg"), "busy_tiles": st.get("n_busy"),
                    "tiles": st.get("tiles")},
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        cb = cpu_baseline(cfg, params_cpu, V, K, args.cpu_views)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = value / cb["value"] if cb["value"] > 0 else None
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
