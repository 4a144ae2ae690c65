#!/usr/bin/env python3
"""Benchmark: rendered frames/s (fwd+bwd) of the MI355X rasterizer on a BASELINE config.

A "step" = one full pass of the hot path over one batch of synthetic input: projection ->
tile binning -> raster fwd -> raster bwd (fixed random cotangents) -> projection bwd.  The
timed steps run capacity-bounded (no host read; `--capacity exact` adds the 32-byte stats
read-back per forward that gsplat's count read-back corresponds to).  Default workload: BASELINE config 3 (3D, 200k Gaussians,
576x512, 6 cameras) -- the shape BASELINE.json's north-star target is quoted on.  Inputs
are resident in HBM before the timed region.  value = views (frames) rendered per second
over the whole job.

Multi-GPU (torchrun, one process per GPU, RCCL over xGMI), SURVEY.md §8(e).  At N > 1 the
line reports the default layout as `value` AND the config's other layout next to it (keys
"weak" / "strong" / "frame_owners", each with its own value, ms_per_step and allreduce_ms):
  * 3D, --shard units (default since round 6, "strong"): ONE C-view job per step -- the same
    job at every N; the C*th (view, tile row) units are cut into `world` contiguous ranges
    balanced by list entries read plus a per-view cost (gsr.multiview.unit_shard); each rank
    projects only the views it touches, bins only its rows, and all-reduces its partial
    v_params in buckets (latency- and exchange-bound at configs 3 and 5: DESIGN.md §5,
    --rank-share).
  * 3D, --shard views ("weak", reported under "weak"): a multi-camera batch -- every rank
    renders C views of its own (ring offset per rank) of the same Gaussians, and the [N,14]
    gradient is all-reduced in Gaussian-range buckets that overlap the projection backward
    (N times the work at N ranks: the data-parallel shape, not the 1 -> N curve of one job).
  * 2D (config 4), --shard units (default, "strong"): 8 frames x 6 views = 48 (frame, view)
    units, round-robin over ranks; each rank renders its units batched per frame bucket and
    all-reduces the [8,N,9] gradient per bucket (async, overlapping the next bucket) -- the
    RCCL Gaussian-gradient all-reduce SURVEY.md §8(e) asks the benchmark to exercise.
  * 2D, --shard frames (reported under "frame_owners"): frame f with all its views on rank
    f % N, no Gaussian-gradient exchange (the frames' sets are disjoint).
  * config 2 (one view, fwd-only): replicas, "weak".
--rank-share N (one GPU, no collectives): times each of the N ranks' shares of the strong
layout one after the other and reports the projected N-GPU time (max share + a ring
all-reduce cost model); no multi-GPU node is needed to size the design.

Launch: the steps run capacity-bounded (gsr.render "bounded": no host synchronisation, every
buffer and grid from the previous step's bounds, overflow checked on the device and by
check_overflow() after the timed region).  On one GPU the K timed steps are captured as ONE
HIP graph (torch.cuda.CUDAGraph) before the timed region and replayed once inside it, with
external HIP timing events around the dominant kernel of every step (--graph 0: eager
launches).  `--gpus N` without a launcher starts N ranks itself (torch.distributed.run).

Also reported: the dominant kernel's roofline (algorithmic bytes per launch, SURVEY.md §8(d),
over its HIP-event-timed average duration, events on the launch stream); roofline.traffic /
.valu from rocprofv3 PMC passes OF THE SAME CONFIG committed under profiles/ (null when none);
the CPU baseline (the oracle, a restatement of the reference semantics, timed on a bounded
sample on this host); and dPSNR = |PSNR(gsr, target) - PSNR(oracle, target)| on a perturbed
target (scripts/utils/evaluate_model.py:240-243).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import platform
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0   # one xGMI link, per direction (ring all-reduce cost model)
N_SIMDS = 256 * 4       # MI355X: 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4         # MI355X maximum engine clock (MI355X_MICROARCH.md)
PROFILES = os.path.join(ROOT, "profiles")
FRAMES_2D = 8           # config 4: 8 frames x 6 views


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--exchange", default="dense", choices=["dense", "rows", "sparse"],
                    help="--shard units (3D): 'dense' (default) = all-reduce the dense gradient in async buckets "
                         "overlapping project_bwd; 'rows' = the device sparse exchange -- each share's backward "
                         "writes only the gradient rows of the Gaussians it composited into a fixed-capacity "
                         "block, the blocks are all-gathered and summed in rank order on the device (no host "
                         "read, graph-capturable; gsr.multiview.rows_backward_units; at config 5, 8 ranks a share "
                         "composites 17-21 %% of the Gaussians, where it breaks even with the dense all-reduce: "
                         "DESIGN.md §5); 'sparse' = the host-synchronising torch variant (exchange only "
                         "the rows each rank touched (gsr.multiview.sparse_sum)")
    ap.add_argument("--shard", default=None, choices=["units", "views", "frames"],
                    help="3D, N>1: 'views' (default) = a multi-camera batch, every rank renders C views of its own "
                         "and the Gaussian gradient is all-reduced (weak scaling); 'units' = the ranks split ONE "
                         "C-view job by (view, tile row) units (strong scaling; latency- and exchange-bound, "
                         "see DESIGN.md §5 and --rank-share).  2D (config 4), N>1: 'units' (default) = (frame, "
                         "view) units round-robin with a per-frame-bucket all-reduce; 'frames' = frame f with all "
                         "its views on rank f %% N, no Gaussian-gradient exchange (the frames' sets are disjoint). "
                         "At N>1 the other layout of the config is timed too and reported in the same line")
    ap.add_argument("--buckets", type=int, default=0,
                    help="all-reduce buckets (3D: Gaussian ranges of v_params; 2D: frame ranges); 0 = default "
                         "(3D 4, 2D 2; 1 on a single GPU)")
    ap.add_argument("--rank-share", type=str, default="",
                    help="one GPU: time each rank's share of the strong layout alone and project N-GPU scaling; "
                         "N or a list N1,N2,... (e.g. 2,4,8)")
    ap.add_argument("--view-cost", type=float, default=0.3,
                    help="3D strong layout: cost of each view a rank touches (its projection fwd+bwd of all N "
                         "Gaussians), in list entries per Gaussian (x N) -- the unit partition balances "
                         "entries read + view_cost x views touched")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU oracle timing")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: every CPU this "
                                                               "process may run on)")
    ap.add_argument("--psnr", type=int, default=1, help="0 disables the dPSNR check")
    ap.add_argument("--loss", default="none", choices=["none", "fused", "torch"],
                    help="3D, 1 GPU: time render + the reference IoU/L1/SSIM training loss "
                         "(train_script.py:127-133) fused into libgsr kernels, or as plain torch ops")
    ap.add_argument("--fwd-lanes", type=int, default=0, choices=[0, 4, 16],
                    help="3D raster forward layout: 0 automatic, 4 or 16 lanes per pixel (gsr_set_fwd_lanes)")
    ap.add_argument("--bwd-layout", type=int, default=0, choices=[0, 1, 2],
                    help="3D raster backward layout: 0 automatic, 1 one pixel per lane, 2 two (gsr_set_bwd_layout)")
    ap.add_argument("--emit-staged", type=int, default=-1, choices=[-1, 0, 1],
                    help="emission layout (gsr_set_emit_staged): 1 LDS-staged per-tile runs, 0 direct "
                         "scatter, -1 library default")
    ap.add_argument("--lazy", type=str, default="",
                    help="MIN_LEN,PREFIX: lazy depth order for 3D lists longer than MIN_LEN, sorted prefix "
                         ">= PREFIX entries (gsr_set_lazy_sort; default 16384,4096; MIN_LEN 0 disables)")
    ap.add_argument("--masks", type=int, default=0, choices=[0, 1],
                    help="3D quadrant masks (gsr.render.set_quadrant_masks): the emission records which 8x8 "
                         "quadrants each list entry reaches and the raster forward gathers only those (same "
                         "outputs bit for bit; off by default: slower end to end, DESIGN.md §4)")
    ap.add_argument("--pmc-dir", default=PROFILES, help="where the per-config rocprofv3 PMC passes live")
    ap.add_argument("--chunk-entries", type=str, default="",
                    help="3D,2D backward work-unit lengths (gsr.render.set_chunk_entries; default 128,512)")
    ap.add_argument("--capacity", default="bounded", choices=["bounded", "exact"],
                    help="bounded: no host sync per step (bounds from the previous step, checked on device); "
                         "exact: one 32-byte stats read-back per forward")
    ap.add_argument("--split", type=int, default=1,
                    help="3D, one GPU: render the views in SPLIT groups, each group's whole fwd+bwd on its own HIP "
                         "stream (forked and joined inside the step, so a captured graph holds SPLIT independent "
                         "branches), gradients summed at the join")
    ap.add_argument("--graph", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: capture the timed steps as one HIP graph (needs --capacity bounded); 0: eager "
                         "launches; -1: 1 on a single GPU with bounded capacity, else 0")
    a = ap.parse_args(argv)
    if a.shard is None:
        # every config but 2 (one fwd-only view: replicas) times the SAME job at every N by default:
        # 3D, the C-view job split into (view, tile row) units; 2D, the 48 (frame, view) units
        # (the 1 -> N curve must not time N times the work at N ranks)
        a.shard = "views" if a.config == 2 else "units"
    if a.shard == "frames" and a.config != 4:
        raise SystemExit("--shard frames is the 2D multi-frame layout (config 4)")
    return a


# ------------------------------------------------------------------ algorithmic bytes (§8(d))

def algorithmic_bytes(kernel: str, C: int, N: int, P: int, I: int, I_eff: int, p: int, rows: int | None = None,
                      fwd_walks: float = 1.0) -> float:
    """Per-launch algorithmic bytes, SURVEY.md §8(d) per-unit figures x the units one launch
    processes: C cameras (units) x N Gaussians projected, P pixels, I intersections, I_eff
    list entries read by the raster.  rows: the (unit, Gaussian) reduced gradient rows the
    backward passes on when fewer than C (2D with several units per parameter set: one row per
    (set, Gaussian), k_raster2d_bwd_frame).  fwd_walks: how many units walk each list in the
    forward (2D shared lists: a set's units all render its first unit's list, while I_eff counts
    that list once)."""
    R = C if rows is None else rows
    if kernel.startswith("raster") and kernel.endswith("_fwd"):
        return 40.0 * I_eff * fwd_walks + 20.0 * P     # read id+xy+conic+opac+colour; write rgb+alpha+last
    if kernel.startswith("raster") and kernel.endswith("_bwd"):
        return 24.0 * P + 40.0 * I_eff + 36.0 * R * N  # cotangents+alpha+last; list; reduced grads
    if kernel.startswith("project") and kernel.endswith("_fwd"):
        return C * N * (4.0 * p + 32.0)
    if kernel.startswith("project") and kernel.endswith("_bwd"):
        return N * (36.0 * R + (32.0 + 8.0 * p) * C)
    if kernel == "bin_sort":
        return 36.0 * I
    return 0.0


def step_bytes(C: int, N: int, P: int, I: int, I_eff: int, p: int, backward: bool = True, sets: int | None = None,
               rows: int | None = None, fwd_walks: float = 1.0) -> float:
    """Whole launch sequence, SURVEY.md §8(d) (P = all pixels of the C units):
    fwd+bwd C*N*(12p+136) + 36*I + 80*I_eff + 44*P; fwd-only C*N*(4p+32) + 36*I + 40*I_eff + 20*P.
    sets: the projections the sequence runs when fewer than C (2D: one per parameter set, the
    frames of the units -- VERDICT r4: config 4 charged its 8 frames' projection 48 times).  The
    per-projection part (params read, record written, params read again, gradient written:
    N*(12p+64)) is then charged `sets` times; the reduced rows (72 B per (unit, Gaussian): written
    by the raster backward, read by the projection backward) `rows` times (default C; 2D with
    several units per set: one per (set, Gaussian), the rows k_raster2d_bwd_frame passes on)."""
    S = C if sets is None else sets
    R = C if rows is None else rows
    if not backward:
        return S * N * (4.0 * p + 32.0) + 36.0 * I + 40.0 * I_eff * fwd_walks + 20.0 * P
    return S * N * (12.0 * p + 64.0) + R * N * 72.0 + 36.0 * I + 40.0 * I_eff * (fwd_walks + 1.0) + 44.0 * P


# libgsr call name (render.py timing brackets) -> substring of its dominant kernel's symbol
KERNEL_SYMBOL = {"raster3d_bwd": "k_raster_bwd", "raster3d_fwd": "k_raster_fwd<false,",
                 "raster2d_bwd": "k_raster2d_bwd_", "raster2d_fwd": "k_raster2d_fwd_pair",
                 "bin_sort": "k_segsort", "project3d_fwd": "k_project3d_fwd", "project3d_bwd": "k_project3d_bwd",
                 "project2d_fwd": "k_project2d_fwd", "project2d_bwd": "k_project2d_bwd", "bin_emit": "k_emit"}


# ------------------------------------------------------------------ PMC passes of THIS config

def pmc_files(config: int, kind: str, pmc_dir: str = PROFILES):
    """Newest round's committed PMC pass(es) of `config`: kind 'traffic' ->
    rNN_pmc_traffic_cfgC.csv; 'sq' -> [rNN_pmc_sq_cfgC_p1.csv, ..._p2.csv].  None if absent:
    no other config's counters are ever substituted."""
    pat = {"traffic": f"r*_pmc_traffic_cfg{config}.csv", "sq": f"r*_pmc_sq_cfg{config}_p1.csv"}[kind]
    found = sorted(glob.glob(os.path.join(pmc_dir, pat)),
                   key=lambda f: int(re.match(r"r(\d+)_", os.path.basename(f)).group(1)))
    if not found:
        return None
    if kind == "traffic":
        return found[-1]
    p1 = found[-1]
    p2 = p1.replace("_p1.csv", "_p2.csv")
    return [p1, p2] if os.path.exists(p2) else None


def traffic_from_csv(path: str, kernel_substr: str):
    """HBM bytes per launch from a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass (KB units;
    FETCH_SIZE doubled per the gfx950 correction in MI355X_MICROARCH.md §HBM, calibrated there
    for 16-B/lane streaming reads.  tools/fetch_probe.hip calibrates this path's 48-B record
    gathers beyond the Infinity Cache (profiles/r02_fetch_probe_*): 1.30 requests per record,
    the 128-B lines a 16-B-aligned 48-B record touches (1.25) tallied at 64 B each, so the
    same x2 gives the line traffic there too -- a gathered record moves >= 128 B)."""
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
    """VALU use of one kernel from rocprofv3 SQ passes, in the cycle model of
    MI355X_MICROARCH.md: a wave64 VALU instruction occupies its SIMD (32 lanes) for 2 cycles,
    and the SQ_ACTIVE_INST_* counters count quad-cycles per wave.  SIMD-cycles = N_SIMDS x
    the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs).
      issue_frac  = SQ_INSTS_VALU x 2 / SIMD-cycles: the share of the SIMDs' VALU issue
                    capacity used (1.0 = VALU-issue-bound; transcendentals cost somewhat more);
      wave_active = SQ_ACTIVE_INST_VALU x 4 / SIMD-cycles: wave-cycles spent in VALU
                    instructions per SIMD-cycle (summed over the waves of a SIMD, so it
                    exceeds 1 when waves overlap -- not a utilisation).
    None when the passes are missing."""
    import csv
    if not paths:
        return None
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
    return {"issue_frac": 2.0 * mean["SQ_INSTS_VALU"] / simd_cycles,
            "wave_active": 4.0 * mean["SQ_ACTIVE_INST_VALU"] / simd_cycles,
            "insts_per_launch": mean["SQ_INSTS_VALU"],
            "source": [os.path.relpath(p, ROOT) for p in paths]}


# ------------------------------------------------------------------ CPU baseline and dPSNR

def cpu_quota() -> int:
    """CPUs of this process's cgroup CPU quota (cgroup v2 cpu.max), 0 if unlimited/unknown.
    The GPU box shows all 256 host CPUs to os.cpu_count() and sched affinity but allots each
    GPU job a 16-CPU quota; threads beyond the quota only queue."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        return 0 if q == "max" else max(1, math.ceil(int(q) / int(period)))
    except (OSError, ValueError):
        return 0


def cpu_threads(requested: int = 0) -> int:
    """Every CPU this process may run on -- sched affinity, capped by the cgroup quota -- unless told."""
    if requested > 0:
        return requested
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = cpu_quota()
    return min(n, q) if q else n


def log(msg: str) -> None:
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_model() -> str:
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def linear_fit(xs, ys):
    """Least squares y = a + b x; returns (a, b, R^2)."""
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    sxy = sum((x - mx) * (y - my) for x, y in zip(xs, ys))
    b = sxy / sxx
    a = my - b * mx
    ss_res = sum((y - (a + b * x)) ** 2 for x, y in zip(xs, ys))
    ss_tot = sum((y - my) ** 2 for y in ys)
    return a, b, 1.0 - ss_res / ss_tot if ss_tot > 0 else 1.0


def cpu_band_rows(cfg) -> tuple:
    """Tile rows of view 0 in the bounded CPU sample: all of them up to config 3; a central
    band of 8 tile rows for config 5 (a whole 1152x1024 view of 2M Gaussians is minutes)."""
    th = (cfg.height + 15) // 16
    if cfg.index == 5:
        return th // 2 - 4, th // 2 + 4
    return 0, th


def cpu_baseline(cfg, params, V, K, threads: int):
    """The oracle (CPU restatement of the reference semantics) on a bounded sample of the
    workload, timed on this host.  Returns (baseline dict, oracle view-0 rgb or None)."""
    from oracle.oracle3d import render3d as oracle_render3d
    from oracle.oracle2d import render2d_dense
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(cfg.seed + 1)
    out = {"unit": "frames/s", "cores": threads, "host_cpus": os.cpu_count(), "cgroup_cpu_quota": cpu_quota() or None,
           "kind": "port", "cpu": cpu_model()}
    if cfg.mode == "3d":
        y0, y1 = cpu_band_rows(cfg)
        th = (cfg.height + 15) // 16
        band = None if (y0, y1) == (0, th) else (y0, y1)
        t0 = time.perf_counter()
        p = params.detach().cpu().clone().requires_grad_(cfg.backward)
        rgb, alpha = oracle_render3d(p, V[:1].cpu(), K[:1].cpu(), cfg.width, cfg.height, torch.ones(3), band=band)
        if cfg.backward:
            vr = torch.randn(rgb.shape, generator=g)
            va = torch.randn(alpha.shape, generator=g)
            ((rgb * vr).sum() + (alpha * va).sum()).backward()
        dt = time.perf_counter() - t0
        frac = (y1 - y0) / th
        out.update(value=frac / dt, seconds=round(dt, 2),
                   sample=(f"view 0 of {cfg.views} of {cfg.name}" +
                           (f", tile rows {y0}-{y1} of {th} (value = row fraction / time)" if band else "") +
                           f", {'fwd+bwd' if cfg.backward else 'fwd'}, oracle/oracle3d.py"))
        return out, rgb.detach()
    # 2D: the dense reference algorithm (src/gaussian_renderer.py:336-427) costs a fixed amount
    # per Gaussian (every Gaussian touches every pixel) and keeps O(N*H*W) autograd state (~18 MB
    # per Gaussian at 576x512), so config 4's 500k Gaussians cannot be run whole.  fwd+bwd is
    # timed at five N, a line t = a + b N is fitted (points and residuals in the line), and the
    # value is 1 / (a + b * 500k): an extrapolation by 500k / max(N) (stated).  The forward alone
    # (no autograd state) is timed at a larger N as a check on the per-Gaussian cost.
    ns = [128, 256, 512, 1024, 1536]
    ts = []
    for n in ns:
        t0 = time.perf_counter()
        p = params[:n].detach().cpu().clone().requires_grad_(True)
        rgb, alpha = render2d_dense(p, cfg.width, cfg.height, torch.ones(3))
        ((rgb * torch.randn(rgb.shape, generator=g)).sum() + (alpha * torch.randn(alpha.shape, generator=g)).sum()
         ).backward()
        ts.append(time.perf_counter() - t0)
        del rgb, alpha, p
    a, b, r2 = linear_fit(ns, ts)
    resid = [t - (a + b * n) for n, t in zip(ns, ts)]
    n_fwd = 4096
    t0 = time.perf_counter()
    with torch.no_grad():
        render2d_dense(params[:n_fwd].detach().cpu(), cfg.width, cfg.height, torch.ones(3))
    t_fwd = time.perf_counter() - t0
    t_full = a + b * cfg.N
    out.update(value=1.0 / t_full, seconds=round(sum(ts) + t_fwd, 2),
               sample=f"one frame-view of {cfg.name}: dense reference algorithm (oracle2d.render2d_dense) fwd+bwd "
                      f"timed at N={ns}, fit t = a + b N, extrapolated {cfg.N / max(ns):.0f}x to N={cfg.N}",
               fit={"N": ns, "seconds": [round(t, 4) for t in ts], "residual_s": [round(r, 4) for r in resid],
                    "a_s": a, "b_s_per_gaussian": b, "r2": r2, "t_full_s": t_full,
                    "extrapolation_factor": cfg.N / max(ns),
                    "fwd_only": {"N": n_fwd, "seconds": round(t_fwd, 3), "s_per_gaussian": t_fwd / n_fwd}})
    return out, None


def psnr(pred_hw3: torch.Tensor, gt_hw3: torch.Tensor) -> float:
    """scripts/utils/evaluate_model.py:240-243 (get_psnr, data_range 1) on [3,H,W] images."""
    pred = pred_hw3.double().permute(2, 0, 1)[None]
    gt = gt_hw3.double().permute(2, 0, 1)[None]
    mse = ((pred - gt) ** 2).mean(dim=(-3, -2, -1))
    return float(10 * torch.log10(1.0 / mse))


def delta_psnr(cfg, params_cpu, V, K, dev, rgb_oracle_view0=None):
    """target = the oracle render of a perturbed copy (means + N(0,0.002),
    colours + N(0,0.05)); dPSNR = |PSNR(gsr, target) - PSNR(oracle, target)|.  3D: view 0 (the
    CPU baseline's band for config 5); 2D: a 16x128 window of frame 0 at full density (the
    dense oracle is O(N) per pixel, so it runs over the Gaussians that can reach the window)."""
    from gsr import render as R
    from oracle.oracle2d import render2d_dense
    from oracle.oracle3d import render3d as oracle_render3d
    g = torch.Generator().manual_seed(cfg.seed + 7)
    with torch.no_grad():
        if cfg.mode == "3d":
            y0, y1 = cpu_band_rows(cfg)
            th = (cfg.height + 15) // 16
            band = None if (y0, y1) == (0, th) else (y0, y1)
            pt = params_cpu.clone()
            pt[:, 0:3] += 0.002 * torch.randn(pt.shape[0], 3, generator=g)
            pt[:, 10:13] += 0.05 * torch.randn(pt.shape[0], 3, generator=g)
            target, _ = oracle_render3d(pt, V[:1], K[:1], cfg.width, cfg.height, torch.ones(3), band=band)
            if rgb_oracle_view0 is None:
                rgb_oracle_view0, _ = oracle_render3d(params_cpu, V[:1], K[:1], cfg.width, cfg.height,
                                                      torch.ones(3), band=band)
            opts = R.RenderOptions3D(band=band) if band else R.RenderOptions3D()
            rgb_gpu, _ = R.render3d(params_cpu.to(dev), V[:1].to(dev), K[:1].to(dev), cfg.width, cfg.height,
                                    torch.ones(3, device=dev), opts)
            rows = slice(16 * y0, min(cfg.height, 16 * y1))
            a, b, t = rgb_gpu[0].cpu()[rows], rgb_oracle_view0[0][rows], target[0][rows]
            sample = f"view 0" + (f", pixel rows {rows.start}-{rows.stop}" if band else "")
        else:
            # the full-density frame (all N Gaussians) in the 16x128 window that
            # tests/test_cfg4_window_vs_oracle checks: the dense reference compositor over every
            # Gaussian that can reach the window (e^-40 * opacity bound), the GPU's full render cropped
            y0, x0 = 240, 192
            y1, x1 = y0 + 16, x0 + 128
            p = params_cpu
            s_max = torch.exp(p[:, 2:4]).amax(1)
            dx = (x0 - p[:, 0]).clamp_min(0) + (p[:, 0] - (x1 - 1)).clamp_min(0)
            dy = (y0 - p[:, 1]).clamp_min(0) + (p[:, 1] - (y1 - 1)).clamp_min(0)
            idx = torch.nonzero((dx * dx + dy * dy) / (2 * s_max * s_max + 1e-8) < 40.0)[:, 0]
            q = p[idx].clone()
            q[:, 0] -= x0
            q[:, 1] -= y0
            qt = q.clone()
            qt[:, 0:2] += 0.002 * torch.randn(q.shape[0], 2, generator=g)
            qt[:, 5:8] += 0.05 * torch.randn(q.shape[0], 3, generator=g)
            nt = torch.get_num_threads()
            torch.set_num_threads(1)   # ~10k tiny per-Gaussian steps: op overhead, not FLOPs
            try:
                t, _ = render2d_dense(qt, x1 - x0, y1 - y0, torch.ones(3))
                b, _ = render2d_dense(q, x1 - x0, y1 - y0, torch.ones(3))
            finally:
                torch.set_num_threads(nt)
            a, _ = R.render2d(params_cpu.to(dev), cfg.width, cfg.height, torch.ones(3, device=dev))
            a = a.cpu()[y0:y1, x0:x1]
            sample = (f"frame 0 at full density ({params_cpu.shape[0]} Gaussians), window rows {y0}-{y1} "
                      f"cols {x0}-{x1} (tests/test_fullsize_gpu.py::test_cfg4_window_vs_oracle); oracle over the "
                      f"{idx.numel()} Gaussians that can reach it")
    pg, po = psnr(a, t), psnr(b, t)
    return {"dpsnr_db": abs(pg - po), "psnr_gsr_db": pg, "psnr_oracle_db": po, "sample": sample,
            "target": "oracle render of means+N(0,0.002), colours+N(0,0.05)",
            "formula": "scripts/utils/evaluate_model.py:240-243"}


# ------------------------------------------------------------------ workloads

def _torch_ssim(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """The reference's SSIM term as plain torch ops (torchmetrics' algorithm: 11-tap Gaussian,
    sigma 1.5, reflect pad + crop, data_range 1.0) -- the `--loss torch` comparison only."""
    import torch.nn.functional as F
    dist = torch.arange(-5.0, 6.0, 1.0, device=x.device)
    g = torch.exp(-torch.pow(dist / 1.5, 2) / 2)
    g = g / g.sum()
    C = x.shape[1]
    kern = torch.matmul(g[:, None], g[None, :]).expand(C, 1, 11, 11)
    p, t = F.pad(x, (5, 5, 5, 5), mode="reflect"), F.pad(y, (5, 5, 5, 5), mode="reflect")
    mp, mt, pp, tt, pt = F.conv2d(torch.cat((p, t, p * p, t * t, p * t)), kern, groups=C).split(x.shape[0])
    full = ((2 * mp * mt + 1e-4) * (2 * (pt - mp * mt) + 9e-4)) / ((mp * mp + mt * mt + 1e-4) *
                                                                  (pp - mp * mp + tt - mt * mt + 9e-4))
    return full[..., 5:-5, 5:-5].reshape(x.shape[0], -1).mean(-1).mean()


class Workload:
    """One rank's share of a config's step.  step() enqueues one step; `units` is the number of
    rendered views (frames) the WHOLE job completes per step; views_here the ones this rank
    renders; launch_C / launch_P the cameras / pixels of the dominant launch sequence."""

    def __init__(self, cfg, dev, world: int, rank: int, shard: str, buckets: int, loss: str, comm: bool,
                 view_cost: float = 0.3, exchange: str = "dense"):
        from gsr import render as R
        from gsr.scenes import gaussians2d, gaussians3d, ring_cameras
        self.R, self.cfg, self.dev, self.world, self.rank = R, cfg, dev, world, rank
        self.view_cost = view_cost * cfg.N   # in list entries (the row weights' unit)
        self.exchange = exchange
        self.comm = comm and world > 1
        C = cfg.views
        g = torch.Generator().manual_seed(cfg.seed + 1)
        self.bg = torch.ones(3, device=dev)
        self.loss = loss
        self.split = 1
        if cfg.mode == "2d":
            F = FRAMES_2D
            self.params_cpu = torch.stack([gaussians2d(cfg.N, cfg.width, cfg.height, cfg.seed + f) for f in range(F)])
            self.V, self.K = ring_cameras(1, cfg.width, cfg.height)
            self.p_dim = 9
            from gsr.multiview import frame_owner_units, frame_view_units
            self.owned = shard == "frames"
            self.units = (frame_owner_units if self.owned else frame_view_units)(F, C, world, rank)
            self.buckets = buckets or (1 if world == 1 or self.owned else 2)
            idx = [f * C + v for f, v in self.units]
            vr = torch.randn(F * C, cfg.height, cfg.width, 3, generator=g)
            va = torch.randn(F * C, cfg.height, cfg.width, generator=g)
            self.v_rgb, self.v_alpha = vr[idx].to(dev), va[idx].to(dev)
            self.units_total = F * C
            self.views_here = len(self.units)
            self.scaling = "strong"
            if world == 1:
                self.layout = f"{F} frames x {C} views batched in one launch sequence"
            elif self.owned:
                self.layout = (f"frame owners: frame f with its {C} views on rank f % {world}, batched in one launch "
                               "sequence; no Gaussian-gradient exchange (disjoint frame sets); the network weight all-reduce "
                               "that frame-parallel training adds is outside the rasterizer and not counted")
            else:
                self.layout = (f"(frame, view) units round-robin over {world} rank(s), batched per frame bucket "
                               f"({self.buckets}), async all-reduce of the [8,N,9] gradient per bucket")
        else:
            self.params_cpu = gaussians3d(cfg.N, cfg.seed)
            self.p_dim = 14
            self.buckets = buckets or (1 if world == 1 else 4)
            th = (cfg.height + 15) // 16
            self.th = th
            if cfg.index == 2 or shard == "views" or world == 1:
                # weak (config 2: replicas of its one fwd-only view; --shard views): every rank
                # renders C views of its own, ring offset per rank
                self.V, self.K = ring_cameras(C, cfg.width, cfg.height, azimuth0=2.0 * math.pi * rank / (C * world))
                self.units_total = C * world
                self.views_here = C
                self.band = (0, -1)
                self.scaling = "weak" if world > 1 else "n/a"
                self.layout = ("single GPU" if world == 1 else
                               f"replicas x{world}" if cfg.index == 2 else
                               f"multi-camera batch: each of {world} ranks renders {C} views of its own, "
                               f"{self.buckets} async all-reduce bucket(s) of the [N,14] gradient overlapping "
                               "project_bwd")
                self.v0, self.v1 = 0, C
            else:
                self.V, self.K = ring_cameras(C, cfg.width, cfg.height)
                self.units_total = C
                self.scaling = "strong"
                self.weights = None
                self.layout = None   # set by balance()
            vr = torch.randn(C, cfg.height, cfg.width, 3, generator=g)
            va = torch.randn(C, cfg.height, cfg.width, generator=g)
            self.v_rgb_all, self.v_alpha_all = vr.to(dev), va.to(dev)
        self.params = self.params_cpu.to(dev).requires_grad_(True)
        self.Vd, self.Kd = self.V.to(dev), self.K.to(dev)
        if cfg.mode == "3d" and self.scaling == "strong":
            self.balance()

    def balance(self, weights=None):
        """(view, row) share of this rank, balanced by per-row list lengths of a full render."""
        from gsr.multiview import unit_shard
        cfg, R = self.cfg, self.R
        if weights is None:
            with torch.no_grad():
                R.render3d(self.params, self.Vd, self.Kd, cfg.width, cfg.height, self.bg)
            tw = (cfg.width + 15) // 16
            weights = [float(x) for x in R.tile_work().reshape(cfg.views * self.th, tw).sum(1).cpu()]
        self.weights = weights
        self.v0, self.v1, self.band = unit_shard(cfg.views, self.th, self.world, self.rank, weights, self.view_cost)
        self.views_here = self.v1 - self.v0
        self.layout = (f"(view, tile-row) units: rank {self.rank} views {self.v0}-{self.v1 - 1} rows {self.band} "
                       f"of {cfg.views}x{self.th}, " +
                       (f"{self.buckets} all-reduce bucket(s) overlapping project_bwd" if self.exchange == "dense" else
                        "device sparse exchange: touched gradient rows in a fixed-capacity block, all-gathered, "
                        "summed in rank order" if self.exchange == "rows" else
                        "sparse exchange of the touched gradient rows (all-gather)"))
        if self.exchange == "rows":
            self._setup_rows()

    def _render_band_rows(self, p, Vs, Ks, band, gr):
        cfg, R = self.cfg, self.R
        return R.render3d(p, Vs, Ks, cfg.width, cfg.height, self.bg, R.RenderOptions3D(band=band, grad_rows=gr))

    def _setup_rows(self):
        """Row-block capacity of the device sparse exchange: this share's touched rows, measured
        once with a block that holds every Gaussian, maximised over the ranks (+25 %)."""
        from gsr.multiview import GradRows, rows_capacity
        touched = 0
        if self.v1 > self.v0:
            probe = GradRows(self.cfg.N, self.dev)
            p = self.params.detach().requires_grad_(True)
            rgb, alpha = self._render_band_rows(p, self.Vd[self.v0:self.v1], self.Kd[self.v0:self.v1], self.band, probe)
            torch.autograd.backward([rgb, alpha], [self.v_rgb_all[self.v0:self.v1], self.v_alpha_all[self.v0:self.v1]])
            touched = probe.count()
            del probe
        self.touched = touched
        self.grad_rows = GradRows(rows_capacity(touched), self.dev)
        # --rank-share (no collectives): the scatter-add runs over `world` copies of this block
        self._gathered = None

    def step(self):
        cfg, R = self.cfg, self.R
        self.params.grad = None
        if cfg.mode == "2d":
            from gsr.multiview import owned_backward_frames, sharded_backward_frames

            def render_units(p, sets):
                return R.render2d_units(p, sets, cfg.width, cfg.height, self.bg)
            if self.comm and self.owned:
                self.params.grad = owned_backward_frames(render_units, self.params, self.units, self.v_rgb,
                                                         self.v_alpha)
            elif self.comm:
                self.params.grad = sharded_backward_frames(render_units, self.params, self.units, self.v_rgb,
                                                           self.v_alpha, self.buckets)
            elif self.units:
                # one rank's share without collectives (single GPU, --rank-share)
                sets = [f for f, _ in self.units]
                rgb, alpha = render_units(self.params, sets)
                torch.autograd.backward([rgb, alpha], [self.v_rgb, self.v_alpha])
            return
        if not cfg.backward:
            with torch.no_grad():   # config 2 is forward-only
                R.render3d(self.params, self.Vd, self.Kd, cfg.width, cfg.height, self.bg)
            return
        if self.loss != "none":
            self._loss_step()
            return
        if self.scaling == "strong" and self.exchange == "rows":
            self._rows_step()
            return
        if self.v1 <= self.v0:
            if self.comm:
                from gsr.multiview import sharded_backward_units
                self.params.grad = sharded_backward_units(None, self.params, self.Vd, self.Kd, self.v_rgb_all,
                                                          self.v_alpha_all, self.th, self.weights, self.buckets,
                                                          view_cost=self.view_cost, exchange=self.exchange)
            return
        if self.comm and self.scaling == "strong":
            from gsr.multiview import sharded_backward_units

            def render_band(p, Vs, Ks, band, hook):
                opts = R.RenderOptions3D(band=band, grad_buckets=self.buckets if hook else 1, grad_hook=hook)
                return R.render3d(p, Vs, Ks, cfg.width, cfg.height, self.bg, opts)
            self.params.grad = sharded_backward_units(render_band, self.params, self.Vd, self.Kd, self.v_rgb_all,
                                                      self.v_alpha_all, self.th, self.weights, self.buckets,
                                                      view_cost=self.view_cost, exchange=self.exchange)
            return
        if self.comm:
            # --shard views: every rank renders its own C views; the gradient is all-reduced in
            # Gaussian-range buckets, each launched as soon as the projection backward has
            # enqueued it (async RCCL), overlapping the rest of the backward
            import torch.distributed as dist
            works, pieces = [], []

            def hook(t):
                pieces.append(t)
                works.append(dist.all_reduce(t, async_op=True))
            opts = R.RenderOptions3D(grad_buckets=self.buckets, grad_hook=hook)
            p = self.params.detach().requires_grad_(True)
            rgb, alpha = R.render3d(p, self.Vd, self.Kd, cfg.width, cfg.height, self.bg, opts)
            torch.autograd.backward([rgb, alpha], [self.v_rgb_all, self.v_alpha_all])
            for wk in works:
                wk.wait()
            # the buckets are slices of the one v_params tensor the backward returned
            full = pieces[0]._base if pieces[0]._base is not None else pieces[0]
            self.params.grad = full.view_as(self.params)
            return
        if self.split > 1 and self.band == (0, -1):
            self._split_step()
            return
        opts = R.RenderOptions3D(band=self.band) if self.band != (0, -1) else R.RenderOptions3D()
        rgb, alpha = R.render3d(self.params, self.Vd[self.v0:self.v1], self.Kd[self.v0:self.v1], cfg.width,
                                cfg.height, self.bg, opts)
        torch.autograd.backward([rgb, alpha], [self.v_rgb_all[self.v0:self.v1], self.v_alpha_all[self.v0:self.v1]])

    def _rows_step(self):
        """Strong layout with the device sparse exchange (gsr.multiview.rows_backward_units).
        Without collectives (--rank-share) the share's own work is timed: its render + backward
        into the row block, then the zero-fill + rank-ordered scatter-add over `world` blocks of
        this block's size (the gathered blocks stand in for the all-gather's output)."""
        from gsr import _lib
        from gsr.multiview import rows_backward_units
        if self.comm:
            self.params.grad = rows_backward_units(self._render_band_rows, self.params, self.Vd, self.Kd,
                                                   self.v_rgb_all, self.v_alpha_all, self.th, self.grad_rows,
                                                   self.weights, view_cost=self.view_cost,
                                                   status=self.R._status_buf(self.dev),
                                                   reuse_output=True)   # (consumed before the next step)
            return
        if self.v1 > self.v0:
            p = self.params.detach().requires_grad_(True)
            rgb, alpha = self._render_band_rows(p, self.Vd[self.v0:self.v1], self.Kd[self.v0:self.v1], self.band,
                                                self.grad_rows)
            torch.autograd.backward([rgb, alpha], [self.v_rgb_all[self.v0:self.v1], self.v_alpha_all[self.v0:self.v1]])
        if self._gathered is None:
            self._gathered = self.grad_rows.block[None].repeat(self.world, 1, 1)
        self._gathered[0].copy_(self.grad_rows.block)
        out = torch.zeros(self.cfg.N, 14, device=self.dev)
        L = _lib.lib()
        _lib.check(L.gsr_rows_scatter_add(self._gathered.data_ptr(), self.world, self.grad_rows.cap, out.data_ptr(),
                                          self.cfg.N, None, torch.cuda.current_stream(self.dev).cuda_stream),
                   "gsr_rows_scatter_add")
        self.params.grad = out

    def _split_step(self):
        """--split G: the views in G groups, each group's fwd+bwd on its own stream; the groups'
        gradients are summed on the step's stream after the join."""
        cfg, R = self.cfg, self.R
        n = self.v1 - self.v0
        G = min(self.split, n)
        if not hasattr(self, "_streams"):
            self._streams = [torch.cuda.Stream(self.dev) for _ in range(G)]
        cur = torch.cuda.current_stream(self.dev)
        grads = []
        for gi in range(G):
            a = self.v0 + n * gi // G
            b = self.v0 + n * (gi + 1) // G
            st = self._streams[gi]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                p = self.params.detach().requires_grad_(True)
                rgb, alpha = R.render3d(p, self.Vd[a:b], self.Kd[a:b], cfg.width, cfg.height, self.bg,
                                        R.RenderOptions3D(tag=gi))
                torch.autograd.backward([rgb, alpha], [self.v_rgb_all[a:b], self.v_alpha_all[a:b]])
                grads.append(p.grad)
        for st in self._streams[:G]:
            cur.wait_stream(st)
        if not torch.cuda.is_current_stream_capturing():   # (a capture's pool is private to the graph)
            for g in grads:
                g.record_stream(cur)
        tot = grads[0]
        for g in grads[1:]:
            tot = tot + g
        self.params.grad = tot

    def _loss_step(self):
        """The reference training loss on the render: IoU + L1 image + ssim_lambda * (1 - SSIM)
        (scripts/training/train_script.py:127-133), fused (libgsr kernels) or as torch ops."""
        cfg, R = self.cfg, self.R
        if not hasattr(self, "timg"):
            g3 = torch.Generator().manual_seed(cfg.seed + 3)
            self.timg = torch.rand(cfg.views, 3, cfg.height, cfg.width, generator=g3).to(self.dev)
            self.tmask = (torch.rand(cfg.views, cfg.height, cfg.width, generator=g3) < 0.3).float().to(self.dev)
        ssim_lambda = 1.0
        if self.loss == "fused":
            from gsr.loss import render3d_iou_l1, ssim
            li, lm, rgb, alpha = render3d_iou_l1(self.params, self.Vd, self.Kd, cfg.width, cfg.height, self.bg,
                                                 self.timg, self.tmask, 1.0)
            ls = ssim_lambda * (1 - ssim(self.timg, rgb))
        else:
            rgb, alpha = R.render3d(self.params, self.Vd, self.Kd, cfg.width, cfg.height, self.bg)
            inter = (alpha * self.tmask).sum(dim=(-2, -1))
            union = (alpha + self.tmask - alpha * self.tmask).sum(dim=(-2, -1))
            li = 1 - ((inter + 1e-6) / (union + 1e-6)).mean()
            lm = torch.abs(self.timg - rgb.permute(0, 3, 1, 2)).sum() / self.tmask.sum()
            ls = ssim_lambda * (1 - _torch_ssim(self.timg, rgb.permute(0, 3, 1, 2)))
        (li + lm + ls).backward()

    def sets_per_launch(self, C: int):
        """Projections one launch sequence runs: 3D one per camera (C); 2D one per parameter set
        (the frames among this rank's units, split over its buckets)."""
        if self.cfg.mode != "2d":
            return C
        frames = len({f for f, _ in self.units})
        nb = self.buckets if self.comm else 1
        return max(1, math.ceil(frames / max(nb, 1)))

    def rows_per_launch(self, C: int):
        """Reduced gradient rows one launch's backward passes on: one per (unit, Gaussian), except
        2D with more units than parameter sets in the launch, whose backward walks each set once
        for all its units and writes one row per (set, Gaussian) (libgsr rows2d_per_set)."""
        if self.cfg.mode != "2d":
            return C
        F = int(self.params_cpu.shape[0])
        return self.sets_per_launch(C) if C > F else C

    def fwd_walks(self, C: int) -> float:
        """Units walking each list in the forward: 2D with more units than sets binds only each
        set's first unit and all its units render that list (libgsr lists2d_per_set), so the
        list entries I_eff counts are walked units / sets times; else 1."""
        r = self.rows_per_launch(C)
        return C / r if r < C else 1.0

    def launch_shape(self):
        """(C, P) of the dominant launch sequence: cameras and pixels one launch covers."""
        cfg = self.cfg
        if cfg.mode == "2d":
            per_bucket = max(1, math.ceil(self.views_here / self.buckets)) if self.comm else self.views_here
            C = max(per_bucket, 1)
            return C, C * cfg.width * cfg.height
        if self.scaling == "strong" and self.world > 1 or getattr(self, "band", (0, -1)) != (0, -1):
            rows = self.band[1] - self.band[0]
            return self.views_here, min(rows * 16 * cfg.width, self.views_here * cfg.width * cfg.height)
        if self.split > 1:   # one launch covers one view group (the last group's stats)
            c = self.views_here - self.views_here * (self.split - 1) // self.split
            return c, c * cfg.width * cfg.height
        return self.views_here, self.views_here * cfg.width * cfg.height


def time_steps(w: Workload, steps: int, warmup: int, dist=None, graph: bool = False):
    """Warm up, name the dominant kernel in a separately profiled pass, then time exactly
    `steps` steps between barrier + synchronize brackets with HIP events around the dominant
    kernel only.  graph: the `steps` steps are captured as ONE HIP graph beforehand (external
    timing events around the dominant kernel of each step become nodes of the graph) and the
    timed region replays it once.  Returns (elapsed_s, breakdown, dom_name, dom (avg_ms,
    launches))."""
    R = w.R
    for _ in range(warmup):
        w.step()
    torch.cuda.synchronize()
    R.enable_kernel_timing(True)
    for _ in range(max(2, min(steps, 5))):
        w.step()
    breakdown = R.kernel_times_ms()
    R.enable_kernel_timing(False)
    dom_name = max(breakdown.items(), key=lambda kv: kv[1][0] * kv[1][1])[0] if breakdown else None
    torch.cuda.synchronize()
    g = None
    if graph:
        # torch's capture rules: warm up on a side stream, then capture on the graph's stream
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                w.step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                w.step()
        torch.cuda.synchronize()
        # one untimed replay first: a graph's first launch also uploads it (its kernel nodes'
        # arguments and resources), a fixed cost the 20-step driver run saw as graph-timed steps
        # slower than the same steps launched eagerly
        g.replay()
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    if g is None:
        R.enable_kernel_timing(True, only={dom_name} if dom_name else None)
    t0 = time.perf_counter()
    if g is not None:
        g.replay()
    else:
        for _ in range(steps):
            w.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if g is not None:
        # ROCm rejects timing events inside a captured graph ("External events are disallowed
        # in rocm"): the dominant kernel is timed with HIP events around each of its launches
        # on its stream over the same number of eager bounded steps (no host sync between
        # them), right after the graph-timed region -- the same kernel on the same inputs
        # Each step starts behind a short GPU spin (torch.cuda._sleep, ~1 ms) so that the host has
        # queued the whole step before the GPU reaches it: without it, a launch whose Python-side
        # preparation outlasts the GPU's queue (the backward after autograd's bookkeeping) is timed
        # from its start event across the host gap (config 3: 124 vs 113.6 us by rocprof).
        R.enable_kernel_timing(True, only={dom_name} if dom_name else None)
        for _ in range(steps):
            torch.cuda._sleep(KTIMING_SPIN_CYCLES)
            w.step()
        torch.cuda.synchronize()
    ktimes = R.kernel_times_ms()
    R.enable_kernel_timing(False)
    R.check_overflow(w.dev)   # a bounded step over its bounds would have rendered NaN: fail loudly
    del g
    return elapsed, breakdown, dom_name, ktimes.get(dom_name, (0.0, 0)) if dom_name else (0.0, 0)


KTIMING_SPIN_CYCLES = 2_000_000   # GPU clock cycles spun before each kernel-timing step


def time_eager(w, steps: int, dist=None) -> float:
    """`steps` eager steps of the already warmed-up workload between barrier + synchronize
    brackets (the slowest rank's time, via the caller's max over ranks)."""
    dev = getattr(w, "dev", "cpu")
    if dist is not None:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        w.step()
    _sync(dev)
    if dist is not None:
        dist.barrier()
    _sync(dev)
    return time.perf_counter() - t0


def headline_timing(w, args, dist, dev, world: int, timer=None, eager_timer=None):
    """The headline line's timing: `args.steps` steps in the run's launch mode (one HIP graph
    of the timed steps at N=1 by default, eager launches at N>1, where the step's collectives
    are not captured), max over ranks.  A graph-timed line ALSO times the same number of eager
    steps right after, so the 1 -> N scaling curve can be read eager to eager (`value_eager`;
    VERDICT r4 item 5): every line states its `launch_mode`."""
    timer = timer or time_steps
    eager_timer = eager_timer or time_eager
    graph = bool(args.graph)
    elapsed, breakdown, dom_name, dom = timer(w, args.steps, args.warmup, dist, graph=graph)
    el_eager = eager_timer(w, args.steps, dist) if graph else elapsed
    if world > 1:
        t = torch.tensor([elapsed, el_eager], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, el_eager = (float(x) for x in t)
    units = w.units_total * args.steps
    timing = {"value": units / elapsed, "ms_per_step": 1000.0 * elapsed / args.steps,
              "launch_mode": "graph" if graph else "eager",
              "value_eager": units / el_eager, "ms_per_step_eager": 1000.0 * el_eager / args.steps}
    return timing, elapsed, breakdown, dom_name, dom


def allreduce_ms(nbytes: int, world: int) -> float:
    """Ring all-reduce cost model over xGMI: 2(n-1)/n * S per GPU at one link's bandwidth
    (a conservative bound: RCCL spreads rings over the 7 links of each MI355X)."""
    if world <= 1:
        return 0.0
    return 2.0 * (world - 1) / world * nbytes / (XGMI_LINK_GBS * 1e9) * 1e3


def roofline(w: Workload, dom_name, dom, args):
    R, cfg = w.R, w.cfg
    st = R.last_stats()
    I, I_eff = st.get("n_isect", 0), R.effective_isect()
    C, P = w.launch_shape()
    dom_ms, dom_n = dom
    alg = algorithmic_bytes(dom_name or "", C, cfg.N, P, I, I_eff, w.p_dim, rows=w.rows_per_launch(C),
                            fwd_walks=w.fwd_walks(C))
    achieved = alg / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    sym = KERNEL_SYMBOL.get(dom_name, "k_" + str(dom_name))
    tfile = pmc_files(cfg.index, "traffic", args.pmc_dir) if dom_name else None
    sq = pmc_files(cfg.index, "sq", args.pmc_dir) if dom_name else None
    traffic = traffic_from_csv(tfile, sym) if tfile else None
    valu = valu_from_csv(sq, sym) if sq else None
    if valu is not None and dom_ms > 0:
        # the kernel's VALU floor: its wave64 VALU instructions (PMC) at 2 cycles each on the
        # 1 024 SIMDs at the 2.4 GHz maximum clock -- the bound of a VALU-issue-bound kernel
        # (config 4's 2D forward: 67 % issue), next to the HBM fraction
        floor_ms = 2.0 * valu["insts_per_launch"] / (N_SIMDS * CLOCK_GHZ * 1e9) * 1e3
        valu.update(floor_ms=floor_ms, frac_of_floor=floor_ms / dom_ms,
                    floor_model=f"SQ_INSTS_VALU x 2 cycles / ({N_SIMDS} SIMDs x {CLOCK_GHZ} GHz)")
    return {"bound": "hbm", "kernel": dom_name, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": os.path.relpath(tfile, ROOT) if traffic is not None else None,
            "algorithmic_bytes": alg, "avg_ms": dom_ms, "launches": dom_n,
            "timing": ("HIP events around each launch on its stream, over the timed steps" if not args.graph else
                       "HIP events around each launch on its stream, over as many eager bounded steps run right "
                       "after the graph-timed region (ROCm rejects timing events inside a captured graph), each "
                       "step queued behind a short GPU spin so no host gap falls inside a timed launch"),
            "valu": valu,
            "units_per_launch": {"C": C, "P": P, "N": cfg.N, "I": I, "I_eff": I_eff}}, (C, P, I, I_eff)


def _sync(dev) -> None:
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)


def measure_allreduce_ms(w, dist, dev, reps: int = 10):
    """The step's Gaussian-gradient collective on its own: `reps` x all_reduce of a buffer the
    size of the gradient the layout exchanges (max over ranks); None for a layout with no
    collective (2D frame owners).  HIP events on the stream on a GPU, wall clock otherwise."""
    if getattr(w, "owned", False):
        return None
    buf = torch.zeros_like(w.params)
    for _ in range(3):
        dist.all_reduce(buf)
    _sync(dev)
    dist.barrier()
    if torch.device(dev).type == "cuda":
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            dist.all_reduce(buf)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
    else:
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(buf)
        ms = 1000.0 * (time.perf_counter() - t0) / reps
    t = torch.tensor([ms], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def other_layouts(cfg, shard: str) -> list:
    """Multi-GPU layouts reported NEXT TO the default one in the same JSON line:
    3D fwd+bwd -- the weak multi-camera batch ('views') and the strong one-job split ('units')
    both; config 4 -- the round-robin (frame, view) units with their all-reduce and the frame
    owners with none.  Config 2 (one fwd-only view) has replicas only."""
    if cfg.mode == "3d" and cfg.backward and cfg.index != 2:
        return [x for x in ("views", "units") if x != shard]
    if cfg.mode == "2d":
        return [x for x in ("units", "frames") if x != shard]
    return []


LAYOUT_KEY = {"views": "weak", "units": "strong", "frames": "frame_owners"}


def measure_layout(cfg, args, dev, world, rank, shard, dist, make_workload=None, timer=None) -> dict:
    """One more layout of the same config on the same ranks, timed like the headline one
    (warmup, barrier-bracketed K steps, max over ranks): value = the units the whole job
    completes per second, plus its own collective timing."""
    make_workload = make_workload or Workload
    timer = timer or time_steps
    w = make_workload(cfg, dev, world, rank, shard, args.buckets, "none", comm=True, view_cost=args.view_cost,
                      exchange=args.exchange)
    elapsed = timer(w, args.steps, args.warmup, dist, graph=False)[0]
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t)
    out = {"value": w.units_total * args.steps / elapsed, "unit": "frames/s",
           "ms_per_step": 1000.0 * elapsed / args.steps, "scaling": w.scaling, "shard": shard,
           "units_per_step": w.units_total, "parallelism": w.layout,
           "launch": "eager launches", "launch_mode": "eager", "allreduce_ms": measure_allreduce_ms(w, dist, dev)}
    del w
    if torch.device(dev).type == "cuda":
        torch.cuda.empty_cache()
    return out


def rank_share_report(cfg, args, dev, n: int, weights=None):
    """--rank-share N: time each rank's share of the strong layout alone on this GPU."""
    from gsr import render as R
    shares = []
    for r in range(n):
        w = Workload(cfg, dev, n, r, args.shard if cfg.mode == "2d" else "units", args.buckets, "none", comm=False,
                     view_cost=args.view_cost, exchange=args.exchange)
        if cfg.mode == "3d" and w.scaling == "strong":
            if weights is None:
                weights = w.weights
            else:
                w.balance(weights)
        el, bd, dom_name, dom = time_steps(w, args.steps, args.warmup, graph=args.graph == 1)
        log(f"share {r}/{n}: {1000.0 * el / args.steps:.3f} ms/step ({w.layout})")
        kern = {k: round(v[0], 4) for k, v in sorted(bd.items())}
        kern_sum = sum(v[0] * v[1] for v in bd.values()) / max(2, min(args.steps, 5))   # per step (breakdown pass)
        touched = None   # Gaussians with a nonzero gradient row in this share (the sparse exchange's rows)
        if cfg.mode == "3d" and getattr(w, "grad_rows", None) is not None:
            touched = w.grad_rows.count() if w.v1 > w.v0 else 0
        elif cfg.mode == "3d" and w.params.grad is not None:
            touched = int(w.params.grad.ne(0).any(1).sum())
        shares.append({"rank": r, "ms_per_step": 1000.0 * el / args.steps, "views_here": w.views_here,
                       "layout": w.layout, "kernels_ms": kern, "kernel_sum_ms": kern_sum,
                       "I": R.last_stats().get("n_isect", 0), "touched_rows": touched,
                       "row_cap": w.grad_rows.cap if getattr(w, "grad_rows", None) is not None else None})
        del w
        torch.cuda.empty_cache()
    grad_bytes = cfg.N * (14 if cfg.mode == "3d" else 9) * 4 * (FRAMES_2D if cfg.mode == "2d" else 1)
    if cfg.mode == "2d" and args.shard == "frames":
        grad_bytes = 0   # frame owners: every frame's gradient is complete on its rank
    ar = allreduce_ms(grad_bytes, n)
    ar7 = ar / 7.0
    worst = max(s["ms_per_step"] for s in shares)
    units = cfg.views * (FRAMES_2D if cfg.mode == "2d" else 1)
    sparse = {}
    if cfg.mode == "3d" and all(s["touched_rows"] is not None for s in shares):
        # the sparse exchange: an all-gather of every rank's touched rows (index + 14 floats, 64 B),
        # padded to one size -- the longest list (sparse_sum) or the common row-block capacity
        # (the device "rows" exchange: the max over ranks of touched + 25 %) -- a ring moves
        # (n-1) of them through each rank's link
        kmax = max(s["touched_rows"] for s in shares)
        caps = [s["row_cap"] for s in shares if s.get("row_cap")]
        kpad = max(caps) + 1 if caps else kmax
        sp_bytes = (n - 1) * kpad * 64
        sp = sp_bytes / (XGMI_LINK_GBS * 1e9) * 1e3
        sparse = {"sparse_exchange": f"all-gather of the touched rows (max {kmax} of {cfg.N}, padded to {kpad}, "
                                     f"64 B each), {sp_bytes / 1e6:.1f} MB through one {XGMI_LINK_GBS:.0f} GB/s link",
                  "sparse_exchange_model_ms": sp, "sparse_exchange_7link_ms": sp / 7.0,
                  "projected_ms_per_step_sparse": worst + sp, "projected_value_sparse": units / ((worst + sp) * 1e-3),
                  "projected_ms_per_step_sparse_7link": worst + sp / 7.0,
                  "projected_value_sparse_7link": units / ((worst + sp / 7.0) * 1e-3)}
    return {"n": n, "shares": shares, "max_share_ms": worst, **sparse, "allreduce_model_ms": ar,
            "allreduce_model": f"ring 2(n-1)/n x {grad_bytes / 1e6:.1f} MB at {XGMI_LINK_GBS:.0f} GB/s (one link), "
                               "not overlapped (upper bound)",
            "allreduce_7link_ms": ar7,
            "projected_ms_per_step": worst + ar, "projected_value": units / ((worst + ar) * 1e-3),
            "projected_ms_per_step_7link": worst + ar7, "projected_value_7link": units / ((worst + ar7) * 1e-3),
            "view_cost": args.view_cost if cfg.mode == "3d" else None,
            "note": "each share timed alone on one GPU, no collectives; projected = max share + all-reduce model "
                    "(one link: upper bound; 7 links: the ring spread over all of a GPU's xGMI links)"}


def _spawn_ranks(args, argv) -> int:
    """`--gpus N` without a launcher: start N ranks (one process per GPU) with
    torch.distributed.run on 127.0.0.1 and return its exit code.  Runs before this process
    touches the GPU, and starts a child instead of exec-ing."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    cmd += list(sys.argv[1:] if argv is None else argv)
    log(f"--gpus {args.gpus} without a launcher: starting {args.gpus} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.call(cmd)


def main(argv=None):
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.rank_share:
        raise SystemExit(_spawn_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and not args.rank_share:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GSR_DIST_BACKEND=gloo + GSR_SAME_DEVICE=1 rehearse N ranks on a single GPU (box tests);
    # the driver's scaling runs use the defaults: backend "nccl" (RCCL), one GPU per rank.
    if os.environ.get("GSR_SAME_DEVICE") == "1":
        local = 0
    dist = None
    backend = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        backend = os.environ.get("GSR_DIST_BACKEND", "nccl")
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    from gsr import render as R
    from gsr import _lib
    from gsr.scenes import CONFIGS
    cfg = CONFIGS[args.config]
    R.set_capacity_mode(args.capacity)
    R.set_quadrant_masks(bool(args.masks))
    if args.chunk_entries:
        c3, c2 = (int(x) for x in args.chunk_entries.split(","))
        R.set_chunk_entries("3d", c3)
        R.set_chunk_entries("2d", c2)
    if args.graph == -1:
        args.graph = int(world == 1 and args.capacity == "bounded" and args.loss == "none")
    if args.graph and args.capacity != "bounded":
        raise SystemExit("--graph 1 needs --capacity bounded (an exact step waits on the host)")
    _lib.check(_lib.lib().gsr_set_fwd_lanes(args.fwd_lanes), "gsr_set_fwd_lanes")
    _lib.check(_lib.lib().gsr_set_bwd_layout(args.bwd_layout), "gsr_set_bwd_layout")
    if args.emit_staged >= 0:
        _lib.check(_lib.lib().gsr_set_emit_staged(args.emit_staged), "gsr_set_emit_staged")
    if args.lazy:
        mn, pf = (int(x) for x in args.lazy.split(","))
        _lib.check(_lib.lib().gsr_set_lazy_sort(mn, pf), "gsr_set_lazy_sort")

    if args.rank_share:
        if world > 1:
            raise SystemExit("--rank-share runs on ONE process")
        ns = [int(x) for x in args.rank_share.split(",")]
        reps = []
        one = None
        for n in ns:
            reps.append(rank_share_report(cfg, args, dev, n))
            log(f"N={n}: max share {reps[-1]['max_share_ms']:.3f} ms, projected {reps[-1]['projected_ms_per_step']:.3f} ms")
        print(json.dumps({"metric": "projected strong scaling (per-rank shares timed on one GPU)",
                          "config": {"workload": cfg.name, "capacity": args.capacity,
                                     "launch": "HIP graph per share" if args.graph else "eager"},
                          "rank_share": reps[0] if len(reps) == 1 else None,
                          "rank_shares": reps}), flush=True)
        return

    if args.loss != "none" and (cfg.mode != "3d" or world > 1):
        raise SystemExit("--loss: 3D configs on one GPU only")
    w = Workload(cfg, dev, world, rank, args.shard, args.buckets, args.loss, comm=True, view_cost=args.view_cost,
                 exchange=args.exchange)
    if args.split > 1:
        if world > 1 or cfg.mode != "3d" or not cfg.backward or args.loss != "none":
            raise SystemExit("--split: 3D fwd+bwd configs on one GPU, loss none")
        w.split = args.split
    timing, elapsed, breakdown, dom_name, dom = headline_timing(w, args, dist, dev, world)

    ar_ms = measure_allreduce_ms(w, dist, dev) if world > 1 else None
    value = timing["value"]
    ms_per_step = timing["ms_per_step"]
    roof, (C, P, I, I_eff) = roofline(w, dom_name, dom, args)
    sb = step_bytes(C, cfg.N, P, I, I_eff, w.p_dim, cfg.backward, sets=w.sets_per_launch(C),
                    rows=w.rows_per_launch(C), fwd_walks=w.fwd_walks(C))
    launches_per_step = max(1, math.ceil(w.views_here / C)) if C else 1
    out = {
        "metric": "rendered frames/sec (%s) at N_gauss x H x W" % ("fwd+bwd" if cfg.backward else "fwd"),
        "value": value,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        # N=1 carries the label of the layout the same command uses at N>1
        "scaling": w.scaling if world > 1 else ("weak" if cfg.index == 2 or args.shard == "views" else "strong"),
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (SURVEY.md §8(d) distributions, seed 1000+config)",
        "config": {"workload": cfg.name, "N_gauss": cfg.N, "width": cfg.width, "height": cfg.height,
                   "views": cfg.views, "frames": FRAMES_2D if cfg.mode == "2d" else 1,
                   "units_per_step": w.units_total, "background": "white", "loss": args.loss,
                   "capacity": args.capacity, "chunk_entries": dict(R._chunk_entries),
                   "launch": (f"one HIP graph of the {args.steps} timed steps, replayed once" if args.graph
                              else "eager launches"),
                   "split": w.split,
                   "parallelism": w.layout + (f"; backend {backend}" + (" (RCCL)" if backend == "nccl" else "")
                                              if backend else "")},
        # the launch mode of this line and, for a graph-timed one, the same steps eager (the
        # mode of the N > 1 lines): a 1 -> N curve compares value_eager with value_eager
        "launch_mode": timing["launch_mode"],
        "value_eager": timing["value_eager"],
        "ms_per_step_eager": timing["ms_per_step_eager"],
        "roofline": roof,
        "kernels_ms": {k: round(v[0], 4) for k, v in sorted(breakdown.items())},
        "allreduce_ms": ar_ms,
        "sets_per_s": value / cfg.views,
        "pair_evals_per_s": 2.0 * 256.0 * I_eff * launches_per_step * world / (ms_per_step * 1e-3),
        "step_roofline": {"algorithmic_bytes": sb * launches_per_step,
                          "achieved": sb * launches_per_step / (ms_per_step * 1e-3) / 1e9,
                          "unit": "GB/s", "frac": sb * launches_per_step / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "formula": ("SURVEY.md 8(d): S*N*(12p+64) + R*N*72 + 36*I + 40*I_eff*(W+1) + 44*P per "
                                      "rank (S = projections: C in 3D, the frames in 2D; R = reduced gradient rows: C, "
                                      "or the frames in 2D when a frame's units share one backward walk; W = forward "
                                      f"walks of each list, {w.fwd_walks(C):g} here: a 2D frame's views each walk "
                                      "its shared list)" if cfg.backward
                                      else "SURVEY.md 8(d) fwd-only: C*N*(4p+32) + 36*I + 40*I_eff + 20*P per rank")},
        "binning": {"I": I, "I_eff": I_eff, "max_list": R.last_stats().get("max_seg"),
                    "busy_tiles": R.last_stats().get("n_busy"), "tiles": R.last_stats().get("tiles")},
    }
    log(f"timed {args.steps} steps: {1000.0 * elapsed / args.steps:.3f} ms/step")
    out["layout"] = LAYOUT_KEY.get(args.shard, args.shard) if cfg.index != 2 else "replicas"
    if world > 1:
        del w
        torch.cuda.empty_cache()
        w = None
        for sh in other_layouts(cfg, args.shard):
            log(f"also timing the '{sh}' layout")
            out[LAYOUT_KEY[sh]] = measure_layout(cfg, args, dev, world, rank, sh, dist)
    if rank == 0 and world == 1 and args.cpu_baseline:
        log(f"CPU baseline on {cpu_threads(args.cpu_threads)} threads")
        cb, rgb_o = cpu_baseline(cfg, w.params_cpu if cfg.mode == "3d" else w.params_cpu[0], w.V, w.K,
                                 cpu_threads(args.cpu_threads))
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu"] = value / cb["value"] if cb["value"] > 0 else None
    else:
        out["cpu_baseline"] = None
        rgb_o = None
    if rank == 0 and world == 1 and args.psnr:
        log("dPSNR vs the oracle")
        p0 = w.params_cpu if cfg.mode == "3d" else w.params_cpu[0]
        out["dpsnr"] = delta_psnr(cfg, p0, w.V, w.K, dev, rgb_o)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
