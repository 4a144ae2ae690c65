"""bench.py host logic that runs without a GPU: the roofline fields read from the committed
rocprofv3 PMC passes of the SAME config (profiles/), the CPU-baseline fit, the PSNR formula
and the §8(d) byte formulas."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_traffic_from_committed_pmc():
    f = bench.pmc_files(3, "traffic")
    assert f is not None and "cfg3" in os.path.basename(f)
    t = bench.traffic_from_csv(f, bench.KERNEL_SYMBOL["raster3d_bwd"])
    assert t is not None and 1e8 < t < 1e9, t
    assert bench.traffic_from_csv(f, "no_such_kernel") is None


def test_no_cross_config_counters(tmp_path):
    """A config without its own PMC pass reports null traffic/valu (never another config's)."""
    assert bench.pmc_files(2, "traffic", str(tmp_path)) is None
    assert bench.pmc_files(2, "sq", str(tmp_path)) is None
    (tmp_path / "r01_pmc_traffic_cfg3.csv").write_text("x\n")
    (tmp_path / "r02_pmc_traffic_cfg3.csv").write_text("x\n")
    (tmp_path / "r10_pmc_traffic_cfg3.csv").write_text("x\n")
    assert bench.pmc_files(2, "traffic", str(tmp_path)) is None
    assert os.path.basename(bench.pmc_files(3, "traffic", str(tmp_path))) == "r10_pmc_traffic_cfg3.csv"
    (tmp_path / "r02_pmc_sq_cfg5_p1.csv").write_text("x\n")
    assert bench.pmc_files(5, "sq", str(tmp_path)) is None          # p2 missing
    (tmp_path / "r02_pmc_sq_cfg5_p2.csv").write_text("x\n")
    assert len(bench.pmc_files(5, "sq", str(tmp_path))) == 2


def test_valu_from_committed_sq_passes():
    sq = bench.pmc_files(3, "sq")
    v = bench.valu_from_csv(sq, bench.KERNEL_SYMBOL["raster3d_bwd"])
    assert v is not None
    assert 0.0 < v["issue_frac"] < 1.0 and v["wave_active"] > v["issue_frac"], v
    assert v["insts_per_launch"] > 1e7
    assert bench.valu_from_csv(sq, "no_such_kernel") is None
    assert bench.valu_from_csv([os.path.join(ROOT, "profiles", "missing.csv")], "k_emit") is None
    assert bench.valu_from_csv(None, "k_emit") is None


def test_linear_fit_and_psnr():
    a, b, r2 = bench.linear_fit([1, 2, 3, 4], [3.0, 5.0, 7.0, 9.0])
    assert abs(a - 1.0) < 1e-12 and abs(b - 2.0) < 1e-12 and abs(r2 - 1.0) < 1e-12
    _, _, r2n = bench.linear_fit([1, 2, 3], [1.0, 3.0, 2.0])
    assert r2n < 1.0
    x = torch.rand(8, 6, 3, dtype=torch.float64)
    y = x + 0.1
    # get_psnr (scripts/utils/evaluate_model.py:240-243): 10 log10(1 / mse), mse = 0.01
    assert abs(bench.psnr(x, y) - 20.0) < 1e-9


def test_byte_formulas_and_allreduce_model():
    # §8(d): fwd+bwd per view N(12p+136) + 36 I + 80 I_eff + 44 P
    assert bench.step_bytes(1, 10, 100, 7, 5, 14) == 10 * (12 * 14 + 136) + 36 * 7 + 80 * 5 + 44 * 100
    # 2D: the projection charged once per parameter set (frame), the rows per unit
    assert bench.step_bytes(48, 10, 100, 7, 5, 9, sets=8) == (8 * 10 * (12 * 9 + 64) + 48 * 10 * 72 + 36 * 7
                                                              + 80 * 5 + 44 * 100)
    assert bench.step_bytes(6, 10, 100, 7, 5, 14, sets=6) == bench.step_bytes(6, 10, 100, 7, 5, 14)
    # ... and the reduced rows per set when the backward walks each set once for its units
    assert bench.step_bytes(48, 10, 100, 7, 5, 9, sets=8, rows=8) == (8 * 10 * (12 * 9 + 64) + 8 * 10 * 72 + 36 * 7
                                                                      + 80 * 5 + 44 * 100)
    assert bench.algorithmic_bytes("raster2d_bwd", 48, 10, 100, 7, 5, 9, rows=8) == 24 * 100 + 40 * 5 + 36 * 8 * 10
    # ... and its lists walked by all six units of a set in the forward (shared lists)
    assert bench.step_bytes(48, 10, 100, 7, 5, 9, sets=8, rows=8, fwd_walks=6.0) == (
        8 * 10 * (12 * 9 + 64) + 8 * 10 * 72 + 36 * 7 + 40 * 5 * 7 + 44 * 100)
    assert bench.algorithmic_bytes("raster2d_fwd", 48, 10, 100, 7, 5, 9, rows=8, fwd_walks=6.0) == 40 * 5 * 6 + 20 * 100
    assert bench.algorithmic_bytes("project2d_bwd", 48, 10, 100, 7, 5, 9, rows=8) == 10 * (36 * 8 + (32 + 72) * 48)
    assert bench.step_bytes(1, 10, 100, 7, 5, 14, backward=False) == 10 * (4 * 14 + 32) + 36 * 7 + 40 * 5 + 20 * 100
    assert bench.algorithmic_bytes("raster3d_bwd", 6, 10, 100, 7, 5, 14) == 24 * 100 + 40 * 5 + 36 * 6 * 10
    assert bench.allreduce_ms(1000, 1) == 0.0
    # 2(n-1)/n S at 153 GB/s: 11.2 MB at n = 8 -> 0.128 ms
    assert abs(bench.allreduce_ms(11_200_000, 8) - 2 * 7 / 8 * 11.2e6 / 153e9 * 1e3) < 1e-12


def test_bench_args_defaults():
    a = bench.parse([])
    # configs 3 and 5 time ONE job at every N (the strong layout) by default
    assert a.config == 3 and a.gpus == 1 and a.shard == "units" and a.cpu_threads == 0
    assert bench.parse(["--config", "5"]).shard == "units" and bench.parse(["--config", "2"]).shard == "views"
    assert a.capacity == "bounded" and a.graph == -1
    assert bench.cpu_threads(3) == 3 and bench.cpu_threads(0) >= 1
    assert a.split == 1
    # config 4 (2D) defaults to the round-robin layout with its all-reduce;
    # frames is a 2D-only layout
    assert bench.parse(["--config", "4"]).shard == "units"
    assert bench.parse(["--config", "4", "--shard", "frames"]).shard == "frames"
    import pytest
    with pytest.raises(SystemExit):
        bench.parse(["--config", "3", "--shard", "frames"])


def test_gpus_without_launcher_spawns_ranks(monkeypatch):
    """`bench.py --gpus 2` with no launcher environment starts 2 ranks itself (never silently
    reports n_gpus 1); a launcher whose WORLD_SIZE disagrees with --gpus is an error."""
    import pytest
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "_spawn_ranks", lambda args, argv: calls.append((args.gpus, argv)) or 7)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2", "--steps", "3"])
    assert e.value.code == 7 and calls == [(2, ["--gpus", "2", "--steps", "3"])]
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2"])
    assert "WORLD_SIZE=4" in str(e.value.code)


def _layout_worker(rank, world, port, q):
    """One rank of a gloo rehearsal of bench.measure_layout with a CPU stand-in workload whose
    step all-reduces its gradient (the host logic only: timing brackets, max over ranks, the
    per-layout collective timing, the JSON keys)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsr.scenes import CONFIGS

        class FakeWorkload:
            def __init__(self, cfg, dev, world, rank, shard, buckets, loss, comm, view_cost, exchange):
                self.params = torch.zeros(64, 14)
                self.owned = shard == "frames"
                self.units_total = cfg.views * (world if shard == "views" else 1) * (8 if cfg.mode == "2d" else 1)
                self.scaling = "weak" if shard == "views" else "strong"
                self.layout = f"fake {shard}"

            def step(self):
                if not self.owned:
                    g = torch.ones_like(self.params)
                    dist.all_reduce(g)

        def timer(w, steps, warmup, dist_, graph=False):
            for _ in range(warmup):
                w.step()
            dist_.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                w.step()
            dist_.barrier()
            return time.perf_counter() - t0, {}, None, (0.0, 0)

        import time
        args = bench.parse(["--steps", "3", "--warmup", "1"])
        res = {}
        for idx in (3, 4):
            cfg = CONFIGS[idx]
            shard = bench.parse(["--config", str(idx)]).shard
            for sh in bench.other_layouts(cfg, shard):
                res[(idx, bench.LAYOUT_KEY[sh])] = bench.measure_layout(cfg, args, "cpu", world, rank, sh, dist,
                                                                        make_workload=FakeWorkload, timer=timer)
        # the headline line's timing at N > 1: eager (graph off by default there), value_eager = value;
        # config 3's default layout is the strong one (the same job at every N)
        hargs = bench.parse(["--steps", "3", "--warmup", "1", "--graph", "0"])
        w = FakeWorkload(CONFIGS[3], "cpu", world, rank, hargs.shard, 1, "none", True, 0.3, "dense")
        res["headline"] = bench.headline_timing(w, hargs, dist, "cpu", world, timer=timer)[0]
        res["headline_layout"] = (bench.LAYOUT_KEY[hargs.shard], w.scaling, w.units_total)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


def test_other_layouts_reported_gloo_world2():
    """at N > 1 one bench.py run reports config 3's strong (default) AND weak
    layouts, and config 4's round-robin all-reduce layout (default) AND the frame owners, each
    with its own value and collective timing -- rehearsed with two gloo ranks on the CPU."""
    import multiprocessing as mp
    import socket
    from gsr.scenes import CONFIGS
    assert bench.parse(["--config", "4"]).shard == "units"   # the all-reduce layout is the default
    assert bench.other_layouts(CONFIGS[3], "units") == ["views"]
    assert bench.other_layouts(CONFIGS[4], "units") == ["frames"]
    assert bench.other_layouts(CONFIGS[2], "views") == []
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_layout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # config 3 at N = 2: value is the strong layout (one 6-view job), the weak one a secondary key
    assert res["headline_layout"] == ("strong", "strong", CONFIGS[3].views), res["headline_layout"]
    weak = res[(3, "weak")]
    assert weak["scaling"] == "weak" and weak["value"] > 0 and weak["allreduce_ms"] is not None
    assert weak["units_per_step"] == 2 * CONFIGS[3].views
    strong = weak
    owners = res[(4, "frame_owners")]
    assert owners["value"] > 0 and owners["allreduce_ms"] is None   # no Gaussian-gradient collective
    assert set(strong) >= {"value", "ms_per_step", "allreduce_ms", "parallelism", "scaling", "launch_mode"}
    assert strong["launch_mode"] == owners["launch_mode"] == "eager"
    head = res["headline"]   # every line states its launch mode
    assert head["launch_mode"] == "eager" and head["value_eager"] == head["value"] > 0
    assert head["ms_per_step_eager"] == head["ms_per_step"]


def test_headline_graph_line_reports_eager_too():
    """A graph-timed N = 1 line also reports the same steps eager (value_eager), so the driver's
    1 -> N curve can divide eager by eager."""
    class W:
        units_total = 6

    calls = []

    def timer(w, steps, warmup, dist_, graph=False):
        calls.append(("timer", graph))
        return 0.010 * steps, {}, None, (0.0, 0)

    def eager_timer(w, steps, dist_):
        calls.append(("eager", steps))
        return 0.012 * steps

    args = bench.parse(["--steps", "4", "--warmup", "1", "--graph", "1"])
    t = bench.headline_timing(W(), args, None, "cpu", 1, timer=timer, eager_timer=eager_timer)[0]
    assert calls == [("timer", True), ("eager", 4)]
    assert t["launch_mode"] == "graph"
    assert abs(t["ms_per_step"] - 10.0) < 1e-9 and abs(t["ms_per_step_eager"] - 12.0) < 1e-9
    assert abs(t["value"] - 600.0) < 1e-6 and abs(t["value_eager"] - 500.0) < 1e-6
