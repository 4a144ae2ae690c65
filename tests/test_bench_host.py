"""bench.py host logic that runs without a GPU: the roofline fields read from the committed
rocprofv3 PMC passes (profiles/), and the §8(d) step-bytes formula."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_traffic_from_committed_pmc():
    t = bench.traffic_from_csv(bench.DEFAULT_TRAFFIC_CSV, bench.KERNEL_SYMBOL["raster3d_bwd"])
    assert t is not None and 1e8 < t < 1e9, t
    assert bench.traffic_from_csv(bench.DEFAULT_TRAFFIC_CSV, "no_such_kernel") is None


def test_valu_from_committed_sq_passes():
    v = bench.valu_from_csv(bench.DEFAULT_SQ_CSVS, bench.KERNEL_SYMBOL["raster3d_bwd"])
    assert v is not None
    assert 0.0 < v["issue_frac"] <= v["active_frac"] + 1e-9 < 1.05, v
    assert v["insts_per_launch"] > 1e7
    assert bench.valu_from_csv(bench.DEFAULT_SQ_CSVS, "no_such_kernel") is None
    assert bench.valu_from_csv([os.path.join(ROOT, "profiles", "missing.csv")], "k_emit") is None
