#!/bin/bash
# round 4: rows exchange tests, then the rank shares with the device rows exchange (cfg 5, 3)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_rows_exchange_gpu.py \
  > gpurun_out/r4e_tests.txt 2>&1 || { tail -40 gpurun_out/r4e_tests.txt; exit 1; }
grep -E "PASS|\[rows\]" gpurun_out/r4e_tests.txt
for c in 5 3; do
  timeout -k 10 600 python -u bench.py --config $c --rank-share 2,4,8 --steps 10 --warmup 3 --cpu-baseline 0 --psnr 0 \
    > gpurun_out/r4_rankshare_rows_cfg$c.json 2> gpurun_out/r4_rankshare_rows_cfg$c.log || { tail -30 gpurun_out/r4_rankshare_rows_cfg$c.log; exit 1; }
  python - $c <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r4_rankshare_rows_cfg{sys.argv[1]}.json").read().strip().splitlines()[-1])
for r in d["rank_shares"]:
    print(sys.argv[1], r["n"], "max share", round(r["max_share_ms"], 3), "sparse 1-link", round(r.get("projected_ms_per_step_sparse", 0), 3),
          "7-link", round(r.get("projected_ms_per_step_sparse_7link", 0), 3), [s["touched_rows"] for s in r["shares"]])
    w = max(r["shares"], key=lambda s: s["ms_per_step"])
    print("   worst share kernels", w["kernels_ms"])
PY
done
