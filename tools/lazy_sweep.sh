#!/bin/bash
# On the GPU box: step time, sort and forward kernel times per lazy-sort setting (MIN_LEN,PREFIX)
# at configs 5, 3 and 2.  Usage: tools/lazy_sweep.sh "0,1 8192,4096 ..."
set -e
cd "$(dirname "$0")/.."
for lz in ${1:-0,1 8192,4096}; do
  for c in 5 3 2; do
    timeout -k 10 100 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 20 --lazy $lz > gpurun_out/lz_${c}_${lz}.json 2>/dev/null
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/lz_*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("lz_")[1][:-5], round(d["ms_per_step"], 4), d["kernels_ms"].get("bin_sort"), d["kernels_ms"].get("raster3d_fwd"))
PY
