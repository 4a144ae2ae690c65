#!/bin/bash
# round 4 v3 (shipped kernels: 2D pair forward + backward, 3D backward layout by shape): PMC
# passes of configs 4 and 5 (their dominant kernels changed) and kernel-trace stats of both
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 4 5; do
  timeout -k 10 400 bash tools/pmc_config.sh 04 $c > gpurun_out/r04_v3_pmc_cfg$c.log 2>&1 || { tail -20 gpurun_out/r04_v3_pmc_cfg$c.log; exit 1; }
  echo "pmc cfg$c done"
done
for c in 4 5; do
  st="--steps 20 --warmup 3"; [ $c = 4 ] && st="--steps 5 --warmup 2"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_v3_trace_cfg$c -o run -- python -u bench.py --config $c $st --cpu-baseline 0 --psnr 0 > gpurun_out/r04_v3_trace_cfg$c.json 2> gpurun_out/r04_v3_trace_cfg$c.err || { tail -20 gpurun_out/r04_v3_trace_cfg$c.err; exit 1; }
  echo "trace cfg$c done"
done
