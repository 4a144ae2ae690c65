#!/bin/bash
# On the GPU box: bench lines for configs 2-5 (cfg3 with the CPU baseline and dPSNR) and the
# rocprofv3 kernel-trace summary of the default (config 3) command.
# Usage: tools/bench_all.sh TAG  -> gpurun_out/TAG_bench_cfgC.json, gpurun_out/TAG_kernel_stats.csv
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=${1:-rNN}
mkdir -p gpurun_out
timeout -k 10 200 python bench.py > gpurun_out/${tag}_bench_cfg3.json 2> gpurun_out/${tag}_bench_cfg3.log
timeout -k 10 200 python bench.py --config 2 > gpurun_out/${tag}_bench_cfg2.json 2> gpurun_out/${tag}_bench_cfg2.log
timeout -k 10 300 python bench.py --config 4 --steps 10 > gpurun_out/${tag}_bench_cfg4.json 2> gpurun_out/${tag}_bench_cfg4.log
timeout -k 10 300 python bench.py --config 5 --steps 10 > gpurun_out/${tag}_bench_cfg5.json 2> gpurun_out/${tag}_bench_cfg5.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --cpu-baseline 0 --psnr 0 > gpurun_out/${tag}_prof.log 2>&1
cp gpurun_out/${tag}_prof/run_kernel_stats.csv gpurun_out/${tag}_kernel_stats.csv
