#!/bin/bash
# On the GPU box: A/B of the default library against build_var/libgsr_*.so at configs 3 and 5
# (kernel times, 20 graph-timed steps), then config-5 view-group split 2, then config-4 rank
# shares of the frame-owner layout at N = 2, 4, 8.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 bash tools/run_variants_cfg.sh "3 5" > gpurun_out/ab_proj.txt 2>&1 || { tail -30 gpurun_out/ab_proj.txt; exit 1; }
cat gpurun_out/ab_proj.txt
CONFIGS=5 SPLITS=2 timeout -k 10 300 bash tools/gpu_split.sh > gpurun_out/split5.txt 2>&1 || { tail -30 gpurun_out/split5.txt; exit 1; }
tail -1 gpurun_out/split5.txt
V=r03s2 CONFIGS=4 timeout -k 10 600 bash tools/gpu_rankshare.sh
