#!/bin/bash
# On the GPU box: graph-branch probe, then config 3 / 5 bench lines with the views rendered in
# 1, 2 or 3 concurrent stream groups (bench.py --split).  Results under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/graph_branch_probe.py > gpurun_out/probe.txt 2>&1 || { cat gpurun_out/probe.txt; exit 1; }
cat gpurun_out/probe.txt
for c in ${CONFIGS:-3}; do
  for s in ${SPLITS:-1 2 3}; do
    timeout -k 10 200 python -u bench.py --config $c --split $s --steps 20 --cpu-baseline 0 --psnr 0 \
      > gpurun_out/split_c${c}_s$s.json 2> gpurun_out/split_c${c}_s$s.err || { tail -30 gpurun_out/split_c${c}_s$s.err; exit 1; }
    python -c "
import json; d = json.loads(open('gpurun_out/split_c${c}_s$s.json').read().strip().splitlines()[-1])
print('cfg$c split $s', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['kernels_ms'])"
  done
done
