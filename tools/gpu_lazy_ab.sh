#!/bin/bash
# On the GPU box: config 3 and 5 steps with the lazy-sort thresholds (gsr_set_lazy_sort via
# bench --lazy MIN_LEN,PREFIX) against the default 16384,4096.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for c in 3 5; do
  for lz in 16384,4096 8192,4096 8192,6144 8192,8192; do
    timeout -k 10 150 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 20 --lazy $lz > gpurun_out/lz_c${c}_${lz/,/_}.json 2> gpurun_out/lz_c${c}_${lz/,/_}.err || { tail -20 gpurun_out/lz_c${c}_${lz/,/_}.err; exit 1; }
    python -c "
import json; d = json.loads(open('gpurun_out/lz_c${c}_${lz/,/_}.json').read().strip().splitlines()[-1])
print('cfg$c lazy $lz', round(d['ms_per_step'], 4), d['kernels_ms'])"
  done
done
