#!/bin/bash
# round 4: quadrant masks -- parity (masks on == off bitwise, mask vs cull), then A/B benches
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_quadrant_masks_gpu.py \
  tests/test_parity_gpu.py tests/test_lazy_gpu.py tests/test_bounded_gpu.py > gpurun_out/r4f_tests.txt 2>&1 \
  || { grep -E "FAIL|Error" gpurun_out/r4f_tests.txt | head; tail -40 gpurun_out/r4f_tests.txt; exit 1; }
grep -E "passed|failed|\[masks\]" gpurun_out/r4f_tests.txt | tail -3
for c in 3 5 2; do
  for m in 0 1 0 1; do
    timeout -k 10 200 python bench.py --config $c --masks $m --cpu-baseline 0 --psnr 0 --steps 20 > gpurun_out/r4f_c${c}_m$m.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/r4f_c${c}_m$m.json').read().strip().splitlines()[-1]); print('c$c m$m', round(d['ms_per_step'],4), d['kernels_ms'])"
  done
done
