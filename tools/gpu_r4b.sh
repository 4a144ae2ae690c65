#!/bin/bash
# round 4 batch: new GPU tests, the pipelined-forward variant (parity + bench), cfg4 dPSNR window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_rows_exchange_gpu.py tests/test_sort_classes_gpu.py tests/test_headline_mode_gpu.py \
  > gpurun_out/r4b_tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/r4b_tests.txt | tail -20
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4b_tests.txt; exit $rc; }
bash tools/gpu_variant_check.sh "3 5 2" || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r4b_cfg4.json 2> gpurun_out/r4b_cfg4.log || exit 1
tail -c 700 gpurun_out/r4b_cfg4.json
