#!/bin/bash
# round 4: new host-side tests, then the forward prefetch variants at configs 3 and 5
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_headline_mode_gpu.py tests/test_bounded_gpu.py tests/test_chunk_units_gpu.py \
  > gpurun_out/r4a_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r4a_tests.txt
[ $rc -eq 0 ] || exit $rc
bash tools/run_variants_cfg.sh "3 5" > gpurun_out/r4a_var.txt 2>&1
tail -8 gpurun_out/r4a_var.txt
