#!/bin/bash
# round 4: the whole GPU suite on the default library, then the pipelined-forward variant
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --maxfail=10 --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r4c_suite.txt 2>&1
rc=$?
grep -E "FAIL|ERROR" gpurun_out/r4c_suite.txt | tail -20
tail -2 gpurun_out/r4c_suite.txt
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_variant_check.sh "3 5 2" || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/r4c_cfg4.json 2> gpurun_out/r4c_cfg4.log || exit 1
tail -c 700 gpurun_out/r4c_cfg4.json
