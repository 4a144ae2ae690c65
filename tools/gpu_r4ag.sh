#!/bin/bash
# round 4: 2D parity with ragged edge tiles (70 x 45) under every forward layout
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "2d_vs_oracle_dense or 3d_small" > gpurun_out/r4ag_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4ag_tests.txt | head -20; tail -30 gpurun_out/r4ag_tests.txt; exit 1; }
tail -1 gpurun_out/r4ag_tests.txt
