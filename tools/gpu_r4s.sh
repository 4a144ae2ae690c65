#!/bin/bash
# round 4: the 3D chunk backward with two pixels per lane (k_raster_bwd_pair3d, build_var p3d) --
# 3D parity suites through the variant library, then configs 3 and 5 against the shipped 4-wave kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GSR_LIBRARY=$PWD/build_var/libgsr_p3d.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_bounded_gpu.py \
  -k "3d or cfg3 or cfg2 or cfg5 or graph" > gpurun_out/r4s_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4s_tests.txt | head -20; tail -30 gpurun_out/r4s_tests.txt; exit 1; }
tail -1 gpurun_out/r4s_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for cfg in 3 5; do
  for v in new p3d new p3d; do
    case $v in
      new) timeout -k 10 300 python bench.py --config $cfg --cpu-baseline 0 --psnr 0 > gpurun_out/r4s_c${cfg}_$v.json 2>/dev/null || exit 1 ;;
      *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config $cfg --cpu-baseline 0 --psnr 0 > gpurun_out/r4s_c${cfg}_$v.json 2>/dev/null || exit 1 ;;
    esac
    show gpurun_out/r4s_c${cfg}_$v.json "c$cfg $v"
  done
done
