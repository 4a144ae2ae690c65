#!/bin/bash
# round 4: per-tile 2D backward -- rows stored by two threads each (ROWS2) vs one; phase trace
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  tests/test_chunk_units_gpu.py tests/test_bounded_gpu.py -k "2d or units" > gpurun_out/r4i_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r4i_tests.txt; exit 1; }
tail -1 gpurun_out/r4i_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for v in new rows1 new rows1; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4i_c4_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4i_c4_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4i_c4_$v.json "c4 $v"
done
timeout -k 10 300 python tools/bwd2d_trace.py 4 > gpurun_out/r4i_trace.txt 2>&1 || { tail -20 gpurun_out/r4i_trace.txt; exit 1; }
cat gpurun_out/r4i_trace.txt
