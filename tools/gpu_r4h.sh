#!/bin/bash
# round 4: per-tile 2D backward variants at config 4 (packed LDS records + grouped survivor slots,
# launch bounds, early prefetch) against the round-start tree (chunk-parallel 2D backward)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  tests/test_chunk_units_gpu.py -k "2d or units" > gpurun_out/r4h_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r4h_tests.txt; exit 1; }
tail -1 gpurun_out/r4h_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for v in base new lds0 minb4 early4 new base; do
  case $v in
    base) (cd build_var/r4base && timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2) > gpurun_out/r4h_c4_$v.json 2>/dev/null || exit 1 ;;
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4h_c4_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4h_c4_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4h_c4_$v.json "c4 $v"
done
