#!/bin/bash
# round 4: pair backward kernels compiled with SLP in their own TU (raster_pairs.o) -- the whole GPU suite, then configs 4, 3, 5 (step and
# per-call kernel times; compare with r04_v3 on the previous box)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4ac_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4ac_tests.txt | head -20; tail -30 gpurun_out/r4ac_tests.txt; exit 1; }
tail -1 gpurun_out/r4ac_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for c in 4 5 4 5; do
  st=""; [ $c = 4 ] && st="--steps 5 --warmup 2"
  timeout -k 10 300 python bench.py --config $c $st --cpu-baseline 0 --psnr 0 > gpurun_out/r4ac_c$c.json 2>/dev/null || exit 1
  show gpurun_out/r4ac_c$c.json "c$c"
done
# the 2D pair forward with SLP at 4 waves per SIMD (build_var f2slp) vs shipped (no SLP, 5)
for v in new f2slp new f2slp; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4ac_c4x_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4ac_c4x_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4ac_c4x_$v.json "c4 $v"
done
