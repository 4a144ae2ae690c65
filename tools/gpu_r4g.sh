#!/bin/bash
# round 4: quadrant masks (3D) + box-forward lane groups / packed records and the per-tile 2D
# backward (ABI 6) -- the whole GPU suite, then A/B benches against the round's starting tree
# (build_var/r4base) and the box-forward build variants (build_var/libgsr_*.so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r4g_tests.txt 2>&1 \
  || { grep -E "FAIL|Error" gpurun_out/r4g_tests.txt | head; tail -40 gpurun_out/r4g_tests.txt; exit 1; }
grep -E "passed|failed|\[masks\]" gpurun_out/r4g_tests.txt | tail -3
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for v in base new lanes0 nok4 base new; do
  case $v in
    base) (cd build_var/r4base && timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2) > gpurun_out/r4g_c4_$v.json 2>/dev/null || exit 1 ;;
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4g_c4_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4g_c4_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4g_c4_$v.json "c4 $v"
done
for c in 3 5; do
  for m in base 0 1 base 0 1; do
    if [ $m = base ]; then
      (cd build_var/r4base && timeout -k 10 200 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 20) > gpurun_out/r4g_c${c}_m$m.json 2>/dev/null || exit 1
    else
      timeout -k 10 200 python bench.py --config $c --masks $m --cpu-baseline 0 --psnr 0 --steps 20 > gpurun_out/r4g_c${c}_m$m.json 2>/dev/null || exit 1
    fi
    show gpurun_out/r4g_c${c}_m$m.json "c$c masks=$m"
  done
done
