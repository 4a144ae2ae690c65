#!/bin/bash
# round 4: 3D records store the conic and L times log2(e) (ABI 12) -- the whole GPU suite, then
# configs 3 and 5 against the unscaled 3D records (build_var v4: GSR_CONIC3D_LOG2E=0), same box
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4ae_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4ae_tests.txt | head -20; tail -30 gpurun_out/r4ae_tests.txt; exit 1; }
tail -1 gpurun_out/r4ae_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for c in 3 5; do
  for v in new v4 new v4 new v4; do
    case $v in
      new) timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 --psnr 0 > gpurun_out/r4ae_c${c}_$v.json 2>/dev/null || exit 1 ;;
      *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config $c --cpu-baseline 0 --psnr 0 > gpurun_out/r4ae_c${c}_$v.json 2>/dev/null || exit 1 ;;
    esac
    show gpurun_out/r4ae_c${c}_$v.json "c$c $v"
  done
done
