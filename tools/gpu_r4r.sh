#!/bin/bash
# round 4: the 2D pair backward at 3 waves per SIMD (shipped default) -- 2D suites, then config 4
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_bounded_gpu.py tests/test_chunk_units_gpu.py tests/test_multiframe_gpu.py \
  tests/test_reference_api_gpu.py -k "2d or cfg4 or units or frame or reference or box or lanes" > gpurun_out/r4r_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4r_tests.txt | head -20; tail -30 gpurun_out/r4r_tests.txt; exit 1; }
tail -1 gpurun_out/r4r_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for v in new new; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4r_c4_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4r_c4_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4r_c4_$v.json "c4 $v"
done
