#!/bin/bash
# round 4: the 2D pixel-pair forward (k_raster2d_fwd_pair) and the 3D backward layout knob
# (ABI 9) -- the 2D suites with the pair forward (build_var
# f2p), then config 4: shipped / previous 2D pair-backward validity form (sc) / pair forward
# (f2p), configs 3
# and 5 with the 3D backward layout automatic / forced
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GSR_LIBRARY=$PWD/build_var/libgsr_f2p.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_bounded_gpu.py tests/test_chunk_units_gpu.py tests/test_multiframe_gpu.py \
  tests/test_reference_api_gpu.py -k "2d or cfg4 or units or frame or reference or box or lanes" > gpurun_out/r4w_tests_f2p.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4w_tests_f2p.txt | head -20; tail -30 gpurun_out/r4w_tests_f2p.txt; exit 1; }
tail -1 gpurun_out/r4w_tests_f2p.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernels_ms']; print('$2', round(d['ms_per_step'],4), {x: k[x] for x in k if 'raster' in x})"; }
for v in new sc f2p new sc f2p; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4w_c4_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4w_c4_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4w_c4_$v.json "c4 $v"
done
for cfg in 3 5; do
  for v in 0 1 2 0 1 2; do
    timeout -k 10 300 python bench.py --config $cfg --cpu-baseline 0 --psnr 0 --bwd-layout $v > gpurun_out/r4w_c${cfg}_$v.json 2>/dev/null || exit 1
    show gpurun_out/r4w_c${cfg}_$v.json "c$cfg layout$v"
  done
done
# timing experiment: the 3D quad forward without its chunk-record stores (build_var nockpt; results wrong)
for v in new nockpt new nockpt; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 3 --cpu-baseline 0 --psnr 0 > gpurun_out/r4w_c3x_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 3 --cpu-baseline 0 --psnr 0 > gpurun_out/r4w_c3x_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4w_c3x_$v.json "c3 $v"
done
