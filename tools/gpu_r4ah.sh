#!/bin/bash
# round 4: the 3D pair backward with half staging (build_var hs: LDS 20.4 KB, 8 workgroups per CU)
# -- 3D parity through the variant (both layouts forced), then config 3 with the layout forced:
# 1 (4-wave), 2 (pair, shipped), 2 via hs; and config 5 auto (pair) shipped vs hs
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
GSR_LIBRARY=$PWD/build_var/libgsr_hs.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py -k "3d" > gpurun_out/r4ah_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4ah_tests.txt | head -20; tail -30 gpurun_out/r4ah_tests.txt; exit 1; }
tail -1 gpurun_out/r4ah_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernels_ms']; print('$2', round(d['ms_per_step'],4), {x: k[x] for x in k if 'raster' in x})"; }
for r in 1 2; do
  timeout -k 10 120 python bench.py --config 3 --cpu-baseline 0 --psnr 0 --bwd-layout 1 > gpurun_out/r4ah_c3_l1.json 2>/dev/null || exit 1; show gpurun_out/r4ah_c3_l1.json "c3 layout1"
  timeout -k 10 120 python bench.py --config 3 --cpu-baseline 0 --psnr 0 --bwd-layout 2 > gpurun_out/r4ah_c3_l2.json 2>/dev/null || exit 1; show gpurun_out/r4ah_c3_l2.json "c3 layout2"
  GSR_LIBRARY=$PWD/build_var/libgsr_hs.so timeout -k 10 120 python bench.py --config 3 --cpu-baseline 0 --psnr 0 --bwd-layout 2 > gpurun_out/r4ah_c3_hs.json 2>/dev/null || exit 1; show gpurun_out/r4ah_c3_hs.json "c3 layout2 hs"
  timeout -k 10 120 python bench.py --config 5 --cpu-baseline 0 --psnr 0 > gpurun_out/r4ah_c5.json 2>/dev/null || exit 1; show gpurun_out/r4ah_c5.json "c5 pair"
  GSR_LIBRARY=$PWD/build_var/libgsr_hs.so timeout -k 10 120 python bench.py --config 5 --cpu-baseline 0 --psnr 0 > gpurun_out/r4ah_c5_hs.json 2>/dev/null || exit 1; show gpurun_out/r4ah_c5_hs.json "c5 pair hs"
done
