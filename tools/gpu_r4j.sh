#!/bin/bash
# round 4: chunk-parallel (3D) backward with packed LDS records + grouped survivor slots vs not;
# config-4 PMC passes of the new 2D kernels
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_bounded_gpu.py tests/test_headline_mode_gpu.py tests/test_lazy_gpu.py \
  > gpurun_out/r4j_tests.txt 2>&1 || { tail -30 gpurun_out/r4j_tests.txt; exit 1; }
tail -1 gpurun_out/r4j_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for c in 3 5; do
  for v in new bwdlds0 new bwdlds0; do
    case $v in
      new) timeout -k 10 200 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 20 > gpurun_out/r4j_c${c}_$v.json 2>/dev/null || exit 1 ;;
      *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 200 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 20 > gpurun_out/r4j_c${c}_$v.json 2>/dev/null || exit 1 ;;
    esac
    show gpurun_out/r4j_c${c}_$v.json "c$c $v"
  done
done
bash tools/pmc_config.sh 04 4 && python3 tools/pmc_summary.py gpurun_out/pmc_cfg4/r04_pmc_*_cfg4*.csv 2>&1 | tail -20
