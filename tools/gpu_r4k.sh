#!/bin/bash
# round 4: 2D records once per parameter set + XCD-aware tile sweep (ABI 7): 2D parity suites,
# config-4 bench, FETCH/WRITE passes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_bounded_gpu.py tests/test_chunk_units_gpu.py tests/test_multiframe_gpu.py \
  tests/test_reference_api_gpu.py -k "2d or cfg4 or units or frame or reference" > gpurun_out/r4k_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r4k_tests.txt | head -20; tail -30 gpurun_out/r4k_tests.txt; exit 1; }
tail -1 gpurun_out/r4k_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms'])"; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4k_c4_$i.json 2>/dev/null || exit 1
  show gpurun_out/r4k_c4_$i.json "c4 sweep"
done
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/r4k_pmc_$ctr -o run -- \
    python3 bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 3 --warmup 1 > gpurun_out/r4k_pmc_$ctr.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/r4k_pmc_*/*counter_collection.csv | grep -A3 "raster\|project2d"
