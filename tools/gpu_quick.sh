set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu ${TESTS:-tests/test_chunk_units_gpu.py tests/test_bounded_gpu.py} > gpurun_out/quick_tests.txt 2>&1 || { tail -40 gpurun_out/quick_tests.txt; exit 1; }
tail -2 gpurun_out/quick_tests.txt
CONFIGS="${CONFIGS:-2 3}" BENCH_ARGS="--cpu-baseline 0 --psnr 0" bash tools/gpu_bench.sh
