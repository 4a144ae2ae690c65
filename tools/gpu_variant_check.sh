#!/bin/bash
# On the GPU box: parity tests against each build_var/libgsr_*.so (GSR_LIBRARY), then the bench
# variants at the given configs.  Usage: tools/gpu_variant_check.sh "3 5" [tests...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cfgs=${1:-3}; shift || true
tests=${*:-tests/test_parity_gpu.py tests/test_lazy_gpu.py tests/test_bounded_gpu.py}
for so in build_var/libgsr_*.so; do
  n=$(basename "$so" .so); n=${n#libgsr_}
  GSR_LIBRARY=$PWD/$so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    $tests > gpurun_out/vcheck_$n.txt 2>&1
  rc=$?
  echo "$n: $(tail -1 gpurun_out/vcheck_$n.txt)"
  [ $rc -eq 0 ] || { tail -30 gpurun_out/vcheck_$n.txt; exit $rc; }
done
bash tools/run_variants_cfg.sh "$cfgs" > gpurun_out/vcheck_bench.txt 2>&1 || { tail -20 gpurun_out/vcheck_bench.txt; exit 1; }
grep -E "^c[0-9]_" gpurun_out/vcheck_bench.txt
