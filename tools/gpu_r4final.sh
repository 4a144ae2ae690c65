#!/bin/bash
# round 4 v4 (pair kernels without the zero-start adds, exp2 2D conic, 36-B rows): the GPU
# suite, config 3 backward-layout A/B, PMC passes of configs 3/4/5 (rows changed), kernel
# stats of configs 4/5, then the bench lines of configs 3, 2, 5, 4.  Results under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
V=r04_v4
timeout -k 10 420 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${V}_gpu_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/${V}_gpu_tests.txt | head -20; tail -30 gpurun_out/${V}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${V}_gpu_tests.txt
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernels_ms']; print('$2', round(d['ms_per_step'],4), {x: k[x] for x in k if 'raster' in x})"; }
for v in 1 2 1 2; do
  timeout -k 10 120 python bench.py --config 3 --cpu-baseline 0 --psnr 0 --bwd-layout $v > gpurun_out/${V}_c3_layout$v.json 2>/dev/null || exit 1
  show gpurun_out/${V}_c3_layout$v.json "c3 layout$v"
done
for c in 3 5 4; do
  timeout -k 10 300 bash tools/pmc_config.sh 04 $c > gpurun_out/${V}_pmc_cfg$c.log 2>&1 || { tail -20 gpurun_out/${V}_pmc_cfg$c.log; exit 1; }
  cp gpurun_out/pmc_cfg$c/r04_pmc_*cfg$c*.csv profiles/
  echo "pmc cfg$c done"
done
for c in 5 4; do
  st="--steps 20 --warmup 3"; [ $c = 4 ] && st="--steps 5 --warmup 2"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${V}_trace_cfg$c -o run -- python -u bench.py --config $c $st --cpu-baseline 0 --psnr 0 > gpurun_out/${V}_trace_cfg$c.json 2> gpurun_out/${V}_trace_cfg$c.err || { tail -20 gpurun_out/${V}_trace_cfg$c.err; exit 1; }
  echo "trace cfg$c done"
done
for c in 3 2 5 4; do
  extra=""; [ "$c" = "4" ] && extra="--steps 10 --warmup 3"
  timeout -k 10 300 python -u bench.py --config $c $extra > gpurun_out/${V}_cfg$c.json 2> gpurun_out/${V}_cfg$c.err || { tail -30 gpurun_out/${V}_cfg$c.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/${V}_cfg$c.json'))
print('cfg$c', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), 'traffic', d['roofline']['traffic'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'dpsnr', (d.get('dpsnr') or {}).get('dpsnr_db'), d['kernels_ms'])"
done
