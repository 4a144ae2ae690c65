#!/bin/bash
# round 4 v3: the whole GPU suite and smoke on the shipped library, then the bench lines of
# configs 3, 2, 5, 4 (CPU baselines and dpsnr included) and a config-3 kernel-trace summary
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04_v3_gpu_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/r04_v3_gpu_tests.txt | head -20; tail -30 gpurun_out/r04_v3_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/r04_v3_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_v3_smoke.txt 2>&1 || { tail -20 gpurun_out/r04_v3_smoke.txt; exit 1; }
tail -1 gpurun_out/r04_v3_smoke.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_v3_trace_cfg3 -o run -- python -u bench.py --config 3 --steps 20 --warmup 3 --cpu-baseline 0 --psnr 0 > gpurun_out/r04_v3_trace_cfg3.json 2> gpurun_out/r04_v3_trace_cfg3.err || { tail -20 gpurun_out/r04_v3_trace_cfg3.err; exit 1; }
for c in 3 2 5 4; do
  extra=""
  [ "$c" = "4" ] && extra="--steps 10 --warmup 3"
  timeout -k 10 600 python -u bench.py --config $c $extra > gpurun_out/r04_v3_cfg$c.json 2> gpurun_out/r04_v3_cfg$c.err || { tail -30 gpurun_out/r04_v3_cfg$c.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/r04_v3_cfg$c.json'))
print('cfg$c', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), 'traffic', d['roofline']['traffic'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'dpsnr', d.get('dpsnr'))"
done
