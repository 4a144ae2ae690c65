#!/bin/bash
# round 4 v5 (shipped, ABI 12): smoke, a config-3 kernel-trace summary, then the bench lines of
# configs 3, 2, 5, 4 (CPU baselines, dpsnr).  The GPU suite of this code: r4ae (181 passed).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
V=r04_v5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${V}_smoke.txt 2>&1 || { tail -20 gpurun_out/${V}_smoke.txt; exit 1; }
tail -1 gpurun_out/${V}_smoke.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${V}_trace_cfg3 -o run -- python -u bench.py --config 3 --steps 20 --warmup 3 --cpu-baseline 0 --psnr 0 > gpurun_out/${V}_trace_cfg3.json 2> gpurun_out/${V}_trace_cfg3.err || { tail -20 gpurun_out/${V}_trace_cfg3.err; exit 1; }
for c in 3 2 5 4; do
  extra=""; [ "$c" = "4" ] && extra="--steps 10 --warmup 3"
  timeout -k 10 300 python -u bench.py --config $c $extra > gpurun_out/${V}_cfg$c.json 2> gpurun_out/${V}_cfg$c.err || { tail -30 gpurun_out/${V}_cfg$c.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/${V}_cfg$c.json'))
print('cfg$c', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), 'traffic', d['roofline']['traffic'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'dpsnr', (d.get('dpsnr') or {}).get('dpsnr_db'), d['kernels_ms'])"
done
