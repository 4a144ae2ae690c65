#!/bin/bash
# round 4: shipped with the half-staged 3D pair backward -- the whole GPU suite, smoke, then the
# bench lines of configs 5 and 3 (v6)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
V=r04_v6
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${V}_gpu_tests.txt 2>&1 \
  || { grep -E "FAIL|Error|error" gpurun_out/${V}_gpu_tests.txt | head -20; tail -30 gpurun_out/${V}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${V}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${V}_smoke.txt 2>&1 || { tail -20 gpurun_out/${V}_smoke.txt; exit 1; }
tail -1 gpurun_out/${V}_smoke.txt
for c in 5 3; do
  timeout -k 10 300 python -u bench.py --config $c > gpurun_out/${V}_cfg$c.json 2> gpurun_out/${V}_cfg$c.err || { tail -30 gpurun_out/${V}_cfg$c.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/${V}_cfg$c.json'))
print('cfg$c', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'dpsnr', (d.get('dpsnr') or {}).get('dpsnr_db'), d['kernels_ms'])"
done
