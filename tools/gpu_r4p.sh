#!/bin/bash
# round 4 v2: config-4 PMC passes + kernel-trace stats of the shipped 2D kernels, bench line of config 4
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 bash tools/pmc_config.sh 04 4 > gpurun_out/r04_v2_pmc_cfg4.log 2>&1 || { tail -20 gpurun_out/r04_v2_pmc_cfg4.log; exit 1; }
cp gpurun_out/pmc_cfg4/r04_pmc_*cfg4*.csv profiles/
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_v2_trace_cfg4 -o run -- python -u bench.py --config 4 --steps 5 --warmup 2 --cpu-baseline 0 --psnr 0 > gpurun_out/r04_v2_trace_cfg4.json 2> gpurun_out/r04_v2_trace_cfg4.err || { tail -20 gpurun_out/r04_v2_trace_cfg4.err; exit 1; }
timeout -k 10 600 python -u bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/r04_v2_cfg4.json 2> gpurun_out/r04_v2_cfg4.err || { tail -30 gpurun_out/r04_v2_cfg4.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/r04_v2_cfg4.json'))
print('cfg4', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), 'traffic', d['roofline']['traffic'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'dpsnr', (d.get('dpsnr') or {}).get('dpsnr_db'), d['kernels_ms'])"
