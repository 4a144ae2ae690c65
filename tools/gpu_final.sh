# Round-end measurement on one box: PMC passes of configs 3, 4 and 5 (copied into profiles/ so
# the bench lines read counters of the shipped kernels), a rocprofv3 kernel-trace summary of
# config 3, the bench lines of configs 3, 2, 5, 4 with their CPU baselines, then rank-share
# projections of configs 3 and 5.  Results under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${V:-r03_v6}
R=${R:-03}
if [ -z "$SKIP_PMC" ]; then
  for c in ${PMC_CONFIGS:-3 5 4}; do
    timeout -k 10 400 bash tools/pmc_config.sh $R $c > gpurun_out/${V}_pmc_cfg$c.log 2>&1 || { tail -20 gpurun_out/${V}_pmc_cfg$c.log; exit 1; }
    cp gpurun_out/pmc_cfg$c/r${R}_pmc_*cfg$c*.csv profiles/
    echo "pmc cfg$c done"
  done
fi
if [ -z "$SKIP_TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${V}_trace_cfg3 -o run -- python -u bench.py --config 3 --steps 20 --warmup 3 --cpu-baseline 0 --psnr 0 > gpurun_out/${V}_trace_cfg3.json 2> gpurun_out/${V}_trace_cfg3.err || { tail -20 gpurun_out/${V}_trace_cfg3.err; exit 1; }
  echo "trace done"
fi
for c in ${CONFIGS:-3 2 5 4}; do
  extra=""
  [ "$c" = "4" ] && extra="--steps 10 --warmup 3"
  timeout -k 10 600 python -u bench.py --config $c $extra > gpurun_out/${V}_cfg$c.json 2> gpurun_out/${V}_cfg$c.err || { tail -30 gpurun_out/${V}_cfg$c.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/${V}_cfg$c.json'))
print('cfg$c', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), 'traffic', d['roofline']['traffic'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'dpsnr', d.get('dpsnr'))"
done
if [ -z "$SKIP_SHARE" ]; then
  V=$V CONFIGS="3 5" timeout -k 10 600 bash tools/gpu_rankshare.sh
fi
