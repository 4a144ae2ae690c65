set -o pipefail
cd $GRAFT_REPO_ROOT
V=${V:-r03_v1}
for c in ${CONFIGS:-3 2 4}; do
  extra=""
  [ "$c" != "3" ] && extra="--cpu-baseline 0"
  [ "$c" = "4" ] && extra="$extra --steps 10 --warmup 3"
  timeout -k 10 300 python -u bench.py --config $c $extra $BENCH_ARGS > gpurun_out/${V}_cfg$c.json 2> gpurun_out/${V}_cfg$c.err || { tail -30 gpurun_out/${V}_cfg$c.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/${V}_cfg$c.json'))
print('cfg$c', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['roofline']['kernel'], round(d['roofline']['avg_ms'], 4), 'frac', round(d['roofline']['frac'], 4), d['kernels_ms'])"
done
