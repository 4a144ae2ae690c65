set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in ${CONFIGS:-2 3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_cfg$c -o run -- python -u bench.py --config $c --steps 20 --warmup 3 --cpu-baseline 0 --psnr 0 > gpurun_out/trace_cfg$c.json 2> gpurun_out/trace_cfg$c.err || { tail -20 gpurun_out/trace_cfg$c.err; exit 1; }
done
find gpurun_out/trace_cfg* -name "*.csv" | head -20
