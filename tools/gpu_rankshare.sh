set -o pipefail
cd $GRAFT_REPO_ROOT
V=${V:-r03_v2}
for c in ${CONFIGS:-3 5 4}; do
  st=20; [ "$c" = "4" ] && st=6
  timeout -k 10 600 python -u bench.py --config $c --rank-share ${NS:-2,4,8} --steps $st --warmup 3 $BENCH_ARGS > gpurun_out/${V}_rankshare_cfg$c.json 2> gpurun_out/${V}_rankshare_cfg$c.err || { tail -20 gpurun_out/${V}_rankshare_cfg$c.err; exit 1; }
  grep "N=" gpurun_out/${V}_rankshare_cfg$c.err
done
