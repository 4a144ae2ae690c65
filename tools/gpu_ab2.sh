# A/B of libgsr variants on one box, interleaved: VARIANTS="base ldsadd" CONFIGS="3" REPS=2
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = "base" ]; then unset GSR_LIBRARY; else export GSR_LIBRARY=$PWD/build_var/libgsr_$v.so; fi
    V=ab_${v}_$r CONFIGS="${CONFIGS:-3}" BENCH_ARGS="--cpu-baseline 0 --psnr 0 $BENCH_ARGS" bash tools/gpu_bench.sh | sed "s/^/$v /" || exit 1
  done
done
