#!/bin/bash
# On the GPU box: bench the default library and each build_var/libgsr_*.so at the given configs
# (kernel times).  Usage: tools/run_variants_cfg.sh "3 5 2" [extra bench args]
set -e
shopt -s nullglob
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cfgs=${1:-3}; shift || true
for c in $cfgs; do
  timeout -k 10 150 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 10 "$@" > gpurun_out/var_c${c}_base.json
  for so in build_var/libgsr_*.so; do
    n=$(basename "$so" .so); n=${n#libgsr_}
    GSR_LIBRARY=$PWD/$so timeout -k 10 150 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 10 "$@" \
      > gpurun_out/var_c${c}_$n.json
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/var_c*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("var_")[1][:-5], round(d["ms_per_step"], 4), d["kernels_ms"])
PY
