#!/bin/bash
# On the GPU box: config-4 (2D) bench of the default library and each build_var/libgsr_*.so.
set -e
shopt -s nullglob
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --config 4 --cpu-baseline 0 --steps 5 > gpurun_out/var2_base.json
for so in build_var/libgsr_*.so; do
  n=$(basename "$so" .so); n=${n#libgsr_}
  GSR_LIBRARY=$PWD/$so timeout -k 10 120 python bench.py --config 4 --cpu-baseline 0 --steps 5 > gpurun_out/var2_$n.json
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/var2_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("var2_")[1][:-5], round(d["ms_per_step"], 4), d["kernels_ms"])
PY
