#!/bin/bash
# On the GPU box: rocprofv3 kernel stats of the emission (staged vs scatter) at configs 2, 3, 5.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for c in 2 3 5; do
  for e in 0 1; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/emit_c${c}_e$e -o run -- \
      python3 bench.py --config $c --steps 10 --cpu-baseline 0 --psnr 0 --emit-staged $e > gpurun_out/emit_c${c}_e$e.log 2>&1
  done
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/emit_c*_e*/run_kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "emit" in r["Name"]:
            print(f.split("/")[1], r["Name"].split("(")[0], r["Calls"], round(float(r["AverageNs"]) / 1000, 1))
PY
