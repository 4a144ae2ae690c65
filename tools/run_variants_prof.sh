#!/bin/bash
# On the GPU box: per-kernel average durations (rocprofv3 kernel trace) of bench.py with the
# default library and each build_var/libgsr_*.so.  Usage: tools/run_variants_prof.sh [bench args]
set -e
shopt -s nullglob
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, library
  rm -rf gpurun_out/vp_$1
  if [ -n "$2" ]; then export GSR_LIBRARY=$2; else unset GSR_LIBRARY; fi
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/vp_$1 -o run \
    --output-format rocpd -- python3 bench.py --cpu-baseline 0 --steps 10 "${@:3}" > gpurun_out/vp_$1.json
  python3 tools/rocpd_stats.py $(find gpurun_out/vp_$1 -name '*.db' | head -1) > gpurun_out/vp_$1.csv
}
run base "" "$@"
for so in build_var/libgsr_*.so; do
  n=$(basename "$so" .so); n=${n#libgsr_}
  run "$n" "$PWD/$so" "$@"
done
python3 - <<'PY'
import csv, glob, json
tabs = {}
for f in sorted(glob.glob("gpurun_out/vp_*.csv")):
    n = f.split("vp_")[1][:-4]
    tabs[n] = {r["Name"].split("(")[0].split("<")[0][-28:]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
    ms = json.loads(open(f[:-4] + ".json").read().strip().splitlines()[-1])["ms_per_step"]
    print(n, "ms/step", round(ms, 4))
names = sorted({k for t in tabs.values() for k in t}, key=lambda k: -tabs.get("base", {}).get(k, 0))
print("kernel".ljust(30) + "".join(n[:10].rjust(11) for n in tabs))
for k in names:
    print(k.ljust(30) + "".join(f"{tabs[n].get(k, float('nan')):11.1f}" for n in tabs))
PY
