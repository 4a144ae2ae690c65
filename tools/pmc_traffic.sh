#!/bin/bash
# On the GPU box: HBM traffic counters of the bench kernels, one rocprofv3 pass per counter
# (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: they cannot share a pass), merged into one CSV
# that bench.py reads for roofline.traffic.  Usage: tools/pmc_traffic.sh OUT.csv [bench args]
# (OUT.csv under gpurun_out/ comes back from the GPU box; copy it to profiles/r01_pmc_counters.csv)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=$1; shift
mkdir -p gpurun_out/pmc_t
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_t/$c -o run -- \
    python3 bench.py --cpu-baseline 0 --steps 3 --warmup 1 --traffic-csv "" "$@" > gpurun_out/pmc_t/$c.log 2>&1
done
python3 - "$out" <<'PY'
import glob, sys
files = sorted(glob.glob("gpurun_out/pmc_t/*/*counter_collection.csv"))
lines = []
for i, f in enumerate(files):
    rows = open(f).read().splitlines()
    lines += rows if i == 0 else rows[1:]
open(sys.argv[1], "w").write("\n".join(lines) + "\n")
print(sys.argv[1], len(lines) - 1, "rows from", files)
PY
