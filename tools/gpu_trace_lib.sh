#!/bin/bash
# rocprofv3 kernel-trace summary of one bench config under a build_var library (cur: in-tree).
# Usage: tools/gpu_trace_lib.sh TAG CONFIG LIB [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; cfg=$2; lib=$3; shift 3
mkdir -p gpurun_out
if [ "$lib" != cur ]; then export GSR_LIBRARY=$PWD/build_var/libgsr_$lib.so; fi
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace_c${cfg}_$lib -o run \
  -- python3 -u bench.py --config $cfg --steps 10 --warmup 3 --cpu-baseline 0 --psnr 0 "$@" > gpurun_out/${tag}_trace_c${cfg}_$lib.json 2>&1 || exit 1
f=$(find gpurun_out/${tag}_trace_c${cfg}_$lib -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith("void gsr") or r["Name"].startswith("gsr"):
        print(f'{r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1000:9.1f} us')
PY
