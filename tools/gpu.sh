#!/bin/bash
# One parametrised recipe for GPU-box runs (replaces the per-experiment tools/gpu_r4*.sh scripts).
# Usage (on the box, from the repo root):   bash tools/gpu.sh TAG STEP [STEP ...]
# Every step runs under its own time limit; the first failing step ends the run (no retries).
#   tests[:K]          pytest -m gpu [-k K]                 -> gpurun_out/TAG_tests.txt
#   smoke              __graft_entry__.smoke()               -> gpurun_out/TAG_smoke.txt
#   ab:C:R:L1,L2,..    R alternations of bench.py --config C over libraries (cur = the in-tree
#                      libgsr.so, NAME = build_var/libgsr_NAME.so), kernel times printed
#   pmc:C[:LIB]        tools/pmc_config.sh passes of config C -> gpurun_out/pmc_cfgC/*.csv
#   trace:C            rocprofv3 --kernel-trace --stats of bench.py --config C
#   bench:C            the full bench line of config C (CPU baseline, dPSNR)
# BENCH_EXTRA (env) is appended to every bench.py command line of ab/pmc/trace/bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
X=${BENCH_EXTRA:-}
withlib() {  # LIB cmd...: run cmd with GSR_LIBRARY pointing at build_var/libgsr_LIB.so (cur: in-tree)
  local L=$1; shift
  if [ "$L" = cur ]; then (unset GSR_LIBRARY; "$@"); else GSR_LIBRARY="$PWD/build_var/libgsr_$L.so" "$@"; fi
}
show() {  # file label
  python3 -c "
import json; d = json.loads(open('$1').read().strip().splitlines()[-1])
k = d.get('kernels_ms', {})
print('$2', round(d['value'], 1), round(d['ms_per_step'], 4), 'ms', k)"
}
steps() { case $1 in 4) echo "--steps 8 --warmup 2";; 5) echo "--steps 20 --warmup 3";; *) echo "--steps 40 --warmup 5";; esac; }
for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  case $kind in
    tests)
      k=(); [ -n "$a" ] && k=(-k "$a")
      timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "${k[@]}" tests \
        > gpurun_out/${TAG}_tests.txt 2>&1 \
        || { grep -E "FAIL|Error|error" gpurun_out/${TAG}_tests.txt | head -20; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
      tail -1 gpurun_out/${TAG}_tests.txt ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.txt ;;
    ab)
      for r in $(seq 1 "$b"); do
        for L in ${c//,/ }; do
          f=gpurun_out/${TAG}_ab_c${a}_${L}_$r.json
          withlib "$L" timeout -k 10 300 python3 -u bench.py --config "$a" $(steps "$a") \
            --cpu-baseline 0 --psnr 0 $X > "$f" 2> "$f.err" || { tail -20 "$f.err"; exit 1; }
          show "$f" "c$a $L #$r"
        done
      done ;;
    pmc)
      withlib "${b:-cur}" timeout -k 10 600 bash tools/pmc_config.sh "${TAG#r}" "$a" $X \
        > gpurun_out/${TAG}_pmc_cfg$a.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_cfg$a.log; exit 1; }
      python3 tools/pmc_summary.py gpurun_out/pmc_cfg$a/${TAG}_pmc_*.csv | grep -E "raster|proj" || true ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace_cfg$a -o run \
        -- python3 -u bench.py --config "$a" $(steps "$a") --cpu-baseline 0 --psnr 0 $X \
        > gpurun_out/${TAG}_trace_cfg$a.json 2> gpurun_out/${TAG}_trace_cfg$a.err \
        || { tail -20 gpurun_out/${TAG}_trace_cfg$a.err; exit 1; }
      echo "trace cfg$a done" ;;
    bench)
      st=""; [ "$a" = 4 ] && st="--steps 10 --warmup 3"
      timeout -k 10 400 python3 -u bench.py --config "$a" $st $X > gpurun_out/${TAG}_cfg$a.json \
        2> gpurun_out/${TAG}_cfg$a.err || { tail -30 gpurun_out/${TAG}_cfg$a.err; exit 1; }
      python3 -c "
import json; d = json.load(open('gpurun_out/${TAG}_cfg$a.json'))
r = d['roofline']
print('cfg$a', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', r.get('kernel'), round(r.get('avg_ms', 0), 4),
      'frac', round(r['frac'], 4), 'traffic', r.get('traffic'), 'cpu', (d.get('cpu_baseline') or {}).get('value'),
      'dpsnr', (d.get('dpsnr') or {}).get('dpsnr_db'), d.get('kernels_ms'))" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
