#!/bin/bash
# On the GPU box: the rocprofv3 PMC passes bench.py reads for roofline.traffic / .valu, for ONE
# config.  One pass per counter group (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: they cannot
# share a pass; the SQ counters fit in two passes of <= 8 SQ counters).
# Usage: tools/pmc_config.sh ROUND CONFIG [extra bench args]
#   -> gpurun_out/pmc_cfgC/rROUND_pmc_traffic_cfgC.csv, rROUND_pmc_sq_cfgC_p{1,2}.csv
#   (copy them to profiles/; bench.py picks the newest round of its own config)
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
round=$1; cfg=$2; shift 2
out=gpurun_out/pmc_cfg$cfg
mkdir -p $out
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o run -- \
    python3 bench.py --config $cfg --cpu-baseline 0 --psnr 0 --steps 3 --warmup 1 $EXTRA > $out/$name.log 2>&1
}
EXTRA="$*"
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU
run sq2 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE
python3 - "$out" "$round" "$cfg" <<'PY'
import glob, sys
out, rnd, cfg = sys.argv[1:]
def merge(parts, dst):
    lines = []
    for i, f in enumerate(parts):
        rows = open(f).read().splitlines()
        lines += rows if i == 0 else rows[1:]
    open(dst, "w").write("\n".join(lines) + "\n")
    print(dst, len(lines) - 1, "rows")
cc = lambda d: sorted(glob.glob(f"{out}/{d}/*counter_collection.csv"))
merge(cc("fetch") + cc("write"), f"{out}/r{rnd}_pmc_traffic_cfg{cfg}.csv")
merge(cc("sq1"), f"{out}/r{rnd}_pmc_sq_cfg{cfg}_p1.csv")
merge(cc("sq2"), f"{out}/r{rnd}_pmc_sq_cfg{cfg}_p2.csv")
PY
