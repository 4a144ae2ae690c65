#!/bin/bash
# On the GPU box: SQ counter passes (LDS / VALU / waits) of the default library and of each
# build_var/libgsr_*.so on one config, for comparing kernel variants.
# Usage: tools/pmc_variants.sh CONFIG  -> gpurun_out/pmcv/<variant>_{sq1,sq2}/..., summary on stdout
set -e
shopt -s nullglob
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
cfg=${1:-3}
out=gpurun_out/pmcv
mkdir -p $out
pass() {  # variant lib name counters...
  local v=$1 lib=$2 name=$3; shift 3
  GSR_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $out/${v}_$name -o run -- \
    python3 bench.py --config $cfg --cpu-baseline 0 --psnr 0 --steps 3 --warmup 1 > $out/${v}_$name.log 2>&1
}
for lib in pose-splatter_amd/gsr/lib/libgsr.so build_var/libgsr_*.so; do
  v=$(basename "$lib" .so); v=${v#libgsr_}; [ "$v" = libgsr ] && v=base
  pass $v $PWD/$lib sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU
  pass $v $PWD/$lib sq2 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE
done
for d in $out/*_sq1; do
  v=$(basename $d _sq1); echo "== $v"
  python3 tools/pmc_summary.py $out/${v}_sq1/*counter_collection.csv $out/${v}_sq2/*counter_collection.csv | grep -A16 "${KERNEL:-k_raster_bwd}" || true
done
