#!/bin/bash
# round 4: config 3 A/B of the 3D pair backward (build_var p3d) vs the shipped 4-wave kernel,
# 4 alternations, then one rocprofv3 kernel-stats pass each
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['ms_per_step'],4), d['kernels_ms']['raster3d_bwd'])"; }
for v in new p3d new p3d new p3d new p3d; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 3 --cpu-baseline 0 --psnr 0 > gpurun_out/r4t_c3_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 3 --cpu-baseline 0 --psnr 0 > gpurun_out/r4t_c3_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4t_c3_$v.json "c3 $v"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4t_prof_new -o run -- python bench.py --config 3 --cpu-baseline 0 --psnr 0 > /dev/null 2>&1 || exit 1
GSR_LIBRARY=$PWD/build_var/libgsr_p3d.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4t_prof_p3d -o run -- python bench.py --config 3 --cpu-baseline 0 --psnr 0 > /dev/null 2>&1 || exit 1
for v in new p3d; do f=$(ls gpurun_out/r4t_prof_$v/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/r4t_prof_$v/run_kernel_stats.csv); grep -E "raster_bwd" $f | cut -c1-160; done
