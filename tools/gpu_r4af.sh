#!/bin/bash
# round 4: the 2D pair forward at 6 waves per SIMD (build_var f6) vs the shipped 5 -- config 4, same box
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernels_ms']; print('$2', round(d['ms_per_step'],4), {x: k[x] for x in k if 'raster' in x})"; }
for v in new f6 new f6 new f6; do
  case $v in
    new) timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4af_c4_$v.json 2>/dev/null || exit 1 ;;
    *) GSR_LIBRARY=$PWD/build_var/libgsr_$v.so timeout -k 10 300 python bench.py --config 4 --cpu-baseline 0 --psnr 0 --steps 5 --warmup 2 > gpurun_out/r4af_c4_$v.json 2>/dev/null || exit 1 ;;
  esac
  show gpurun_out/r4af_c4_$v.json "c4 $v"
done
