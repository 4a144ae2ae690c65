set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # name lib config chunk_entries
  GSR_LIBRARY=$2 timeout -k 10 200 python -u bench.py --config $3 --steps ${STEPS:-8} --warmup 3 --cpu-baseline 0 --psnr 0 --chunk-entries $4 > gpurun_out/units_$1.json 2> gpurun_out/units_$1.err || { tail -20 gpurun_out/units_$1.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/units_$1.json'))
k = d['kernels_ms']; print('$1', round(d['ms_per_step'], 4), 'ms', {n: k[n] for n in k if 'raster' in n or 'project' in n})"
}
L0=pose-splatter_amd/gsr/lib/libgsr.so
L5=build_var/libgsr_v5.so
run c4_u128 $L0 4 128,128
run c4_u512 $L0 4 128,512
run c4_u512_v5 $L5 4 128,512
run c4_u256 $L0 4 128,256
run c4_u256_v5 $L5 4 128,256
run c4_u1024_v5 $L5 4 128,1024
STEPS=30 run c3_u128 $L0 3 128,512
STEPS=30 run c3_u256 $L0 3 256,512
STEPS=30 run c3_u256_v5 $L5 3 256,512
