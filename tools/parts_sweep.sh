set -o pipefail
# Sweep of the split 2D per-set backward's target workgroups (gsr_set_bwd2d_parts via GSR_BWD2D_PART_WGS, read by gsr/_lib.py):
# config 4 one-frame shares (--shard frames --rank-share 8) and the eight-frame step.  Output: profiles/r05_ab5_bwd2d_parts_sweep.txt
mkdir -p gpurun_out
for t in 1 4608 9216 18432; do
  GSR_BWD2D_PART_WGS=$t timeout -k 10 200 python3 -u bench.py --config 4 --shard frames --rank-share 8 --steps 5 --warmup 2 > gpurun_out/rs_$t.json 2> gpurun_out/rs_$t.err || exit 1
  python3 -c "
import json
d=json.loads(open('gpurun_out/rs_$t.json').read().strip().splitlines()[-1]); r=d['rank_share']
print('share t=$t', round(r['max_share_ms'],3), [round(s['kernels_ms']['raster2d_bwd'],3) for s in r['shares']][:4])"
done
for t in 4608 18432 36864 4608 18432 36864; do
  GSR_BWD2D_PART_WGS=$t timeout -k 10 300 python3 -u bench.py --config 4 --steps 8 --warmup 2 --cpu-baseline 0 --psnr 0 > gpurun_out/c4_$t.json 2> gpurun_out/c4_$t.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c4_$t.json').read().strip().splitlines()[-1]); k=d['kernels_ms']
print('c4 t=$t', round(d['value'],1), round(d['ms_per_step'],3), k['raster2d_bwd'], k['raster2d_fwd'])"
done
