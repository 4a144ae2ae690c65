# A/B of two libgsr builds on config 4's one-frame shares (--shard frames --rank-share 8) and a
# single-camera 2D render (the drop-in's call): bash tools/rr_ab.sh LIB_A LIB_B (build_var/libgsr_*.so)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    GSR_LIBRARY=$PWD/build_var/libgsr_$L.so timeout -k 10 200 python3 -u bench.py --config 4 --shard frames --rank-share 8 \
      --steps 5 --warmup 2 > gpurun_out/rr_${L}_$r.json 2> gpurun_out/rr_${L}_$r.err || exit 1
    GSR_LIBRARY=$PWD/build_var/libgsr_$L.so timeout -k 10 200 python3 -u tools/dropin2d_timing.py > gpurun_out/d2_${L}_$r.txt 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/rr_${L}_$r.json').read().strip().splitlines()[-1]); r=d['rank_share']
k=[s['kernels_ms'] for s in r['shares']]
print('$L #$r share', round(r['max_share_ms'],3), 'fwd', round(max(x['raster2d_fwd'] for x in k),3), 'bwd', round(max(x['raster2d_bwd'] for x in k),3))"
    tail -1 gpurun_out/d2_${L}_$r.txt
  done
done
