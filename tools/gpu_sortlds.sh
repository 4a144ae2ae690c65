set -o pipefail
cd $GRAFT_REPO_ROOT
run() {  # name lib config
  GSR_LIBRARY=$2 timeout -k 10 200 python -u bench.py --config $3 --steps ${STEPS:-30} --warmup 3 --cpu-baseline 0 --psnr 0 > gpurun_out/sl_$1.json 2> gpurun_out/sl_$1.err || { tail -20 gpurun_out/sl_$1.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/sl_$1.json'))
k = d['kernels_ms']; print('$1', round(d['ms_per_step'], 4), 'ms', {n: k[n] for n in k if 'bin' in n or 'raster' in n}, d['binning']['max_list'])"
}
L0=pose-splatter_amd/gsr/lib/libgsr.so
for c in 3 5 2; do
  run c${c}_16k $L0 $c
  run c${c}_8k build_var/libgsr_s8192.so $c
  run c${c}_4k build_var/libgsr_s4096.so $c
done
