set -e
cd /root/repo
for lz in 0,1 16384,8192 16384,6144 16384,4096 8192,6144 8192,4096 12288,6144; do
  for c in 5 3; do
    timeout -k 10 100 python bench.py --config $c --cpu-baseline 0 --psnr 0 --steps 20 --lazy $lz > gpurun_out/lz_${c}_${lz}.json 2>/dev/null
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/lz_*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("lz_")[1][:-5], round(d["ms_per_step"], 4), d["kernels_ms"].get("bin_sort"), d["kernels_ms"].get("raster3d_fwd"))
PY
