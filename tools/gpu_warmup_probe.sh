set -o pipefail
for r in 1 2; do for W in 5 200; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup $W --cpu-baseline 0 --psnr 0 > gpurun_out/wu_${W}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/wu_${W}_$r.json').read().strip().splitlines()[-1]); print('W=$W #$r', round(d['value']), round(d['ms_per_step'],4), d['roofline']['avg_ms'], d.get('kernels_ms'))"
done; done
