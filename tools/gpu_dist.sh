set -o pipefail
cd $GRAFT_REPO_ROOT
# two ranks on the one GPU of the box (gloo): rehearses the N>1 code paths of bench.py
for shard in views units sparse; do
  args="--shard $shard"; [ "$shard" = "sparse" ] && args="--shard units --exchange sparse"
  GSR_DIST_BACKEND=gloo GSR_SAME_DEVICE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 $args > gpurun_out/dist_$shard.json 2> gpurun_out/dist_$shard.err || { tail -30 gpurun_out/dist_$shard.err; exit 1; }
  python -c "
import json; d = json.loads(open('gpurun_out/dist_$shard.json').read().strip().splitlines()[-1])
print('$shard', d['n_gpus'], round(d['value']), d['scaling'], d.get('launch_mode'), round(d.get('value_eager', 0)), d['config']['parallelism'][:90])"
done
GSR_DIST_BACKEND=gloo GSR_SAME_DEVICE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29518 bench.py --config 4 --gpus 2 --steps 3 --warmup 1 > gpurun_out/dist_cfg4.json 2> gpurun_out/dist_cfg4.err || { tail -30 gpurun_out/dist_cfg4.err; exit 1; }
tail -c 300 gpurun_out/dist_cfg4.json
