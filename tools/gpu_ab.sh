set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
summ() { python -c "
import json; d = json.load(open('$1'))
print('$2', round(d['value']), 'fps', round(d['ms_per_step'], 4), 'ms', d['kernels_ms'])"; }
(cd build_var/r02 && timeout -k 10 200 python -u bench.py --steps 50 --cpu-baseline 0 --psnr 0 > ../../gpurun_out/ab_r02_cfg3.json 2> ../../gpurun_out/ab_r02_cfg3.err) || { tail -20 gpurun_out/ab_r02_cfg3.err; exit 1; }
summ gpurun_out/ab_r02_cfg3.json r02_cfg3
timeout -k 10 200 python -u bench.py --steps 50 --cpu-baseline 0 --psnr 0 --graph 0 --capacity exact > gpurun_out/ab_r03_exact_cfg3.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
summ gpurun_out/ab_r03_exact_cfg3.json r03_exact_eager_cfg3
timeout -k 10 200 python -u bench.py --steps 50 --cpu-baseline 0 --psnr 0 --graph 0 > gpurun_out/ab_r03_bounded_cfg3.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
summ gpurun_out/ab_r03_bounded_cfg3.json r03_bounded_eager_cfg3
timeout -k 10 200 python -u bench.py --steps 50 --cpu-baseline 0 --psnr 0 > gpurun_out/ab_r03_graph_cfg3.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
summ gpurun_out/ab_r03_graph_cfg3.json r03_graph_cfg3
(cd build_var/r02 && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ../../gpurun_out/prof_ab_r02 -o run -- python -u bench.py --steps 30 --cpu-baseline 0 --psnr 0 > /dev/null 2>&1) || { echo rocprof r02 failed; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab_r03 -o run -- python -u bench.py --steps 30 --cpu-baseline 0 --psnr 0 > /dev/null 2>&1 || { echo rocprof r03 failed; exit 1; }
find gpurun_out/prof_ab_r02 gpurun_out/prof_ab_r03 -name "*kernel_stats.csv" | head
