set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu $T > gpurun_out/r03_gpu_tests.txt 2>&1 || { tail -60 gpurun_out/r03_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r03_gpu_tests.txt
V=${V:-r03_v1}
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > gpurun_out/${V}_cfg3.json 2> gpurun_out/${V}_cfg3.err || { tail -30 gpurun_out/${V}_cfg3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 5 --cpu-baseline 0 > gpurun_out/${V}_cfg2.json 2> gpurun_out/${V}_cfg2.err || { tail -30 gpurun_out/${V}_cfg2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/${V}_cfg4.json 2> gpurun_out/${V}_cfg4.err || { tail -30 gpurun_out/${V}_cfg4.err; exit 1; }
python - <<P
import json
for f in ["${V}_cfg3", "${V}_cfg2", "${V}_cfg4"]:
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, round(d["value"]), "fps", round(d["ms_per_step"], 4), "ms", d["roofline"]["kernel"], round(d["roofline"]["avg_ms"], 4), d["kernels_ms"])
P
