set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc/p1 -o p1 -- python3 bench.py --cpu-baseline 0 --steps 3 --warmup 1 > gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/p2 -o p2 -- python3 bench.py --cpu-baseline 0 --steps 3 --warmup 1 > gpurun_out/pmc/p2.log 2>&1
