#!/bin/bash
# GPU-box profiling pass: integer op rates (ubench_int) and SQ PMC passes over the C2 bench.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
true || timeout -k 10 120 ./build/ubench_int > gpurun_out/ubench_int.txt 2>&1
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc1 -o run -- $B > gpurun_out/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc2 -o run -- $B > gpurun_out/pmc2.log 2>&1
echo done
