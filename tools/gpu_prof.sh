#!/bin/bash
# GPU-box profiling pass: SQ / GRBM PMC passes over a short C2 bench (one pass per counter set,
# each under its own kill timer).  Summarise with tools/pmc_table.py.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_LDS" \
         "SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_LEVEL_WAVES SQ_INST_CYCLES_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc$i -o run -- $B > gpurun_out/pmc$i.log 2>&1
done
echo done
