#!/bin/bash
# Counters of one workload's kernels: one rocprofv3 --pmc pass per counter set (the gfx950 slot
# limits: 8 SQ, 4 TCC -- FETCH_SIZE and WRITE_SIZE in separate passes, 2 GRBM), each under its
# own kill timer, then a --kernel-trace --stats run of the same bench.
# usage: tools/pmc_kernel.sh <workload> <tag>      (summarise: tools/pmc_table.py gpurun_out/<tag>)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
W=${1:-c2}; T=${2:-$W}
mkdir -p gpurun_out/$T
B="python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-exact"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU" \
         "WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/$T/pmc_$i -o run -- $B > gpurun_out/$T/pmc_$i.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats -o run -- python3 bench.py --workload $W --steps 20 --no-cpu-baseline --no-latency --no-exact > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
echo done
