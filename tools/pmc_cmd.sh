#!/bin/bash
# Counters of any command's kernels: the same four rocprofv3 --pmc passes as tools/pmc_kernel.sh
# (gfx950 slot limits: 8 SQ, 4 TCC -- FETCH_SIZE and WRITE_SIZE in separate passes), each under
# its own kill timer.   usage: tools/pmc_cmd.sh <tag> <command ...>    outputs: gpurun_out/<tag>/
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU" \
         "WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/$T/pmc_$i -o run -- "$@" > gpurun_out/$T/pmc_$i.log 2>&1
done
echo done
