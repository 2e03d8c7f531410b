#!/bin/bash
# The fused hand-off (pss_generate_mapped) under rocprofv3: a kernel trace with --stats over
# tools/prof_handoff.py (C2 V2, C2 V1, C5 V2: 20 epochs after 4 warm-up epochs each) and the
# counter passes of the same driver (3 epochs each: one pass per counter set, the gfx950 slot
# limits -- FETCH_SIZE and WRITE_SIZE in separate passes), each under its own kill timer.
# usage: tools/pmc_handoff.sh <tag>        (outputs under gpurun_out/<tag>/)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-handoff}; mkdir -p gpurun_out/$T
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o run -- \
  python3 tools/prof_handoff.py > gpurun_out/$T/trace.json 2> gpurun_out/$T/trace.err
P="python3 tools/prof_handoff.py --epochs 3"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU" \
         "WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/$T/pmc_$i -o run -- $P > gpurun_out/$T/pmc_$i.log 2>&1
done
echo done
