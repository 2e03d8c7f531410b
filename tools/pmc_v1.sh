#!/bin/bash
# V1 window kernel counters on the C2 V1 workload (k_v1_lds<8,512>): one rocprofv3 --pmc pass per
# counter set, each under its own kill timer.  Summarise with tools/pmc_table.py --match k_v1.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --workload c2v1 --steps 3 --warmup 1 --no-cpu-baseline --no-latency"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU" \
         "WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcv1_$i -o run -- $B > gpurun_out/pmcv1_$i.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profv1 -o run -- python3 bench.py --workload c2v1 --steps 20 --no-cpu-baseline --no-latency > gpurun_out/bench_v1.json 2> gpurun_out/bench_v1.err
echo done
