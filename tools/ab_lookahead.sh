#!/bin/bash
# A/B of the V2 epoch lookahead: off / side stream at the least priority / at the greatest,
# interleaved, C2 bench line each.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-latency --steps 100"
for i in 1 2 3; do
PSS_V2_LOOKAHEAD=0 timeout -k 10 120 $B > gpurun_out/ab_off$i.json 2> gpurun_out/ab_off$i.err
timeout -k 10 120 $B > gpurun_out/ab_lo$i.json 2> gpurun_out/ab_lo$i.err
PSS_V2_LOOKAHEAD_PRIO=hi timeout -k 10 120 $B > gpurun_out/ab_hi$i.json 2> gpurun_out/ab_hi$i.err
done
echo done
