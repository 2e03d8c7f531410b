#!/bin/bash
# Depth-2 lookahead: default vs 512-thread last-occurrence workgroups vs side stream at the
# greatest priority; C2 bench line, 200 steps, interleaved.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-latency --steps 200"
for i in 1 2; do
timeout -k 10 120 $B > gpurun_out/k2_def_$i.json 2> gpurun_out/k2.err
PSS_V2_LASTOCC_NT=512 timeout -k 10 120 $B > gpurun_out/k2_nt512_$i.json 2> gpurun_out/k2.err
PSS_V2_LOOKAHEAD_PRIO=hi timeout -k 10 120 $B > gpurun_out/k2_hi_$i.json 2> gpurun_out/k2.err
done
echo done
