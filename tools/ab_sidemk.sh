#!/bin/bash
# A/B: per-kernel events on the lookahead stream (PSS_PROFILE_LOOKAHEAD=1) or not, C2 bench line.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-latency --steps 200"
for i in 1 2 3; do
PSS_PROFILE_LOOKAHEAD=1 timeout -k 10 120 $B > gpurun_out/sm_on$i.json 2> gpurun_out/sm.err
timeout -k 10 120 $B > gpurun_out/sm_off$i.json 2> gpurun_out/sm.err
done
echo done
