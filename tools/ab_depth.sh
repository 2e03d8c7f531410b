#!/bin/bash
# Epoch lookahead depth A/B (PSS_V2_LOOKAHEAD_DEPTH 1 / 2) on the C2 bench line, interleaved;
# plus the host-step probe (no per-kernel events) at each depth.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-latency --steps 200"
for i in 1 2 3; do
for d in 1 2; do
PSS_V2_LOOKAHEAD_DEPTH=$d timeout -k 10 120 $B > gpurun_out/dep${d}_$i.json 2> gpurun_out/dep.err
done
done
for d in 1 2; do PSS_V2_LOOKAHEAD_DEPTH=$d timeout -k 10 120 python -u tools/host_step.py >> gpurun_out/dep_host.log 2>&1; done
echo done
