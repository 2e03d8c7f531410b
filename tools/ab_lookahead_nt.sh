#!/bin/bash
# With the epoch lookahead on: threads per last-occurrence workgroup (256 / 512 / 1024),
# interleaved, C2 bench line each (the pass co-runs with the replay in the LDS the replay leaves).
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-latency --steps 100"
for i in 1 2 3; do
for nt in 256 512 1024; do
PSS_V2_LASTOCC_NT=$nt timeout -k 10 120 $B > gpurun_out/abnt_${nt}_$i.json 2> gpurun_out/abnt_${nt}_$i.err
done
done
echo done
