#!/bin/bash
# A/B of the last-occurrence pass variants on the C2 bench (one line per variant)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "256" "512" "1024"; do
  PSS_V2_LASTOCC_NT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-latency 2>/dev/null | tail -1 > gpurun_out/ab_$v.json
done
echo done
