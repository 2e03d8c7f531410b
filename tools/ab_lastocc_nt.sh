#!/bin/bash
# Interleaved A/B of the last-occurrence workgroup size on the whole C2 step (3 runs each)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 256 512; do
    PSS_V2_LASTOCC_NT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --no-latency 2>/dev/null | tail -1 > gpurun_out/abnt_${v}_$r.json
  done
done
echo done
