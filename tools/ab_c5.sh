#!/bin/bash
# Interleaved A/B of the big-pool emit's XCD grouping on C5 (PSS_V2BIG_XCD), 2 runs each
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    PSS_V2BIG_XCD=$v timeout -k 10 120 python tools/bench_configs.py c5 2>/dev/null | tail -1 > gpurun_out/abc5_${v}_$r.json
  done
done
echo done
