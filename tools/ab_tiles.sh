#!/bin/bash
# A/B of the V2 tile length (PSS_V2_TILE_MULT = tile length in pools) on the C2 bench
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in 0 6 4 3; do
  if [ $m = 0 ]; then unset PSS_V2_TILE_MULT; else export PSS_V2_TILE_MULT=$m; fi
  timeout -k 10 100 python bench.py --no-cpu-baseline --no-latency 2>/dev/null | tail -1 > gpurun_out/tile_$m.json
done
echo done
