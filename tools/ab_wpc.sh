#!/bin/bash
# A/B of the emit waves per CU (PSS_V2_WPC) on the C2 bench
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for w in 0 4; do
  if [ $w = 0 ]; then unset PSS_V2_WPC; else export PSS_V2_WPC=$w; fi
  timeout -k 10 100 python bench.py --no-cpu-baseline --no-latency 2>/dev/null | tail -1 > gpurun_out/wpc_$w.json
done
echo done
