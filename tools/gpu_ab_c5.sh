#!/bin/bash
# C5 bench lines (k_g_emit), three passes; outputs under gpurun_out/ab_c5/<tag>_<i>.json
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_c5; mkdir -p $O; export TMPDIR=/tmp
T=${1:-cur}
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --workload c5 --steps 100 --no-cpu-baseline --no-latency --no-exact > $O/${T}_$i.json 2> $O/${T}_$i.err
done
echo done
