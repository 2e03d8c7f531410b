#!/bin/bash
# A/B of k_v1_feistel's occupancy and work per wave (c2v1): PSS_V1_PER_WAVE super-blocks of 256
# positions per wave x PSS_V1_WAVES_PER_CU resident waves (an LDS claim), two interleaved passes.
# Outputs under gpurun_out/ab_v1occ/.
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_v1occ; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for cfg in "16 0" "191 8" "96 16" "48 32" "16 8" "32 12"; do
    set -- $cfg
    PSS_V1_PER_WAVE=$1 PSS_V1_WAVES_PER_CU=$2 timeout -k 10 200 python bench.py --workload c2v1 --steps 100 --no-cpu-baseline --no-latency --no-exact > $O/p$1_w$2_$i.json 2> $O/p$1_w$2_$i.err
  done
done
echo done
