#!/bin/bash
# A/B of the V1 pair-store layout (PSS_V1_PAIRS=1, default) against 8-byte stores (=0), c2v1
# bench lines interleaved three times.  Outputs under gpurun_out/ab_v1/.
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_v1; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for v in 0 1; do
    PSS_V1_PAIRS=$v timeout -k 10 200 python bench.py --workload c2v1 --steps 100 --no-cpu-baseline --no-latency > $O/pairs${v}_$i.json 2> $O/pairs${v}_$i.err
  done
done
echo done
