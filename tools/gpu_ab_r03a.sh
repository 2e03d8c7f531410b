#!/bin/bash
# Round-3 A/B: C5 grouped replay with / without the straddle path (PSS_G_STRADDLE), and V1's
# resident waves per CU at one round (PSS_V1_WAVES_PER_CU); interleaved, two passes each.
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_r03a; mkdir -p $O; export TMPDIR=/tmp
B="python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact"
for i in 1 2; do
  for v in 1 0; do PSS_G_STRADDLE=$v timeout -k 10 200 $B --workload c5 > $O/c5_st${v}_$i.json 2> $O/c5_st${v}_$i.err; done
  for w in 8 4 12 16 24 32; do PSS_V1_WAVES_PER_CU=$w timeout -k 10 200 $B --workload c2v1 > $O/v1_w${w}_$i.json 2> $O/v1_w${w}_$i.err; done
done
echo done
