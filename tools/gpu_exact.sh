#!/bin/bash
# Exact-order measurements on one GPU box: tools/bench_configs.py lines of the exact orders
# (c2x, c2v1x, c5x, c5v1x) and rocprofv3 --kernel-trace --stats of each.  Outputs under
# gpurun_out/exact/.  usage: tools/gpu_exact.sh [configs...]
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/exact; mkdir -p $O; export TMPDIR=/tmp
CF=("$@"); [ ${#CF[@]} -eq 0 ] && CF=(c2x c2v1x c5x c5v1x)
for c in "${CF[@]}"; do
  timeout -k 10 300 python tools/bench_configs.py $c > $O/$c.json 2> $O/$c.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- python3 tools/bench_configs.py $c > $O/stats_$c.log 2>&1
done
echo done
