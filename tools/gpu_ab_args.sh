#!/bin/bash
# Same-box A/B of bench.py argument sets on one workload, three interleaved runs each.
# usage: tools/gpu_ab_args.sh <workload> <tag> "<args1>" "<args2>" ...     outputs: gpurun_out/aba_<tag>/
set -e
cd "$GRAFT_REPO_ROOT"; W=$1; O=gpurun_out/aba_$2; shift 2; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  j=0
  for a in "$@"; do
    j=$((j+1))
    timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency $a > $O/v${j}_$i.json 2>/dev/null
  done
done
echo done
