#!/bin/bash
# A/B on one box: the in-tree libpss.so against build/libpss_alt.so (PSS_LIB) on one workload
# usage: tools/gpu_ab_lib.sh <workload> <alt .so> <tag>
set -e
cd "$GRAFT_REPO_ROOT"; W=${1:-c5}; ALT=${2:-build/libpss_head.so}; O=gpurun_out/ab_${3:-lib}; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/new_$i.json 2>/dev/null
  PSS_LIB=$GRAFT_REPO_ROOT/$ALT timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/alt_$i.json 2>/dev/null
done
echo done
