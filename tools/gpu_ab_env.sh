#!/bin/bash
# Same-box A/B of run-time knobs: the in-tree libpss.so under each environment setting, three
# interleaved bench runs each on one workload (and the PSS_LIB build given as "lib:<path>").
# usage: tools/gpu_ab_env.sh <workload> <tag> <setting>...     e.g. "X=1" "lib:build/libpss_head.so" "-"
#        ("-" = no change)                                          outputs: gpurun_out/abe_<tag>/
set -e
cd "$GRAFT_REPO_ROOT"; W=$1; O=gpurun_out/abe_$2; shift 2; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  j=0
  for v in "$@"; do
    j=$((j+1))
    case $v in
      -) timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/v${j}_$i.json 2>/dev/null ;;
      lib:*) PSS_LIB=$GRAFT_REPO_ROOT/${v#lib:} timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/v${j}_$i.json 2>/dev/null ;;
      *) env $v timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/v${j}_$i.json 2>/dev/null ;;
    esac
  done
done
echo done
