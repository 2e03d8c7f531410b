#!/bin/bash
# bench.py with one epoch in flight against two (--pipeline 2), interleaved on one box
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_pipeline; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for w in c2 c5 c2v1; do
    for p in 1 2; do
      timeout -k 10 300 python bench.py --workload $w --steps 100 --pipeline $p --no-cpu-baseline --no-latency --no-exact > $O/p${p}_${w}_$i.json 2> $O/p${p}_${w}_$i.err || exit $?
    done
  done
done
echo done
