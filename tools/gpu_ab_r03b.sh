#!/bin/bash
# Round-3 A/B: C5 on this build vs the round-2 library (PSS_LIB=build/r02/libpss.so, built from
# 9ba71c5's csrc), and the exact tile decode at 8 vs 16 outputs per thread (PSS_V2X_OUT).
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_r03b; mkdir -p $O; export TMPDIR=/tmp
B="python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload c5"
for i in 1 2; do
  timeout -k 10 200 $B > $O/c5_cur_$i.json 2> $O/c5_cur_$i.err
  PSS_LIB=build/r02/libpss.so timeout -k 10 200 $B > $O/c5_r02_$i.json 2> $O/c5_r02_$i.err
  for o in 8 16; do PSS_V2X_OUT=$o timeout -k 10 200 python tools/bench_configs.py c2x > $O/c2x_o${o}_$i.json 2> $O/c2x_o${o}_$i.err; done
done
echo done
