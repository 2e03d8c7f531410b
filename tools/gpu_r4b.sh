#!/bin/bash
# round-4 check: the -m gpu suite, the MT round clocks (build/stamp_mt), the exact-order lines
# with kernel stats, and the c2v1 bench line.  Stops at a crash / abort / timeout.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4b; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1"; exit $1 ;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" > $O/rc.txt; stop $rc
timeout -k 10 120 ./build/stamp_mt > $O/stamp_mt.txt 2>&1; stop $?
for c in c5x c5v1x; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- python3 tools/bench_configs.py $c > $O/$c.json 2> $O/$c.err; stop $?
done
timeout -k 10 300 python bench.py --workload c2v1 --steps 50 --no-cpu-baseline --no-latency --no-exact > $O/c2v1.json 2> $O/c2v1.err; stop $?
echo done
