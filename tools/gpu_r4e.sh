#!/bin/bash
# exact-order subset + exact-order kernel stats (after a kernel change)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4e; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1"; exit $1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x -k "exact or golden or knob" > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" > $O/rc.txt; stop $rc
for c in c5x c2x; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- python3 tools/bench_configs.py $c > $O/$c.json 2> $O/$c.err; stop $?
done
echo done
