#!/bin/bash
# exact-order subset of the suite at the new MT defaults, the MT clocks, then counter passes of
# the exact-order workloads (tools/pmc_cmd.sh: 4 rocprofv3 --pmc passes each)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4d; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1"; exit $1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x -k "exact or golden or knob" > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" > $O/rc.txt; stop $rc
timeout -k 10 120 ./build/stamp_mt > $O/stamp_mt.txt 2>&1; stop $?
for c in c5x c5v1x c2x; do
  bash tools/pmc_cmd.sh r4d/pmc_$c python3 tools/bench_configs.py $c > /dev/null 2>&1; stop $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- python3 tools/bench_configs.py $c > $O/$c.json 2> $O/$c.err; stop $?
done
echo done
