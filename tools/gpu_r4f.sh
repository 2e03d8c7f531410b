#!/bin/bash
# exact subset (tail draws folded into the workgroup draws), c5x without the profiler, then the
# one-shot V1 lane-width variants against the in-tree library
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4f; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1"; exit $1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x -k "exact or golden or knob" > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" > $O/rc.txt; stop $rc
for i in 1 2 3; do timeout -k 10 300 python tools/bench_configs.py c5x > $O/c5x_$i.json 2> $O/c5x_$i.err; stop $?; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5x -o run -- python3 tools/bench_configs.py c5x > $O/c5x_prof.json 2> $O/c5x_prof.err; stop $?
bash tools/gpu_ab_lib.sh r4f/v1os2 build/ab/v1os2/libpss.so c2v1; stop $?
bash tools/gpu_ab_lib.sh r4f/v1os8 build/ab/v1os8/libpss.so c2v1; stop $?
echo done
