#!/bin/bash
# exact V2 decode tiles: the first three merge levels in registers for 64-bit entries too (C5):
# the exact-order GPU tests, then C5 exact A/B against HEAD's build
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4l; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x -k "exact or golden" > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/rc.txt; stop $rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh r4l/t build/ab/t0/libpss.so c5x; stop $?
echo done >> $O/rc.txt
