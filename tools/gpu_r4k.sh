#!/bin/bash
# exact V2: global merge writing from registers, last level writing the pool2 ranks / the ids itself:
# against HEAD's build
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4k; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x -k "exact or golden" > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/rc.txt; stop $rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh r4k/gm build/ab/gm0/libpss.so c5x c2x; stop $?
echo done >> $O/rc.txt
