#!/bin/bash
# the C2 replay's super-batch loop unrolled 2 / 4 times (compiler interleave) against 1: C2 / C3 A/B
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4s; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
bash tools/gpu_ab_lib.sh r4s/un2 build/ab/un2/libpss.so c2 c3; stop $?
bash tools/gpu_ab_lib.sh r4s/un4 build/ab/un4/libpss.so c2; stop $?
echo done >> $O/rc.txt
