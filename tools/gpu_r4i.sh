#!/bin/bash
# same-box A/Bs: exact C5 with the tail draws folded into the workgroup MT launch (current) vs
# the separate tail kernel (8903149); one-shot V1 at 2 / 8 positions per lane vs 4
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4i; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
bash tools/gpu_ab_lib.sh r4i/fold build/ab/prefold/libpss.so c5x; stop $?
bash tools/gpu_ab_lib.sh r4i/v1os2 build/ab/v1os2/libpss.so c2v1; stop $?
bash tools/gpu_ab_lib.sh r4i/v1os8 build/ab/v1os8/libpss.so c2v1; stop $?
echo done >> $O/rc.txt
