#!/bin/bash
# one-shot V1 workgroups running 2 / 4 iterations of 1024 positions behind one prologue: the GPU
# suite under the 2-iteration build, then C2 V1 A/B of both against 1
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4q; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
PSS_LIB=build/ab/it2/libpss.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_it2.txt 2>&1; rc=$?; echo "it2 suite rc=$rc" >> $O/rc.txt; stop $rc
bash tools/gpu_ab_lib.sh r4q/it2 build/ab/it2/libpss.so c2v1; stop $?
bash tools/gpu_ab_lib.sh r4q/it4 build/ab/it4/libpss.so c2v1; stop $?
echo done >> $O/rc.txt
