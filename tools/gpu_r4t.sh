#!/bin/bash
# one-shot V1 through the keyed-carry packed Feistel: the GPU suite, then C2 V1 A/B against HEAD
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4t; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1; rc=$?; echo "suite rc=$rc" >> $O/rc.txt; stop $rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_lib.sh r4t/ab build/ab/kc0/libpss.so c2v1; stop $?
echo done >> $O/rc.txt
