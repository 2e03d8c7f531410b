#!/bin/bash
# MT draw workgroups of 12 / 16 waves (11 / 15 consumers) against 10: the exact-order tests under
# each build, then C5 exact V2 / V1 A/B
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4n; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
for v in mt1024 mt768; do
  PSS_LIB=build/ab/$v/libpss.so timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x -k "exact or golden" > $O/pytest_$v.txt 2>&1; rc=$?; echo "$v pytest rc=$rc" >> $O/rc.txt; stop $rc
  [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_ab_lib.sh r4n/ab1024 build/ab/mt1024/libpss.so c5x c5v1x; stop $?
bash tools/gpu_ab_lib.sh r4n/ab768 build/ab/mt768/libpss.so c5x; stop $?
echo done >> $O/rc.txt
