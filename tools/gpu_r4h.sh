#!/bin/bash
# replay pacing against a whole tile: per-wave stamps (beside the pass / alone) of the current
# source and of HEAD, then C2 / C3 bench A/B against the round-3 pacing build
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4h; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
for m in pass alone; do
  timeout -k 10 120 ./build/stamp_v2x $m > $O/stamp_cur_$m.txt 2>&1; stop $?
  timeout -k 10 120 ./build/stamp_v2x_base $m > $O/stamp_base_$m.txt 2>&1; stop $?
done
bash tools/gpu_ab_lib.sh r4h/ab build/ab/pace_nvalid/libpss.so c2 c3; stop $?
echo done >> $O/rc.txt
