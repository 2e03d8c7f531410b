#!/bin/bash
# the MT round-size / window-margin variants of build/stamp_mt_* (tools/stamp_mt.hip), twice each
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/mt_ab; rm -rf $O; mkdir -p $O
for i in 1 2; do for v in r8sd6 r8sd4 r4sd4 r6sd4 r10sd4; do
  echo "== $v" >> $O/stamp.txt
  timeout -k 10 120 ./build/stamp_mt_$v >> $O/stamp.txt 2>&1 || exit $?
done; done
echo done
