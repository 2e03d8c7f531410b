#!/bin/bash
# the exact-order GPU tests (+ knob children) and the split timing (V2, V1)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "exact or knob or golden or c5 or split" > $O/suite.txt 2>&1 || { echo "suite rc=$?"; tail -30 $O/suite.txt; exit 1; }
tail -3 $O/suite.txt
bash tools/gpu_split.sh $1 timing timingv1 profv1
