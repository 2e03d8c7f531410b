#!/bin/bash
# kernel trace of cold C5 exact epochs with the split draws (pss_v2split.h)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 tools/bench_configs.py c5x > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
echo done
