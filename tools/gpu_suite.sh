#!/bin/bash
# the whole -m gpu suite and smoke() on the current tree -> gpurun_out/suite/
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/suite; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/rc.txt
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?" >> $O/rc.txt
