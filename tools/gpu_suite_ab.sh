#!/bin/bash
# The -m gpu suite, then (unless it died by a fault or a time limit) a same-box A/B of the
# in-tree library against another build on bench workloads:
#   bash tools/gpu_suite_ab.sh <name> <other libpss.so> <workload> [...]
# A failing test does not stop the A/B; a crash / abort / timeout (rc 124, 134, 137, 139) does.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/suite; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc" > $O/pytest_rc.txt
case $rc in 124|134|137|139) echo "suite ended by signal/timeout rc=$rc"; exit $rc ;; esac
[ -n "$1" ] && bash tools/gpu_ab_lib.sh "$@"
echo done
