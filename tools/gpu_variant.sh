#!/bin/bash
# A kernel variant built by tools/build_variant.sh: its parity subset (pytest -k EXPR under
# PSS_LIB), then the same-box A/B against the in-tree library on bench workloads.
#   bash tools/gpu_variant.sh <name> "<pytest -k expr>" <workload> [...]
cd "$GRAFT_REPO_ROOT"; name=$1; expr=$2; shift 2
O=gpurun_out/var_$name; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
PSS_LIB=$PWD/build/ab/$name/libpss.so timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -k "$expr" --timeout 300 --timeout-method thread > $O/pytest_variant.txt 2>&1
rc=$?; echo "variant pytest rc=$rc" > $O/pytest_rc.txt
case $rc in 124|134|137|139) echo "ended by signal/timeout rc=$rc"; exit $rc ;; esac
bash tools/gpu_ab_lib.sh var_$name/ab build/ab/$name/libpss.so "$@"
echo done
