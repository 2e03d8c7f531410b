#!/bin/bash
# parity tests of the V2 kernels, then a same-box A/B against build/libpss_head.so
# usage: tools/gpu_test_ab.sh <workload> <tag>
set -e
cd "$GRAFT_REPO_ROOT"; W=${1:-c5}; T=${2:-ab}
mkdir -p gpurun_out/ab_$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_$T/pytest_gpu.txt 2>&1
bash tools/gpu_ab_lib.sh $W build/libpss_head.so $T
