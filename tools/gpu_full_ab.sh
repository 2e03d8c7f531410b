#!/bin/bash
# full -m gpu suite, then same-box A/Bs (C2, C5) against build/libpss_head.so
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/full
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.txt 2>&1
bash tools/gpu_ab_lib.sh c2 build/libpss_head.so h24c2
bash tools/gpu_ab_lib.sh c5 build/libpss_head.so h24c5
