#!/bin/bash
# fused-map check: parity + sampler GPU tests, then the mapped kernels' durations
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/map; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_sampler.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hof -o run -- python3 tools/prof_handoff.py > $O/hof.log 2>&1
echo done
