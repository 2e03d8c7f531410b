#!/bin/bash
# A/B of V1 window workgroup shapes on the C2 files (bench_configs c2v1) + V1 GPU parity tests
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in 256 512 1024; do
  PSS_V1_NT=$v timeout -k 10 100 python tools/bench_configs.py c2v1 2>/dev/null > gpurun_out/v1_$v.json
  PSS_V1_NT=$v timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -q -k "oracle_twin and 1" --timeout 120 --timeout-method thread > gpurun_out/v1t_$v.log 2>&1
done
echo done
