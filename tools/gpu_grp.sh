#!/bin/bash
# grouped-pool round: device Feistel check, the grouped / big-pool parity tests, C5 bench
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 60 ./tools/check_feistel > gpurun_out/chk.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "large_pool or c5 or cpu_mode or streams_match or lookahead or wide" > gpurun_out/grp_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py --workload c5 --steps 50 --no-cpu-baseline --no-latency > gpurun_out/c5_$i.json 2>/dev/null
done
echo ok
