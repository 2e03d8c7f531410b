#!/bin/bash
# C5 change check: grouped-pool GPU tests, two C5 benches, C5 kernel stats
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/c5x; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py --workload c5 --steps 50 --no-cpu-baseline --no-latency > $O/c5_$i.json 2>/dev/null
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python3 bench.py --workload c5 --steps 20 --no-cpu-baseline --no-latency > $O/stats_c5.log 2>&1
echo done
