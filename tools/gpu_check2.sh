#!/bin/bash
# full -m gpu suite + C2 (twice) and C5 benches, C2 kernel stats (quick confirmation of a change)
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/chk; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 50 --no-cpu-baseline --no-latency > $O/c2_$i.json 2>/dev/null
done
timeout -k 10 120 python bench.py --workload c5 --steps 50 --no-cpu-baseline --no-latency > $O/c5.json 2>/dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-latency > $O/stats_c2.log 2>&1
echo done
