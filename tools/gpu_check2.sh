#!/bin/bash
# full -m gpu suite + one C2 and one C5 bench (quick confirmation of a change)
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/chk; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 120 python bench.py --steps 50 --no-cpu-baseline --no-latency > $O/c2.json 2>/dev/null
timeout -k 10 120 python bench.py --workload c5 --steps 50 --no-cpu-baseline --no-latency > $O/c5.json 2>/dev/null
echo done
