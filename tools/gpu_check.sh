#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.  Each GPU step has its
# own time limit; the first failure ends the script.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-latency > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo done
