#!/bin/bash
# Full measurement pass for the round's record: parity tests, smoke, the bench line (with CPU
# baseline and latency), per-config throughput, kernel-trace stats, WRITE_SIZE / FETCH_SIZE
# passes.  Each GPU step has its own limit; the first failure ends the script.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python -u tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-latency"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- $B > gpurun_out/pmc_w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- $B > gpurun_out/pmc_f.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-latency > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo done
