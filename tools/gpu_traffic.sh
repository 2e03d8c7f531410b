#!/bin/bash
# HBM traffic of the bench kernels: WRITE_SIZE and FETCH_SIZE in separate rocprofv3 --pmc passes
# (MI355X_MICROARCH.md: they cannot share a pass), summarised into profiles/pmc_traffic.json by
# tools/pmc_summary.py (run on the CPU side after the merge), plus a kernel-trace stats run.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-latency"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- $B > gpurun_out/pmc_w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- $B > gpurun_out/pmc_f.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-latency > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo done
