#!/bin/bash
# Same-box A/B: the in-tree libpss.so against another build of it (PSS_LIB), three interleaved
# bench runs each on one workload; --tests runs the full -m gpu suite first.
# usage: tools/gpu_ab_lib.sh <workload> <alt .so> <tag> [--tests]      outputs: gpurun_out/ab_<tag>/
# (alt build: git archive <rev> ... | tar -x -C /tmp/x; make -C .../csrc OBJDIR=... OUT=<alt .so>)
set -e
cd "$GRAFT_REPO_ROOT"; W=${1:-c2}; ALT=${2:-build/libpss_head.so}; O=gpurun_out/ab_${3:-lib}
rm -rf $O; mkdir -p $O
if [ "$4" = "--tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
fi
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/new_$i.json 2>/dev/null
  PSS_LIB=$GRAFT_REPO_ROOT/$ALT timeout -k 10 120 python bench.py --workload $W --steps 50 --no-cpu-baseline --no-latency > $O/alt_$i.json 2>/dev/null
done
echo done
