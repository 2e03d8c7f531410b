#!/bin/bash
# Same-box A/B of one workload: the in-tree library against build/head (HEAD's csrc) and
# build/r02 (round 2's), three interleaved runs each; optional -m gpu suite first (--tests).
# usage: tools/gpu_ab3.sh <workload> <tag> [--tests]     outputs: gpurun_out/ab_<tag>/
set -e
cd "$GRAFT_REPO_ROOT"; W=$1; O=gpurun_out/ab_$2; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
if [ "$3" = "--tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
fi
B="python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload $W"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/new_$i.json 2> $O/new_$i.err
  PSS_LIB=$GRAFT_REPO_ROOT/build/head/libpss.so timeout -k 10 200 $B > $O/head_$i.json 2> $O/head_$i.err
  if [ -f build/r02/libpss.so ]; then PSS_LIB=$GRAFT_REPO_ROOT/build/r02/libpss.so timeout -k 10 200 $B > $O/r02_$i.json 2> $O/r02_$i.err; fi
done
echo done
