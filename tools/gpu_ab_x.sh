#!/bin/bash
# Same-box A/B of one tools/bench_configs.py config (e.g. c2x): the in-tree library against
# build/head, three interleaved runs each; optional pytest -k filter of the -m gpu suite first.
# usage: tools/gpu_ab_x.sh <config> <tag> [pytest -k expr]     outputs: gpurun_out/abx_<tag>/
set -e
cd "$GRAFT_REPO_ROOT"; C=$1; O=gpurun_out/abx_$2; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$3" > $O/pytest_gpu.txt 2>&1
fi
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_configs.py $C > $O/new_$i.json 2> $O/new_$i.err
  PSS_LIB=$GRAFT_REPO_ROOT/build/head/libpss.so timeout -k 10 200 python tools/bench_configs.py $C > $O/head_$i.json 2> $O/head_$i.err
done
echo done
