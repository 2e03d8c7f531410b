#!/bin/bash
# Round-3 check of the working tree: the -m gpu suite, then same-box A/B against build/head
# for C5 (k_g_emit), C2 V1 (k_v1_feistel) and C2 exact (c2x).   outputs: gpurun_out/r03ab/
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03ab; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for i in 1 2; do
  for w in c5 c2v1 c2; do
    B="python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload $w"
    timeout -k 10 200 $B > $O/${w}_new_$i.json 2> $O/${w}_new_$i.err
    PSS_LIB=$GRAFT_REPO_ROOT/build/head/libpss.so timeout -k 10 200 $B > $O/${w}_head_$i.json 2> $O/${w}_head_$i.err
  done
  PSS_LIB=$GRAFT_REPO_ROOT/build/exp/libpss.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload c5 > $O/c5_nofeistel_$i.json 2> $O/c5_nofeistel_$i.err
  PSS_V2_PAIR2=1 timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload c2 > $O/c2_pair2_$i.json 2> $O/c2_pair2_$i.err
  timeout -k 10 200 python tools/bench_configs.py c2x > $O/c2x_new_$i.json 2> $O/c2x_new_$i.err
  PSS_LIB=$GRAFT_REPO_ROOT/build/head/libpss.so timeout -k 10 200 python tools/bench_configs.py c2x > $O/c2x_head_$i.json 2> $O/c2x_head_$i.err
  PSS_V2X_OUT=16 timeout -k 10 200 python tools/bench_configs.py c2x > $O/c2x_o16_$i.json 2> $O/c2x_o16_$i.err
done
timeout -k 10 200 python tools/bench_configs.py c5x > $O/c5x_new_1.json 2> $O/c5x_new_1.err
PSS_LIB=$GRAFT_REPO_ROOT/build/head/libpss.so timeout -k 10 200 python tools/bench_configs.py c5x > $O/c5x_head_1.json 2> $O/c5x_head_1.err
echo done
