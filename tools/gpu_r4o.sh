#!/bin/bash
# epochs on two streams: the new stream tests, the whole suite, bench --pipeline 2 coverage on
# V1 / V2 / C5, and C2 / C2V1 A/B against HEAD's build (the cross-stream ordering's cost)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4o; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "ended by signal/timeout rc=$1" | tee -a $O/rc.txt; exit $1 ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -v --timeout 250 --timeout-method thread > $O/pytest_streams.txt 2>&1; rc=$?; echo "streams rc=$rc" >> $O/rc.txt; stop $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?; echo "suite rc=$rc" >> $O/rc.txt; stop $rc
for w in c2v1 c2 c5; do
  timeout -k 10 200 python bench.py --workload $w --steps 100 --pipeline 2 --no-cpu-baseline --no-latency --no-exact > $O/p2_$w.json 2> $O/p2_$w.err; stop $?
done
bash tools/gpu_ab_lib.sh r4o/ab build/ab/head0/libpss.so c2 c2v1; stop $?
echo done >> $O/rc.txt
