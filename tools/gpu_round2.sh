#!/bin/bash
# Round-2 GPU pass: full -m gpu suite, smoke, the default bench line (CPU baseline, latency,
# data path), benches of the other workloads, rocprofv3 kernel stats and counter passes
# (tools/pmc_kernel.sh) of c2 and c5, and the 2-process same-GPU rehearsal of the multi-GPU
# path (c2 weak, c3 strong).  Outputs under gpurun_out/r02/.
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r02; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
for w in c5 c2v1 c3; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-latency > $O/bench_$w.json 2> $O/bench_$w.err
done
for w in c2 c5; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o run -- python3 bench.py --workload $w --steps 20 --no-cpu-baseline --no-latency > $O/stats_$w.log 2>&1
  bash tools/pmc_kernel.sh $w r02/pmc_$w > /dev/null
done
PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-latency > $O/rehearse_c2.json 2> $O/rehearse_c2.err
PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --workload c3 --steps 5 --warmup 2 --no-latency > $O/rehearse_c3.json 2> $O/rehearse_c3.err
echo done
