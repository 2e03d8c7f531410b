#!/bin/bash
# Round-2 GPU pass: full -m gpu suite, smoke, benches of every workload, rocprofv3 kernel stats
# of the default bench, separate WRITE_SIZE / FETCH_SIZE passes, and the 2-process same-GPU
# rehearsal of the multi-GPU path (c2 weak, c3 strong).  Outputs under gpurun_out/r02/.
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r02; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err
for w in c5 c2v1 c3; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --no-cpu-baseline --no-latency > $O/bench_$w.json 2> $O/bench_$w.err
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-latency > $O/stats_c2.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5 -o run -- python3 bench.py --workload c5 --steps 20 --no-cpu-baseline --no-latency > $O/stats_c5.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > $O/pmc_write.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > $O/pmc_fetch.log 2>&1
PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-latency > $O/rehearse_c2.json 2> $O/rehearse_c2.err
PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --workload c3 --steps 5 --warmup 2 --no-latency > $O/rehearse_c3.json 2> $O/rehearse_c3.err
echo done
