#!/bin/bash
# Round-3 GPU pass, in two parts (each well inside one gpurun call):
#   part a: full -m gpu suite, smoke, the default bench line (CPU baseline, latency, data path,
#           exact-order figures), bench lines of c5 / c2v1 / c3, rocprofv3 kernel stats of
#           c2 / c5 / c2v1, the 2-process same-GPU rehearsal of the multi-GPU path
#   part b: counter passes (tools/pmc_kernel.sh) of c2 / c5 / c2v1, exact-order stats
# usage: tools/gpu_round3.sh a|b          outputs: gpurun_out/r03/
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r03; mkdir -p $O; export TMPDIR=/tmp
if [ "$1" = "a" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
  timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
  for w in c5 c2v1 c3; do
    timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-latency --no-exact > $O/bench_$w.json 2> $O/bench_$w.err
  done
  for w in c2 c5 c2v1; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o run -- python3 bench.py --workload $w --steps 20 --no-cpu-baseline --no-latency --no-exact > $O/stats_$w.log 2>&1
  done
  PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-latency > $O/rehearse_c2.json 2> $O/rehearse_c2.err
else
  for w in c2 c5 c2v1; do bash tools/pmc_kernel.sh $w r03/pmc_$w > /dev/null; done
  bash tools/gpu_exact.sh > /dev/null
fi
echo done
