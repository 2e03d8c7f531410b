#!/bin/bash
# Round-4 GPU pass, in two parts (each well inside one gpurun call):
#   part a: full -m gpu suite, smoke, the default bench line (CPU baseline, latency, hand-off,
#           exact-order figures), bench lines of c5 / c2v1 / c3, rocprofv3 kernel stats of
#           c2 / c5 / c2v1, the 2-process same-GPU rehearsal of the multi-GPU path
#   part b: counter passes (tools/pmc_kernel.sh) of c2 / c5 / c2v1, exact-order stats
# A crash / abort / timeout ends the part.   usage: tools/gpu_round4.sh a|b   outputs: gpurun_out/r04/
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
stop() { case $1 in 0) ;; 124|134|137|139) echo "ended by signal/timeout rc=$1"; exit $1 ;; *) echo "step rc=$1" ;; esac; }
if [ "$1" = "a" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; stop $?
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; stop $?
  timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err; stop $?
  for w in c5 c2v1 c3; do
    timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-latency --no-exact > $O/bench_$w.json 2> $O/bench_$w.err; stop $?
  done
  for w in c2 c5 c2v1; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o run -- python3 bench.py --workload $w --steps 20 --no-cpu-baseline --no-latency --no-exact > $O/stats_$w.log 2>&1; stop $?
  done
  PSS_BENCH_SAME_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-latency > $O/rehearse_c2.json 2> $O/rehearse_c2.err; stop $?
else
  for w in c2 c5 c2v1; do bash tools/pmc_kernel.sh $w r04/pmc_$w > /dev/null 2>&1; stop $?; done
  for c in c2x c2v1x c5x c5v1x; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- python3 tools/bench_configs.py $c > $O/$c.json 2> $O/$c.err; stop $?
  done
fi
echo done
