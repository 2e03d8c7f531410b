#!/bin/bash
# One parameterised GPU-box pass (replaces the per-experiment gpu_r4*.sh scripts of round 4).
#   usage: tools/gpu_run.sh <outdir> <step> [<step> ...]      outputs: gpurun_out/<outdir>/
# steps (run in order; each under its own time limit; a signal / timeout / abort ends the pass,
# another failure is recorded in rc.txt and the pass goes on):
#   suite              the whole -m gpu suite (tests/, -v, per-test timeout)
#   suite:<expr>       the -m gpu tests selected by pytest -k <expr>
#   smoke              __graft_entry__.smoke()
#   bench              the default bench line (CPU baseline, latency, hand-off, exact order)
#   bench:<w>          bench line of workload w (c2 c5 c2v1 c3), generation figures only
#   stats:<w>          rocprofv3 --kernel-trace --stats of 20 bench steps of workload w
#   xstats:<cfg>       rocprofv3 --kernel-trace --stats of tools/bench_configs.py <cfg> (c2x ...)
#   pmc:<w>            the counter passes of workload w (tools/pmc_kernel.sh)
#   gpus2              bench.py --gpus 2 with no launcher (2 ranks on cuda:0, gloo)
#   ab:<lib>:<w>       3 interleaved runs of bench workload w: in-tree library vs <lib> (PSS_LIB)
#   abx:<lib>:<cfg>    the same for a tools/bench_configs.py config (c2x, c5x, c2v1x, ...)
#   env:<K=V>:<w>      3 interleaved runs of bench workload w: as is vs with K=V
#   envx:<K=V>:<cfg>   the same for a tools/bench_configs.py config
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O; export TMPDIR=/tmp
BN="--no-cpu-baseline --no-latency --no-exact"
run() {   # run <limit s> <log> <cmd...>
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2> $O/$log.err; local rc=$?
  echo "$log rc=$rc" >> $O/rc.txt
  case $rc in 124|134|137|139) echo "ended by signal/timeout rc=$rc ($log)"; exit $rc ;; esac
  return 0
}
for s in "$@"; do
  IFS=: read -r kind a b <<< "$s"
  case $kind in
    suite) if [ -n "$a" ]; then run 700 pytest_${a//[^a-z0-9]/_}.txt python -u -m pytest tests -m gpu -v -k "$a" --timeout 300 --timeout-method thread
           else run 900 pytest_gpu.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; fi ;;
    smoke) run 150 smoke.txt python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) if [ -n "$a" ]; then run 240 bench_$a.json python bench.py --workload $a $BN
           else run 500 bench_c2.json python bench.py; fi ;;
    stats) run 200 stats_$a.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$a -o run -- python3 bench.py --workload $a --steps 20 $BN ;;
    xstats) run 300 xstats_$a.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/xstats_$a -o run -- python3 tools/bench_configs.py $a ;;
    pmc) run 600 pmc_$a.log bash tools/pmc_kernel.sh $a ${O#gpurun_out/}/pmc_$a ;;
    gpus2) run 300 gpus2.json env PSS_BENCH_SAME_GPU=1 python bench.py --gpus 2 --steps 10 --warmup 2 --no-latency --no-exact ;;
    ab) t=$(basename $(dirname $a))
        for i in 1 2 3; do
          run 240 ab_${t}_cur_${b}_$i.json python bench.py --steps 100 --workload $b $BN
          run 240 ab_${t}_alt_${b}_$i.json env PSS_LIB=$a python bench.py --steps 100 --workload $b $BN
        done ;;
    abx) t=$(basename $(dirname $a))
         for i in 1 2 3; do
           run 300 abx_${t}_cur_${b}_$i.json python tools/bench_configs.py $b
           run 300 abx_${t}_alt_${b}_$i.json env PSS_LIB=$a python tools/bench_configs.py $b
         done ;;
    envx) for i in 1 2 3; do
           run 300 envx_cur_${b}_$i.json python tools/bench_configs.py $b
           run 300 envx_alt_${b}_$i.json env "$a" python tools/bench_configs.py $b
         done ;;
    env) for i in 1 2 3; do
           run 240 env_cur_${b}_$i.json python bench.py --steps 100 --workload $b $BN
           run 240 env_alt_${b}_$i.json env "$a" python bench.py --steps 100 --workload $b $BN
         done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
