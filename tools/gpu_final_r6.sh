#!/bin/bash
# Round-6 final pass, in parts (each under gpurun's 1200 s limit):
#   part a: the whole -m gpu suite, smoke, the default bench line, C5 / C2 V1 / C3 bench lines
#   part b: rocprofv3 --kernel-trace --stats of the C2 / C5 / C2 V1 benches + the hand-off trace
#   part c: counter passes (tools/pmc_kernel.sh) of C2 and C5, hand-off counters
# usage: bash tools/gpu_final_r6.sh <a|b|c>   (outputs under gpurun_out/final6/)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/final6; mkdir -p $O; export TMPDIR=/tmp
step() {   # step <limit s> <log> <cmd...>: a signal / timeout ends the pass
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2> $O/$log.err; local rc=$?
  echo "$log rc=$rc" >> $O/rc.txt
  case $rc in 124|134|137|139) echo "ended by signal/timeout rc=$rc ($log)"; exit $rc ;; esac
  return 0
}
case $1 in
  a)
    step 900 pytest_gpu.txt python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    step 150 smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
    step 300 bench_c2.json python bench.py
    step 200 bench_c5.json python bench.py --workload c5 --no-cpu-baseline
    step 200 bench_c2v1.json python bench.py --workload c2v1 --no-cpu-baseline
    step 300 bench_c3.json python bench.py --workload c3 --steps 20 --no-cpu-baseline
    ;;
  b)
    for w in c2 c5 c2v1; do
      step 200 stats_$w.json rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o run -- \
        python3 bench.py --workload $w --steps 40 --no-cpu-baseline --no-latency --no-exact
    done
    step 300 handoff_trace.json rocprofv3 --kernel-trace --stats --output-format csv -d $O/handoff -o run -- \
      python3 tools/prof_handoff.py
    ;;
  c)
    step 400 pmc_c2.txt bash tools/pmc_kernel.sh c2 final6/pmc_c2
    step 400 pmc_c5.txt bash tools/pmc_kernel.sh c5 final6/pmc_c5
    ;;
  *) echo "usage: $0 a|b|c"; exit 2 ;;
esac
echo done
