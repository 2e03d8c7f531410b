#!/bin/bash
# One GPU-box check of a change: the full -m gpu suite, then per workload argument a bench line
# (50 steps), and on request rocprofv3 kernel stats of each (--stats) and the host-prologue
# timing (--prologue).  Each step has its own time limit; the first failure ends the script.
# usage: tools/gpu_check.sh [c2|c2v1|c3|c5 ...] [--stats] [--prologue]     outputs: gpurun_out/chk/
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/chk; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
WL=(); STATS=0; PRO=0
for a in "$@"; do
  case $a in --stats) STATS=1 ;; --prologue) PRO=1 ;; *) WL+=("$a") ;; esac
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for w in "${WL[@]}"; do
  timeout -k 10 200 python bench.py --workload $w --steps 50 --no-cpu-baseline --no-latency > $O/$w.json 2> $O/$w.err
  if [ $STATS = 1 ]; then
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o run -- python3 bench.py --workload $w --steps 20 --no-cpu-baseline --no-latency > $O/stats_$w.log 2>&1
  fi
done
if [ $PRO = 1 ]; then timeout -k 10 300 python tools/host_prologue.py > $O/prologue.txt 2>&1; fi
echo done
