#!/bin/bash
# Round-6 GPU pass: the whole -m gpu suite, smoke, the default bench line, hand-off profile.
#   usage: tools/gpu_r6.sh <outdir>    (outputs under gpurun_out/<outdir>/)
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
step() {   # step <limit s> <log> <cmd...>: a signal / timeout ends the pass
  local lim=$1 log=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$log 2> $O/$log.err; local rc=$?
  echo "$log rc=$rc" >> $O/rc.txt
  case $rc in 124|134|137|139) echo "ended by signal/timeout rc=$rc ($log)"; exit $rc ;; esac
  return 0
}
for s in "${@:2}"; do
  case $s in
    suite) step 900 pytest_gpu.txt python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) step 150 smoke.txt python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step 600 bench_c2.json python bench.py ;;
    bench20) step 600 bench_c2_20.json python bench.py --steps 20 --warmup 5 ;;
    handoff) step 300 handoff.json python tools/prof_handoff.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
