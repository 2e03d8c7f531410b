#!/bin/bash
# Split exact V2 draws (pss_v2split.h): parity subset, cold C5 exact split vs workgroup form, and a
# kernel trace of the cold split epochs.
#   usage: tools/gpu_split.sh <outdir> [tests] [timing] [prof]
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O; export TMPDIR=/tmp
for what in "$@"; do
  case $what in
  tests) timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread \
           -k "big_pool_exact_order or c5_pool_exact or (bench_shape and c5)" > $O/tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.txt; exit 1; } ;;
  timing) for i in 1 2; do
      timeout -k 10 200 env PSS_EXACT_LOOKAHEAD=0 python tools/bench_configs.py c5x > $O/cold_split_$i.json 2> $O/cold_split_$i.err || exit 1
      timeout -k 10 200 env PSS_EXACT_LOOKAHEAD=0 PSS_EXACT_SPLIT=0 python tools/bench_configs.py c5x > $O/cold_wg_$i.json 2> $O/cold_wg_$i.err || exit 1
    done ;;
  timingv1) for i in 1 2; do
      timeout -k 10 200 env PSS_EXACT_LOOKAHEAD=0 python tools/bench_configs.py c5v1x > $O/cold_v1split_$i.json 2> $O/cold_v1split_$i.err || exit 1
      timeout -k 10 200 env PSS_EXACT_LOOKAHEAD=0 PSS_EXACT_SPLIT=0 python tools/bench_configs.py c5v1x > $O/cold_v1wg_$i.json 2> $O/cold_v1wg_$i.err || exit 1
    done ;;
  profv1) PSS_EXACT_LOOKAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profv1 -o run -- \
          python3 tools/bench_configs.py c5v1x > $O/profv1.log 2>&1 || { echo "prof rc=$?"; exit 1; } ;;
  prof) PSS_EXACT_LOOKAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
          python3 tools/bench_configs.py c5x > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; } ;;
  proflib:*) n=${what#proflib:}; PSS_LIB=build/ab/$n/libpss.so PSS_EXACT_LOOKAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
          --output-format csv -d $O/prof_$n -o run -- python3 tools/bench_configs.py c5x > $O/prof_$n.log 2>&1 || { echo "prof rc=$?"; exit 1; } ;;
  runlib:*) n=${what#runlib:}; PSS_LIB=build/ab/$n/libpss.so PSS_EXACT_LOOKAHEAD=0 timeout -k 10 200 \
          python3 tools/bench_configs.py c5x > $O/run_$n.log 2>&1 || { echo "run rc=$?"; exit 1; } ;;
  esac
done
echo done
