# Interleaved same-box A/B of the in-tree library against another build (e.g. HEAD's csrc built
# into build/base with `git archive HEAD partiallyshuffledistributedsampler_amd/csrc include`):
#   bash tools/gpu_ab_lib.sh <name> <other libpss.so> <workload|config> [...]
# bench.py workloads (c2, c5, c2v1, c3) run 100 steps; anything else is a tools/bench_configs.py
# config (c2x, c5x, ...).  Outputs gpurun_out/<name>/{cur,alt}_<w>_<i>.json; tools/ab_summary.py
set -e
cd "$GRAFT_REPO_ROOT"; name=$1; lib=$2; shift 2; O=gpurun_out/$name; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for w in "$@"; do
    case $w in
      c2|c5|c2v1|c3) cmd="python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload $w" ;;
      *) cmd="python tools/bench_configs.py $w" ;;
    esac
    timeout -k 10 300 $cmd > $O/cur_${w}_$i.json 2> $O/cur_${w}_$i.err
    PSS_LIB=$lib timeout -k 10 300 $cmd > $O/alt_${w}_$i.json 2> $O/alt_${w}_$i.err
  done
done
echo done
