# interleaved same-box A/B of one environment knob on one workload:
#   bash tools/gpu_ab_env.sh <name> <workload> VAR=value [VAR=value ...]
set -e
name=$1; wl=$2; shift 2
mkdir -p gpurun_out/$name
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload $wl > gpurun_out/$name/cur_$i.json 2>/dev/null
  env "$@" timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload $wl > gpurun_out/$name/alt_$i.json 2>/dev/null
done
