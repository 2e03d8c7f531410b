set -e
mkdir -p gpurun_out/sc0
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload c5 > gpurun_out/sc0/cur_$i.json 2>/dev/null
  PSS_LIB=$GRAFT_REPO_ROOT/build/sc0/libpss.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload c5 > gpurun_out/sc0/sc0_$i.json 2>/dev/null
done
