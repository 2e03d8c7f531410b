set -e
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 120 python bench.py --workload c5 --steps 50 --no-cpu-baseline --no-latency > gpurun_out/c5_split_$i.json 2>/dev/null
  PSS_V2_GRP_SPLIT=0 timeout -k 10 120 python bench.py --workload c5 --steps 50 --no-cpu-baseline --no-latency > gpurun_out/c5_inline_$i.json 2>/dev/null
done
bash tools/pmc_kernel.sh c5 pmc_c5
bash tools/pmc_kernel.sh c2v1 pmc_c2v1
bash tools/pmc_kernel.sh c2 pmc_c2
