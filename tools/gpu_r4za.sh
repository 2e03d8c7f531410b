# k_v1_os computing its window's round keys itself (-DPSS_V1OS_INKEYS: no k_v1_keys kernel per
# epoch) against HEAD (build/ab/v1rv), same box: C2 V1; then the V1 GPU tests on the variant
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/inkeys
for r in 1 2 3; do
  for n in v1rv inkeys; do
    PSS_LIB=build/ab/$n/libpss.so timeout -k 10 200 python3 bench.py --workload c2v1 --steps 200 --no-cpu-baseline --no-latency --no-exact > gpurun_out/inkeys/${n}_c2v1_$r.json 2>> gpurun_out/inkeys/err.txt
  done
done
PSS_LIB=build/ab/inkeys/libpss.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "v1 or V1 or stream" --timeout 300 --timeout-method thread > gpurun_out/inkeys/pytest_gpu.txt 2>&1
