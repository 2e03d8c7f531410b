# V1 one-shot generation with the ranks' descriptors as kernel arguments (no upload kernel per
# epoch) against HEAD, same box: C2 V1, C2; then the V1 / stream GPU tests on the new build
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/v1rv
for r in 1 2 3; do
  for n in head v1rv; do
    for w in c2v1 c2; do
      PSS_LIB=build/ab/$n/libpss.so timeout -k 10 200 python3 bench.py --workload $w --steps 200 --no-cpu-baseline --no-latency --no-exact > gpurun_out/v1rv/${n}_${w}_$r.json 2>> gpurun_out/v1rv/err.txt
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/v1rv/pytest_gpu.txt 2>&1
