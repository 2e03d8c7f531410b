set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for i in 1 2; do
timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-latency --steps 50 > gpurun_out/b_on$i.json 2> gpurun_out/b_on$i.err
PSS_V2_LOOKAHEAD=0 timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-latency --steps 50 > gpurun_out/b_off$i.json 2> gpurun_out/b_off$i.err
done
echo done
