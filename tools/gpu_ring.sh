set -e
export TMPDIR=/tmp
O=gpurun_out/ring; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_handoff.py tests/test_gpu_streams.py > $O/tests.log 2>&1
for i in 1 2; do timeout -k 10 150 python tools/prof_handoff.py > $O/h$i.json 2>&1; done
timeout -k 10 200 python bench.py --workload c3 --steps 20 --no-cpu-baseline --no-exact > $O/c3.json 2>/dev/null
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/prof_handoff.py --cfg c2v2 > $O/tr.json 2> $O/tr.err
echo ok
