set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/rs
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_handoff.py tests/test_gpu_configs.py > gpurun_out/rs/tests.log 2>&1
timeout -k 10 120 python tools/prof_handoff.py > gpurun_out/rs/handoff.json 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rs/trace -o run -- python3 tools/ab_rank_shared.py > gpurun_out/rs/rs.json 2> gpurun_out/rs/rs.err
echo ok
