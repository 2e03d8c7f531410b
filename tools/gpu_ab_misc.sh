# exact-order GPU tests (default, then the one-wave draws forced), then same-box env-knob A/Bs:
# the V2 exact q2 grid (c5x), the V1 exact fused bucket count (c5v1x), the last-occurrence
# workgroup size (c2)
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/misc; mkdir -p $O
PSS_V2X_Q2_XCD=1 PSS_V1X_FUSED_COUNT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "exact" --timeout 300 --timeout-method thread > $O/pytest_exact.txt 2>&1
PSS_V2X_Q2_XCD=1 PSS_V1X_FUSED_COUNT=1 PSS_V1X_DRAWS_WG=0 PSS_V2X_DRAWS_WG=0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "exact" --timeout 300 --timeout-method thread > $O/pytest_exact_wave_forced.txt 2>&1
mkdir -p $O/q2 $O/fcount
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py c5v1x > $O/fcount/cur_c5v1x_$i.json 2> /dev/null
  PSS_V1X_FUSED_COUNT=1 timeout -k 10 300 python tools/bench_configs.py c5v1x > $O/fcount/alt_c5v1x_$i.json 2> /dev/null
done
PSS_V1X_FUSED_COUNT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5v1x -o run -- python3 tools/bench_configs.py c5v1x > $O/stats_c5v1x.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py c5x > $O/q2/cur_c5x_$i.json 2> /dev/null
  PSS_V2X_Q2_XCD=1 timeout -k 10 300 python tools/bench_configs.py c5x > $O/q2/alt_c5x_$i.json 2> /dev/null
done
PSS_V2X_Q2_XCD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_c5x -o run -- python3 tools/bench_configs.py c5x > $O/stats_c5x.log 2>&1
bash tools/gpu_ab_env.sh misc/nt512 c2 PSS_V2_LASTOCC_NT=512
echo done
