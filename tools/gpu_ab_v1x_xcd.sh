set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/xcdv1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "exact" --timeout 300 --timeout-method thread > $O/pytest_exact.txt 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py c5v1x > $O/cur_c5v1x_$i.json 2> $O/cur_$i.err
  PSS_V1X_XCD=0 timeout -k 10 300 python tools/bench_configs.py c5v1x > $O/alt_c5v1x_$i.json 2> $O/alt_$i.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/bench_configs.py c5v1x > $O/stats.log 2>&1
echo done
