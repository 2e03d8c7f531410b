# exact-order parity (default dispatch, then the workgroup draws forced everywhere) and an
# interleaved A/B of the exact-order configs against a baseline library:
#   bash tools/gpu_ab_exact.sh <name> <baseline libpss.so> [configs...]
set -e
cd "$GRAFT_REPO_ROOT"; name=$1; base=$2; shift 2; O=gpurun_out/$name; mkdir -p $O
CF=("$@"); [ ${#CF[@]} -eq 0 ] && CF=(c5x c5v1x)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "exact" --timeout 300 --timeout-method thread > $O/pytest_exact.txt 2>&1
PSS_V2X_DRAWS_WG=1 PSS_V1X_DRAWS_WG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "exact" --timeout 300 --timeout-method thread > $O/pytest_exact_wg_forced.txt 2>&1
for i in 1 2; do
  for c in "${CF[@]}"; do
    timeout -k 10 300 python tools/bench_configs.py $c > $O/cur_${c}_$i.json 2> $O/cur_${c}_$i.err
    PSS_LIB=$base timeout -k 10 300 python tools/bench_configs.py $c > $O/base_${c}_$i.json 2> $O/base_${c}_$i.err
  done
done
echo done
