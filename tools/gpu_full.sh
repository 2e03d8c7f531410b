set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err
echo done
