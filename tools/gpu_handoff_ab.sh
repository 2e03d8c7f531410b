set -e
mkdir -p gpurun_out/ho
for i in 1 2; do
  for L in cur head r02; do
    if [ $L = cur ]; then LIB=""; else LIB=$GRAFT_REPO_ROOT/build/$L/libpss.so; fi
    PSS_LIB=$LIB timeout -k 10 120 python -c "
import sys, json; sys.path.insert(0, '.')
import bench
print(json.dumps(bench.handoff_figures(0)))" > gpurun_out/ho/${L}_$i.json 2> gpurun_out/ho/${L}_$i.err
  done
done
