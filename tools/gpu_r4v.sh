# C2 step with the replay stream's event wait / record removed one at a time (diagnostic builds,
# racy VAL reuse: timing only), same-box against the default build
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/noev2
for r in 1 2 3; do
  for n in base noev nowait norec; do
    PSS_LIB=build/ab/$n/libpss.so timeout -k 10 200 python3 bench.py --steps 200 --no-cpu-baseline --no-latency --no-exact > gpurun_out/noev2/${n}_$r.json 2>> gpurun_out/noev2/err.txt
  done
done
