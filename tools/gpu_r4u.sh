# C2 replay-stream gaps with and without the replay stream's event wait/record (diagnostic build,
# racy VAL reuse: timing only): kernel traces + same-box bench A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/noev
for n in base noev; do
  lib=build/ab/$n/libpss.so
  PSS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/noev/$n -o $n -- python3 bench.py --steps 40 --no-cpu-baseline --no-latency --no-exact > gpurun_out/noev/${n}_trace_bench.json 2> gpurun_out/noev/${n}_trace_err.txt
done
for r in 1 2 3; do
  for n in base noev; do
    PSS_LIB=build/ab/$n/libpss.so timeout -k 10 200 python3 bench.py --steps 200 --no-cpu-baseline --no-latency --no-exact > gpurun_out/noev/${n}_$r.json 2>> gpurun_out/noev/err.txt
  done
done
