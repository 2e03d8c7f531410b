# kernel timelines of the default C2 bench under lookahead variants (gaps between replays)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace/$n -o $n -- python3 bench.py --steps 40 --no-cpu-baseline --no-latency --no-exact > gpurun_out/trace/${n}_bench.json 2> gpurun_out/trace/${n}_err.txt
}
run d2 PSS_V2_LOOKAHEAD_DEPTH=2
run d1 PSS_V2_LOOKAHEAD_DEPTH=1
run hi PSS_V2_LOOKAHEAD_PRIO=h
