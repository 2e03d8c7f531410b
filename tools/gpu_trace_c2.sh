# kernel timelines of the default C2 bench, with and without the epoch lookahead (gaps between replays)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace/$n -o $n -- python3 bench.py --steps 40 --no-cpu-baseline --no-latency --no-exact > gpurun_out/trace/${n}_bench.json 2> gpurun_out/trace/${n}_err.txt
}
run la PSS_V2_LOOKAHEAD=1
run nola PSS_V2_LOOKAHEAD=0
