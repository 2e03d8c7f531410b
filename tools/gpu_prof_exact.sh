#!/bin/bash
# rocprofv3 kernel stats of the exact-order configs, one run per config (c2x, c2v1x, c5x, c5v1x).
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/prof_exact; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for c in c2x c2v1x c5x c5v1x; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- python3 tools/bench_configs.py $c > $O/$c.json 2> $O/$c.err
done
echo done
