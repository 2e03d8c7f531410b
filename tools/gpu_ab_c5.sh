#!/bin/bash
# Same-box C5 A/B: this build, this build with PSS_G_STRADDLE=0, and the round-2 library
# (PSS_LIB=build/r02/libpss.so, built from 9ba71c5's csrc), three interleaved runs each.
set -e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab_c5; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
B="python bench.py --steps 100 --no-cpu-baseline --no-latency --no-exact --workload c5"
for i in 1 2 3; do
  timeout -k 10 200 $B > $O/cur_$i.json 2> $O/cur_$i.err
  PSS_G_STRADDLE=0 timeout -k 10 200 $B > $O/nostr_$i.json 2> $O/nostr_$i.err
  PSS_LIB=$GRAFT_REPO_ROOT/build/r02/libpss.so timeout -k 10 200 $B > $O/r02_$i.json 2> $O/r02_$i.err
done
echo done
