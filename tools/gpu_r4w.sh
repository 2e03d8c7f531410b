# C2 step with the lookahead events created device-scope (hipEventReleaseToDevice) or without the
# system fence, and (racy, timing only) without the replay stream's events, same-box against the default
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/evfl
for r in 1 2 3; do
  for n in base rdev nosys noev; do
    PSS_LIB=build/ab/$n/libpss.so timeout -k 10 200 python3 bench.py --steps 200 --no-cpu-baseline --no-latency --no-exact > gpurun_out/evfl/${n}_$r.json 2>> gpurun_out/evfl/err.txt
  done
done
