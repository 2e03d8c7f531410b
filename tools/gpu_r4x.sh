# the shared-state ordering event (SharedUse, one record per call on V1 / grouped / non-lookahead
# paths) without the system-scope fence, same-box against the default: C2 V1, C5, C2
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/shev
for r in 1 2 3; do
  for n in base2 shnf; do
    for w in c2v1 c5 c2; do
      PSS_LIB=build/ab/$n/libpss.so timeout -k 10 200 python3 bench.py --workload $w --steps 200 --no-cpu-baseline --no-latency --no-exact > gpurun_out/shev/${n}_${w}_$r.json 2>> gpurun_out/shev/err.txt
    done
  done
done
