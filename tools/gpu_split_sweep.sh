#!/bin/bash
# cold C5 exact (V2 and V1) for the in-tree library and build/ab/<variant> libraries, interleaved
#   usage: tools/gpu_split_sweep.sh <outdir> <variant> [<variant> ...]
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for v in cur "$@"; do
    lib=""; [ $v != cur ] && lib=build/ab/$v/libpss.so
    for c in c5x c5v1x; do
      timeout -k 10 200 env PSS_EXACT_LOOKAHEAD=0 ${lib:+PSS_LIB=$lib} python tools/bench_configs.py $c > $O/${v}_${c}_$i.json 2>&1 || exit 1
    done
  done
done
python - "$O" <<'PY'
import glob, json, os, sys, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    v, c, i = os.path.basename(f)[:-5].rsplit("_", 2)
    r[(v, c)].append(json.loads(open(f).read().strip().splitlines()[-1])["ms_per_step"])
for k in sorted(r): print(k, [round(x, 3) for x in r[k]])
PY
