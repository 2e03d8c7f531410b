# same-box A/B of libpss builds on the exact order at C3 (tools/prof_exact_c3.py), interleaved
# usage: bash tools/gpu_ab_x.sh <outdir> name=lib ...   (lib "-" = the in-tree build)
set -e
O=gpurun_out/$1; shift; mkdir -p $O
for i in 1 2 3; do
  for spec in "$@"; do
    n=${spec%%=*}; l=${spec#*=}
    if [ "$l" = "-" ]; then unset PSS_LIB; else export PSS_LIB=$l; fi
    timeout -k 10 200 python tools/prof_exact_c3.py > $O/${n}_x$i.json 2>&1
    timeout -k 10 200 python tools/prof_exact_c3.py --cfg c2 --epochs 20 > $O/${n}_c2_$i.json 2>&1
  done
done
unset PSS_LIB
echo ok
