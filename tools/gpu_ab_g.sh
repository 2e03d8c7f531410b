# same-box A/B of libpss builds: mapped hand-off (tools/prof_handoff.py, configs $HCFG, default
# c5v2) and, unless NOBENCH=1, the C5 ids bench, interleaved rounds
# usage: bash tools/gpu_ab_g.sh <outdir> name=lib ...   (lib "-" = the in-tree build)
set -e
O=gpurun_out/$1; shift; mkdir -p $O
for i in 1 2 3; do
  for spec in "$@"; do
    n=${spec%%=*}; l=${spec#*=}
    if [ "$l" = "-" ]; then unset PSS_LIB; else export PSS_LIB=$l; fi
    timeout -k 10 150 python tools/prof_handoff.py --cfg ${HCFG:-c5v2} > $O/${n}_h$i.json 2>&1
    if [ "${NOBENCH:-0}" != 1 ]; then
      timeout -k 10 200 python bench.py --workload ${BENCHW:-c5} --steps 100 --no-cpu-baseline --no-latency --no-exact > $O/${n}_b$i.json 2>/dev/null
    fi
  done
done
unset PSS_LIB
echo ok
