#!/bin/bash
# Build libpss.so from another commit's csrc into build/ab/<name>/ (same-box A/B through PSS_LIB):
#   bash tools/build_ref_variant.sh <name> <git-ref> [-DFLAG ...]
set -e
cd "$(dirname "$0")/.."
name=$1; ref=$2; shift 2
S=build/ab/$name/src; O=build/ab/$name; rm -rf $O; mkdir -p $S $O/obj
git archive "$ref" partiallyshuffledistributedsampler_amd/csrc include | tar -x -C $S
cd $S/partiallyshuffledistributedsampler_amd/csrc
for f in pss_kernels.hip pss_v2.hip pss_v2grp.hip pss_v1exact.hip pss_v2exact.hip pss_runtime.cpp pss_cpu.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c -o ../../../obj/$f.o $f &
done
wait
cd ../../..
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libpss.so obj/*.o
rm -rf obj src
echo built build/ab/$name/libpss.so
