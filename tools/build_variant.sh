#!/bin/bash
# Build libpss.so with extra compile definitions into build/ab/<name>/ (same-box A/B of a kernel
# variant through PSS_LIB; build/ab travels with gpurun, build/obj does not):
#   bash tools/build_variant.sh <name> -DFLAG=1 [...]
set -e
cd "$(dirname "$0")/../partiallyshuffledistributedsampler_amd/csrc"
name=$1; shift
O=../../build/ab/$name; mkdir -p $O/obj
for f in pss_kernels.hip pss_v2.hip pss_v2grp.hip pss_v1exact.hip pss_v2exact.hip pss_runtime.cpp pss_cpu.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c -o $O/obj/$f.o $f &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $O/libpss.so $O/obj/*.o
rm -rf $O/obj
echo built $O/libpss.so
