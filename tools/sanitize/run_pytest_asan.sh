#!/bin/bash
# pytest -m "not gpu" against the ASan + UBSan build of libpss.so (make -C tools/sanitize pylib):
# the clang ASan runtime preloaded into the interpreter, PSS_LIB pointing the ctypes binding at the
# instrumented library.  Leak detection is off (CPython keeps its arenas); ASan/UBSan errors abort.
cd "$(dirname "$0")/../.."
ASAN_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export LD_PRELOAD=$ASAN_RT
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:detect_odr_violation=0:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export PSS_LIB=$PWD/build/sanitize/asan/libpss.so
exec python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
