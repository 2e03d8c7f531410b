"""ctypes binding of libpss.so (include/pss.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).  There is no
fallback: if the library is missing or a call fails, an exception is raised.  (The CPU mode,
device="cpu", is part of the same library: PSS_DEVICE_CPU handles.)
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSS_LIB: another build of the library (same-box A/B of kernel variants); default the in-tree one
LIB_PATH = os.environ.get("PSS_LIB") or os.path.join(_HERE, "libpss.so")

PSS_OK = 0
PSS_DEVICE_CPU = -1
_c_i64p = ctypes.POINTER(ctypes.c_int64)
_c_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p
_i32, _i64, _u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64

# name -> (argtypes, restype); kept in sync with include/pss.h (tests check both directions)
SIGNATURES = {
    "pss_last_error": ([], ctypes.c_char_p),
    "pss_abi_version": ([], ctypes.c_int),
    "pss_schedule_version": ([], ctypes.c_int),
    "pss_create": ([_c_i64p, _i64, _i64, _i32, _i64, _i32, _i32, _u64, _i32,
                    ctypes.POINTER(_vp)], ctypes.c_int),
    "pss_destroy": ([_vp], ctypes.c_int),
    "pss_num_samples": ([_vp, _c_i64p], ctypes.c_int),
    "pss_init_iter": ([_vp, _i64], ctypes.c_int),
    "pss_file_order": ([_vp, _c_i32p], ctypes.c_int),
    "pss_blocks": ([_vp, _c_i32p], ctypes.c_int),
    "pss_rank_starts": ([_vp, _c_i64p, _c_i64p], ctypes.c_int),
    "pss_prepare": ([_vp, _vp], ctypes.c_int),
    "pss_generate": ([_vp, _i32, _i32, _i64, _i64, _vp, _vp], ctypes.c_int),
    "pss_map": ([_vp, _vp, _i64, _vp, _vp, _vp], ctypes.c_int),
    "pss_partition": ([_vp, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp], ctypes.c_int),
    "pss_digest": ([_vp, _i64, _vp, _vp], ctypes.c_int),
    "pss_digest_range": ([_i64, _i64, _vp, _vp], ctypes.c_int),
    "pss_check": ([_vp, _vp], ctypes.c_int),
    "pss_profile": ([_vp, _i32], ctypes.c_int),
    "pss_set_emit_path": ([_vp, _i32], ctypes.c_int),
    "pss_emit_path": ([_vp, _c_i32p], ctypes.c_int),
    "pss_set_order_mode": ([_vp, _i32], ctypes.c_int),
    "pss_order_mode": ([_vp, _c_i32p], ctypes.c_int),
    "pss_profile_read": ([_vp, ctypes.POINTER(ctypes.c_double), _c_i64p, _i32], ctypes.c_int),
    "pss_debug_wave_scan": ([_vp, _vp, _i64, _vp], ctypes.c_int),
    "pss_digest_host": ([_vp, _i64, _vp], ctypes.c_int),
    "pss_digest_range_host": ([_i64, _i64, _vp], ctypes.c_int),
    "pss_device": ([_vp, _c_i32p], ctypes.c_int),
    "pss_error_snapshot": ([_vp, _vp, _vp], ctypes.c_int),
    "pss_map_prefix_host": ([_vp, _i64, _vp, _i64, _vp, _vp], ctypes.c_int),
    "pss_generate_mapped": ([_vp, _i32, _i32, _i64, _i64, _vp, _vp, _vp], ctypes.c_int),
    "pss_gather": ([_vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp], ctypes.c_int),
    "pss_set_lookahead": ([_vp, _i32, _i64, _i32], ctypes.c_int),
    "pss_workspace_bytes": ([_vp, _c_i64p], ctypes.c_int),
    "pss_lookahead_stats": ([_vp, _c_i64p], ctypes.c_int),
}

_lib = None


class PSSError(RuntimeError):
    pass


def load():
    """Load libpss.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libpss.so is not built (%s). Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` -- there is no fallback."
            % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (argt, rest) in SIGNATURES.items():
        if os.environ.get("PSS_LIB") and not hasattr(lib, name):
            continue   # (same-box A/B against an older build: entry points it lacks stay unbound)
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rest
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != PSS_OK:
        msg = load().pss_last_error().decode(errors="replace")
        raise PSSError("%s failed (code %d): %s" % (what or "libpss call", rc, msg))


def call(name, *args):
    check(getattr(load(), name)(*args), name)
