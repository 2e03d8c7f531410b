"""TEST INFRASTRUCTURE ONLY -- Python side of the CPU oracle (see pss_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker.  The product package never imports it.

Contents:
  * ctypes bindings of oracle/_build/libpss_oracle.so (built by oracle/Makefile);
  * `RefHistory`: restatement of the reference's stateful init_iter bookkeeping --
    cumulative file-order shuffles (V1:116-117,122-125 / V2:143-144,149-152), V1's cumulative
    block shuffle (V1:118-121), V2's reset-then-shuffle blocks and old/new start (V2:135-148);
  * `ref_batches`: restatement of the reference __next__ mapping/grouping semantics
    (V1:178-259, V2:181-254) on top of an id stream: lazy exclusive scan, reflection,
    grouping by first appearance, the `tmp_count == 1` StopIteration quirk;
  * `rank_id_ranges` / `partition_segments`: a rank's id ranges (V1:158-163, V2:110-114,135-138)
    cut at the shuffled files' exclusive prefix sums (V1:181-214) -- the checker of pss_partition.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libpss_oracle.so")
_lib = None

I64P = ctypes.POINTER(ctypes.c_int64)
I32P = ctypes.POINTER(ctypes.c_int32)
U32P = ctypes.POINTER(ctypes.c_uint32)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "pss_oracle.c"))):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_mt_new.restype = ctypes.c_void_p
        L.orc_mt_free.argtypes = [ctypes.c_void_p]
        L.orc_mt_u32.argtypes = [ctypes.c_void_p]
        L.orc_mt_u32.restype = ctypes.c_uint32
        L.orc_mt_seed_i64.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.orc_mt_seed_words.argtypes = [ctypes.c_void_p, U32P, ctypes.c_int64]
        L.orc_mt_randbelow.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.orc_mt_randbelow.restype = ctypes.c_uint64
        L.orc_mt_shuffle_i64.argtypes = [ctypes.c_void_p, I64P, ctypes.c_int64]
        L.orc_seeded_shuffle_i32.argtypes = [ctypes.c_int64, I32P, ctypes.c_int64]
        L.orc_num_samples.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.orc_num_samples.restype = ctypes.c_int64
        L.orc_v1_exact_stream.argtypes = [ctypes.c_int64] * 5 + [ctypes.c_int, ctypes.c_int64, I64P]
        L.orc_v1_exact_stream.restype = ctypes.c_int64
        L.orc_v2_exact_stream.argtypes = [ctypes.c_int64] * 7 + [I64P]
        L.orc_v2_exact_stream.restype = ctypes.c_int64
        L.orc_v2_exact_prefix.argtypes = [ctypes.c_int64] * 7 + [I64P]
        L.orc_v2_exact_prefix.restype = ctypes.c_int64
        L.orc_v2_exact_stream_rs.argtypes = [ctypes.c_int64] * 7 + [I64P]
        L.orc_v2_exact_stream_rs.restype = ctypes.c_int64
        L.orc_philox4x32.argtypes = [U32P, ctypes.c_uint64, U32P]
        L.orc_mix64.argtypes = [ctypes.c_uint64]
        L.orc_mix64.restype = ctypes.c_uint64
        L.orc_epoch_key.argtypes = [ctypes.c_uint64, ctypes.c_int64]
        L.orc_epoch_key.restype = ctypes.c_uint64
        L.orc_feistel.argtypes = [ctypes.c_uint32, ctypes.c_uint32, U32P]
        L.orc_feistel.restype = ctypes.c_uint32
        L.orc_v1_philox_stream.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [ctypes.c_int64] * 4 + \
            [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, I64P]
        L.orc_v1_philox_stream.restype = ctypes.c_int64
        L.orc_v2_philox_stream.argtypes = [ctypes.c_uint64, ctypes.c_uint32] + [ctypes.c_int64] * 5 + [I64P]
        L.orc_v2_philox_stream.restype = ctypes.c_int64
        L.orc_v2_slots.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, U32P]
        L.orc_map.argtypes = [I64P, ctypes.c_int64, I64P, ctypes.c_int64, I32P, I64P]
        L.orc_digest.argtypes = [I64P, ctypes.c_int64]
        L.orc_digest.restype = ctypes.c_uint64
        L.orc_digest_range.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.orc_digest_range.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _p64(a):
    return a.ctypes.data_as(I64P)


def _p32(a):
    return a.ctypes.data_as(I32P)


def _pu32(a):
    return a.ctypes.data_as(U32P)


# ------------------------------------------------------------------------------------------
# MT19937 (CPython-exact)
# ------------------------------------------------------------------------------------------
class MT:
    def __init__(self, seed=0):
        self._h = ctypes.c_void_p(lib().orc_mt_new())
        self.seed(seed)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_mt_free(self._h)

    def seed(self, a):
        a = abs(int(a))
        if a < 2 ** 63:
            lib().orc_mt_seed_i64(self._h, a)
        else:
            words = []
            while a:
                words.append(a & 0xFFFFFFFF)
                a >>= 32
            w = np.array(words, dtype=np.uint32)
            lib().orc_mt_seed_words(self._h, _pu32(w), len(words))

    def u32(self):
        return lib().orc_mt_u32(self._h)

    def randbelow(self, n):
        return lib().orc_mt_randbelow(self._h, n)

    def shuffle(self, x):
        a = np.ascontiguousarray(x, dtype=np.int64)
        lib().orc_mt_shuffle_i64(self._h, _p64(a), len(a))
        return a


def seeded_shuffle(seed, n_or_arr):
    a = np.arange(n_or_arr, dtype=np.int32) if np.isscalar(n_or_arr) else \
        np.ascontiguousarray(n_or_arr, dtype=np.int32).copy()
    lib().orc_seeded_shuffle_i32(int(seed), _p32(a), len(a))
    return a


def num_samples(N, R):
    return lib().orc_num_samples(N, R)


# ------------------------------------------------------------------------------------------
# init_iter history
# ------------------------------------------------------------------------------------------
class RefHistory:
    """State of one reference sampler across init_iter calls (files order, blocks, start)."""

    def __init__(self, version, num_files, R, rank, N, shuffle=True):
        self.version = version
        self.F = num_files
        self.R = R
        self.rank = rank
        self.N = N
        self.ns = num_samples(N, R)
        self.shuffle = shuffle if version == 1 else True
        self.order = np.arange(num_files, dtype=np.int32)   # positions into dataset.files
        self.blocks = np.arange(R, dtype=np.int32)
        self.start = self.ns * int(self.blocks[rank])        # V1:53 / V2:49
        self.old_start = self.start

    def init_iter(self, epoch):
        self.old_start = self.start
        if self.version == 1:
            if self.shuffle:                                   # V1:113-125
                fid = seeded_shuffle(epoch + 1, self.F)
                self.blocks = seeded_shuffle(epoch + 2, self.blocks)
                self.start = self.ns * int(self.blocks[self.rank])
                self.order = self.order[fid]
        else:                                                  # V2:142-152
            fid = seeded_shuffle(epoch, self.F)
            self.blocks = seeded_shuffle(epoch + 1, np.arange(self.R, dtype=np.int32))
            self.start = self.ns * int(self.blocks[self.rank])
            self.order = self.order[fid]


def v1_exact_stream(epoch, start, ns, B, N, shuffle=True, resume_pos=-1):
    out = np.empty(ns, dtype=np.int64)
    n = lib().orc_v1_exact_stream(epoch, start, ns, B, N, int(bool(shuffle)), resume_pos, _p64(out))
    if n < 0:
        raise IndexError("reference raises IndexError on this resume position")
    return out[:n]


def v2_exact_stream(epoch, old_start, new_start, ns, B, N, skip=0):
    out = np.empty(ns, dtype=np.int64)
    n = lib().orc_v2_exact_stream(epoch, old_start, new_start, ns, B, N, skip, _p64(out))
    return out[:n]


def v2_exact_stream_rs(epoch, old_start, new_start, ns, B, N, skip=0):
    """The same stream as v2_exact_stream with rank-select bitmaps in place of list.remove:
    O(log B) per draw, the checker for pools far beyond the list.remove restatement's reach."""
    out = np.empty(ns, dtype=np.int64)
    n = lib().orc_v2_exact_stream_rs(epoch, old_start, new_start, ns, B, N, skip, _p64(out))
    return out[:n]


def v2_exact_prefix(epoch, old_start, new_start, ns, B, N, limit):
    out = np.empty(limit, dtype=np.int64)
    n = lib().orc_v2_exact_prefix(epoch, old_start, new_start, ns, B, N, limit, _p64(out))
    return out[:n]


# ------------------------------------------------------------------------------------------
# Philox twin
# ------------------------------------------------------------------------------------------
def epoch_key(seed, epoch):
    return lib().orc_epoch_key(seed & 0xFFFFFFFFFFFFFFFF, epoch)


def philox4x32(ctr, key64):
    c = np.array(ctr, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib().orc_philox4x32(_pu32(c), key64, _pu32(o))
    return o


def feistel(x, n, rk):
    r = np.ascontiguousarray(rk, dtype=np.uint32)
    return lib().orc_feistel(x, n, _pu32(r))


def v1_philox_stream(key64, rank, start, ns, B, N, shuffle=True, pos_lo=0, count=None):
    if count is None:
        count = ns - pos_lo
    out = np.empty(max(count, 0), dtype=np.int64)
    n = lib().orc_v1_philox_stream(key64, rank, start, ns, B, N, int(bool(shuffle)), pos_lo,
                                   count, _p64(out))
    return out[:n]


def v2_philox_stream(key64, rank, old_start, new_start, ns, B, N):
    out = np.empty(ns, dtype=np.int64)
    lib().orc_v2_philox_stream(key64, rank, old_start, new_start, ns, B, N, _p64(out))
    return out


def v2_slots(key64, rank, P1, T):
    out = np.empty(max(T, 1), dtype=np.uint32)
    lib().orc_v2_slots(key64, rank, P1, T, _pu32(out))
    return out[:T]


def map_ids(prefix, ids):
    prefix = np.ascontiguousarray(prefix, dtype=np.int64)
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    fpos = np.empty(len(ids), dtype=np.int32)
    off = np.empty(len(ids), dtype=np.int64)
    lib().orc_map(_p64(prefix), len(prefix) - 1, _p64(ids), len(ids), _p32(fpos), _p64(off))
    return fpos, off


def rank_id_ranges(version, old_start, new_start, ns, B, N, T=None):
    """The id ranges a rank's epoch draws from, in stream order: V1 its block [new, new + ns)
    (V1:158-163); V2 the first two pools from the previous start [old, old + min(2B, ns))
    (V2:135-138) and the later windows of the new one [new + min(2B, ns), new + ns)
    (V2:110-112).  Each range wraps at N (V1:161-163, V2:113-114) and is clipped to the scanned
    total T (ids past it are reflected by the map, V1:191-196, and own no file segment)."""
    T = N if T is None else T
    if version == 1:
        parts = [(int(new_start), ns)]
    else:
        a = min(2 * B, ns)
        parts = [(int(old_start), a)] + ([(int(new_start) + a, ns - a)] if ns > a else [])
    out = []
    for lo, ln in parts:
        lo %= N
        while ln > 0:
            take = min(N - lo, ln)
            hi = min(lo + take, T)
            if lo < hi:
                out.append((lo, hi))
            ln -= take
            lo = 0
    return out


def partition_segments(version, prefix, old_start, new_start, ns, B, N):
    """(file position, lo, hi) segments of the shuffled files a rank's epoch reads, in stream
    order of its id ranges (rank_id_ranges): each range cut at the exclusive prefix sums of the
    shuffled file order (V1:181-190's past_files_samples, here complete); empty files own no
    segment.  Offsets are within the file, as V1:210-214's `i - past_files_samples[...]`."""
    prefix = np.asarray(prefix, dtype=np.int64)
    F = len(prefix) - 1
    sf, sl, sh = [], [], []
    for a, b in rank_id_ranges(version, old_start, new_start, ns, B, N, int(prefix[-1])):
        f0 = int(np.searchsorted(prefix, a, side="right")) - 1
        f1 = min(int(np.searchsorted(prefix, b - 1, side="right")) - 1, F - 1)
        fs = np.arange(f0, f1 + 1)
        fs = fs[prefix[fs + 1] > prefix[fs]]
        sf.append(fs.astype(np.int32))
        sl.append(np.maximum(a, prefix[fs]) - prefix[fs])
        sh.append(np.minimum(b, prefix[fs + 1]) - prefix[fs])
    if not sf:
        return np.zeros(0, np.int32), np.zeros(0, np.int64), np.zeros(0, np.int64)
    return np.concatenate(sf), np.concatenate(sl), np.concatenate(sh)


def digest(ids):
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    return lib().orc_digest(_p64(ids), len(ids))


def digest_range(lo, hi):
    return lib().orc_digest_range(lo, hi)


def mix64(x):
    return lib().orc_mix64(x & 0xFFFFFFFFFFFFFFFF)


# ------------------------------------------------------------------------------------------
# __next__ mapping/grouping semantics (V1:178-259, V2:181-254)
# ------------------------------------------------------------------------------------------
def ref_batches(stream, bs, files, length_of):
    """Yield per-batch (read_files, per-file offsets) exactly as the reference groups them.

    `files` is the sampler's current (shuffled) file list, `length_of(path)` the length the
    reference would use (files_len entry or reader probe).  Reflection (V1:191-196) appends
    the reflected id to the batch and maps it after the others.  A batch that maps exactly
    one id raises StopIteration (V1:225-226) -- here: generation stops.
    """
    prefix = [0]
    for i in range(0, len(stream), bs):
        indices = [int(x) for x in stream[i:i + bs]]
        read_files, offs = [], []
        tmp = 0
        j = 0
        while j < len(indices):
            bid = indices[j]
            j += 1
            while bid >= prefix[-1] and len(prefix) <= len(files):
                prefix.append(prefix[-1] + length_of(files[len(prefix) - 1]))
            if bid >= prefix[-1]:
                bid = prefix[-1] * 2 - bid
                if bid == prefix[-1]:
                    bid = prefix[-1] - 1
                indices.append(bid)
                continue
            # largest f with prefix[f] <= bid < prefix[f+1]
            lo, hi = 0, len(prefix) - 1
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if prefix[mid] <= bid:
                    lo = mid
                else:
                    hi = mid
            f = lo
            path = files[f]
            tmp += 1
            if path in read_files:
                offs[read_files.index(path)].append(bid - prefix[f])
            else:
                read_files.append(path)
                offs.append([bid - prefix[f]])
        if tmp == 1:
            return
        yield read_files, offs
