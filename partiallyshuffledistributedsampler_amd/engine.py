"""IndexEngine: one libpss sampler handle plus the torch plumbing around it.

torch is used only for device memory and streams; every index is produced by libpss.so
(include/pss.h): the HIP kernels on a GPU handle, or the library's CPU mode when the engine
is created with device="cpu" (the same counter schedule on host threads, bit-identical to the
GPU; BASELINE configs[0] runs there without a GPU).  A GPU engine never falls back to the CPU:
its device methods raise without a ROCm GPU.
"""
import ctypes

import numpy as np
import torch

from . import _lib

_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)


def _stream_ptr(stream, device):
    if device.type == "cpu":
        return ctypes.c_void_p(0)
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return ctypes.c_void_p(stream.cuda_stream)


def is_cpu(device):
    return device == "cpu" or (isinstance(device, torch.device) and device.type == "cpu")


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("partiallyshuffledistributedsampler_amd needs a ROCm GPU for index "
                           "generation (no CPU fallback)")


class IndexEngine:
    """Device index generator of one sampler configuration (all R logical ranks)."""

    def __init__(self, files_len, total_size, num_replicas, shuffle_buffer, version,
                 shuffle=True, seed=0, device=0, order="counter"):
        """device: a HIP device ordinal (or torch.device("cuda", i)), or "cpu" for the CPU
        mode of the same schedule."""
        lib = _lib.load()
        fl = np.ascontiguousarray(files_len, dtype=np.int64)
        self.num_files = len(fl)
        self.total_size = int(total_size)
        self.num_replicas = int(num_replicas)
        self.shuffle_buffer = int(shuffle_buffer)
        self.version = int(version)
        self.cpu = is_cpu(device)
        if isinstance(device, torch.device) and not self.cpu:
            device = device.index if device.index is not None else 0
        self.device = -1 if self.cpu else int(device)
        h = ctypes.c_void_p()
        _lib.check(lib.pss_create(fl.ctypes.data_as(_i64p), len(fl), self.total_size,
                                  self.num_replicas, self.shuffle_buffer, self.version,
                                  int(bool(shuffle)), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                  self.device, ctypes.byref(h)), "pss_create")
        self._h = h
        ns = ctypes.c_int64()
        _lib.check(lib.pss_num_samples(h, ctypes.byref(ns)), "pss_num_samples")
        self.num_samples = ns.value
        self.epoch = None
        if order != "counter":
            self.set_order_mode(order)

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().pss_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- host-side epoch history ---------------------------------------------------------
    def init_iter(self, epoch):
        _lib.call("pss_init_iter", self._h, int(epoch))
        self.epoch = int(epoch)

    def file_order(self):
        o = np.empty(self.num_files, dtype=np.int32)
        _lib.call("pss_file_order", self._h, o.ctypes.data_as(_i32p))
        return o

    def blocks(self):
        b = np.empty(self.num_replicas, dtype=np.int32)
        _lib.call("pss_blocks", self._h, b.ctypes.data_as(_i32p))
        return b

    def rank_starts(self):
        o = np.empty(self.num_replicas, dtype=np.int64)
        n = np.empty(self.num_replicas, dtype=np.int64)
        _lib.call("pss_rank_starts", self._h, o.ctypes.data_as(_i64p), n.ctypes.data_as(_i64p))
        return o, n

    # ---- device --------------------------------------------------------------------------
    def _dev(self):
        if self.cpu:
            return torch.device("cpu")
        require_gpu()
        return torch.device("cuda", self.device)

    def prepare(self, stream=None):
        d = self._dev()
        _lib.call("pss_prepare", self._h, _stream_ptr(stream, d))

    def generate(self, rank_lo, rank_hi, pos_lo=0, count=None, out=None, stream=None):
        """int64 ids of positions [pos_lo, pos_lo+count) for ranks [rank_lo, rank_hi)."""
        d = self._dev()
        if count is None:
            count = self.num_samples - pos_lo
        count = max(0, int(count))
        nr = rank_hi - rank_lo
        if out is None:
            out = torch.empty((nr, count), dtype=torch.int64, device=d)
        assert out.is_contiguous() and out.dtype == torch.int64 and out.numel() >= nr * count
        _lib.call("pss_generate", self._h, int(rank_lo), int(rank_hi), int(pos_lo), count,
                  ctypes.c_void_p(out.data_ptr()), _stream_ptr(stream, d))
        return out

    def map(self, ids, fpos=None, off=None, stream=None):
        d = self._dev()
        ids = ids.contiguous()
        n = ids.numel()
        if fpos is None:
            fpos = torch.empty(n, dtype=torch.int32, device=d)
        if off is None:
            off = torch.empty(n, dtype=torch.int64, device=d)
        _lib.call("pss_map", self._h, ctypes.c_void_p(ids.data_ptr()), n,
                  ctypes.c_void_p(fpos.data_ptr()), ctypes.c_void_p(off.data_ptr()),
                  _stream_ptr(stream, d))
        return fpos, off

    def generate_mapped(self, rank_lo, rank_hi, pos_lo=0, count=None, stream=None, out=None):
        """(file_pos, offset) int32 tensors [ranks, count] of positions [pos_lo, pos_lo+count):
        the fused hand-off (pss_generate_mapped) -- 8 bytes per id, no int64 id pass.
        out: an optional (file_pos, offset) pair of contiguous int32 tensors to write into."""
        d = self._dev()
        if count is None:
            count = self.num_samples - pos_lo
        count = max(0, int(count))
        nr = rank_hi - rank_lo
        if out is None:
            fpos = torch.empty((nr, count), dtype=torch.int32, device=d)
            off = torch.empty((nr, count), dtype=torch.int32, device=d)
        else:
            fpos, off = out
            for t in (fpos, off):
                if not (t.is_contiguous() and t.dtype == torch.int32 and t.numel() >= nr * count
                        and t.device == d):
                    raise ValueError("generate_mapped: out tensors must be contiguous int32 "
                                     "[ranks, count] on the engine's device")
        _lib.call("pss_generate_mapped", self._h, int(rank_lo), int(rank_hi), int(pos_lo), count,
                  ctypes.c_void_p(fpos.data_ptr()), ctypes.c_void_p(off.data_ptr()),
                  _stream_ptr(stream, d))
        return fpos, off

    def gather(self, data, base_rows, fpos, off, out=None, stream=None):
        """Rows of device-resident files (pss_gather): data [rows, ...] holds every dataset file's
        samples, file f starting at row base_rows[f] (dataset order); returns data rows of the
        (file_pos, offset) pairs, in their order (the on-GPU form of V1:243-248)."""
        d = self._dev()
        fpos = fpos.reshape(-1).contiguous()
        off = off.reshape(-1).to(torch.int32).contiguous()
        base_rows = base_rows.to(device=d, dtype=torch.int64).contiguous()
        assert data.device == d and data.is_contiguous() and fpos.device == d
        n = fpos.numel()
        row_bytes = data[0].numel() * data.element_size() if data.dim() > 0 and data.shape[0] else 0
        if out is None:
            out = torch.empty((n,) + tuple(data.shape[1:]), dtype=data.dtype, device=d)
        _lib.call("pss_gather", self._h, ctypes.c_void_p(data.data_ptr()), row_bytes,
                  ctypes.c_void_p(base_rows.data_ptr()), ctypes.c_void_p(fpos.data_ptr()),
                  ctypes.c_void_p(off.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                  _stream_ptr(stream, d))
        return out

    def partition(self, rank_lo, rank_hi, stream=None):
        """Host arrays (seg_off[n+1], seg_file, seg_lo, seg_hi) of the ranks' file segments."""
        d = self._dev()
        nr = rank_hi - rank_lo
        sp = _stream_ptr(stream, d)
        seg_off = torch.zeros(nr + 1, dtype=torch.int64, device=d)
        null = ctypes.c_void_p(0)
        _lib.call("pss_partition", self._h, rank_lo, rank_hi, ctypes.c_void_p(seg_off.data_ptr()),
                  null, null, null, 0, sp)
        total = int(seg_off[-1].item())
        sf = torch.empty(max(total, 1), dtype=torch.int32, device=d)
        sl = torch.empty(max(total, 1), dtype=torch.int64, device=d)
        sh = torch.empty(max(total, 1), dtype=torch.int64, device=d)
        _lib.call("pss_partition", self._h, rank_lo, rank_hi, ctypes.c_void_p(seg_off.data_ptr()),
                  ctypes.c_void_p(sf.data_ptr()), ctypes.c_void_p(sl.data_ptr()),
                  ctypes.c_void_p(sh.data_ptr()), max(total, 1), sp)
        self.check(stream)
        return (seg_off.cpu().numpy(), sf[:total].cpu().numpy(), sl[:total].cpu().numpy(),
                sh[:total].cpu().numpy())

    def check(self, stream=None):
        d = self._dev()
        _lib.call("pss_check", self._h, _stream_ptr(stream, d))

    EMIT_PATHS = {"auto": 0, "xchg": 1, "probe": 2}

    def set_emit_path(self, path):
        """V2 replay kernel: "auto", "xchg" (one LDS exchange per step) or "probe"."""
        _lib.call("pss_set_emit_path", self._h, self.EMIT_PATHS[path])

    def emit_path(self):
        v = ctypes.c_int32()
        _lib.call("pss_emit_path", self._h, ctypes.byref(v))
        return {0: "cpu", 1: "xchg", 2: "probe"}[v.value]

    ORDER_MODES = {"counter": 0, "exact": 1}

    def set_order_mode(self, mode):
        """Order of ids inside a pool: "counter" (the counter-based schedule, default) or
        "exact" (the reference's own CPython-MT19937 draws: V1 windows shuffled as
        V1:102,114-115,165-171 do, V2's choice / remove / append of V2:96-116 -- the id stream is
        bit-identical to the reference's)."""
        _lib.call("pss_set_order_mode", self._h, self.ORDER_MODES[mode])

    def order_mode(self):
        v = ctypes.c_int32()
        _lib.call("pss_order_mode", self._h, ctypes.byref(v))
        return {0: "counter", 1: "exact"}[v.value]

    def set_lookahead(self, exact_depth=-1, exact_max_bytes=1 << 30, v2_depth=-1):
        """Bounds of the work done ahead of the calls (pss_set_lookahead): exact-order epochs
        drawn ahead (-1: by geometry), the bytes all exact draw slots may hold, V2 passes queued
        ahead (-1: 2, 0: in line).  Results never depend on them."""
        _lib.call("pss_set_lookahead", self._h, int(exact_depth), int(exact_max_bytes), int(v2_depth))

    def workspace_bytes(self):
        """Device bytes the handle holds (tables, workspaces, VAL ring, draw slots)."""
        v = ctypes.c_int64()
        _lib.call("pss_workspace_bytes", self._h, ctypes.byref(v))
        return v.value

    def lookahead_stats(self):
        """{exact_made, exact_used, v2_queued, v2_used} since create."""
        a = (ctypes.c_int64 * 4)()
        _lib.call("pss_lookahead_stats", self._h, a)
        return dict(zip(("exact_made", "exact_used", "v2_queued", "v2_used"), list(a)))

    KERNEL_KINDS = ("scan", "v1_window", "v2_lastocc", "v2_emit", "v2_tail", "map",
                    "partition", "digest")

    def profile(self, enable=True, generation_only=False, every=1):
        """Bracket every launch of this handle with HIP events on its stream (generation_only:
        only the index-generation kernels, two events per timed generate, every `every`-th)."""
        mode = 0 if not enable else (1 + max(1, int(every)) if generation_only else 1)
        _lib.call("pss_profile", self._h, mode)

    def profile_read(self):
        """{kind: (total_ms, launches)} since the last read (synchronises on the events)."""
        n = len(self.KERNEL_KINDS)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        _lib.call("pss_profile_read", self._h, ms, cnt, n)
        return {k: (ms[i], cnt[i]) for i, k in enumerate(self.KERNEL_KINDS) if cnt[i]}


def digest(ids, acc=None, stream=None):
    """acc (1-element int64 tensor holding a uint64 bit pattern, on ids' device) +=
    sum(splitmix64(ids)).  Device ids: one kernel; host ids: the library's host loop."""
    d = ids.device
    ids = ids.contiguous()
    if acc is None:
        acc = torch.zeros(1, dtype=torch.int64, device=d)
    if d.type == "cpu":
        _lib.call("pss_digest_host", ctypes.c_void_p(ids.data_ptr()), ids.numel(),
                  ctypes.c_void_p(acc.data_ptr()))
        return acc
    require_gpu()
    _lib.call("pss_digest", ctypes.c_void_p(ids.data_ptr()), ids.numel(),
              ctypes.c_void_p(acc.data_ptr()), _stream_ptr(stream, d))
    return acc


def digest_range(lo, hi, device, acc=None, stream=None):
    """acc += sum(splitmix64(i)) for i in [lo, hi); device: a GPU ordinal / device or "cpu"."""
    if is_cpu(device):
        if acc is None:
            acc = torch.zeros(1, dtype=torch.int64)
        _lib.call("pss_digest_range_host", int(lo), int(hi), ctypes.c_void_p(acc.data_ptr()))
        return acc
    require_gpu()
    d = torch.device("cuda", device) if isinstance(device, int) else device
    if acc is None:
        acc = torch.zeros(1, dtype=torch.int64, device=d)
    _lib.call("pss_digest_range", int(lo), int(hi), ctypes.c_void_p(acc.data_ptr()),
              _stream_ptr(stream, d))
    return acc


def as_u64(t):
    """Read a 1-element int64 tensor as the uint64 digest it stores."""
    return int(t.item()) & 0xFFFFFFFFFFFFFFFF
