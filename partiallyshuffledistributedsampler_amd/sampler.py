"""Drop-in `torch.utils.data.Sampler` facade over the MI355X index engine.

Same constructor, methods, return format and errors as the reference samplers
(V1 = DistributedSamplerViaLocallyShuffle.py, V2 = ...V2.py); index generation and the
id -> (file, offset) map run in libpss.so (engine.py): on the GPU, or in the library's CPU mode
with device="cpu".  The file reader and cache stay on the host (assembler.py).

Differences from the reference, all deliberate:
  * within-pool order comes from the counter-based schedule, not from the global `random`
    module: file order, blocks, start_num (the file -> rank assignment) and every rank's
    per-epoch multiset are bit-identical to the reference, the order inside a pool is an
    independent shuffle of the same law.  The global `random` state is never touched.
    `order="exact"` instead replays the reference's own CPython-MT draws: the id stream is
    then bit-identical too.
  * find_ckpt_position is an O(1) skip-ahead on the same stream (V1's reference resume
    leaves the current window unshuffled, V1:139; V2's replays every draw, V2:121-122).
  * no per-batch gc.collect() (V1:258, V2:253); eviction collects only with gc_on_evict.
Extensions (keyword-only): seed, device ("cpu" or a GPU), order, ranks=(lo, hi) -- the block of
logical ranks this process owns (one process per GPU owning R / G ranks; block_indices()),
copy_chunk, gc_on_evict, lookahead=(exact_depth, exact_max_bytes, v2_depth) -- bounds of the
device work and memory the engine spends ahead of the calls (pss_set_lookahead).
"""
import math
from collections.abc import Sequence

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import Sampler

from . import _lib
from .assembler import FileCache, gather, order_and_group
from .engine import IndexEngine, is_cpu, require_gpu


class _FileOrder(Sequence):
    """`self.files` of the reference (V1:122-125): the dataset's files in the epoch's shuffled
    order, as a view over the engine's order array -- no O(F) list rebuild per epoch."""

    def __init__(self, base, order):
        self._base = base
        self._order = order

    def __len__(self):
        return len(self._order)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._base[j] for j in self._order[i].tolist()]
        return self._base[int(self._order[i])]

    def __eq__(self, other):
        return len(self) == len(other) and all(a == b for a, b in zip(self, other))

    def __repr__(self):
        return repr(list(self))


class _LazyScan:
    """The reference's lazily extended `past_files_samples` (V1:126,182-190): exclusive prefix
    over the shuffled files, extended file by file -- length from files_len, else probed with
    reader(path, get_data=False) -- only as far as a batch needs.  Reset every epoch, so the
    probe calls come in the reference's order."""

    def __init__(self, files, files_len, reader):
        self.files = files
        self.files_len = files_len
        self.reader = reader
        self.prefix = np.zeros(len(files) + 1, dtype=np.int64)
        self.n = 0                                    # files scanned

    def extend_to(self, max_id):
        while max_id >= self.prefix[self.n] and self.n < len(self.files):
            path = self.files[self.n]
            ln = self.files_len[path] if path in self.files_len else self.reader(path, get_data=False)
            self.prefix[self.n + 1] = self.prefix[self.n] + int(ln)
            self.n += 1


class _PartialShuffleSampler(Sampler):
    _VERSION = 1

    def __init__(self, dataset, reader, num_replicas=None, rank=None, shuffle=True,
                 shuffle_buffer=None, total_size=None, batch_size=1, file_buffer=10,
                 debug=False, files_len=None, *, seed=0, device=None, copy_chunk=1 << 18,
                 gc_on_evict=False, order="counter", ranks=None, lookahead=None):
        if num_replicas is None:                                    # V1:19-26
            if not dist.is_available():
                raise RuntimeError("Requires distributed package to be available")
            num_replicas = dist.get_world_size()
        if rank is None:
            if ranks is not None:
                rank = int(ranks[0])
            else:
                if not dist.is_available():
                    raise RuntimeError("Requires distributed package to be available")
                rank = dist.get_rank()
        self.files_len = dict()
        self.ori_total_size = total_size
        if files_len is not None:                                   # V1:29-31
            self.files_len = files_len
            self.ori_total_size = int(sum(files_len[k] for k in files_len.keys()))
        self.dataset = dataset
        self.reader = reader
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.shuffle_buffer = shuffle_buffer
        self.batch_size = batch_size
        self.file_buffer = file_buffer
        self.debug = debug
        assert total_size is not None, 'total size must be provided'    # V1:41
        self.num_samples = int(math.ceil(self.ori_total_size * 1.0 / self.num_replicas))
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        if self._VERSION == 1 and shuffle_buffer is None:
            # V1:45 builds list(range(shuffle_buffer)) in the constructor
            raise TypeError("'NoneType' object cannot be interpreted as an integer")
        self.files = list(self.dataset.files)
        self.blocks = list(range(self.num_replicas))
        self.start_num = self.num_samples * self.blocks[self.rank]    # V1:52-53
        self.count_batches = 0
        self.warm_start = False
        self.seed = seed
        self.order = order     # "counter" or "exact" (the reference's own draws)
        self.device = device
        lo, hi = (rank, rank + 1) if ranks is None else (int(ranks[0]), int(ranks[1]))
        if not (0 <= lo <= rank < hi <= num_replicas):
            raise ValueError("ranks=(lo, hi) must hold rank and lie in [0, num_replicas)")
        self.ranks = (lo, hi)
        self.copy_chunk = int(copy_chunk)
        # (exact_depth, exact_max_bytes, v2_depth) for pss_set_lookahead; None: the defaults
        self.lookahead = None if lookahead is None else tuple(lookahead)
        self._engine = None
        self._cache = FileCache(reader, file_buffer, debug, rank, gc_on_evict)
        self._pos = 0
        self._end = 0
        self._block = None     # [hi - lo, ns] ids of the rank block, generated on first request
        self._ids = None       # [ns] ids of this rank's epoch, generated on first request
        self._dev = None       # (file_pos, offset) of this rank's epoch (None in lazy mode)
        self._iterated = False
        self._host = None      # host copies of (file_pos, offset) or (ids,) + per-chunk events
        self._err = None       # pinned int32: the device error word after this epoch's kernels
        self._scan = None      # lazy-length mode: the epoch's _LazyScan
        self._history = []     # epochs of every init_iter so far (file order / blocks are cumulative)
        # every dataset file's length known up front -> device map; else lazy probing in scan
        # order (V1:186-190) with the library's host map over the scanned prefix
        self._lazy = any(p not in self.files_len for p in self.dataset.files)
        # the fused hand-off (pss_generate_mapped: int32 file position + int32 offset, 8 bytes per
        # id, no id pass) unless an offset could need 64 bits; else generate + pss_map
        self._fused = not self._lazy and all(int(self.files_len[p]) < (1 << 31) for p in self.dataset.files)

    # ---- engine ---------------------------------------------------------------------------
    def _lengths(self):
        # lazy mode: unknown lengths are never read by the engine (no device map)
        return np.array([self.files_len.get(p, 0) for p in self.dataset.files], dtype=np.int64)

    def _get_engine(self):
        if self._engine is None:
            if self.shuffle_buffer is None:     # V2 fails at its first init_iter (V2:135-136)
                raise TypeError("unsupported operand type(s) for +: 'int' and 'NoneType'")
            if is_cpu(self.device):
                self.device = "cpu"
            else:
                require_gpu()
                dev = self.device if self.device is not None else torch.cuda.current_device()
                self.device = int(dev.index if isinstance(dev, torch.device) else dev)
            self._engine = IndexEngine(self._lengths(), self.ori_total_size, self.num_replicas,
                                       self.shuffle_buffer, self._VERSION, shuffle=self.shuffle,
                                       seed=self.seed, device=self.device, order=self.order)
            if self.lookahead is not None:
                self._engine.set_lookahead(*self.lookahead)
        return self._engine

    # ---- epoch ----------------------------------------------------------------------------
    def init_iter(self):
        """One init_iter (V1:100-132 / V2:124-159): the host history, then this rank's whole
        epoch as (file position, offset) pairs -- generated and mapped in one pass on the device
        (pss_generate_mapped, 8 bytes per id) -- and an asynchronous copy of them to the host.
        The ids themselves (device_indices, block_indices) are generated only when asked for."""
        self.dataset.reset()
        eng = self._get_engine()
        eng.init_iter(self.epoch)
        self._history.append(int(self.epoch))
        self.files = _FileOrder(self.dataset.files, eng.file_order())
        self.blocks = eng.blocks().tolist()
        _, new = eng.rank_starts()
        self.start_num = int(new[self.rank])
        if self.debug:
            print(str(self.rank) + ': start number ' + str(self.start_num))
        self.count_batches = 0
        self._pos = 0
        ns = self.num_samples
        cpu = eng.cpu
        dev = torch.device("cpu") if cpu else torch.device("cuda", self.device)
        stream = None if cpu else torch.cuda.current_stream(dev)
        self._block = None
        self._ids = None
        self._iterated = True
        if self._lazy:
            # lengths probed in scan order on the host (V1:186-190): ids only
            self._dev = None
            self._scan = _LazyScan(self.files, self.files_len, self.reader)
            payload = (self._rank_ids(stream),)
        elif self._fused:
            fpos, off = eng.generate_mapped(self.rank, self.rank + 1, stream=stream)
            self._dev = (fpos[0], off[0])
            payload = self._dev
        else:
            ids = self._rank_ids(stream)
            fpos, off = eng.map(ids, stream=stream)
            self._dev = (fpos, off)
            payload = self._dev
        self._copy_to_host(eng, payload, stream, cpu)
        self._end = ns
        wraps = (self.ori_total_size - self.start_num) < self.num_samples     # V1:79-80
        self._cache.reset(self.files, len(self.files) // self.num_replicas if wraps else 0)

    def _copy_to_host(self, eng, payload, stream, cpu):
        ns = self.num_samples
        if cpu:
            self._host = (tuple(t.numpy() for t in payload), [])
            return
        if self._err is None:
            self._err = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        _lib.call("pss_error_snapshot", eng._h, ctypes_ptr(self._err), ctypes_stream(stream))
        bufs = self._host[0] if self._host is not None else None
        if bufs is None or len(bufs) != len(payload) or bufs[0].numel() < ns:
            bufs = tuple(torch.empty(ns, dtype=t.dtype, pin_memory=True) for t in payload)
        events = []
        for a in range(0, ns, self.copy_chunk):
            b = min(ns, a + self.copy_chunk)
            for h, d in zip(bufs, payload):
                h[a:b].copy_(d[a:b], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            events.append((b, ev))
        self._host = (bufs, events)

    def find_ckpt_position(self, step):
        """Resume at batch `step` of the current epoch: O(1) skip-ahead (V1:134-140)."""
        self.warm_start = True
        self.init_iter()
        self._pos = min(step * self.batch_size, self._end)

    def state_dict(self):
        """Resume point (extension; the reference only has find_ckpt_position(step)): the epochs
        of every init_iter so far -- the file order and V1's blocks are cumulative over them
        (V1:122-125, V2:149-152) -- the stream position reached, and what positions mean: the
        order mode, and for the counter order the seed and libpss's schedule version."""
        return {"history": list(self._history), "position": int(self._pos),
                "sampler_version": self._VERSION, "num_replicas": self.num_replicas,
                "rank": self.rank, "shuffle_buffer": self.shuffle_buffer,
                "total_size": self.ori_total_size, "order": self.order, "seed": int(self.seed),
                # V2 always shuffles (its shuffle flag is ignored, V2:142-152)
                "shuffle": bool(self.shuffle) if self._VERSION == 1 else True,
                "num_files": len(self.files),
                "schedule_version": _lib.load().pss_schedule_version()}

    def load_state_dict(self, sd):
        """Continue exactly where state_dict() was taken: the init_iter history is replayed on
        the host (O(F) each, no generation), then the last epoch is generated and iteration
        resumes at the recorded position -- the next __iter__ is a warm start.  A state of
        another configuration, or of another counter schedule (pss_schedule_version), raises
        ValueError: its positions would index a different permutation."""
        mine = self.state_dict()
        for k in ("sampler_version", "num_replicas", "rank", "shuffle_buffer", "total_size", "order",
                  "shuffle", "num_files"):
            if k not in sd:
                if k in ("shuffle", "num_files"):
                    # recorded since round 5 only; a state of an earlier build (the same schedule
                    # version, checked below) resumes as before, without these two checks
                    continue
                raise ValueError("state_dict has no %r: it was taken by another build" % k)
            if sd[k] != mine[k]:
                raise ValueError("state_dict was taken with %s=%r, this sampler has %r"
                                 % (k, sd[k], mine[k]))
        if self.order == "counter":
            for k in ("seed", "schedule_version"):
                if sd[k] != mine[k]:
                    raise ValueError("state_dict was taken with %s=%r, this sampler has %r: the "
                                     "counter-order positions would not continue the same "
                                     "permutation" % (k, sd[k], mine[k]))
        if not sd["history"]:
            return
        if self._history:
            raise ValueError("load_state_dict needs a sampler that has not iterated yet")
        eng = self._get_engine()
        for e in sd["history"][:-1]:
            eng.init_iter(e)
        self._history = list(sd["history"][:-1])
        self.epoch = sd["history"][-1]
        self.warm_start = True
        self.init_iter()
        self._pos = min(int(sd["position"]), self._end)

    def __iter__(self):
        if not self.warm_start:
            self.init_iter()
        else:
            print(self._warm_msg())
            self.warm_start = False
        return self

    def _warm_msg(self):
        return str(self.rank) + ': warm start!! ' + str(self.epoch)

    def _wait_host(self, hi):
        events = self._host[1]
        while events and events[0][0] < hi:
            events.pop(0)[1].synchronize()
        if events:
            events[0][1].synchronize()
        if self._err is not None and int(self._err[0]):
            raise RuntimeError("partiallyshuffledistributedsampler_amd: a kernel flagged device "
                               "error %d while generating this epoch" % int(self._err[0]))

    def _host_batch(self, lo, hi):
        """(file_pos, offset) of stream positions [lo, hi) on the host."""
        bufs = self._host[0]
        if not self._lazy:
            return (np.asarray(bufs[0][lo:hi]), np.asarray(bufs[1][lo:hi]))
        ids = np.ascontiguousarray(np.asarray(bufs[0][lo:hi]), dtype=np.int64)
        sc = self._scan
        sc.extend_to(int(ids.max()))
        fpos = np.empty(len(ids), dtype=np.int32)
        off = np.empty(len(ids), dtype=np.int64)
        _lib.call("pss_map_prefix_host", sc.prefix.ctypes.data, sc.n, ids.ctypes.data, len(ids),
                  fpos.ctypes.data, off.ctypes.data)
        return fpos, off

    def __next__(self):
        if self._pos >= self._end:
            raise StopIteration
        lo, hi = self._pos, min(self._pos + self.batch_size, self._end)
        self._wait_host(hi)
        fpos, off = self._host_batch(lo, hi)
        groups, n_mapped, n_refl = order_and_group(fpos, off)
        self._pos = hi
        if n_refl:
            print(str(self.rank) + ': ' + 'the number of the whole dataset might be larger than '
                  'the real number')
        if n_mapped == 1:                                            # V1:225-226
            raise StopIteration
        out = gather(groups, self.files, self._cache)
        self.count_batches += 1
        return out

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch):
        self.epoch = epoch

    # ---- extensions -----------------------------------------------------------------------
    def _rank_ids(self, stream=None):
        """This rank's epoch ids (generated once per epoch, on first request)."""
        if self._ids is None:
            if self._block is not None:
                self._ids = self._block[self.rank - self.ranks[0]]
            else:
                eng = self._engine
                if stream is None and not eng.cpu:
                    stream = torch.cuda.current_stream(torch.device("cuda", self.device))
                self._ids = eng.generate(self.rank, self.rank + 1, stream=stream)[0]
        return self._ids

    def device_indices(self):
        """(ids, file_pos, offset) tensors of this rank's current epoch, in stream order (on
        the GPU, or host tensors in CPU mode) -- the hand-off for an on-GPU gather (positions of
        file_pos index self.files; negative entries are reflected ids, see pss_map).  file_pos
        and offset come from the epoch's fused hand-off (int32 both; int64 offsets when a file
        holds 2^31 samples or more); the ids are generated on the first call of the epoch.  With
        lazily probed lengths only ids exist before the scan: (ids, None, None)."""
        if not self._iterated:
            raise RuntimeError("call iter(sampler) first")
        ids = self._rank_ids()
        if self._dev is None:
            return (ids, None, None)
        return (ids,) + tuple(self._dev)

    def device_batches(self, data, base_rows):
        """This rank's remaining batches of the epoch gathered on the device: yields
        (rows, file_pos, offset) with rows = data[base_rows[file] + offset] for the batch's ids
        in stream order (pss_gather) -- no host round trip.  `data` holds every dataset file's
        samples on the sampler's device, file f (dataset order) starting at row base_rows[f]."""
        if self._dev is None:
            raise RuntimeError("device_batches needs iter(sampler) first and every file length "
                               "in files_len")
        eng = self._engine
        fpos, off = self._dev
        while self._pos < self._end:
            lo, hi = self._pos, min(self._pos + self.batch_size, self._end)
            self._pos = hi
            self.count_batches += 1
            yield eng.gather(data, base_rows, fpos[lo:hi], off[lo:hi]), fpos[lo:hi], off[lo:hi]

    def block_indices(self):
        """[hi - lo, num_samples] ids of every logical rank of the block ranks=(lo, hi), in one
        launch (generated on the first call of the epoch)."""
        if not self._iterated:
            raise RuntimeError("call iter(sampler) first")
        if self._block is None:
            eng = self._engine
            stream = None if eng.cpu else torch.cuda.current_stream(torch.device("cuda", self.device))
            lo, hi = self.ranks
            self._block = eng.generate(lo, hi, stream=stream)
        return self._block

    def indices(self):
        """Host numpy copy of this rank's epoch ids in stream order (debug / parity)."""
        return self.device_indices()[0].cpu().numpy()

    def workspace_bytes(self):
        """Device bytes the sampler's engine holds (pss_workspace_bytes: workspaces, the V2
        lookahead's VAL ring, exact-order draw slots, epoch tables); 0 before the first epoch."""
        return 0 if self._engine is None else self._engine.workspace_bytes()


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


def ctypes_stream(stream):
    import ctypes
    return ctypes.c_void_p(0 if stream is None else stream.cuda_stream)
