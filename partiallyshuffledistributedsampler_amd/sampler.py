"""Drop-in `torch.utils.data.Sampler` facade over the MI355X index engine.

Same constructor, methods, return format and errors as the reference samplers
(V1 = DistributedSamplerViaLocallyShuffle.py, V2 = ...V2.py); index generation and the
id -> (file, offset) map run on the GPU (engine.py -> libpss.so), the file reader and cache
stay on the host (assembler.py).

Differences from the reference, all deliberate:
  * within-pool order comes from the counter-based Philox schedule, not from the global
    `random` module: file order, blocks, start_num (the file -> rank assignment) and every
    rank's per-epoch multiset are bit-identical to the reference, the order inside a pool is
    an independent uniform shuffle.  The global `random` state is never touched.
    `order="exact"` (V1) instead shuffles every window with CPython's MT19937 exactly as the
    reference does (V1:102,114-115,165-171): the id stream is then bit-identical too.
  * find_ckpt_position is an O(1) skip-ahead on the same stream (V1's reference resume
    leaves the current window unshuffled, V1:139; V2's replays every draw, V2:121-122).
  * file lengths missing from files_len are probed for every file at the first __iter__
    (the reference probes lazily while scanning, V1:186-189).
  * no per-batch gc.collect() (V1:258, V2:253); eviction still collects.
"""
import math

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import Sampler

from .assembler import FileCache, gather, order_and_group
from .engine import IndexEngine, require_gpu


class _PartialShuffleSampler(Sampler):
    _VERSION = 1

    def __init__(self, dataset, reader, num_replicas=None, rank=None, shuffle=True,
                 shuffle_buffer=None, total_size=None, batch_size=1, file_buffer=10,
                 debug=False, files_len=None, *, seed=0, device=None, copy_chunk=1 << 18,
                 gc_on_evict=False, order="counter"):
        if num_replicas is None:                                    # V1:19-26
            if not dist.is_available():
                raise RuntimeError("Requires distributed package to be available")
            num_replicas = dist.get_world_size()
        if rank is None:
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
        self.order = order     # "counter" or "exact" (V1: the reference's own window order)
        self.device = device
        self.copy_chunk = int(copy_chunk)
        self._engine = None
        self._cache = FileCache(reader, file_buffer, debug, rank, gc_on_evict)
        self._pos = 0
        self._end = 0
        self._dev = None       # (ids, file_pos, offset) device tensors of the current epoch
        self._host = None      # pinned host copies + per-chunk events

    # ---- engine ---------------------------------------------------------------------------
    def _lengths(self):
        out = np.empty(len(self.dataset.files), dtype=np.int64)
        for i, p in enumerate(self.dataset.files):
            out[i] = self.files_len[p] if p in self.files_len else self.reader(p, get_data=False)
        return out

    def _get_engine(self):
        if self._engine is None:
            if self.shuffle_buffer is None:     # V2 fails at its first init_iter (V2:135-136)
                raise TypeError("unsupported operand type(s) for +: 'int' and 'NoneType'")
            require_gpu()
            dev = self.device if self.device is not None else torch.cuda.current_device()
            self.device = int(dev.index if isinstance(dev, torch.device) else dev)
            self._engine = IndexEngine(self._lengths(), self.ori_total_size, self.num_replicas,
                                       self.shuffle_buffer, self._VERSION, shuffle=self.shuffle,
                                       seed=self.seed, device=self.device, order=self.order)
        return self._engine

    # ---- epoch ----------------------------------------------------------------------------
    def init_iter(self):
        """One init_iter (V1:100-132 / V2:124-159) followed by device generation of this
        rank's whole epoch and an asynchronous pinned copy to the host."""
        self.dataset.reset()
        eng = self._get_engine()
        eng.init_iter(self.epoch)
        base = self.dataset.files
        self.files = [base[i] for i in eng.file_order()]
        self.blocks = eng.blocks().tolist()
        _, new = eng.rank_starts()
        self.start_num = int(new[self.rank])
        if self.debug:
            print(str(self.rank) + ': start number ' + str(self.start_num))
        self.count_batches = 0
        self._pos = 0
        ns = self.num_samples
        dev = torch.device("cuda", self.device)
        stream = torch.cuda.current_stream(dev)
        ids = eng.generate(self.rank, self.rank + 1, stream=stream).view(-1)
        fpos, off = eng.map(ids, stream=stream)
        self._dev = (ids, fpos, off)
        if self._host is None or self._host[0].numel() < ns:
            self._host = (torch.empty(ns, dtype=torch.int32, pin_memory=True),
                          torch.empty(ns, dtype=torch.int64, pin_memory=True), [])
        h_f, h_o, _ = self._host
        events = []
        for lo in range(0, ns, self.copy_chunk):
            hi = min(ns, lo + self.copy_chunk)
            h_f[lo:hi].copy_(fpos[lo:hi], non_blocking=True)
            h_o[lo:hi].copy_(off[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            events.append((hi, ev))
        self._host = (h_f, h_o, events)
        self._end = ns
        wraps = (self.ori_total_size - self.start_num) < self.num_samples     # V1:79-80
        self._cache.reset(self.files, len(self.files) // self.num_replicas if wraps else 0)

    def find_ckpt_position(self, step):
        """Resume at batch `step` of the current epoch: O(1) skip-ahead (V1:134-140)."""
        self.warm_start = True
        self.init_iter()
        self._pos = min(step * self.batch_size, self._end)

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
        for end, ev in self._host[2]:
            ev.synchronize()
            if end >= hi:
                break

    def __next__(self):
        if self._pos >= self._end:
            raise StopIteration
        lo, hi = self._pos, min(self._pos + self.batch_size, self._end)
        self._wait_host(hi)
        groups, n_mapped, n_refl = order_and_group(self._host[0][lo:hi].numpy(),
                                                   self._host[1][lo:hi].numpy())
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
    def device_indices(self):
        """(ids, file_pos, offset) device tensors of this rank's current epoch, in stream
        order -- the hand-off for an on-GPU gather (positions of file_pos index self.files;
        negative entries are reflected ids, see pss_map)."""
        if self._dev is None:
            raise RuntimeError("call iter(sampler) first")
        return self._dev

    def indices(self):
        """Host numpy copy of this rank's epoch ids in stream order (debug / parity)."""
        return self.device_indices()[0].cpu().numpy()
