"""TEST / BENCH INFRASTRUCTURE ONLY -- a pure-Python restatement of the reference's per-batch
loops, used by bench.py's cpu_baseline leg to time the reference algorithm on the GPU box's host
cores (the reference itself is not on that box; BASELINE.md "CPU-baseline plan").  Nothing in
the product imports this module.

  V1Loop  -- V1 __next__ (DistributedSamplerViaLocallyShuffle.py:151-259): window shuffles with
             the process-global `random` module (V1:157-172), the lazy exclusive scan and
             cursor walk (V1:181-221), numpy gather of the rows (V1:243-248) and the per-batch
             gc.collect() (V1:258), switchable for the gc-on / gc-off figures.
  V2Draws -- V2 get_index (DistributedSamplerViaLocallyShuffleV2.py:96-116): choice + list.remove
             pools, reseeded per window (and per draw once pool2 is spent).
  V2Loop  -- V2 __next__ (V2:170-254): a batch of get_index draws, then the same map, gather and
             per-batch gc.collect() as V1's (V2:181-253 repeat V1:178-259).
All follow the reference's arithmetic exactly (same seeds, same calls into `random`), so their
id streams are the reference's (checked against tests/golden in tests/test_oracle_golden.py).
"""
import gc
import random


class _MapGather:
    """The reference's id -> (file, offset) walk and row gather (V1:181-248, V2:184-248) over
    a lazily extended exclusive prefix of the epoch's file lengths (no reflection: the bench's
    files_len is complete)."""

    def _init_map(self, files_len_in_order, data, use_gc):
        self.lens = files_len_in_order          # lengths in the epoch's shuffled file order
        self.data = data                        # file position -> dict of arrays
        self.use_gc = use_gc
        self.past = [0]

    def _map_gather(self, indices):
        read, ids = [], []
        for bid in indices:                                      # V1:181-221
            while bid >= self.past[-1] and len(self.past) <= len(self.lens):
                self.past.append(self.past[-1] + self.lens[len(self.past) - 1])
            lo, hi = 0, len(self.past) - 1
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if self.past[mid] <= bid:
                    lo = mid
                else:
                    hi = mid
            if lo in read:
                ids[read.index(lo)].append(bid - self.past[lo])
            else:
                read.append(lo)
                ids.append([bid - self.past[lo]])
        out = [{k: v[i] for k, v in self.data(f).items()} for f, i in zip(read, ids)]   # V1:243-248
        if self.use_gc:
            gc.collect()                                         # V1:258 / V2:253
        return out


class V1Loop(_MapGather):
    def __init__(self, start, ns, B, N, files_len_in_order, data, epoch=0, bs=1024, use_gc=True):
        self.start, self.ns, self.B, self.N = start, ns, B, N
        self._init_map(files_len_in_order, data, use_gc)
        self.epoch, self.bs = epoch, bs
        self.batch_ids = list(range(min(B, ns)))                 # V1:102
        random.seed(epoch)                                       # V1:114-115
        random.shuffle(self.batch_ids)
        self.buffers = 0
        self.batch_position = 0

    def next_batch(self):
        if len(self.batch_ids) == 0:
            return None
        indices = []
        for _ in range(self.bs):                                 # V1:158-172
            if len(self.batch_ids) == 0:
                break
            index = self.batch_ids[self.batch_position] + self.B * self.buffers + self.start
            if index >= self.N:
                index -= self.N
            self.batch_position += 1
            if self.batch_position >= len(self.batch_ids):
                self.buffers += 1
                self.batch_ids = list(range(min(self.B, self.ns - self.buffers * self.B)))
                random.seed(self.epoch + self.buffers * 10000)
                random.shuffle(self.batch_ids)
                self.batch_position = 0
            indices.append(index)
        self.last_indices = indices
        return self._map_gather(indices)


class V2Draws:
    """get_index of one rank (V2:96-116), seeded like init_iter (V2:135-148).  N: wrap ids at
    N (V2:113-114); None leaves them unwrapped."""

    def __init__(self, old_start, new_start, ns, B, epoch=0, N=None):
        self.ns, self.B, self.new, self.epoch, self.N = ns, B, new_start, epoch, N
        self.pool1 = list(range(old_start, old_start + min(B, ns)))
        self.pool2 = list(range(old_start + B, min(old_start + 2 * B, old_start + ns)))
        self.buffers = 0
        random.seed(epoch + 2)

    def empty(self):
        return len(self.pool1) == 0 and len(self.pool2) == 0

    def get_index(self):
        index = random.choice(self.pool1)
        self.pool1.remove(index)
        if len(self.pool2) != 0:
            index2 = random.choice(self.pool2)
            self.pool2.remove(index2)
            self.pool1.append(index2)
        if len(self.pool2) == 0:
            random.seed(self.epoch + self.buffers * 10000)
            self.buffers += 1
            self.pool2 = list(range(self.new + (self.buffers + 1) * self.B,
                                    min(self.new + (self.buffers + 2) * self.B, self.new + self.ns)))
        if self.N is not None and index >= self.N:
            index -= self.N
        return index


class V2Loop(_MapGather):
    def __init__(self, old_start, new_start, ns, B, N, files_len_in_order, data, epoch=0,
                 bs=1024, use_gc=True):
        self.draws = V2Draws(old_start, new_start, ns, B, epoch, N)
        self._init_map(files_len_in_order, data, use_gc)
        self.bs = bs

    def next_batch(self):
        if self.draws.empty():                                   # V2:171-172
            return None
        indices = []
        for _ in range(self.bs):                                 # V2:98-116
            if self.draws.empty():
                break
            indices.append(self.draws.get_index())
        self.last_indices = indices
        return self._map_gather(indices)
