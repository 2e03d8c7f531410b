"""TEST / BENCH INFRASTRUCTURE ONLY -- a pure-Python restatement of the reference's per-batch
loops, used by bench.py's cpu_baseline leg to time the reference algorithm on the GPU box's host
cores (the reference itself is not on that box; BASELINE.md "CPU-baseline plan").  Nothing in
the product imports this module.

  V1Loop  -- V1 __next__ (DistributedSamplerViaLocallyShuffle.py:151-259): window shuffles with
             the process-global `random` module (V1:157-172), the lazy exclusive scan and
             cursor walk (V1:181-221), numpy gather of the rows (V1:243-248) and the per-batch
             gc.collect() (V1:258), switchable for the gc-on / gc-off figures.
  V2Draws -- V2 get_index (DistributedSamplerViaLocallyShuffleV2.py:96-116): choice + list.remove
             pools, reseeded per window.
Both follow the reference's arithmetic exactly (same seeds, same calls into `random`), so their
id streams are the reference's (checked against tests/golden in tests/test_oracle_golden.py).
"""
import gc
import random


class V1Loop:
    def __init__(self, start, ns, B, N, files_len_in_order, data, epoch=0, bs=1024, use_gc=True):
        self.start, self.ns, self.B, self.N = start, ns, B, N
        self.lens = files_len_in_order          # lengths in the epoch's shuffled file order
        self.data = data                        # file position -> dict of arrays
        self.epoch, self.bs, self.use_gc = epoch, bs, use_gc
        self.batch_ids = list(range(min(B, ns)))                 # V1:102
        random.seed(epoch)                                       # V1:114-115
        random.shuffle(self.batch_ids)
        self.buffers = 0
        self.batch_position = 0
        self.past = [0]
        self.last = 0

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
        read, ids = [], []
        for bid in indices:                                      # V1:181-221 (no reflection)
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
            gc.collect()                                         # V1:258
        return out


class V2Draws:
    """get_index of one rank (V2:96-116), seeded like init_iter (V2:135-148)."""

    def __init__(self, old_start, new_start, ns, B, epoch=0):
        self.ns, self.B, self.new, self.epoch = ns, B, new_start, epoch
        self.pool1 = list(range(old_start, old_start + min(B, ns)))
        self.pool2 = list(range(old_start + B, min(old_start + 2 * B, old_start + ns)))
        self.buffers = 0
        random.seed(epoch + 2)

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
        return index
