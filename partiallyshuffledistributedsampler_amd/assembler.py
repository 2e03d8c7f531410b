"""Host-side batch assembly: (file position, offset) pairs -> the reference's batch format.

Mirrors the reference's __next__ tail (V1:178-259, V2:181-254) on top of ids that the GPU
already mapped (pss_map):
  * reflected ids (flagged file_pos = -1 - f) are moved behind the others, as V1:195 appends
    them to `indices` and maps them last;
  * rows are grouped per file in order of first appearance (V1:216-221);
  * a batch that maps exactly one id ends the epoch (V1:225-226);
  * files are loaded through a FIFO-evicting cache of `file_buffer` entries with a one-thread
    prefetcher of the next file in the shuffled order (V1:58-98), and rows are gathered with
    numpy fancy indexing (V1:243-248).
The file reader and cache stay host-side (BASELINE.json north_star).
"""
import gc
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def order_and_group(fpos, off):
    """Reorder one batch like the reference and group it by file.

    Returns (groups, n_mapped, n_reflected): groups is a list of (file_position, offsets)
    in first-appearance order."""
    fpos = np.asarray(fpos)
    off = np.asarray(off)
    refl = fpos < 0
    n_refl = int(refl.sum())
    if n_refl:
        idx = np.concatenate([np.flatnonzero(~refl), np.flatnonzero(refl)])
        f = np.where(refl, -1 - fpos, fpos)[idx]
        o = off[idx]
    else:
        f, o = fpos, off
    if len(f) == 0:
        return [], 0, n_refl
    uniq, first, inv = np.unique(f, return_index=True, return_inverse=True)
    rank_of_file = np.empty(len(uniq), dtype=np.int64)
    rank_of_file[np.argsort(first, kind="stable")] = np.arange(len(uniq))
    g = rank_of_file[inv]
    perm = np.argsort(g, kind="stable")
    bounds = np.flatnonzero(np.diff(g[perm])) + 1
    files_in_order = uniq[np.argsort(first, kind="stable")]
    chunks = np.split(o[perm], bounds)
    return list(zip(files_in_order.tolist(), chunks)), len(f), n_refl


class FileCache:
    """`file_buffer`-bounded cache of reader(path, True) results with one prefetch thread
    (V1:55,58-98).  Eviction scans cached files in shuffled-order position and drops them
    until the count is back within file_buffer, keeping -- for a rank whose block wraps past
    the dataset end -- the first len(files)//R files (V1:79-81)."""

    def __init__(self, reader, file_buffer, debug=False, rank=0, gc_on_evict=False):
        self.reader = reader
        self.file_buffer = file_buffer
        self.debug = debug
        self.rank = rank
        # the reference runs gc.collect() after every eviction (V1:85); refcounting already
        # frees the arrays, so it is opt-in here (it dominated the reference's wall time)
        self.gc_on_evict = gc_on_evict
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="file_reader_")
        self.reset([], keep_head=0)

    def reset(self, files, keep_head):
        self.files = files
        self.data = {}
        self.loaded = 0
        self.keep_head = keep_head        # positions < keep_head are never evicted
        self.pending_pos = None
        self.pending = None

    def shutdown(self):
        self.pool.shutdown(wait=True)

    def _log(self, msg):
        if self.debug:
            try:
                import psutil
                rss = psutil.Process(os.getpid()).memory_info().rss / 1024 / 1024
            except Exception:  # psutil is optional here
                rss = -1
            print("%d: %s memory used:%s" % (self.rank, msg, rss))

    def get(self, pos):
        if pos in self.data:
            self._log("use cache data from %s" % (self.files[pos],))
            return self.data[pos]
        path = self.files[pos]
        self._log("load data from %s" % (path,))
        if self.pending_pos == pos:
            d, _ = self.pending.result()
        else:
            d, _ = self.reader(path, True)
        nxt = pos + 1
        if nxt < len(self.files) and nxt not in self.data:
            self.pending_pos = nxt
            self.pending = self.pool.submit(self.reader, self.files[nxt], True)
        self.data[pos] = d
        self.loaded += 1
        if self.loaded > self.file_buffer:
            for p in sorted(self.data):
                if p < self.keep_head:
                    continue
                del self.data[p]
                if self.gc_on_evict:
                    gc.collect()
                self.loaded -= 1
                if self.loaded <= self.file_buffer:
                    break
        return d


def gather(groups, files, cache):
    """[target_datas, None, read_files] of one grouped batch (V1:232-259)."""
    read_files, target = [], []
    for pos, offs in groups:
        d = cache.get(pos)
        target.append({k: v[offs] for k, v in d.items()})
        read_files.append(files[pos])
    return [target, None, read_files]
