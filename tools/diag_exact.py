"""Diagnostic: per-window comparison of the exact-order V1 stream against the oracle."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle as O
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
for B in (4096, 1024, 700, 600, 500):
    F, R = 8, 2
    lengths = np.full(F, 3000)
    N = int(lengths.sum())
    eng = IndexEngine(lengths, N, R, B, 1, seed=7, device=0, order="exact")
    ns = eng.num_samples
    eng.init_iter(0)
    _, new = eng.rank_starts()
    out = eng.generate(0, R).cpu().numpy()
    ref = O.v1_exact_stream(0, int(new[0]), ns, B, N, True)
    bad = []
    for w in range((ns + B - 1) // B):
        a, b = out[0][w * B:(w + 1) * B], ref[w * B:(w + 1) * B]
        if not np.array_equal(a, b):
            d = np.nonzero(a != b)[0]
            bad.append((w, len(a), len(d), int(d[0]), int(d[-1])))
    print("B", B, "ns", ns, "bad windows (w, n, ndiff, first, last):", bad[:6])
