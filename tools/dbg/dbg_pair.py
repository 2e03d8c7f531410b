import sys, zlib
import numpy as np, torch
sys.path.insert(0, ".")
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
for (kind, R, B, extra) in [("varied", 5, 1024, 0), ("varied", 4, 4096, 0), ("varied", 3, 1000, 0)]:
    rng = np.random.default_rng(zlib.crc32(repr((kind, R, B, extra)).encode()))
    lengths = rng.integers(3000, 12000, 40)
    N = int(lengths.sum()) + extra
    eng = IndexEngine(lengths, N, R, B, 2, seed=11, device=0)
    ns = eng.num_samples
    eng.init_iter(0)
    ids = eng.generate(0, R)
    f, o = eng.map(ids.reshape(-1)); f = f.reshape(R, -1).cpu().numpy(); o = o.reshape(R, -1).cpu().numpy()
    f2, o2 = eng.generate_mapped(0, R); f2 = f2.cpu().numpy(); o2 = o2.cpu().numpy()
    idn = ids.cpu().numpy()
    print(kind, R, B, "ns", ns, "N", N)
    for r in range(R):
        bad = np.nonzero((f[r] != f2[r]) | (o[r] != o2[r]))[0]
        print(" rank", r, "bad", len(bad), "first", bad[:8].tolist(), "last", bad[-4:].tolist() if len(bad) else [])
        for i in bad[:5]:
            print("   pos", i, "id", idn[r, i], "want", f[r, i], o[r, i], "got", f2[r, i], o2[r, i])
    eng.close()
