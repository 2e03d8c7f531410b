import sys, numpy as np
sys.path.insert(0, '/root/repo')
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
from oracle import oracle as O
M32 = 0xFFFFFFFF
def slot_hash(t, s0, s1):
    x = (t ^ s0) & M32; x ^= x >> 16; x = (x * 0x21F0AAAD) & M32; x ^= x >> 15; x ^= s1
    x = (x * 0x735A2D97) & M32; x ^= x >> 15; return x
B, R, F, lo, hi = 4096, 3, 40, 5000, 9000
rng = np.random.default_rng(B + R)
lengths = rng.integers(lo, hi, F); N = int(lengths.sum())
eng = IndexEngine(lengths, N, R, B, 2, seed=99, device=0)
eng.set_emit_path("probe")
ns = eng.num_samples; P1 = B; T = ns - P1
eng.init_iter(4)
old, new = eng.rank_starts()
full = eng.generate(0, R).cpu().numpy()
key = O.epoch_key(99, 4)
L = 16384; G = (T + L - 1) // L; tlo = (G - 1) * L
for r in range(R):
    ref = O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N)
    bad = np.nonzero(full[r] != ref)[0]
    sk = O.philox4x32([0, 0, r, 2], key)
    draws = {}
    hist = {}
    for t in range(tlo - 3 * L, T):
        k = (slot_hash(t, int(sk[0]), int(sk[1])) * P1) >> 32
        hist.setdefault(k, []).append(t)
    tk = np.concatenate([O.philox4x32([0, 0, r, 4], key), O.philox4x32([0, 1, r, 4], key)])
    for pos in bad:
        j = pos - T
        s = O.feistel(j, P1, tk)
        h = [t - tlo for t in hist.get(s, [])][-6:]
        print("rank", r, "pos", pos, "slot", s, "draw steps rel. last tile", h, "gpu", full[r][pos], "ref", ref[pos])
