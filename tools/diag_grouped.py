"""Where a grouped-pool (P1 > 16384) GPU stream first departs from the oracle twin."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
from oracle import oracle as O

def main():
    cases = [(10_000, 10_000, 8, 1 << 20), (400, 10000, 1, 1 << 18), (400, 10000, 2, 100000), (40, 20000, 2, 65536)]
    for F, L, R, B in cases:
        N = F * L
        eng = IndexEngine(np.full(F, L), N, R, B, 2, seed=0, device=0)
        ns = eng.num_samples
        eng.init_iter(0)
        old, new = eng.rank_starts()
        out = eng.generate(0, R).cpu().numpy()
        eng.check()
        P1 = min(B, ns); T = ns - P1
        for r in range(min(R, 2)):
            ref = O.v2_philox_stream(O.epoch_key(0, 0), r, int(old[r]), int(new[r]), ns, B, N)
            bad = np.nonzero(out[r] != ref)[0]
            G = (P1 + 4095) // 4096
            print(F, L, R, B, "rank", r, "ns", ns, "T", T, "G", G, "mismatches", len(bad),
                  "first", bad[:8].tolist(), "in tail", int((bad >= T).sum()))
            if len(bad):
                t = int(bad[0]); print("   t", t, "burst", t // 16, "group", (t // 16) % G, "u", (t // 16 // G) * 16 + t % 16,
                                       "got", int(out[r][t]), "want", int(ref[t]))
        eng.close()

main()
