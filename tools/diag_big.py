"""Diagnostic: the big-pool V2 configuration of test_streams_match_oracle_twin (cfg9) with the
handle's device error flag checked after each epoch (bounds guards in pss_v2big.hip)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle as O
from partiallyshuffledistributedsampler_amd.engine import IndexEngine
F, lo, hi, R, B = 20, 5000, 20000, 2, 20000
rng = np.random.default_rng(F * 1000 + R)
lengths = rng.integers(lo, hi, F)
N = int(lengths.sum())
eng = IndexEngine(lengths, N, R, B, 2, seed=1234, device=0)
print("ns", eng.num_samples, "path", eng.emit_path(), flush=True)
for epoch in (0, 3):
    eng.init_iter(epoch)
    old, new = eng.rank_starts()
    out = eng.generate(0, R)
    try:
        eng.check()
        print("epoch", epoch, "device flag clear", flush=True)
    except Exception as e:
        print("epoch", epoch, "CHECK:", e, flush=True)
    o = out.cpu().numpy()
    key = O.epoch_key(1234, epoch)
    for r in range(R):
        ref = O.v2_philox_stream(key, r, int(old[r]), int(new[r]), eng.num_samples, B, N)
        print("epoch", epoch, "rank", r, "match", bool(np.array_equal(o[r], ref)), flush=True)
