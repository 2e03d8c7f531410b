"""Parity subset run in a child process under a forced environment knob (tests/test_knobs.py).

The library reads its PSS_* switches once per process, before the first GPU call, so each
forced setting needs a fresh interpreter: `python -m tests.knob_worker <check> [device]` exits 0
when every check passes and prints the first mismatch otherwise.

Checks:
  exact     order="exact" against the reference-captured fixtures (tests/golden/big) and the
            exact oracle: V1 windows through HBM (2^17 and 2^20 entries) and V2 pools beyond one
            decode tile (2^16) over consecutive epochs -- the paths PSS_V1X_DRAWS_WG /
            PSS_V2X_DRAWS_WG switch between, and the draw lookahead PSS_EXACT_LOOKAHEAD turns off
  counter   the counter order (V2 small pools with the lookahead ring over consecutive epochs,
            grouped pools, V1) against the oracle twin -- the path PSS_V2_LOOKAHEAD switches
  cpu       CPU mode, exact and counter order, against the oracle (PSS_CPU_THREADS)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
from tests.golden_util import big_lengths, check_stream, load_big  # noqa: E402
from partiallyshuffledistributedsampler_amd.engine import IndexEngine  # noqa: E402


def _gen(eng, lo, hi, **kw):
    out = eng.generate(lo, hi, **kw)
    if not eng.cpu:
        eng.check()
    return out.cpu().numpy()


def _fixture(name, device):
    fx = load_big(name)
    lens = big_lengths(fx)
    eng = IndexEngine(lens, int(lens.sum()), fx["R"], fx["B"], fx["version"], device=device,
                      order="exact")
    count = fx["prefix"] if fx["kind"] == "prefix" else None
    for i, er0 in enumerate(fx["ranks"][0]["epochs"]):
        eng.init_iter(er0["epoch"])
        for rr in fx["ranks"]:
            er = rr["epochs"][i]
            got = _gen(eng, rr["rank"], rr["rank"] + 1, pos_lo=0, count=count)[0]
            check_stream(got, er, fx, "%s r%d e%d" % (name, rr["rank"], er["epoch"]))
    eng.close()


def _two_rank_shape(B, pad=1):
    R, ns = 2, int(3.5 * B)
    N, F = ns * R - pad, 70
    lens = np.full(F, N // F, dtype=np.int64)
    lens[-1] += N - lens.sum()
    return lens, N, R


def check_exact(device):
    for name in ("c1_v1", "c1_v2", "v2_b65536_r0_e5", "v2_b65536_r1_e4294967294", "v1_c5_r0"):
        _fixture(name, device)
    for version, B in ((1, 1 << 17), (2, 1 << 16), (2, 5000)):
        lens, N, R = _two_rank_shape(B)
        eng = IndexEngine(lens, N, R, B, version, device=device, order="exact")
        ns = eng.num_samples
        for epoch in (3, 4, 5, 6):   # consecutive: from epoch 5 on the draws were made ahead
            eng.init_iter(epoch)
            old, new = eng.rank_starts()
            out = _gen(eng, 0, R)
            for r in range(R):
                ref = (O.v1_exact_stream(epoch, int(new[r]), ns, B, N) if version == 1 else
                       O.v2_exact_stream_rs(epoch, int(old[r]), int(new[r]), ns, B, N))
                assert np.array_equal(out[r], ref), ("exact", version, B, epoch, r)
        eng.close()


def check_counter(device):
    shapes = [  # (F, L, R, B, version): small pools (lookahead ring; tiles of 4 pools: walks
        # back over several tiles), grouped pools, V1
        (1000, 10_000, 8, 4096, 2), (300, 7_001, 5, 1000, 2), (200, 3_001, 3, 100, 2),
        (20, 10_000, 1, 4096, 2), (500, 20_000, 4, 1 << 17, 2), (1000, 10_000, 8, 4096, 1)]
    for F, L, R, B, version in shapes:
        lens = np.full(F, L, dtype=np.int64)
        N = int(lens.sum())
        eng = IndexEngine(lens, N, R, B, version, device=device, seed=5)
        ns = eng.num_samples
        for epoch in range(4):      # consecutive epochs: the lookahead passes are consumed
            eng.init_iter(epoch)
            old, new = eng.rank_starts()
            out = _gen(eng, 0, R)
            key = O.epoch_key(5, epoch)
            for r in sorted({0, R - 1, epoch % R}):
                ref = (O.v1_philox_stream(key, r, int(new[r]), ns, B, N) if version == 1 else
                       O.v2_philox_stream(key, r, int(old[r]), int(new[r]), ns, B, N))
                assert np.array_equal(out[r], ref), ("counter", F, R, B, version, epoch, r)
                if r == R - 1:   # a position range of the same stream
                    lo = ns // 3
                    part = _gen(eng, r, r + 1, pos_lo=lo, count=ns // 2)[0]
                    assert np.array_equal(part, ref[lo:lo + ns // 2]), ("range", F, R, B, epoch)
        eng.close()


def check_cpu(_device):
    check_exact("cpu")
    check_counter("cpu")


CHECKS = {"exact": check_exact, "counter": check_counter, "cpu": check_cpu}


def main(argv):
    check = argv[0]
    device = "cpu" if check == "cpu" else int(argv[1]) if len(argv) > 1 else 0
    CHECKS[check](device)
    print("knob_worker %s ok (%s)" % (check, " ".join("%s=%s" % (k, v) for k, v in
                                                       sorted(os.environ.items())
                                                       if k.startswith("PSS_"))))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
