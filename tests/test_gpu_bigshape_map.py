"""The prologue kernels at the true C3 / C4 shapes on the GPU: the device
prefix scan over 100K shuffled files (multi-chunk), the bucket-indexed id -> (file, offset) map
(C4: N = 2,594,705,250 > 2^31, 64-bit prefixes, kb ~ 14), the file -> rank partition and the
fused hand-off, through the C-ABI.

The file order they scan is the engine's, itself pinned to the reference's own order at these
shapes (tests/golden/big/assign_c3.json / assign_c4.json, captured from the reference).  Against
that order's exclusive prefix (V1:181-190, computed here on the host):
  * pss_map of whole rank streams (rank 0, the ranks whose block wraps at N, ranks whose ids all
    lie above 2^31) == the oracle's map (oracle.map_ids, V1:181-221), element for element;
  * pss_partition of EVERY rank == the oracle's segments (oracle.partition_segments), and each
    picked rank's segment lengths == the per-file counts of its mapped stream;
  * every id of every rank: the map characterised on the device (prefix[f] + off == id,
    0 <= off < len[f]) and pss_generate_mapped == pss_generate + pss_map.
Both versions (V1 windows and V2 two-pool ranges), two epochs of the cumulative history.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.golden_util import load_big, sha256_i64
import workloads as W

pytestmark = pytest.mark.gpu

pss = pytest.importorskip("partiallyshuffledistributedsampler_amd.engine")


def _picks(version, old, new, ns, B, N, R):
    wrap = [r for r in range(R) if int(new[r]) + ns > N or (version == 2 and int(old[r]) + 2 * B > N)]
    lo_v2 = (lambda r: min(int(old[r]), int(new[r]) + 2 * B)) if version == 2 else (lambda r: int(new[r]))
    hi = [r for r in range(R) if lo_v2(r) > 2 ** 31][:2]
    return sorted({0, R - 1} | set(wrap[:2]) | set(hi)), hi


@pytest.mark.parametrize("cfg,version", [("c4", 2), ("c4", 1), ("c3", 2)])
def test_scan_map_partition_at_bench_shape(cfg, version):
    lengths, N, R, B, _ = W.shape(cfg)
    fx = load_big("assign_" + cfg)
    assert fx["N"] == N and fx["R"] == R
    eng = pss.IndexEngine(lengths, N, R, B, version, device=0, seed=0)
    ns = eng.num_samples
    for rec in fx["versions"]["v%d" % version][:2]:            # init_iter(0), init_iter(1)
        eng.init_iter(rec["epoch"])
        order = eng.file_order()
        assert sha256_i64(order.astype(np.int64)) == rec["order_sha256"]   # the reference's order
        prefix = np.concatenate([[0], np.cumsum(lengths[order])]).astype(np.int64)
        old, new = eng.rank_starts()
        picks, hi = _picks(version, old, new, ns, B, N, R)
        if cfg == "c4":
            assert hi, "no rank with ids above 2^31"
        # whole rank streams: device map == oracle map; fused hand-off == generate + map
        for r in picks:
            ids = eng.generate(r, r + 1)
            eng.check()
            f, o = eng.map(ids.view(-1))
            rf, ro = O.map_ids(prefix, ids.cpu().numpy().reshape(-1))
            assert np.array_equal(f.cpu().numpy(), rf), (cfg, version, rec["epoch"], r)
            assert np.array_equal(o.cpu().numpy(), ro), (cfg, version, rec["epoch"], r)
            fm, om = eng.generate_mapped(r, r + 1)
            eng.check()
            assert torch.equal(fm.view(-1), f) and torch.equal(om.view(-1).long(), o), r
            lo, cnt = ns // 3 + 5, ns // 2               # a ragged position range
            f2, o2 = eng.generate_mapped(r, r + 1, lo, cnt)
            assert torch.equal(f2.view(-1), f[lo:lo + cnt]) and torch.equal(o2.view(-1).long(), o[lo:lo + cnt])
        if cfg == "c4":
            assert int(eng.generate(hi[0], hi[0] + 1).min()) > 2 ** 31
        # the partition of every rank == the oracle's segments
        seg_off, sf, sl, sh = eng.partition(0, R)
        for r in range(R):
            a, b = int(seg_off[r]), int(seg_off[r + 1])
            wf, wl, wh = O.partition_segments(version, prefix, int(old[r]), int(new[r]), ns, B, N)
            assert np.array_equal(sf[a:b], wf) and np.array_equal(sl[a:b], wl) and np.array_equal(sh[a:b], wh), r
        for r in picks:     # segments == what the rank's stream reads, file by file
            a, b = int(seg_off[r]), int(seg_off[r + 1])
            f, _ = eng.map(eng.generate(r, r + 1).view(-1))
            cnt = np.bincount(f.cpu().numpy(), minlength=len(lengths))
            seg = np.zeros(len(lengths), dtype=np.int64)
            np.add.at(seg, sf[a:b], sh[a:b] - sl[a:b])
            assert np.array_equal(cnt, seg), r
        # every id of every rank, on the device
        pre_d = torch.from_numpy(prefix).cuda()
        len_d = torch.from_numpy(lengths[order].astype(np.int64)).cuda()
        chunk = 512
        for lo in range(0, R, chunk):
            ids = eng.generate(lo, min(R, lo + chunk)).view(-1)
            f, o = eng.map(ids)
            fl = f.long()
            assert bool((f >= 0).all())                  # files_len complete: nothing reflects
            assert bool(((o >= 0) & (o < len_d[fl])).all())
            assert torch.equal(pre_d[fl] + o, ids)
            del fl
            fm, om = eng.generate_mapped(lo, min(R, lo + chunk))
            assert torch.equal(fm.view(-1), f) and torch.equal(om.view(-1).long(), o), lo
            del ids, f, o, fm, om
        eng.check()
    eng.close()
