#!/usr/bin/env python
"""Golden vectors of the reference's lazy length probing (run in the build container only).

When a file's length is not in `files_len`, the reference probes it with
reader(path, get_data=False) while it extends `past_files_samples` in shuffled scan order
(V1:182-190, V2:185-193), and it restarts that scan every epoch (V1:126).  This script runs
the reference (imported read-only from /root/reference with gen_golden.py's harness shims) and
records, per rank and epoch, the ordered list of probe calls and the batches' file groups,
for files_len absent and partially given.  Output: tests/golden/probes_{v1,v2}.json (data only).

Usage:  python tools/gen_golden_probes.py
"""
import json
import os
import sys

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402


def run(mod, cfg, rank):
    calls = []
    reader = G.make_reader(cfg["lengths"], calls)
    kw = dict(num_replicas=cfg["R"], rank=rank, shuffle_buffer=cfg["B"],
              total_size=cfg["total_size"], batch_size=cfg["bs"])
    if cfg.get("files_len_dict") is not None:
        kw["files_len"] = dict(cfg["files_len_dict"])
    s = mod.DistributedSamplerViaLocallyShuffle(G.Dataset(cfg["files"]), reader, **kw)
    rec = {"rank": rank, "epochs": []}
    for ep in cfg["epochs"]:
        s.set_epoch(ep)
        it = iter(s)
        del calls[:]
        groups = []
        while True:
            try:
                out = next(it)
            except StopIteration:
                break
            groups.append(list(out[2]))
        probes = [p for p, get_data in calls if not get_data]
        rec["epochs"].append({"epoch": ep, "probes": probes, "read_files": groups})
    return rec


def main():
    v1 = G._load("ref_v1", G.V1_FILE)
    v2 = G._load("ref_v2", G.V2_FILE)
    files, lens = G.cfg_lengths([17, 29, 3, 41, 8, 55, 12, 30, 6, 19])
    total = sum(lens.values())
    partial = {p: n for i, (p, n) in enumerate(lens.items()) if i % 3 == 0}
    scen = [
        dict(name="none", files=files, lengths=lens, R=3, B=9, bs=5, epochs=[0, 1, 2],
             total_size=total, files_len_dict=None),
        # a partial table: N is the sum of its values only (V1:29-31); files missing from it
        # are probed as the scan reaches them
        dict(name="partial", files=files, lengths=lens, R=2, B=16, bs=8, epochs=[0, 1],
             total_size=1, files_len_dict=partial),
    ]
    for ver, mod in (("v1", v1), ("v2", v2)):
        out = {"version": ver, "scenarios": []}
        for cfg in scen:
            recs = [run(mod, cfg, r) for r in range(cfg["R"])]
            out["scenarios"].append({"name": cfg["name"],
                                     "config": {k: v for k, v in cfg.items() if k != "name"},
                                     "ranks": recs})
        with open(os.path.join(G.OUT, "probes_%s.json" % ver), "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print("wrote probes_%s.json" % ver)


if __name__ == "__main__":
    main()
