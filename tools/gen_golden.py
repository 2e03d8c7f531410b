#!/usr/bin/env python
"""Generate golden vectors from the *reference* sampler (run in the build container only).

This script imports the two reference modules read-only from ``/root/reference`` and records
what they produce on small synthetic inputs.  It is the only place the reference is executed;
the fixtures it writes (``tests/golden/*.json``) are data (inputs + expected outputs), and the
reference never travels with the repo.

Harness-side shims (reference files untouched):
  * ``torch.utils.data.Sampler.__init__`` accepts ``data_source`` again (torch 2.x removed it;
    the reference calls ``super().__init__(dataset)`` at V1:18 / V2:18).
  * the modules' ``gc`` global is replaced by a no-op ``collect`` (V1:85,109,258; V2:81,133,253)
    purely for speed -- it has no semantic effect.

Raw id streams are captured observationally with ``sys.settrace``: at V1:178 / V2:181
(``batch_ids = []``) the local ``indices`` holds the batch's generated ids before mapping.

Usage:  python tools/gen_golden.py   (writes tests/golden/)
"""
import importlib.util
import json
import os
import random
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

V1_FILE = os.path.join(REF, "DistributedSamplerViaLocallyShuffle.py")
V2_FILE = os.path.join(REF, "DistributedSamplerViaLocallyShuffleV2.py")
V1_CAPTURE_LINE = 178   # `batch_ids = []` right after the V1 generation loop (V1:157-172)
V2_CAPTURE_LINE = 181   # `batch_ids = []` right after `indices = self.get_index()` (V2:176)


def _load(name, path):
    import torch.utils.data as tud
    tud.Sampler.__init__ = lambda self, data_source=None: None
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.gc = types.SimpleNamespace(collect=lambda: 0)
    return mod


class Dataset:
    """The reference's `dataset` protocol: `.files` + `.reset()` (V1:101, V1:271-278)."""

    def __init__(self, files):
        self.files = list(files)

    def reset(self):
        pass


def make_reader(lengths, calls=None):
    """Reader protocol (README.md:17-33): reader(path, get_data=False) -> len | (dict, len)."""
    index = {p: i for i, p in enumerate(sorted(lengths))}

    def reader(path, get_data=False):
        n = lengths[path]
        if calls is not None:
            calls.append((path, bool(get_data)))
        if not get_data:
            return n
        return {"fid": np.full(n, index[path], dtype=np.int64),
                "off": np.arange(n, dtype=np.int64)}, n
    return reader


def next_with_capture(it, path, line):
    cap = {}

    def local(frame, event, arg):
        if event == "line" and frame.f_lineno == line and "indices" not in cap:
            cap["indices"] = [int(x) for x in frame.f_locals["indices"]]
        return local

    def glob(frame, event, arg):
        if frame.f_code.co_filename == path and frame.f_code.co_name in ("__next__",):
            return local
        return None

    sys.settrace(glob)
    try:
        out = next(it)
        stop = False
    except StopIteration:
        out, stop = None, True
    finally:
        sys.settrace(None)
    return cap.get("indices"), out, stop


def encode_output(out):
    target_datas, none, read_files = out
    assert none is None
    return {"read_files": list(read_files),
            "off": [[int(x) for x in d["off"]] for d in target_datas],
            "fid": [[int(x) for x in d["fid"]] for d in target_datas]}


def run_epochs(mod, path, line, cfg, rank, outputs=True):
    lengths = cfg["lengths"]
    files = cfg["files"]
    reader = make_reader(lengths)
    kw = dict(num_replicas=cfg["R"], rank=rank, shuffle=cfg.get("shuffle", True),
              shuffle_buffer=cfg["B"], total_size=cfg.get("total_size", 1),
              batch_size=cfg["bs"], file_buffer=cfg.get("file_buffer", 10))
    if cfg.get("files_len", True):
        kw["files_len"] = dict(cfg.get("files_len_dict", lengths))
    s = mod.DistributedSamplerViaLocallyShuffle(Dataset(files), reader, **kw)
    rec = {"rank": rank, "num_samples": s.num_samples, "ori_total_size": s.ori_total_size,
           "len": len(s), "epochs": []}
    for ep in cfg["epochs"]:
        er = {}
        if isinstance(ep, dict):           # {"epoch": e, "resume_step": k}
            s.set_epoch(ep["epoch"])
            er["epoch"] = ep["epoch"]
            er["resume_step"] = ep["resume_step"]
            er["old_start"] = s.start_num
            s.find_ckpt_position(ep["resume_step"])
        else:
            s.set_epoch(ep)
            er["epoch"] = ep
            er["old_start"] = s.start_num
        it = iter(s)
        er["files"] = list(s.files)
        er["blocks"] = list(s.blocks)
        er["start_num"] = s.start_num
        batches, outs = [], []
        nb = 0
        while True:
            idx, out, stop = next_with_capture(it, path, line)
            if idx is not None:
                batches.append(idx)
            if stop:
                break
            if outputs and nb < cfg.get("max_out_batches", 10 ** 9):
                outs.append(encode_output(out))
            nb += 1
        er["batches"] = batches
        er["num_batches"] = nb
        if outputs:
            er["outputs"] = outs
        rec["epochs"].append(er)
    return rec


def mt_kats():
    r = random.Random()
    seeds = [0, 1, 7, 10007, 2 ** 32 - 1, 2 ** 32, 2 ** 32 + 5, 10 ** 10, 2 ** 64 + 3,
             123456789012345678901234567890, -5, 30000, 1230002]
    out = {"genrand": [], "shuffle": [], "randbelow": [], "choice": []}
    for s in seeds:
        r.seed(s)
        out["genrand"].append({"seed": s, "u32": [r.getrandbits(32) for _ in range(700)]})
    for s in (0, 3, 20001):
        for n in (1, 2, 3, 4, 5, 17, 100, 1023, 1024, 1025, 4096):
            r.seed(s)
            x = list(range(n))
            r.shuffle(x)
            out["shuffle"].append({"seed": s, "n": n, "perm": x})
    r.seed(42)
    ns = [1, 2, 3, 5, 7, 8, 9, 1000, 4095, 4096, 4097, 65536, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 1]
    out["randbelow"] = {"seed": 42, "n": ns * 5, "r": [r._randbelow(n) for n in ns * 5]}
    r.seed(9)
    ns2 = [1, 3, 10, 300, 4096, 5000] * 10
    out["choice"] = {"seed": 9, "n": ns2, "r": [r.choice(list(range(n))) for n in ns2]}
    return out


def cfg_lengths(lens, prefix="f"):
    files = ["%s%03d" % (prefix, i) for i in range(len(lens))]
    return files, dict(zip(files, lens))


def main():
    os.makedirs(OUT, exist_ok=True)
    v1 = _load("ref_v1", V1_FILE)
    v2 = _load("ref_v2", V2_FILE)

    with open(os.path.join(OUT, "mt_kats.json"), "w") as f:
        json.dump(mt_kats(), f)

    rng = np.random.default_rng(12345)
    scen = {}

    files, lens = cfg_lengths([37, 120, 5, 64, 200, 1, 99, 33])
    scen["small"] = dict(files=files, lengths=lens, R=3, B=16, bs=7, epochs=[0, 1, 2, 2, 5])
    scen["noshuffle"] = dict(files=files, lengths=lens, R=3, B=16, bs=7, epochs=[0, 1, 3],
                             shuffle=False)
    # files_len has keys that are not in dataset.files -> N > scanned total -> reflection
    # (V1:191-196); the extra key is sorted last so it is also out of the file order.
    extra = dict(lens)
    extra["zz_extra"] = 50
    scen["reflect"] = dict(files=files, lengths=lens, files_len_dict=extra, R=2, B=32, bs=16,
                           epochs=[0, 1])
    files, lens = cfg_lengths([int(x) for x in rng.integers(100, 300, 64)])
    scen["c1_small"] = dict(files=files, lengths=lens, R=2, B=64, bs=32, epochs=[0, 1, 2],
                            max_out_batches=4)
    files, lens = cfg_lengths([int(x) for x in np.clip(rng.zipf(1.5, 60) * 15, 1, 900)])
    scen["zipf"] = dict(files=files, lengths=lens, R=7, B=40, bs=64, epochs=[0, 1, 2],
                        max_out_batches=3)
    files, lens = cfg_lengths([10, 11, 12, 13])
    scen["tiny_ns_lt_B"] = dict(files=files, lengths=lens, R=2, B=100, bs=5, epochs=[0, 4])
    scen["ns_between_B_2B"] = dict(files=files, lengths=lens, R=2, B=15, bs=4, epochs=[0, 1])
    scen["bs1"] = dict(files=files, lengths=lens, R=2, B=8, bs=1, epochs=[0])
    scen["resume"] = dict(files=files, lengths=lens, R=2, B=6, bs=4,
                          epochs=[0, {"epoch": 1, "resume_step": 3}, 2])
    files, lens = cfg_lengths([17, 29, 3, 41, 8])
    scen["no_files_len"] = dict(files=files, lengths=lens, R=2, B=9, bs=5, epochs=[0, 1],
                                files_len=False, total_size=98)
    scen["exact_div"] = dict(files=files, lengths=lens, R=2, B=7, bs=7, epochs=[3])

    for name, cfg in scen.items():
        for ver, mod, path, line in (("v1", v1, V1_FILE, V1_CAPTURE_LINE),
                                     ("v2", v2, V2_FILE, V2_CAPTURE_LINE)):
            if name == "noshuffle" and ver == "v2":
                pass  # V2 ignores shuffle (V2:142-152); still recorded as a quirk fixture
            recs = [run_epochs(mod, path, line, cfg, r) for r in range(cfg["R"])]
            fx = {"version": ver, "name": name,
                  "config": {k: v for k, v in cfg.items() if k not in ("lengths",)},
                  "lengths": cfg["lengths"], "ranks": recs}
            with open(os.path.join(OUT, "%s_%s.json" % (ver, name)), "w") as f:
                json.dump(fx, f, separators=(",", ":"))
            print("wrote", ver, name)


if __name__ == "__main__":
    main()
