"""Helpers shared by tests that read the reference golden fixtures (tests/golden/*.json)."""
import glob
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def scenario_names(version):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, version + "_*.json"))):
        out.append(os.path.basename(p)[:-5])
    return out


def fixture_params(fx):
    """(files, lengths, files_len_dict, N, R, B, bs, shuffle) of one fixture."""
    cfg = fx["config"]
    lengths = fx["lengths"]
    files = cfg["files"]
    use_fl = cfg.get("files_len", True)
    fl = cfg.get("files_len_dict", lengths) if use_fl else {}
    N = sum(fl.values()) if use_fl else cfg["total_size"]
    return files, lengths, fl, N, cfg["R"], cfg["B"], cfg["bs"], cfg.get("shuffle", True)


def length_of_fn(lengths, fl):
    def f(path):
        return fl[path] if path in fl else lengths[path]
    return f
