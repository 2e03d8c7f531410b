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


# ---- bench-scale fixtures (tests/golden/big, tools/gen_golden_big.py) ----------------------
BIG = os.path.join(GOLDEN, "big")


def big_names(kind=None):
    out = []
    for p in sorted(glob.glob(os.path.join(BIG, "*.json"))):
        name = os.path.basename(p)[:-5]
        if kind is None or load_big(name)["kind"] == kind:
            out.append(name)
    return out


def load_big(name):
    with open(os.path.join(BIG, name + ".json")) as f:
        return json.load(f)


def load_big_streams(name):
    """Full raw streams of a fixture stored whole ({"r<rank>_e<epoch>": int64 array})."""
    import numpy as np
    with np.load(os.path.join(BIG, name + ".npz")) as z:
        return {k: z[k].astype(np.int64) for k in z.files}


def sha256_i64(a):
    """sha256 of an id array as little-endian int64 (the fixtures' stream digest)."""
    import hashlib
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i8").tobytes()).hexdigest()


def big_lengths(fx):
    """files_len (dataset order) of a bench-scale fixture; checked against its recorded hash."""
    import numpy as np
    if "lengths" in fx:
        return np.asarray(fx["lengths"], dtype=np.int64)
    if "uniform" in fx:
        F, L = fx["uniform"]
        return np.full(F, L, dtype=np.int64)
    import workloads as W
    ln = W.lengths(fx["config"]).astype(np.int64)
    assert sha256_i64(ln) == fx["lengths_sha256"], "workloads.py no longer makes the fixture's files"
    return ln


def check_stream(got, er, fx, what=""):
    """Assert one rank-epoch id stream equals the fixture record (whole-stream sha256; a prefix
    fixture compares its first `prefix` ids).  On a mismatch, say where it starts."""
    import numpy as np
    got = np.asarray(got, dtype=np.int64)
    if fx["kind"] == "prefix":
        got = got[:fx["prefix"]]
        assert len(got) == fx["prefix"], what
    else:
        assert len(got) == er["count"], (what, len(got), er["count"])
    if sha256_i64(got) == er["sha256"]:
        return
    head = np.asarray(er.get("head", []), dtype=np.int64)
    bad = np.nonzero(got[:len(head)] != head)[0]
    where = "head[%d]" % bad[0] if len(bad) else "after the head"
    if "window_sha256" in er:
        B = fx["B"]
        ws = [sha256_i64(got[w:w + B]) for w in range(0, len(got), B)]
        where += "; windows differing: %s" % [i for i, (a, b) in
                                             enumerate(zip(ws, er["window_sha256"])) if a != b]
    raise AssertionError("%s: stream differs from the reference (%s)" % (what, where))


def check_multiset(got, er, what=""):
    import numpy as np
    got = np.asarray(got, dtype=np.int64)
    assert len(got) == er["count"], what
    assert sha256_i64(np.sort(got)) == er["sorted_sha256"], "%s: multiset differs" % what
