"""CPU-side checks of the C-ABI library: it loads, exports exactly what include/pss.h
declares, validates arguments, and its host-side epoch history (CPython-MT file order,
blocks, start_num -- pss_init_iter) matches the reference goldens.  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
from tests.golden_util import fixture_params, load, scenario_names

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pss.h")

_lib = pytest.importorskip("partiallyshuffledistributedsampler_amd._lib")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pss_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert _declared() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.pss_abi_version() == 2


def test_create_validates_arguments():
    lib = _lib.load()
    fl = np.array([3, 4], dtype=np.int64)
    p = fl.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    h = ctypes.c_void_p()
    assert lib.pss_create(p, 2, 7, 0, 4, 1, 1, 0, 0, ctypes.byref(h)) == 1   # R = 0
    assert b"num_replicas" in lib.pss_last_error()
    assert lib.pss_create(p, 2, 7, 2, 0, 1, 1, 0, 0, ctypes.byref(h)) == 1   # B = 0
    assert lib.pss_create(p, 2, 7, 2, 4, 3, 1, 0, 0, ctypes.byref(h)) == 1   # version 3
    assert lib.pss_create(p, 2, 7, 2, 4, 1, 1, 0, 0, ctypes.byref(h)) == 0
    # device work before init_iter is a state error (and touches no GPU)
    assert lib.pss_prepare(h, None) == 4
    assert lib.pss_destroy(h) == 0


@pytest.mark.parametrize("name", scenario_names("v1") + scenario_names("v2"))
def test_host_history_matches_reference(name):
    from partiallyshuffledistributedsampler_amd.engine import IndexEngine
    fx = load(name)
    files, lengths, fl, N, R, B, bs, shuffle = fixture_params(fx)
    version = 1 if fx["version"] == "v1" else 2
    lens = [fl.get(p, lengths[p]) if fl else lengths[p] for p in files]
    eng = IndexEngine(lens, N, R, B, version, shuffle=shuffle)
    assert eng.num_samples == fx["ranks"][0]["num_samples"]
    for i, er0 in enumerate(fx["ranks"][0]["epochs"]):
        eng.init_iter(er0["epoch"])
        assert [files[j] for j in eng.file_order()] == er0["files"]
        assert eng.blocks().tolist() == er0["blocks"]
        old, new = eng.rank_starts()
        for rrec in fx["ranks"]:
            er = rrec["epochs"][i]
            assert (int(old[rrec["rank"]]), int(new[rrec["rank"]])) == (er["old_start"], er["start_num"])


def test_host_history_large_matches_oracle():
    from partiallyshuffledistributedsampler_amd.engine import IndexEngine
    F, R = 100_000, 1024
    N = 1_000_000_000
    for version in (1, 2):
        eng = IndexEngine(np.full(F, N // F), N, R, 4096, version)
        hist = [O.RefHistory(version, F, R, r, N) for r in (0, 517, 1023)]
        for ep in (0, 1, 1, 9):
            eng.init_iter(ep)
            for h in hist:
                h.init_iter(ep)
            assert np.array_equal(eng.file_order(), hist[0].order)
            assert np.array_equal(eng.blocks(), hist[0].blocks)
            old, new = eng.rank_starts()
            for h in hist:
                assert (old[h.rank], new[h.rank]) == (h.old_start, h.start)
