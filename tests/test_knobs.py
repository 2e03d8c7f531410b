"""Every environment switch the library reads is run by a test.

The C++/HIP sources read their PSS_* switches once per process, so each forced setting runs
tests/knob_worker.py in a child interpreter with the variable set before any GPU call:

  PSS_V1X_DRAWS_WG / PSS_V2X_DRAWS_WG  0 / 1 force the one-wave / workgroup MT draws of the
                                       exact orders (by default chosen by geometry)
  PSS_V1X_GRID2D=1                     the exact V1 HBM path's kernels on their 2-D grids (window
                                       slot in blockIdx.y) instead of the XCD-major flat grids
  PSS_V2_LOOKAHEAD=0                   no epoch lookahead: the V2 last-occurrence passes run in
                                       line on the caller's stream
  PSS_EXACT_LOOKAHEAD=0                no exact-order draw lookahead: every exact V2 call makes its
                                       own MT draws
  PSS_EXACT_SPLIT=0 / 1                  the exact V2 draws of a call without a prepared slot: the
                                       workgroup form / the split form (pss_v2split.h) even for
                                       short windows (by default the split form for long windows)
  PSS_CPU_THREADS=1 / 3                host threads of the CPU mode

`test_every_knob_is_covered` fails when a source gains a getenv that is not listed here.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "partiallyshuffledistributedsampler_amd", "csrc")

GPU_CASES = [
    ("exact", {"PSS_V1X_DRAWS_WG": "0", "PSS_V2X_DRAWS_WG": "0"}),
    ("exact", {"PSS_V1X_DRAWS_WG": "1", "PSS_V2X_DRAWS_WG": "1"}),
    ("exact", {"PSS_V1X_GRID2D": "1"}),
    ("exact", {"PSS_EXACT_LOOKAHEAD": "0"}),
    ("exact", {"PSS_EXACT_SPLIT": "0"}),
    ("exact", {"PSS_EXACT_SPLIT": "1", "PSS_EXACT_LOOKAHEAD": "0"}),
    ("counter", {"PSS_V2_LOOKAHEAD": "0"}),
]
CPU_CASES = [("cpu", {"PSS_CPU_THREADS": "1"}), ("cpu", {"PSS_CPU_THREADS": "3"})]


def _source_knobs():
    names = set()
    for f in os.listdir(CSRC):
        if f.endswith((".cpp", ".hip", ".h")):
            names |= set(re.findall(r'getenv\("(PSS_[A-Z0-9_]+)"\)', open(os.path.join(CSRC, f)).read()))
    return names


def _run(check, env):
    e = dict(os.environ)
    for k in list(e):
        if k.startswith("PSS_"):
            del e[k]
    e.update(env)
    r = subprocess.run([sys.executable, "-m", "tests.knob_worker", check], cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (env, r.stdout[-2000:], r.stderr[-4000:])
    assert "knob_worker %s ok" % check in r.stdout


def test_every_knob_is_covered():
    covered = {k for _, env in GPU_CASES + CPU_CASES for k in env}
    assert _source_knobs() == covered


@pytest.mark.parametrize("check,env", CPU_CASES, ids=lambda x: str(x))
def test_cpu_mode_under_forced_knob(check, env):
    _run(check, env)


@pytest.mark.gpu
@pytest.mark.parametrize("check,env", GPU_CASES, ids=lambda x: str(x))
def test_gpu_parity_under_forced_knob(check, env):
    _run(check, env)
