#!/usr/bin/env python
"""Summarise rocprofv3 --pmc passes into profiles/pmc_traffic.json (read by bench.py).

Usage: python tools/pmc_summary.py OUT.json WORKLOAD PASS_DIR [PASS_DIR ...]
(merges the workload's entry into OUT.json: {workload: {kernel: ...}}, the bench.py workload names)

Each PASS_DIR holds one rocprofv3 counter-collection run (csv output).  Per kernel we average
the counters over its dispatches and convert them to HBM bytes per launch the way
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes:
  * WRITE_SIZE and FETCH_SIZE are in KiB;
  * on gfx950 FETCH_SIZE reports half of the bytes of a wide coalesced read, so it is doubled
    (reads are a small share of this path's traffic: O(files + ranks) + the VAL tables);
  * hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Accesses narrower than 16 B per lane are uncalibrated in the guide; the raw counters are
kept next to the derived number.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    base = name.split("(")[0]
    base = base.replace("void ", "").strip()
    return base.split("::")[-1].split("<")[0]


def load(pass_dir):
    """Per kernel, the counters of its dispatches of the LARGEST grid only: a process may launch
    one kernel name at several sizes (torch's fill_ on the 800 MB output and on tiny buffers),
    and averaging them together describes neither."""
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    for p in glob.glob(os.path.join(pass_dir, "**", "*counter_collection*.csv"), recursive=True):
        with open(p) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", ""))
                grid = int(float(row.get("Grid_Size", 0) or 0))
                acc[k][grid][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, grids in acc.items():
        g = max(grids)
        out[k] = grids[g]
        if len(grids) > 1:
            print("%s: counters of grid %d only (other grids: %s)" % (k, g, sorted(x for x in grids if x != g)))
    return out


def main():
    out, workload, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    merged = defaultdict(dict)
    for d in dirs:
        for k, ctrs in load(d).items():
            for c, vals in ctrs.items():
                merged[k][c] = sum(vals) / len(vals)
    res = {}
    for k, c in merged.items():
        ws, fs = c.get("WRITE_SIZE"), c.get("FETCH_SIZE")
        hbm = None
        if ws is not None and fs is not None:
            hbm = (2.0 * fs + ws) * 1024.0
        res[k] = {"counters_per_launch": c, "hbm_bytes_per_launch": hbm,
                  "write_bytes_per_launch": ws * 1024.0 if ws is not None else None,
                  "fetch_bytes_per_launch_corrected": 2.0 * fs * 1024.0 if fs is not None else None}
    try:
        with open(out) as f:
            allres = json.load(f)
    except (OSError, ValueError):
        allres = {}
    allres[workload] = {k: v for k, v in res.items() if k.startswith("k_")}
    with open(out, "w") as f:
        json.dump(allres, f, indent=1, sort_keys=True)
    for k, v in sorted(res.items()):
        print(k, v["hbm_bytes_per_launch"], v["counters_per_launch"])


if __name__ == "__main__":
    main()
