#!/usr/bin/env python
"""Per-kernel launch times from a rocprofv3 --kernel-trace CSV, split by grid size.

rocprofv3's --stats table averages every dispatch of a kernel name together, so a kernel that
runs at two sizes in one process (torch's fill_ on the 800 MB output and on a few tiny buffers)
reports a mean that describes neither (24 fill_ dispatches, 3 of them
tiny).  This groups the trace's dispatches by (kernel, grid size) instead.

Usage: python tools/trace_by_grid.py <rocprofv3 output dir or kernel_trace.csv> [bytes] [name-substring ...]
  bytes: algorithmic bytes of the largest-grid dispatch of each listed kernel (default 800000000,
         the C2 / C5 epoch's 100M int64 ids), reported as GB/s and as a fraction of 8 TB/s.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

PEAK = 8000.0


def trace_files(path):
    if os.path.isfile(path):
        return [path]
    return glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)


def main(argv):
    path = argv[0]
    nbytes = float(argv[1]) if len(argv) > 1 else 8e8
    pats = argv[2:]
    acc = defaultdict(list)
    for f in trace_files(path):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if pats and not any(p in name for p in pats):
                    continue
                grid = int(float(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
                dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3   # us
                acc[(name, grid)].append(dt)
    largest = {}
    for (name, grid) in acc:
        largest[name] = max(largest.get(name, 0), grid)
    print("%-70s %10s %6s %10s %10s %10s" % ("kernel", "grid", "n", "mean us", "min us", "GB/s*"))
    for (name, grid), v in sorted(acc.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        mean = sum(v) / len(v)
        rate = ""
        if grid == largest[name]:
            rate = "%.0f (%.3f)" % (nbytes / (mean * 1e-6) / 1e9, nbytes / (mean * 1e-6) / 1e9 / PEAK)
        print("%-70s %10d %6d %10.1f %10.1f %s" % (name[:70], grid, len(v), mean, min(v), rate))
    print("* GB/s of the largest-grid dispatches at %.0f algorithmic bytes each, "
          "(fraction of the 8 TB/s spec)" % nbytes)


if __name__ == "__main__":
    main(sys.argv[1:])
