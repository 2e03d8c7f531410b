#!/usr/bin/env python
"""Print per-kernel mean counter values from rocprofv3 --pmc pass directories.
Usage: python tools/pmc_table.py DIR [DIR ...] [--match SUBSTR]"""
import csv
import glob
import os
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args = [a for a in args if a != match]
acc = defaultdict(lambda: defaultdict(list))
for d in args:
    for p in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if match and match not in k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print("   %-28s %16.0f" % (c, sum(v) / len(v)))
