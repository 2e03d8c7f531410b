"""Summary of a tools/gpu_split.sh output directory: cold C5 exact ms per epoch (split / workgroup
form) and, from the kernel trace, the last cold epoch's split-draw launches."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "cold_*.json"))):
    line = open(f).read().strip().splitlines()[-1]
    print(os.path.basename(f), round(json.loads(line)["ms_per_step"], 3))
tr = os.path.join(d, "prof", "run_kernel_trace.csv")
if os.path.exists(tr):
    t = sorted(csv.DictReader(open(tr)), key=lambda x: int(x["Start_Timestamp"]))
    last_gen = max(i for i, x in enumerate(t) if "sp_gen" in x["Kernel_Name"])
    b = int(t[last_gen]["Start_Timestamp"])
    for x in t[last_gen:]:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        print(f'{(s - b) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {x["Kernel_Name"].split("(")[0][:40]} grid={x["Grid_Size_X"]}x{x["Grid_Size_Y"]}')
