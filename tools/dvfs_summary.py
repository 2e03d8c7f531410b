"""Replay launch durations of tools/dvfs_probe.py's trace, per phase of 40 epochs."""
import csv
import sys

t = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in t
     if "k_v2_emit_x" in x["Kernel_Name"] and x["Grid_Size_X"] == "131072"]
for i, name in enumerate(("back to back", "3 ms idle after each", "back to back again")):
    p = d[40 * i:40 * (i + 1)]
    if p:
        print(f"{name:24s} n {len(p)}  mean {sum(p) / len(p):6.1f} us  min {min(p):6.1f}  max {max(p):6.1f}  "
              f"first 5 {[round(x, 1) for x in p[:5]]}")
