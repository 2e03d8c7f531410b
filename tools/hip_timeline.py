"""Merged host-API / kernel timeline of a rocprofv3 --hip-trace --kernel-trace run around the
n-th launch of a kernel (how the host paces a loop: blocking calls against kernel spans).
usage: python tools/hip_timeline.py <rocprofv3 output dir> <kernel-name substring> [n] [before_us] [after_us]"""
import csv
import glob
import os
import sys


def main(d, key, n=14, before=600.0, after=300.0):
    api = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])))
    kt = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in kt)
    main_ = [(s, e) for s, e, k in ev if key in k]
    t0 = main_[n][0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API " + r["Function"]) for r in api]
    rows += [(s, e, "GPU " + k[-50:]) for s, e, k in ev]
    for s, e, k in sorted(rows):
        if t0 - before * 1e3 <= s < t0 + after * 1e3 and (e - s > 2000 or k.startswith("GPU")):
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {k}")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], *(int(a[2]),) if len(a) > 2 else (), *(float(x) for x in a[3:5]))
