"""Summarise an A/B directory of bench lines: G idx/s and dominant-kernel launch time per run."""
import glob
import json
import sys

for d in sys.argv[1:]:
    rows = {}
    for f in sorted(glob.glob(d + "/*.json")):
        try:
            j = json.loads(open(f).read().strip().splitlines()[-1])
        except Exception:
            print(f, "unreadable")
            continue
        tag = f.rsplit("/", 1)[1].rsplit("_", 1)[0]
        rows.setdefault(tag, []).append((j["value"], j["roofline"]["launch_ms"] * 1e3))
    for tag, v in rows.items():
        print("%-10s G idx/s %s   launch us %s" % (tag, " ".join("%.1f" % a for a, _ in v),
                                                  " ".join("%.1f" % b for _, b in v)))
