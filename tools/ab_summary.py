"""Summarise an A/B directory (tools/gpu_run.sh ab:/env: steps): per tag,
G idx/s and the dominant kernel's launch time (bench.py lines) or ms per epoch
(tools/bench_configs.py lines), one column per run."""
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
        if "roofline" in j:
            rows.setdefault(tag, []).append((j["value"], "launch us", j["roofline"]["launch_ms"] * 1e3))
        else:
            rows.setdefault(tag, []).append((j["G_idx_per_s"], "ms/epoch", j["ms_per_step"]))
    for tag, v in rows.items():
        print("%-14s G idx/s %s   %s %s" % (tag, " ".join("%.2f" % a for a, _, _ in v), v[0][1],
                                          " ".join("%.2f" % c for _, _, c in v)))
