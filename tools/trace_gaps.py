"""Timeline of a rocprofv3 kernel trace: per-dispatch start/end relative to the first replay,
and the idle gap between consecutive launches of the named kernel (tools/gpu_trace_c2.sh)."""
import csv, sys

def main(path, key):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:], r["Queue_Id"]) for r in rows)
    t0 = next(s for s, e, n, q in ev if key in n)
    main_ = [(s, e) for s, e, n, q in ev if key in n]
    gaps = [main_[i + 1][0] - main_[i][1] for i in range(len(main_) - 1)]
    for s, e, n, q in ev:
        if s >= t0 and s < t0 + 60 * 200000:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{q} {n}")
    g = sorted(gaps[5:])
    print(f"{key}: launches {len(main_)}, dur mean {sum(e - s for s, e in main_[5:]) / len(main_[5:]) / 1e3:.1f} us,"
          f" gap median {g[len(g) // 2] / 1e3:.1f} us mean {sum(g) / len(g) / 1e3:.1f} max {g[-1] / 1e3:.1f}")
    per = [(main_[i + 1][0] - main_[i][0]) for i in range(5, len(main_) - 1)]
    print(f"start-to-start mean {sum(per) / len(per) / 1e3:.1f} us")

if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
