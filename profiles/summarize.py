"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (per-call and share)."""
import csv
import sys


def main(path, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}")
    for r in rows[:top]:
        name = r["Name"].replace("(anonymous namespace)::", "")[:60]
        print(f"{name:60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['TotalDurationNs']) / 1e6:9.3f} {100 * float(r['TotalDurationNs']) / tot:6.2f}")
    print(f"total GPU kernel time {tot / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
