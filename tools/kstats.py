"""Summarise a rocprofv3 --stats kernel_stats.csv: short names, calls, average and total time, share."""
import csv
import sys


def short(name: str) -> str:
    if "::" in name:
        name = name.split("::")[-1] if "anonymous" not in name else name.split("::", 1)[1]
    return name.split("(")[0][:40]


def main(path, top=16):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':40s} {'calls':>7s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}")
    for r in rows[:top]:
        print(f"{short(r['Name']):40s} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['TotalDurationNs']) / 1e6:9.2f} {float(r['TotalDurationNs']) / tot * 100:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 16)
