"""Print the kernel timeline around one mid-run k_policy_step of a rocprofv3 kernel trace (CSV):
start/end relative to that launch, duration, queue id, name.   python tools/steptrace.py trace.csv [count]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 24

    def name(r):
        m = re.search(r"(k_[a-z_0-9]+)", r["Kernel_Name"])
        return m.group(1) if m else r["Kernel_Name"][:30]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), name(r)) for r in rows)
    idx = [i for i, e in enumerate(ev) if e[3] == "k_policy_step"]
    i0 = idx[len(idx) // 2]
    t0 = ev[i0][0]
    for s, e, q, n in ev[i0 - 2:i0 + cnt]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:>3s}  {n}")


if __name__ == "__main__":
    main()
