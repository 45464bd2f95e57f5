"""Timeline / gap analysis of a rocprofv3 kernel trace (CSV): per-kernel mean duration and
mean gap before each kernel, over the LAST N occurrences of a marker kernel's epoch.
    python tools/timeline.py gpurun_out/trace_a/trace_kernel_trace.csv"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
    # an epoch = 16 k_policy_step (rollout) followed by the update ending at a k_apply
    # that is the 64th in a run; take the second-to-last complete epoch (graph-replayed)
    applies = [i for i, e in enumerate(ev) if e[2] == "k_apply"]
    ends = [applies[k] for k in range(len(applies)) if k + 1 == len(applies) or applies[k + 1] - applies[k] > 4]
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    end = ends[which]
    pol = [i for i, e in enumerate(ev[:end]) if e[2] == "k_policy_step"]
    start = pol[-16]
    seg = ev[start:end + 1]
    dur = defaultdict(list)
    gap = defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(seg, seg[1:]):
        gap[n1].append(s1 - e0)
    for s, e, n in seg:
        dur[n].append(e - s)
    total = (seg[-1][1] - seg[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in seg) / 1e3
    print(f"epoch span {total:.1f} us, kernel busy {busy:.1f} us, gaps {total - busy:.1f} us, {len(seg)} kernels")
    print(f"{'kernel':24s} {'n':>4s} {'mean us':>8s} {'sum us':>8s} {'gap-before us':>14s} {'gap sum':>8s}")
    for n in sorted(dur, key=lambda k: -sum(dur[k])):
        d = dur[n]
        g = gap.get(n, [0])
        print(f"{n:24s} {len(d):4d} {sum(d) / len(d) / 1e3:8.2f} {sum(d) / 1e3:8.1f} {sum(g) / len(g) / 1e3:14.2f} "
              f"{sum(g) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
