"""Condense a rocprofv3 --kernel-trace CSV into one rollout epoch's timeline (the last epoch's 16 env steps):
kernel, queue, start / end relative to the epoch's first k_step_begin, in us.  Prints per-step spans and the
idle time on the GPU (no kernel running) inside the rollout.
    python tools/rollout_timeline.py <kernel_trace.csv> <out.csv>"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id", r.get("Stream_Id", ""))
        ks.append((s, e, name, q))
    ks.sort()
    # the rollout windows: from a k_step_begin to the first k_mb_grad after it
    begins = [i for i, k in enumerate(ks) if "k_step_begin" in k[2]]
    grads = [i for i, k in enumerate(ks) if "k_mb_grad" in k[2]]
    # rollouts: runs of 16 step_begins between gradient kernels; the last one with no timing spin kernel in
    # it (the bench's graph-replayed epochs, not its eager launch-timing epoch)
    groups, cur = [], []
    gi = 0
    for b in begins:
        while gi < len(grads) and grads[gi] < b:
            gi += 1
            if cur:
                groups.append(cur)
                cur = []
        cur.append(b)
    if cur:
        groups.append(cur)
    cands = []
    for g in groups:
        if len(g) < 16 or not any(x > g[-1] for x in grads):
            continue
        a = ks[g[0]][0]
        z = ks[min(x for x in grads if x > g[-1])][0]
        if not any("spin_kernel" in k[2] for k in ks if a <= k[0] < z):
            cands.append(g[-16:])
    bs = cands[-1]
    t0 = ks[bs[0]][0]
    t_end = ks[min(g for g in grads if g > bs[-1])][0]
    print("queues in the window:", sorted({k[3] for k in ks if t0 <= k[0] < t_end}))
    win = [k for k in ks if t0 <= k[0] < t_end]
    with open(sys.argv[2], "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "queue", "start_us", "end_us", "dur_us"])
        for s, e, n, q in win:
            short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
            w.writerow([short, q, f"{(s - t0) / 1e3:.2f}", f"{(e - t0) / 1e3:.2f}", f"{(e - s) / 1e3:.2f}"])
    # busy union
    busy, cur_s, cur_e = 0, None, None
    for s, e, n, q in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - t0
    print(f"rollout window {span / 1e3:.1f} us, GPU busy (any kernel) {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")
    steps = [ks[b][0] for b in bs] + [t_end]
    for i in range(16):
        print(f"step {i:2d}: {(steps[i + 1] - steps[i]) / 1e3:7.1f} us")


if __name__ == "__main__":
    main()
