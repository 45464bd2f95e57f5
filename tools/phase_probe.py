"""Per-phase timing of the instrumented kernels (k_mb_grad, k_field_wave) on the
bench workload.  Needs the probe build (lib/libusv_hip_probe.so, built by
`_capi.build(probe=True)`); run on the GPU box:  python tools/phase_probe.py"""
import ctypes
import os
import sys

os.environ["USV_HIP_PROBE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from omniisaacgymenvs_loop_amd import _capi  # noqa: E402


def read(tu):
    buf = np.zeros((4096, 16), np.uint64)
    rc = getattr(_capi.lib(), f"usv_probe_read_{tu}")(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    return buf.astype(np.int64)


def report(name, buf, nblk, phases, extra_col=None):
    b = buf[:nblk]
    ok = b[:, 0] > 0
    b = b[ok]
    t0 = b[:, 0:1]
    print(f"{name}: {len(b)} workgroups (wall_clock64 ticks = 10 ns)")
    prev = 0
    for k in range(1, phases):
        d = (b[:, k] - t0[:, 0]) / 100.0
        print(f"  phase {k}: t = {d.mean():8.2f} us (max {d.max():8.2f})  delta {d.mean() - prev:8.2f} us")
        prev = d.mean()
    if extra_col is not None:
        it = b[:, extra_col]
        print(f"  iterations: mean {it.mean():.1f} min {it.min()} max {it.max()}")
        print(f"  obstacle/table setup: {np.mean(b[:, 12] - b[:, 0]) / 100:.2f} us")
        dclk = (b[:, 14] - b[:, 13]).astype(np.float64)
        dwall = (b[:, 2] - b[:, 1]).astype(np.float64) / 100e6
        print(f"  shader clock during the sweeps: {np.mean(dclk / dwall) / 1e9:.2f} GHz "
              f"({np.mean(dclk / np.maximum(it, 1)):.0f} cycles per iteration)")


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    _capi.build(probe=True)
    env, task, agent = bench.build(envs, 0, 1, 42)
    agent.obs = agent.env_reset()
    for _ in range(4):
        agent.train_epoch()
    torch.cuda.synchronize()
    pb = read("ppo")
    out = os.environ.get("USV_PROBE_DUMP")
    if out:   # raw per-workgroup stamps of the last k_mb_grad launch (wall_clock64 ticks) for offline analysis
        np.save(out, pb[:agent.minibatch_size // 32])
    report("k_mb_grad (last launch)", pb, agent.minibatch_size // 32, 9)
    b = pb[:agent.minibatch_size // 32]
    b = b[b[:, 0] > 0]
    for k, what in ((9, "layer 1 done"), (10, "W2 committed"), (11, "layer-2 MFMA loop done"),
                    (12, "layer 2 done"), (2, "heads done"), (3, "losses done"), (4, "dz2 done"),
                    (13, "dW2 MFMA loop done"), (5, "dW2 stored"), (6, "dh1 done"), (7, "dz1 done"),
                    (8, "dW1 done"), (14, "fold: group arrived"), (15, "fold: slice written")):
        if np.all(b[:, k] == 0):   # not stamped by this build
            continue
        print(f"  slot {k:2d} {what:24s} t = {np.mean(b[:, k] - b[:, 0]) / 100:7.2f} us "
              f"(max {np.max(b[:, k] - b[:, 0]) / 100:7.2f})")
    last = 15 if np.any(b[:, 15] != 0) else 8
    print(f"  launch span (first start -> last slot-{last} stamp): {(b[:, last].max() - b[:, 0].min()) / 100:7.2f} us; "
          f"start spread {(b[:, 0].max() - b[:, 0].min()) / 100:5.2f} us")
    # k_reduce_partials: stamps 0 start, 1 row sums (thread 0's loads landed), 2 LDS fold, 3 Adam + stores
    # issued, 4 end; against the gradient kernel's stamps of the same minibatch (the last one of the epoch)
    rb = read("red")[:167]
    rb = rb[rb[:, 0] > 0]
    if len(rb):
        g0 = pb[:agent.minibatch_size // 32]
        g0 = g0[g0[:, 0] > 0]
        gend = g0[:, 8].max()
        print(f"k_reduce_partials (last launch): {len(rb)} workgroups; first start {(rb[:, 0].min() - gend) / 100:+.2f} us "
              f"after the gradient kernel's last dW1 stamp, start spread {(rb[:, 0].max() - rb[:, 0].min()) / 100:.2f} us")
        for k, what in ((1, "row sums"), (2, "LDS fold"), (3, "Adam + stores issued"), (4, "end")):
            d = (rb[:, k] - rb[:, 0]) / 100.0
            print(f"  stamp {k} {what:22s} t = {d.mean():6.2f} us (max {d.max():6.2f})")
        print(f"  launch span (first start -> last end stamp): {(rb[:, 4].max() - rb[:, 0].min()) / 100:.2f} us")
    pp = read("pol")
    b = pp[pp[:, 0] > 0]
    ntiles = (agent.num_actors + 31) // 32
    per = ntiles / max(len(b), 1)
    print(f"k_policy_step (last launch, {len(b)} workgroups, {per:.2f} tiles per workgroup; slots 1-4 are the last tile):")
    print(f"  last tile starts at t = {np.mean(b[:, 1] - b[:, 0]) / 100:7.2f} us (launch mean per tile "
          f"{np.mean(b[:, 4] - b[:, 0]) / 100 / per:6.2f} us)")
    for k, what in ((2, "obs staged"), (3, "forward done"), (4, "sampled + stored")):
        print(f"  slot {k} {what:18s} +{np.mean(b[:, k] - b[:, k - 1]) / 100:6.2f} us")
    if np.any(b[:, 5:10] != 0):   # per-phase sums over the workgroup's tiles (wave 0's view)
        tot = b[:, 5:10].sum(axis=1).mean()
        for k, what in enumerate(("tile setup (obs prefetch issue)", "layer 1 + barrier", "layer 2 + barrier",
                                  "heads + barrier", "epilogue / next obs + barrier")):
            m = b[:, 5 + k].mean() / 100 / per
            print(f"  per tile: {what:32s} {m:6.2f} us ({b[:, 5 + k].mean() / tot:5.1%})")
        print(f"  launch span {(b[:, 4].max() - b[:, 0].min()) / 100:7.2f} us; start spread "
              f"{(b[:, 0].max() - b[:, 0].min()) / 100:5.2f} us")
    cnt = int(task.ctl[0].item())
    print("reset count of the last step:", cnt)
    report("k_field_wave (last launch)", read("field"), min(cnt, 512), 4, extra_col=15)


if __name__ == "__main__":
    main()
