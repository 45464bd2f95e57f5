"""Do parallel branches of a captured HIP graph run concurrently on this stack?  Two spin kernels on
two streams inside one torch.cuda.graph capture (fork / join by events), replay timed against the
same two kernels captured on one stream.  Run on the GPU box: python tools/graph_branches.py"""
import time

import torch


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    cyc = 20_000_000     # ~8-10 ms per spin kernel
    s2 = torch.cuda.Stream()
    torch.cuda.synchronize()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        s1 = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(s1)
        s2.wait_event(ev)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        ev2 = torch.cuda.Event()
        ev2.record(s2)
        s1.wait_event(ev2)
    print(f"one stream: {timed(g1):.2f} ms per replay; two branches: {timed(g2):.2f} ms per replay")
    # eager, two streams
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ev = torch.cuda.Event(); ev.record(); s2.wait_event(ev)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
        torch.cuda.current_stream().wait_stream(s2)
    torch.cuda.synchronize()
    print(f"eager two streams: {(time.perf_counter() - t0) / 10 * 1e3:.2f} ms per pair")


if __name__ == "__main__":
    main()
