#!/usr/bin/env python3
"""Launch-gap probe (diagnostic): wall time per C2 step for K plain launches,
for K replays of a one-launch HIP graph, and for one replay of a graph of K
launches, next to the event-timed kernel time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ix_amd import ixgrx, traces
    dev = torch.device("cuda:0")
    wl = bench.Workload("c2", seed=0x1B0002, dev=dev)
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, 0), device=0)
    s = torch.cuda.Stream()
    K = 50
    with torch.cuda.stream(s):
        for _ in range(10):
            wl.launch(eng, s.cuda_stream)
    torch.cuda.synchronize()

    def wall(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e3
    res = {}
    with torch.cuda.stream(s):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            wl.launch(eng, s.cuda_stream)
        res["host_per_launch_ms"] = (time.perf_counter() - t0) / K * 1e3
        torch.cuda.synchronize()
        res["plain"] = wall(lambda: [wl.launch(eng, s.cuda_stream) for _ in range(K)])
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, stream=s):
            wl.launch(eng, s.cuda_stream)
        res["graph1_xK"] = wall(lambda: [g1.replay() for _ in range(K)])
        gk = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gk, stream=s):
            for _ in range(K):
                wl.launch(eng, s.cuda_stream)
        res["graphK_x1"] = wall(lambda: gk.replay())
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for a, b in ev:
            a.record(s)
            wl.launch(eng, s.cuda_stream)
            b.record(s)
    torch.cuda.synchronize()
    res["kernel_events"] = sum(a.elapsed_time(b) for a, b in ev) / K
    print({k: round(v, 4) for k, v in res.items()})
    eng.close()


if __name__ == "__main__":
    main()
