#!/usr/bin/env python3
"""Which clock moves during the launch-settling transient?

Fresh process; launch order as bench.py's (W warm-ups, then timed
launches). Before every launch, tools/clock_probe.hip's one-wave kernel
measures the shader clock (shader-clock counter / 100 MHz real-time counter
over a fixed dependent loop) and the latency of a dependent chain of loads
through cold lines (HBM miss latency, in ns: follows the memory and fabric
clocks). Modes:
  c2     probe, C2 launch (HIP events around it), probe, ...
  idle   probes only, ~0.25 ms apart (no C2 work)
  plain  C2 launches with events only (no probe), for comparison
usage: clock_trace.py MODE [LAUNCHES] [OUT.json]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

HOPS = 16
SPIN = 2000


def main():
    import torch
    import bench
    from ix_amd import ixgrx, traces
    mode = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    dst = sys.argv[3] if len(sys.argv) > 3 else None
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(HERE, "libclock_probe.so"))
    lib.clk_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_void_p]
    # the chain: probes x HOPS random 64-byte lines of a 1 GiB buffer
    lines = (1 << 30) // 64
    n_probe = k + 1
    g = torch.Generator().manual_seed(7)
    pick = torch.randperm(lines, generator=g)[:n_probe * (HOPS + 1)].to(torch.int64) * 16
    chase = torch.zeros(1 << 28, dtype=torch.int32)
    pr = pick.view(n_probe, HOPS + 1)
    chase[pr[:, :-1].reshape(-1)] = pr[:, 1:].reshape(-1).to(torch.int32)
    chase = chase.to(dev)
    starts = pr[:, 0].tolist()
    out = torch.zeros((n_probe, 4), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    wl = eng = None
    if mode != "idle":
        wl = bench.Workload("c2", seed=0x1B0002, dev=dev)
        eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, wl.flags), device=0)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]

    def probe(i):
        lib.clk_launch(out[i].data_ptr(), chase.data_ptr(), starts[i], HOPS, SPIN, s.cuda_stream)
    t0 = time.perf_counter()
    for i in range(k):
        if mode != "plain":
            probe(i)
        if mode == "idle":
            torch.cuda.synchronize()
            while time.perf_counter() - t0 < 0.00025 * (i + 1):
                pass
            continue
        a, b = ev[i]
        a.record(s)
        wl.launch(eng, s.cuda_stream)
        b.record(s)
    if mode != "plain":
        probe(k)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    res = {"mode": mode, "launches": k}
    if mode != "idle":
        res["kernel_ms"] = [round(a.elapsed_time(b), 4) for a, b in ev]
    if mode != "plain":
        res["sclk_mhz"] = [round(float(t) / float(r) * 100.0, 1) if r else None for t, r, _, _ in o]
        res["hbm_miss_ns"] = [round(float(c) * 10.0 / HOPS, 1) for _, _, c, _ in o]
    print(json.dumps(res))
    if dst:
        with open(dst, "w") as f:
            json.dump(res, f)
    if eng:
        eng.close()


if __name__ == "__main__":
    main()
