#!/usr/bin/env python3
"""C2's memory pattern alone (tools/probe_c2mem.hip): chunks in flight per
wave (AHEAD) x grid size, next to the product's C2 launch time."""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch
    import bench
    from ix_amd import ixgrx, traces
    lib = ctypes.CDLL(os.path.join(HERE, "libprobe_c2mem.so"))
    lib.pm_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    wl = bench.Workload("c2", seed=0x1B0002, dev=dev)
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, flags=wl.flags))
    n = wl.n
    s = torch.cuda.current_stream()
    names = ["ahead0", "ahead1", "ahead2", "ahead3", "run2_ahead1", "run2_ahead2", "run2_ahead3"]
    cfgs = [("product", None, None)] + [(f"{names[a]}_g{g}", a, g) for a in range(7) for g in (2048, 4096, 8192)]
    times = {c[0]: [] for c in cfgs}
    for r in range(10):
        for nm, a, g in cfgs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            if a is None:
                wl.launch(eng, s.cuda_stream)
            else:
                lib.pm_launch(a, wl.blob.data_ptr(), wl.len.data_ptr(), wl.out.data_ptr(), n, g, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                times[nm].append(e0.elapsed_time(e1))
    res = {k: {"ms": round(float(np.median(v)), 4), "frac72": round(n * 72 / (np.median(v) * 1e-3) / 8e12, 4)}
           for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
