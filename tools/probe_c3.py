#!/usr/bin/env python3
"""Memory ceiling of C3's (or argv[1]'s workload's) byte pattern (diagnostic): tools/probe_c3.hip's
whole-span reads next to the product's C3 launch on the same buffers."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch
    import bench
    from ix_amd import ixgrx, traces
    so = os.path.join(HERE, "libprobe_c3.so")
    lib = ctypes.CDLL(so)
    lib.p3_launch.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p,
                                                                        ctypes.c_uint32, ctypes.c_void_p]
    lib.p3_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    wname = sys.argv[1] if len(sys.argv) > 1 else "c3"
    wl = bench.Workload(wname, seed=0x1B0002, dev=dev)
    zero = torch.zeros(4096, dtype=torch.uint8, device=dev)
    out = torch.empty((wl.n, 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, wl.flags), device=0)
    span = int(wl.off[-1].item()) + int(wl.len[-1].item())
    res = {}

    def timeit(fn, k=10):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        torch.cuda.synchronize()
        for a, b in ev:
            a.record(s)
            fn()
            b.record(s)
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))
    for rep in range(2):
        res.setdefault("product", []).append(timeit(lambda: wl.launch(eng, s.cuda_stream)))
        for w in range(lib.p3_count()):
            for g in (1024, 2048, 4096):
                name = f"{lib.p3_name(w).decode()}_g{g}"
                t = timeit(lambda: lib.p3_launch(w, wl.blob.data_ptr(), wl.off.data_ptr(), wl.len.data_ptr(),
                                                 out.data_ptr(), wl.n, zero.data_ptr(), g, s.cuda_stream))
                res.setdefault(name, []).append(t)
    print(json.dumps({"workload": wname, "span_bytes": span, "n": wl.n,
                      "ms": {k: round(min(v), 4) for k, v in res.items()},
                      "tbps_span_read": {k: round(span / (min(v) * 1e-3) / 1e12, 2) for k, v in res.items()}}))
    eng.close()


if __name__ == "__main__":
    main()
