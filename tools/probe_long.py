#!/usr/bin/env python3
"""Memory ceiling of the C4 byte pattern (diagnostic): tools/probe_long.hip's
decompositions, and the product kernel on the same buffer for comparison."""
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
    so = os.path.join(HERE, "libprobe_long.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                        os.path.join(HERE, "probe_long.hip"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.pl_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint32] * 4 + [ctypes.c_void_p]
    lib.pl_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    n, L, S = 8 * 1024 * 1024, 1514, 1516
    src = torch.randint(0, 255, (n * S + 64,), dtype=torch.uint8, device=dev)
    rec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    cfgs = [(w, lib.pl_name(w).decode(), g) for w in range(lib.pl_count()) for g in (1024, 2048, 4096)]
    times = {c: [] for c in cfgs}
    for r in range(6):
        for c in cfgs:
            w, nm, g = c
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            lib.pl_launch(w, src.data_ptr(), rec.data_ptr(), n, L, S, g, s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                times[c].append(a.elapsed_time(b) * 1e-3)
    res = {}
    for c, ts in times.items():
        t = float(np.median(ts))
        res[f"{c[1]}_g{c[2]}"] = {"ms": round(t * 1e3, 4), "frac1532": round(n * 1532 / t / 8e12, 4)}
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
