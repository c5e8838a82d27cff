#!/usr/bin/env python3
"""Memory-ceiling calibration for the C2 byte pattern (diagnostic, not product).
Builds tools/libprobe.so and times the probe kernels with events, interleaved."""
import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "libprobe.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                    os.path.join(HERE, "probe_stream.hip"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib.probe_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    n, S = 16 * 1024 * 1024, 60
    blob = torch.randint(0, 255, (n * S + 64,), dtype=torch.uint8, device=dev)
    ln = torch.full((n,), 60, dtype=torch.int16, device=dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    cfgs = [(w, g) for w in range(lib.probe_count()) for g in (1024, 2048, 4096)]
    times = {c: [] for c in cfgs}
    for r in range(10):
        for c in cfgs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            lib.probe_launch(c[0], blob.data_ptr(), ln.data_ptr(), out.data_ptr(), n, S, c[1], s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                times[c].append(a.elapsed_time(b) * 1e-3)
    res = {}
    for (w, g), ts in times.items():
        nm = lib.probe_name(w).decode()
        t = float(np.median(ts))
        rd = n * (S + 2) if nm.startswith("rw") else (n * S if nm.startswith("read") else 0)
        wr = n * 16 if (nm.startswith("rw") or nm.startswith("write")) else 0
        res[f"{nm}_g{g}"] = {"ms": round(t * 1e3, 4), "TBps": round((rd + wr) / t / 1e12, 3),
                             "equiv_frac72": round(n * 72 / t / 8e12, 4) if nm.startswith("rw") else None}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
