#!/usr/bin/env python3
"""Plain HBM -> HBM copy ceiling (diagnostic): tools/probe_copy.hip's
variants over 6 GiB, next to torch's copy. TB/s counts read + write."""
import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    lib = ctypes.CDLL(os.path.join(HERE, "libprobe_copy.so"))
    lib.pc_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                              ctypes.c_void_p]
    lib.pc_name.restype = ctypes.c_char_p
    n = 6 << 30
    a = torch.ones(n, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    s = torch.cuda.current_stream()

    def timeit(fn, k=8):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        torch.cuda.synchronize()
        for x, y in ev:
            x.record(s)
            fn()
            y.record(s)
        torch.cuda.synchronize()
        return float(np.median([x.elapsed_time(y) for x, y in ev]))
    res = {"torch": timeit(lambda: b.copy_(a))}
    for w in range(lib.pc_count()):
        for g in (1024, 2048, 4096, 8192):
            res[f"{lib.pc_name(w).decode()}_g{g}"] = timeit(
                lambda: lib.pc_launch(w, a.data_ptr(), b.data_ptr(), n // 16, g, s.cuda_stream))
    print(json.dumps({k: round(2 * n / (v * 1e-3) / 1e12, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
