#!/usr/bin/env python3
"""HBM ceiling for read/write mixes (diagnostic): copy vs the C2 byte mix."""
import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    so = os.path.join(HERE, "libprobe2.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                    os.path.join(HERE, "probe2.hip"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.p2_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint32] * 3 + [ctypes.c_void_p]
    lib.p2_name.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    n = 16 * 1024 * 1024
    src = torch.randint(0, 255, (n * 64 + 64,), dtype=torch.uint8, device=dev)   # 1 GiB
    dst = torch.empty((n * 64 // 16 * 16 + 64,), dtype=torch.uint8, device=dev)  # 1 GiB (copy target)
    rec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    cfgs = []
    only = os.environ.get("P2_ONLY")
    for w in range(lib.p2_count()):
        nm = lib.p2_name(w).decode()
        if only and nm not in only.split(","):
            continue
        for g in (1024, 2048, 4096, 8192):
            if nm.startswith("copy"):
                cfgs.append((w, nm, g, n * 4, 0, n * 64 * 2))             # 1 GiB copied
            elif nm.startswith("mixw") or nm.startswith("mx"):
                S = int(nm[-2:])
                cfgs.append((w, nm, g, n, S, n * (S + 16)))
            else:
                for S in (60, 64):
                    cfgs.append((w, f"{nm}_S{S}", g, n, S, n * (S + 16)))
    times = {c: [] for c in cfgs}
    for r in range(8):
        for c in cfgs:
            w, nm, g, items, S, byt = c
            out = dst if nm.startswith("copy") else rec
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            lib.p2_launch(w, src.data_ptr(), out.data_ptr(), items, S, g, s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                times[c].append(a.elapsed_time(b) * 1e-3)
    res = {}
    for c, ts in times.items():
        w, nm, g, items, S, byt = c
        t = float(np.median(ts))
        e = {"ms": round(t * 1e3, 4), "TBps": round(byt / t / 1e12, 3)}
        if not nm.startswith("copy"):
            e["c2_equiv_frac72"] = round(n * 72 / t / 8e12, 4)
        res[f"{nm}_g{g}"] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
