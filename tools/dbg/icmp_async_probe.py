"""Probe: the asynchronous path with IXG_ASYNC_ICMP_REFLECT over icmp.npz's
frames; prints which records carry IXG_RF_REPLY and which mbufs were
rewritten (GPU box)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ix_amd import ixgrx, traces  # noqa: E402

g = dict(np.load("tests/golden/icmp.npz"))
for direct in (True, False):
    tr = traces.Trace(blob=g["blob"].copy(), off=g["off"], len=g["len"], stride=0)
    arena, ptrs = ixgrx.make_mbufs(tr)
    before = arena.copy()
    eng = ixgrx.RxEngine(ixgrx.Config(bytes(g["key"])))
    eng.async_init(batch_frames=48, batch_bytes=1 << 20, max_wait_us=10000000, depth=3, direct=direct,
                   icmp_reflect=True)
    eng.register_memory(arena.ctypes.data, arena.nbytes)
    eng.set_icmp_reply(bytes(g["mac"]), int(g["host_addr"]))
    assert eng.submit_mbufs(ptrs[:48]) == 48
    eng.flush()
    m, r = eng.poll(100, wait=True)
    st = eng.async_stats()
    eng.close()
    rr = r.view(np.uint8).reshape(-1, 16)
    refl = g["reflected"].astype(bool)[:48]
    changed = [(arena[int(p) - arena.ctypes.data + 64:int(p) - arena.ctypes.data + 64 + 64] !=
                before[int(p) - arena.ctypes.data + 64:int(p) - arena.ctypes.data + 64 + 64]).any() for p in ptrs[:48]]
    print("direct", direct, "n", len(r), "reflected(golden)", int(refl.sum()),
          "flag set", int(((rr[:, 3] & 0x40) != 0).sum()), "mbufs changed", int(np.sum(changed)),
          "verdicts", np.unique(rr[:, 2], return_counts=True), "batches", st["batches"], flush=True)
