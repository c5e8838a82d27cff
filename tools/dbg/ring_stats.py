"""One-off: the ring kernel's cycle counters (build: tools/build_variant.sh
rstats "(lambda ns: (exec(open('tools/dbg/ring_stats_patch.py').read(), ns), ns['out'])[1])({'s': s})")."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import bench
from ix_amd import ixgrx, traces
lib = os.path.join(ROOT, "tools", "ablib", "rstats.so")
for wname in sys.argv[1:] or ["c3"]:
    dev = torch.device("cuda:0")
    wl = bench.Workload(wname, seed=0x1B0002, dev=dev)
    e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, flags=wl.flags), lib_path=lib)
    st = (ctypes.c_ulonglong * 16)()
    f = e._lib.ixgrx_ring_stats
    s = torch.cuda.current_stream()
    for _ in range(10):
        wl.launch(e, s.cuda_stream)
    f(st, 1)
    K = 10
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(s)
    for _ in range(K):
        wl.launch(e, s.cuda_stream)
    ev1.record(s)
    torch.cuda.synchronize()
    f(st, 0)
    v = list(st)
    nchunks = (wl.n + 63) // 64 * K
    ms = ev0.elapsed_time(ev1) / K
    nl = max(v[10], 1)  # loader waves (all launches)
    print(f"{wname}: {ms:.4f} ms/launch; per loader wave per launch: total {v[0]/nl:.0f} cyc, "
          f"blocked {v[1]/nl:.0f} ({v[3]/nl:.0f} spins), header waits {v[2]/nl:.0f}; "
          f"per chunk: ready wait {v[4]/max(v[7],1):.0f}, phase R {v[5]/max(v[7],1):.0f}, phase P {v[6]/max(v[7],1):.0f} cyc; "
          f"chunks {v[7]/K:.0f} (of {nchunks/K:.0f}); consumer wave total {v[8]/max(v[9],1):.0f} cyc; "
          f"phase R parts: header {v[11]/max(v[7],1):.0f}, prefix+edges {v[12]/max(v[7],1):.0f}, tails {v[13]/max(v[7],1):.0f}")
