"""Run one bench workload a few times through a given library build (for
rocprofv3 counter passes of A/B variants): run_lib.py LIB WORKLOAD [N]."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
from ix_amd import ixgrx, traces
lib, w = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 3
wl = bench.Workload(w, seed=0x1B0002, dev=torch.device("cuda:0"))
import ctypes
full = os.path.join(ROOT, lib)
v = ctypes.CDLL(full).ixg_abi_version()  # (a build of an older revision: its own ABI version)
cur, ixgrx.ABI_VERSION = ixgrx.ABI_VERSION, v
ixgrx.load_library(full)
ixgrx.ABI_VERSION = cur
e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, flags=wl.flags), lib_path=full)
s = torch.cuda.current_stream()
for _ in range(n):
    wl.launch(e, s.cuda_stream)
torch.cuda.synchronize()
print("ok", lib, w)
