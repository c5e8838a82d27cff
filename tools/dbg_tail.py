"""Debug: residual words for frames with short segment tails (GPU vs oracle)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from ix_amd import ixgrx, traces
from oracle import oracle
import make_golden as mg
frames = []
for pl in range(40, 80):
    frames.append(mg.ipv4(proto=6, payload=bytes((7 * k + 3) & 0xff for k in range(pl))))
tr = traces.pack(frames)
er, ec = oracle.rx_trace(tr, traces.RSS_KEY)
for mode in ("auto", "general"):
    e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY), split=mode)
    rec, cs = e.batch_trace(tr, want_csum=True)
    for k in range(len(frames)):
        L = len(frames[k])
        if cs[k] != ec[k]:
            print(mode, "L", L, "seg_end", L, "gpu", hex(cs[k] >> 16), "exp", hex(ec[k] >> 16),
                  "diff", hex(((cs[k] >> 16) - (ec[k] >> 16)) & 0xffff))
    print(mode, "mismatches", int((cs != ec).sum()), "of", len(frames))
