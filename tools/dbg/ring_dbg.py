"""One-off: which frames the ring kernel gets wrong, and their residuals."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from ix_amd import ixgrx, traces
from oracle import oracle
KEY = traces.RSS_KEY
e = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, 0))
for n, seed in ((64, 0x1B5000 + 64), (64, 5), (64, 6), (128, 7), (64 * 40, 8)):
    tr = traces.make_trace("imix", n, seed=seed, bad_ip=0.01, bad_l4=0.01)
    dev = torch.device("cuda:0")
    blob = torch.zeros(tr.blob.size + 64, dtype=torch.uint8, device=dev)
    blob[:tr.blob.size] = torch.from_numpy(tr.blob)
    off = torch.from_numpy(tr.offsets().astype(np.int64)).to(dev)
    lens = torch.from_numpy(tr.len.view(np.int16)).to(dev)
    out = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
    cs = torch.zeros(n, dtype=torch.int32, device=dev)
    e.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, out.data_ptr(), cs.data_ptr(), None)
    torch.cuda.synchronize()
    info = e.launch_info()
    rec = out.cpu().numpy(); c = cs.cpu().numpy().view(np.uint32)
    er, ec = oracle.rx_batch(KEY, 128, 0, 0, tr.blob, tr.offsets(), tr.len)
    bad = np.nonzero((rec != er).any(axis=1))[0]
    offs = tr.offsets()
    b16 = int(offs[0]) & ~15
    print(f"n={n} seed={seed} info={info} bad={bad.tolist()}")
    for i in bad[:10]:
        ra = 1024 + int(offs[i]) - b16
        print(f"  frame {i} L={tr.len[i]} rel={int(offs[i]) - b16} ring_slots {ra // 1024}..{(ra + int(tr.len[i])) // 1024}"
              f" res gpu {c[i] >> 16:#06x} exp {ec[i] >> 16:#06x} diff {((c[i] >> 16) - (ec[i] >> 16)) & 0xffff:#06x}")
