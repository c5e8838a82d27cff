#!/usr/bin/env python3
"""Per-launch kernel times of one bench workload, in launch order (HIP events
on the launch stream): shows warm-up / clock ramp effects behind bench.py's
mean-vs-min spread. usage: launch_times.py WORKLOAD [K] [W]
LT_PRE=touch: read every 4 KiB page of the batch and write the records
buffer first; LT_PRE=busy: keep the GPU busy ~100 ms on other memory
first (separates translation / first-touch effects from clock ramp-up)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ix_amd import ixgrx, traces
    w = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda:0")
    wl = bench.Workload(w, seed=0x1B0002, dev=dev)
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, wl.flags), device=0)
    s = torch.cuda.current_stream()
    pre = os.environ.get("LT_PRE", "")
    if pre == "touch":
        pages = wl.blob.view(-1)[::4096].to(torch.int32).sum()
        wl.out.zero_()
        if wl.off is not None:
            pages += wl.off[::512].sum().to(torch.int32)
        pages += wl.len[::2048].to(torch.int32).sum()
        torch.cuda.synchronize()
    elif pre == "busy":
        a = torch.randn(4096, 4096, device=dev)
        for _ in range(60):
            a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()
    for _ in range(warm):
        wl.launch(eng, s.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    torch.cuda.synchronize()
    for a, b in ev:
        a.record(s)
        wl.launch(eng, s.cuda_stream)
        b.record(s)
    torch.cuda.synchronize()
    t = [round(a.elapsed_time(b), 4) for a, b in ev]
    print(w, pre or "none", "ms per launch:", t)
    eng.close()


if __name__ == "__main__":
    main()
