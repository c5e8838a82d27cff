import torch, time
d = torch.device("cuda:0")
for gb in (1, 6):
    n = gb * (1 << 30)
    a = torch.empty(n, dtype=torch.uint8, device=d); b = torch.empty_like(a)
    a.fill_(1)
    for _ in range(3): b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): b.copy_(a)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e-3
    print(f"copy {gb} GiB: {t*1e3:.3f} ms, {2*n/t/1e12:.2f} TB/s (read+write)")
    del a, b
