import torch, time
x = torch.empty(300_000_000, dtype=torch.float64, device='cuda').uniform_()
a, b = x[:150_000_000], x[150_000_000:]
c = torch.empty(150_000_000, dtype=torch.float64, device='cuda')
for name, fn, by in [("add r2.4G w1.2G", lambda: torch.add(a, b, out=c), 3.6e9),
                     ("copy r1.2G w1.2G", lambda: c.copy_(a), 2.4e9),
                     ("sum r2.4G", lambda: x.sum(), 2.4e9)]:
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{name}: {ms:.3f} ms  {by/ms/1e9:.0f} GB/s")
