import torch, time
d = torch.device("cuda", 0)
for mb in (256, 1024):
    n = mb * 2**20 // 2
    a = torch.randn(n, device=d).bfloat16(); b = torch.empty_like(a)
    for _ in range(3): b.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(20): b.copy_(a)
    e.record(); e.synchronize()
    t = s.elapsed_time(e) / 20
    print("copy %d MB: %.3f ms  %.2f TB/s (read+write)" % (mb, t, 2 * mb * 2**20 / t / 1e9))
    s.record()
    for _ in range(20): a.add_(b)
    e.record(); e.synchronize()
    t = s.elapsed_time(e) / 20
    print("a+=b %d MB: %.3f ms  %.2f TB/s (2 reads + write)" % (mb, t, 3 * mb * 2**20 / t / 1e9))
