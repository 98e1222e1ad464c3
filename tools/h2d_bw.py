import torch, time
for mb in (16, 64, 168, 336, 672):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(s): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    reps = max(4, 2048 // mb)
    t = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(reps): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"{mb:4d} MB x {reps}: {n*reps/dt/1e9:.1f} GB/s  ({dt/reps*1e3:.3f} ms per copy)", flush=True)
