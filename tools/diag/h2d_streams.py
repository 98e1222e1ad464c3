"""Pinned H2D bandwidth with 1, 2 and 4 concurrent streams (copy engines)."""
import time
import torch

n = 256 << 20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
for ns in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    part = n // ns
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(4):
            for k, s in enumerate(streams):
                with torch.cuda.stream(s):
                    d[k * part:(k + 1) * part].copy_(h[k * part:(k + 1) * part], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        if rep == 1:
            print(f"{ns} streams: {n * 4 / dt / 1e9:.1f} GB/s", flush=True)
