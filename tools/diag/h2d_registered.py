"""Pinned H2D rate: torch pin_memory (hipHostMalloc) vs a numpy array
page-locked with hipHostRegister (how the e2e bench pins the receiver's
UTF-8 buffers), 176 MB (one wide batch's text)."""
import time
import numpy as np
import torch
from twitter_stream_ml_amd.ops._native import hip

n = 176 << 20
d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
s = torch.cuda.Stream()


def rate(src_t, label):
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(6):
                d.copy_(src_t, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    print(f"{label}: {n * 6 / dt / 1e9:.1f} GB/s", flush=True)


rate(torch.empty(n, dtype=torch.uint8).pin_memory(), "pin_memory")
a = np.empty(n, dtype=np.uint8)
a[:] = 1
hip().host_register(int(a.ctypes.data), n)
rate(torch.from_numpy(a), "numpy + hipHostRegister")
b = np.empty(n + 4096, dtype=np.uint8)[1234:1234 + n]   # not page aligned
b[:] = 1
hip().host_register(int(b.ctypes.data), n)
rate(torch.from_numpy(b), "numpy (unaligned) + hipHostRegister")
hip().host_unregister(int(a.ctypes.data))
hip().host_unregister(int(b.ctypes.data))
