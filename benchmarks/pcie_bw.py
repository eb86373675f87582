#!/usr/bin/env python3
"""PCIe ceiling of the box: pinned 4 GiB H2D, D2H and both directions at once
(two streams); the reference point for host-streamed cipher throughput
(config 5, docs/PERF.md)."""
import os

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # before torch / HIP: dmabuf IPC only on this host driver (as bench.py)

import torch, time, json
n = 4 << 30
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def t(f, reps=3):
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps
h2d = t(lambda: d.copy_(h, non_blocking=True))
d2h = t(lambda: h.copy_(d, non_blocking=True))
def both():
    with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
bi = t(both)
print(json.dumps({"h2d_gbps": n / h2d / 1e9, "d2h_gbps": n / d2h / 1e9, "bidir_each_gbps": n / bi / 1e9}))
