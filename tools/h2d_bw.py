"""Host->device copy bandwidth of this box's MI355X link (pinned and
registered host memory), to bound the PCIe-inclusive verify rate."""
import json
import time

import torch

out = {}
dev = torch.device("cuda:0")
for mb in (22, 256):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    out[f"h2d_pinned_{mb}MB_GBps"] = round(n * reps / (time.perf_counter() - t0) / 1e9, 2)
    t0 = time.perf_counter()
    for _ in range(reps):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    out[f"d2h_pinned_{mb}MB_GBps"] = round(n * reps / (time.perf_counter() - t0) / 1e9, 2)
print(json.dumps(out))
