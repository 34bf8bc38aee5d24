#!/usr/bin/env python3
"""HBM bandwidth probe: write (fill_), read (sum), copy on a big buffer, and the
same-buffer rewrite case (MALL-resident) -- context for the obs-write numbers."""
import torch

dev = torch.device("cuda")
for nbytes in (77 * 2**20, 256 * 2**20, 2 * 2**30, 8 * 2**30):
    n = nbytes // 4
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty(n, dtype=torch.float32, device=dev)
    a.fill_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(3, int(4e9 // nbytes))
    for name, fn, mult in (("write(fill)", lambda: a.fill_(2.0), 1), ("read(sum)", lambda: a.sum(), 1),
                           ("copy", lambda: b.copy_(a), 2)):
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        dt = e0.elapsed_time(e1) / 1e3 / reps
        print(f"{nbytes / 2**20:8.0f} MiB {name:12s} {mult * nbytes / dt / 1e12:6.2f} TB/s", flush=True)
    del a, b
