#!/usr/bin/env python3
"""Achievable HBM write bandwidth on this GPU (torch fill_ of 2 GiB) vs read+write copy,
for judging write-bound kernels (the channel observation kernel)."""
import torch
x = torch.empty(2**30, dtype=torch.int16, device="cuda")
y = torch.empty_like(x)
for name, fn, nbytes in (("fill (write)", lambda: x.fill_(1), 2 * x.numel()),
                         ("copy (read+write)", lambda: y.copy_(x), 4 * x.numel())):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print("%-18s %.3f ms  %.2f TB/s" % (name, ms, nbytes / ms / 1e9))
