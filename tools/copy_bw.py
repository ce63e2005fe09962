#!/usr/bin/env python3
"""Streaming bandwidth references on this GPU: the library's 16-byte copy (sl_copy16,
what bench.py reports as copy_GBps), torch's device copy and a torch fill, for 1 GiB."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "safelife-k2_amd"))
import torch  # noqa: E402
from safelife_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
L = _lib.lib()
x = torch.empty(2 ** 29, dtype=torch.int16, device=dev)
y = torch.empty_like(x)
nb = 2 * x.numel()
sp = _lib.stream_ptr(dev)
for name, fn, moved in (
        ("sl_copy16 (read+write)", lambda: L.sl_copy16(_lib.ptr(x), _lib.ptr(y), nb // 16, sp), 2 * nb),
        ("torch copy_ (read+write)", lambda: y.copy_(x), 2 * nb),
        ("torch fill_ (write)", lambda: x.fill_(1), nb)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    print("%-26s %.3f ms  %.2f TB/s" % (name, ms, moved / ms / 1e9))
