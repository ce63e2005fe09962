#!/usr/bin/env python3
"""Per-phase wave timings of the 64x64 step kernel (tuning builds with
-DSL_BITS_TIMING=1): runs the bench workload for a few steps with each given
variant library and prints, for the sampled waves of the last step, the mean
s_memtime delta of every phase and the wave lifetime against the kernel span.

usage: phase_timing.py lib1.so [lib2.so ...]   (one subprocess per library)
"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["rec+dma+goal loads issue", "goals phase", "wait_vm", "action", "board rule",
         "scoring", "stores", "epilogue", "reset queue"]


def child(lib):
    sys.path.insert(0, os.path.join(REPO, "safelife-k2_amd"))
    import numpy as np
    import torch
    from safelife_amd import SafeLifeVecEnv, LevelPool, _lib
    dev = torch.device("cuda", 0)
    pool = LevelPool.load(os.path.join(REPO, "tests", "golden", "pools", "c3_prune_still_64.npz"))
    B = 65536
    env = SafeLifeVecEnv(pool, B, dev, time_limit=1000, view_shape=(33, 33), output_channels=None,
                         penalty_coef=1.0, min_performance=0.01, rng="philox", seed=1234,
                         level_order="random", augment_roll=True, compute_obs=False)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    env.st_t["episode_length"].copy_(torch.randint(0, 1000, (B,), device=dev, generator=g,
                                                   dtype=torch.int32))
    for _ in range(300):
        env.step_async(torch.randint(0, 9, (B,), dtype=torch.int32, device=dev, generator=g))
    torch.cuda.synchronize(dev)
    L = _lib.lib()
    L.sl_debug_phase_times.argtypes = [ctypes.c_void_p]
    buf = np.zeros((1024, 10), dtype=np.uint64)
    assert L.sl_debug_phase_times(buf.ctypes.data) == 0
    t = buf.astype(np.float64)
    d = np.diff(t, axis=1)
    life = t[:, 9] - t[:, 0]
    span = t[:, 9].max() - t[:, 0].min()
    print("%s: wave lifetime mean %.0f  p50 %.0f  p90 %.0f cycles; kernel span %.0f cycles;"
          " span/life %.1f" % (os.path.basename(lib), life.mean(), np.median(life),
                               np.percentile(life, 90), span, span / life.mean()))
    for k, name in enumerate(NAMES):
        print("   %-26s mean %7.0f  p50 %7.0f  p90 %7.0f  (%.1f%%)" % (
            name, d[:, k].mean(), np.median(d[:, k]), np.percentile(d[:, k], 90),
            100 * d[:, k].mean() / life.mean()))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        rc = 0
        for lib in sys.argv[1:]:
            env = dict(os.environ, SAFELIFE_HIP_LIB=os.path.abspath(lib))
            r = subprocess.run([sys.executable, __file__, "--child", lib], env=env, timeout=300)
            rc = rc or r.returncode
        sys.exit(rc)
