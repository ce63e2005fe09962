#!/usr/bin/env python3
"""Per-phase wave timings of the 128x128 step kernel (tuning builds with
-DSL_B128_TIMING=1): runs the c5 workload for a few hundred steps with each given
library and prints, for the sampled waves of the last step, the mean s_memtime
cycles of every phase (band phases summed over the four bands).

usage: phase_timing128.py lib1.so [lib2.so ...]   (one subprocess per library)
"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["record + halo loads", "goals phase", "action", "band: load P + edits",
         "band: rule", "band: start planes", "band: scores", "band: stores",
         "totals + wait stores", "epilogue"]


def child(lib):
    sys.path.insert(0, os.path.join(REPO, "safelife-k2_amd"))
    import numpy as np
    import torch
    from safelife_amd import SafeLifeVecEnv, LevelPool, _lib
    dev = torch.device("cuda", 0)
    pool = LevelPool.load(os.path.join(REPO, "tests", "golden", "pools", "c5_navigation_128.npz"))
    B = 65536
    env = SafeLifeVecEnv(pool, B, dev, time_limit=1000, view_shape=(33, 33), output_channels=None,
                         penalty_coef=1.0, min_performance=0.01, rng="philox", seed=1234,
                         level_order="random", augment_roll=True, compute_obs=False)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    env.st_t["episode_length"].copy_(torch.randint(0, 1000, (B,), device=dev, generator=g,
                                                   dtype=torch.int32))
    for _ in range(200):
        env.step_async(torch.randint(0, 9, (B,), dtype=torch.int32, device=dev, generator=g))
    torch.cuda.synchronize(dev)
    L = _lib.lib()
    L.sl_debug_phase_times128.argtypes = [ctypes.c_void_p]
    buf = np.zeros((1024, 12), dtype=np.uint64)
    assert L.sl_debug_phase_times128(buf.ctypes.data) == 0
    t = buf.astype(np.float64)
    life = t[:, 10] - t[:, 0]
    span = t[:, 10].max() - t[:, 0].min()
    d = [t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 4], t[:, 5], t[:, 6],
         t[:, 7], t[:, 8], t[:, 9] - t[:, 3] - t[:, 4:9].sum(1), t[:, 10] - t[:, 9]]
    print("%s: wave lifetime mean %.0f  p50 %.0f  p90 %.0f cycles; kernel span %.0f cycles;"
          " span/life %.1f" % (os.path.basename(lib), life.mean(), np.median(life),
                               np.percentile(life, 90), span, span / life.mean()))
    for x, name in zip(d, NAMES):
        print("   %-24s mean %8.0f  p50 %8.0f  p90 %8.0f  (%.1f%%)" % (
            name, x.mean(), np.median(x), np.percentile(x, 90), 100 * x.mean() / life.mean()))


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
