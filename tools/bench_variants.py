#!/usr/bin/env python3
"""Run bench.py once per tuning variant library (safelife-k2_amd/build/variants/*.so)
in separate processes, rounds interleaved, and print value / kernel ms per variant."""
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = sorted(glob.glob(os.path.join(REPO, "safelife-k2_amd", "build", "variants", "*.so")))
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
extra = sys.argv[2:]
res = {os.path.basename(l): [] for l in libs}
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, SAFELIFE_HIP_LIB=lib)
        out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "60",
                              "--warmup", "10", "--no-cpu-baseline", "--burnin", "300"] + extra,
                             env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(os.path.basename(lib), "FAILED", out.stderr[-2000:], flush=True)
            continue
        d = json.loads(line[-1])
        res[os.path.basename(lib)].append((d["value"], d["roofline"]["kernel_ms"]))
        print(r, os.path.basename(lib), "%.1f M/s" % (d["value"] / 1e6),
              "kernel %.4f ms" % d["roofline"]["kernel_ms"], flush=True)
for k, v in res.items():
    if v:
        print("%-10s best %.1f M/s  kernel %.4f ms" % (k, max(x[0] for x in v) / 1e6,
                                                       min(x[1] for x in v)))
