"""Debug: one step of fast vs generic kernels on the sprinkled-spawner pool; dump diffs."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "safelife-k2_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import torch
from test_gpu_parity import _sprinkled_pool
from safelife_amd import SafeLifeVecEnv
path = os.path.join(REPO, "tests", "golden", "pools", "c3_prune_still_64.npz")
rng = np.random.RandomState(11)
pool = _sprinkled_pool(path, rng)
B = 64
kw = dict(time_limit=70, view_shape=(33, 33), output_channels=None, penalty_coef=0.7,
          min_performance=0.01, rng="philox", seed=42, level_order="random", augment_roll=True)
fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
fast.reset(); gen.reset()
g0 = fast.goals.cpu().numpy().copy()
a = torch.zeros(B, dtype=torch.int32, device="cuda:0")
fast.step(a); gen.step(a)
gf, gg = fast.goals.cpu().numpy(), gen.goals.cpu().numpy()
bf, bg = fast.board.cpu().numpy(), gen.board.cpu().numpy()
print("board diffs", int((bf != bg).sum()), "goal diffs", int((gf != gg).sum()))
d = np.argwhere(gf != gg)
for e, y, x in d[:40]:
    print("env %d y %d x %d  before %d fast %d gen %d" % (e, y, x, g0[e, y, x], gf[e, y, x], gg[e, y, x]))
print("goal cells changed by gen:", int((gg != g0).sum()), " by fast:", int((gf != g0).sum()))
import oracle
sp = float(pool.spawn_prob[0])
print("spawn_prob", sp, "thr", float(np.float32(sp)))
for e, y, x in d[:40]:
    nb = np.array([[g0[e, (y + dy) % 64, (x + dx) % 64] for dx in (-1, 0, 1)] for dy in (-1, 0, 1)])
    print("env", e, (y, x), "\n", nb)
    for st in (0, 1):
        print("   step", st, "u", oracle.philox_uniform(int(y * 64 + x), int(e), st, 1, 42))
