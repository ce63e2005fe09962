#!/usr/bin/env python3
"""
Capture golden vectors from the REFERENCE itself (run in the build container only;
needs /root/reference).  The outputs under tests/golden/ are data (inputs and
expected outputs); no reference source is copied into the repository.

How the reference is made importable here:
  * the C extension ``speedups`` is compiled from /root/reference by oracle/Makefile
    into oracle/_ref/ (git-ignored);
  * oracle/_ref/pkg/safelife/ is a symlink farm onto /root/reference/safelife/*.py
    and levels/, plus the compiled extension;
  * two third-party packages are absent from the image: ``gym`` (base classes only:
    Env, Wrapper attribute forwarding, spaces, seeding) and ``pyemd`` (EMD, needed only
    at episode end by the logging wrapper, which these fixtures do not run).  Minimal
    import stand-ins written below provide just those names; pyemd.emd raises, so no
    EMD value is ever produced or pinned.

Fixtures and synthetic level pools (§8(d)):
  advance_known_answers.npz   G1  random all-bit boards, p in {0, 1}
  advance_stream.npz          G2  spawner boards, seeded reference stream, 50 steps
  traj_<name>.npz             G3/G4 full PPO wrapper chain trajectories
  densities.npz               G5  _add_cell_distribution rollout densities
  levels/<name>.npz           benchmark levels used by the tests (data)
  pools/<name>.npz            proc-gen level pools for the benchmark configs
  advance_known_answers_128.npz  G1 at 128x128, C5's board size (round 5)
  advance_stream_128.npz         G2 at 128x128: C5 navigation levels, seeded stream
  traj_nav128_*.npz              G4 at 128x128: PPO-chain trajectories on C5 levels
  g7_ppo_loop_*.npz              G7: the PPO rollout loop (ppo.py:436-452), 16 envs,
                                 action draws and spawn refills in one global stream

Usage: python tests/golden/make_golden.py [--only g1,g2,traj,dens,pools,pool128,
                                                  g1_128,g2_128,traj128,g7]
"""
import argparse
import hashlib
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
REFPKG = os.path.join(REPO, "oracle", "_ref", "pkg")
STUBS = os.path.join(REPO, "oracle", "_ref", "stubs")

GYM_STUB = '''
import numpy as _np
class Env(object):
    def seed(self, seed=None):
        return []
    def close(self):
        pass
class Wrapper(Env):
    def __init__(self, env):
        self.env = env
        self.action_space = getattr(env, "action_space", None)
        self.observation_space = getattr(env, "observation_space", None)
    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)
    def step(self, action):
        return self.env.step(action)
    def reset(self, **kw):
        return self.env.reset(**kw)
    def close(self):
        return self.env.close()
def register(**kw):
    pass
'''
SPACES_STUB = '''
class Discrete(object):
    def __init__(self, n):
        self.n = n
class Box(object):
    def __init__(self, low, high, shape=None, dtype=None):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype
'''
SEEDING_STUB = '''
import numpy as _np, os as _os
def np_random(seed=None):
    if seed is None:
        seed = int.from_bytes(_os.urandom(4), "little")
    return _np.random.RandomState(seed), seed
'''
VR_STUB = '''
class VideoRecorder(object):
    def __init__(self, *a, **k):
        raise RuntimeError("video recording is not available in the fixture build")
'''
PYEMD_STUB = '''
def emd(*a, **k):
    raise RuntimeError("pyemd is not installed; EMD values are not pinned")
'''


def _write(path, text):
    if os.path.exists(path) and open(path).read() == text:
        return
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def setup_reference(build=True):
    if build:
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    pk = os.path.join(REFPKG, "safelife")
    os.makedirs(pk, exist_ok=True)
    src = os.path.join(REF, "safelife")
    for name in os.listdir(src):
        if name.endswith(".py") or name in ("levels",):
            dst = os.path.join(pk, name)
            if not os.path.lexists(dst):
                os.symlink(os.path.join(src, name), dst)
    import sysconfig
    so = "speedups" + sysconfig.get_config_var("EXT_SUFFIX")
    dst = os.path.join(pk, so)
    if not os.path.lexists(dst):
        os.symlink(os.path.join(REPO, "oracle", "_ref", so), dst)
    _write(os.path.join(STUBS, "gym", "__init__.py"), GYM_STUB + "\nfrom . import spaces, utils, wrappers\n")
    _write(os.path.join(STUBS, "gym", "spaces.py"), SPACES_STUB)
    _write(os.path.join(STUBS, "gym", "utils", "__init__.py"), "from . import seeding\n")
    _write(os.path.join(STUBS, "gym", "utils", "seeding.py"), SEEDING_STUB)
    _write(os.path.join(STUBS, "gym", "wrappers", "__init__.py"), "from . import monitoring\n")
    _write(os.path.join(STUBS, "gym", "wrappers", "monitoring", "__init__.py"),
           "from . import video_recorder\n")
    _write(os.path.join(STUBS, "gym", "wrappers", "monitoring", "video_recorder.py"), VR_STUB)
    _write(os.path.join(STUBS, "pyemd", "__init__.py"), PYEMD_STUB)
    sys.path.insert(0, STUBS)
    sys.path.insert(0, REFPKG)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------------------------
def gen_g1(out):
    from safelife import speedups
    rng = np.random.RandomState(1234)
    sizes = [2, 3, 4, 5, 7, 16, 25, 26, 31, 64]
    used = np.uint16(0b1000111111111111)   # bits 0-11 and 15 ("13 used bits")
    ins, outs, shapes, probs = [], [], [], []
    for i in range(600):
        H = int(rng.choice(sizes))
        W = int(rng.choice(sizes))
        dens = rng.uniform(0.05, 0.95)
        mode = i % 3
        if mode == 0:      # all used bits, random
            b = rng.randint(0, 1 << 16, size=(H, W)).astype(np.uint16) & used
        elif mode == 1:    # life-like soup with sparse special cells
            b = np.where(rng.rand(H, W) < 0.5, 9, 1).astype(np.uint16)
            b |= (rng.randint(0, 8, size=(H, W)) << 9).astype(np.uint16)
            special = rng.rand(H, W) < 0.1
            b[special] |= rng.choice([16, 32, 64, 128, 152, 256, 4, 32768],
                                     size=special.sum()).astype(np.uint16)
        else:              # every bit pattern, including unused bits 12-14
            b = rng.randint(0, 1 << 16, size=(H, W)).astype(np.uint16)
        b = (b * (rng.rand(H, W) < dens)).astype(np.uint16)
        p = float([0.0, 1.0][i % 2])
        o = speedups.advance_board(b, p)
        ins.append(b.ravel()); outs.append(o.ravel()); shapes.append((H, W)); probs.append(p)
    np.savez_compressed(out, boards_in=np.concatenate(ins), boards_out=np.concatenate(outs),
                        shapes=np.array(shapes, np.int64), spawn_prob=np.array(probs))
    print("G1", len(shapes), "boards ->", out)


def gen_g1_128(out):
    """G1 at C5's board size: random 128x128 boards (all used bits, life-like soups
    with special cells, every bit pattern), one advance each at p in {0, 1} (no draw
    decides anything).  Consecutive pairs share p, so a device test can step pair k
    as one env's board and goals."""
    from safelife import speedups
    rng = np.random.RandomState(128)
    used = np.uint16(0b1000111111111111)
    ins, outs, probs = [], [], []
    H = W = 128
    for i in range(54):
        dens = rng.uniform(0.05, 0.95)
        mode = (i // 2) % 3
        if mode == 0:
            b = rng.randint(0, 1 << 16, size=(H, W)).astype(np.uint16) & used
        elif mode == 1:
            b = np.where(rng.rand(H, W) < 0.5, 9, 1).astype(np.uint16)
            b |= (rng.randint(0, 8, size=(H, W)) << 9).astype(np.uint16)
            special = rng.rand(H, W) < 0.1
            b[special] |= rng.choice([16, 32, 64, 128, 152, 256, 4, 32768],
                                     size=special.sum()).astype(np.uint16)
        else:
            b = rng.randint(0, 1 << 16, size=(H, W)).astype(np.uint16)
        b = (b * (rng.rand(H, W) < dens)).astype(np.uint16)
        p = float([0.0, 1.0][(i // 2) % 2])
        speedups.seed(i)
        ins.append(b)
        outs.append(speedups.advance_board(b, p))
        probs.append(p)
    np.savez_compressed(out, boards_in=np.array(ins), boards_out=np.array(outs),
                        spawn_prob=np.array(probs))
    print("G1-128", len(ins), "boards ->", out)


def gen_g2_128(out):
    """G2 at 128x128: speedups.seed(s), then 30 advances of a C5 navigation level's
    board and goals (board first), the level's own spawn_prob."""
    from safelife import speedups
    pool = np.load(os.path.join(HERE, "pools", "c5_navigation_128.npz"))
    rec = {}
    for s, k in ((21, 0), (22, 3)):
        b0, g0 = pool["board"][k].copy(), pool["goals"][k].copy()
        p = float(pool["spawn_prob"][k])
        speedups.seed(s)
        b, g = b0.copy(), g0.copy()
        hb, hg = [], []
        for t in range(30):
            b = speedups.advance_board(b, p)
            g = speedups.advance_board(g, p)
            hb.append(b)
            hg.append(g)
        key = "s%d_l%d" % (s, k)
        rec[key + "_board0"], rec[key + "_goals0"] = b0, g0
        rec[key + "_boards"], rec[key + "_goals"] = np.array(hb), np.array(hg)
        rec[key + "_p"] = np.float64(p)
    np.savez_compressed(out, **rec)
    print("G2-128 ->", out)


def _spawner_boards(rng):
    from safelife.safelife_game import SafeLifeGame
    lv = np.load(os.path.join(REF, "safelife/levels/benchmarks/v1.0/append-spawn.npz"))["levels"]
    nav = np.load(os.path.join(REF, "safelife/levels/benchmarks/v1.0/navigation.npz"))["levels"]
    boards = [(lv[0]["board"], lv[0]["goals"]), (lv[1]["board"], lv[1]["goals"]),
              (nav[0]["board"], nav[0]["goals"])]
    H, W = 20, 31
    b = np.where(rng.rand(H, W) < 0.2, 9, 0).astype(np.uint16)
    b |= (rng.randint(0, 8, size=(H, W)) << 9).astype(np.uint16) * (b > 0)
    b[rng.rand(H, W) < 0.05] = 152 | (rng.randint(0, 8) << 9)
    b[rng.rand(H, W) < 0.02] = 128 | 16                  # hard spawner
    b[rng.rand(H, W) < 0.02] = 64                        # inhibitor
    boards.append((b, np.zeros_like(b)))
    del SafeLifeGame
    return boards


def gen_g2(out):
    from safelife import speedups
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    rng = np.random.RandomState(99)
    rec = {}
    for s in (0, 1, 2):
        for k, (b0, g0) in enumerate(_spawner_boards(rng)):
            speedups.seed(s)
            b, g = b0.copy(), g0.copy()
            counts, hb, hg = [], [], []
            for t in range(50):
                nb = oracle.count_eligible(b)
                b = speedups.advance_board(b, 0.3)
                ng = oracle.count_eligible(g)
                g = speedups.advance_board(g, 0.3)
                counts.append((nb, ng)); hb.append(b); hg.append(g)
            key = "s%d_b%d" % (s, k)
            rec[key + "_board0"] = b0
            rec[key + "_goals0"] = g0
            rec[key + "_boards"] = np.array(hb)
            rec[key + "_goals"] = np.array(hg)
            rec[key + "_counts"] = np.array(counts, np.int64)
    np.savez_compressed(out, **rec)
    print("G2 ->", out)


# ----------------------------------------------------------------------------
TRAJ_SPECS = [
    # name, level source, kwargs
    ("append_still_v01", ("npz", "benchmarks/v0.1/append-still-1.npz", None),
     dict(steps=1100, penalty=1.0, min_perf=0.01, seed=1, view=(33, 33))),
    ("prune_still_v10", ("archive", "benchmarks/v1.0/prune-still.npz", 0),
     dict(steps=1100, penalty=0.5, min_perf=-1.0, seed=2, view=(33, 33))),
    ("append_spawn_v10", ("archive", "benchmarks/v1.0/append-spawn.npz", 3),
     dict(steps=600, penalty=1.0, min_perf=0.01, seed=3, view=(15, 15))),
    ("prune_spawn_v10", ("archive", "benchmarks/v1.0/prune-spawn.npz", 1),
     dict(steps=600, penalty=1.0, min_perf=-1.0, seed=4, view=(33, 33))),
    ("navigation_v10", ("archive", "benchmarks/v1.0/navigation.npz", 2),
     dict(steps=600, penalty=0.0, min_perf=-1.0, seed=5, view=(33, 33))),
    ("append_dynamic_v10", ("archive", "benchmarks/v1.0/append-dynamic.npz", 4),
     dict(steps=600, penalty=1.0, min_perf=0.3, seed=6, view=(33, 33))),
    ("sokoban_example", ("npz", "examples/sokuban.npz", None),
     dict(steps=600, penalty=1.0, min_perf=-1.0, seed=7, view=(15, 15))),
    ("prune_still_64", ("pool", "pools/c3_prune_still_64.npz", 0),
     dict(steps=350, penalty=1.0, min_perf=0.01, seed=8, view=(33, 33), time_limit=100)),
    # exit-seeking policies: exercise can_exit / game_over / ContinuingEnv resets
    ("navigation_seek", ("archive", "benchmarks/v1.0/navigation.npz", 5),
     dict(steps=800, penalty=0.25, min_perf=-1.0, seed=9, view=(33, 33), seek=0.85)),
    ("prune_still_seek", ("archive", "benchmarks/v1.0/prune-still.npz", 7),
     dict(steps=800, penalty=1.0, min_perf=-1.0, seed=10, view=(33, 33), seek=0.85)),
    ("append_still_seek", ("archive", "benchmarks/v1.0/append-still.npz", 2),
     dict(steps=800, penalty=1.0, min_perf=0.0, seed=11, view=(15, 15), seek=0.85)),
]
# G4-128 (round 5): C5's board size -- 128x128 proc-gen navigation levels with
# spawners and oscillators, the bench's wrapper settings, episodes short enough that
# resets fall inside the trajectory
TRAJ128_SPECS = [
    ("nav128_c5", ("pool", "pools/c5_navigation_128.npz", 0),
     dict(steps=400, penalty=1.0, min_perf=0.01, seed=12, view=(33, 33), time_limit=150)),
    ("nav128_seek", ("pool", "pools/c5_navigation_128.npz", 3),
     dict(steps=320, penalty=1.0, min_perf=0.01, seed=13, view=(33, 33), time_limit=120,
          seek=0.8)),
]


def load_level_data(src):
    kind, path, idx = src
    if kind == "npz":
        d = np.load(os.path.join(REF, "safelife/levels", path))
        return {k: d[k] for k in d.files}
    if kind == "archive":
        lv = np.load(os.path.join(REF, "safelife/levels", path))["levels"][idx]
        return {k: lv[k] for k in lv.dtype.names if k != "name"}
    d = np.load(os.path.join(HERE, path))
    return {"board": d["board"][idx], "goals": d["goals"][idx],
            "agent_loc": d["agent_loc"][idx], "orientation": d["orientation"][idx],
            "spawn_prob": d["spawn_prob"][idx], "min_performance": d["min_performance"][idx],
            "class": "safelife.safelife_game.SafeLifeGame"}


def _seek_action(game, rng):
    """A move that shortens the wrapped distance to the (first) exit, if any."""
    ey, ex = game.exit_locs
    if len(ey) == 0:
        return None
    H, W = game.board.shape
    x0, y0 = game.agent_loc
    dy = (int(ey[0]) - y0 + H // 2) % H - H // 2
    dx = (int(ex[0]) - x0 + W // 2) % W - W // 2
    opts = []
    if dy < 0: opts.append(1)
    if dy > 0: opts.append(3)
    if dx > 0: opts.append(2)
    if dx < 0: opts.append(4)
    if not opts:
        return None
    return int(rng.choice(opts))


def run_traj(name, src, steps, penalty, min_perf, seed, view, time_limit=1000, seek=0.0):
    from safelife import speedups
    from safelife.safelife_env import SafeLifeEnv
    from safelife.safelife_game import SafeLifeGame
    from safelife import env_wrappers as ew

    data = load_level_data(src)
    level_data = dict(data)

    def level_iter():
        while True:
            yield SafeLifeGame.loaddata(level_data)

    env0 = SafeLifeEnv(level_iter(), view_shape=view, time_limit=time_limit)
    env = ew.MovementBonusWrapper(env0)
    env = ew.SimpleSideEffectPenalty(env, penalty_coef=penalty, min_performance=min_perf)
    env = ew.ContinuingEnv(env)
    speedups.seed(seed)                       # the spawn stream: RandomState(seed)
    arng = np.random.RandomState(1000 + seed)  # actions: a separate generator
    p_act = np.array([0.04] + [0.17] * 4 + [0.03] * 4)
    p_act /= p_act.sum()

    def packed_obs():
        oc = env0.output_channels
        env0.output_channels = None
        o = env0.get_obs()
        env0.output_channels = oc
        return o

    obs = env.reset()
    rec = {k: [] for k in ("action", "reward", "done", "times_up", "agent_loc", "orientation",
                           "points", "perf", "side_effect", "board", "goals", "obs",
                           "game_over", "episode_length")}
    obs0_packed = packed_obs()
    rec_obs0 = obs0_packed
    assert np.array_equal(obs0_packed & 0x7FFF,
                          (obs.astype(np.uint32) << np.arange(15)).sum(-1).astype(np.uint16))
    pen_wrapper = env.env
    for t in range(steps):
        a = int(arng.choice(9, p=p_act))
        if seek > 0 and arng.rand() < seek:
            sa = _seek_action(env0.game, arng)
            if sa is not None:
                a = sa
        obs, r, done, info = env.step(a)
        # ContinuingEnv resets on game over, so read it from the episode counter
        game_over = (env0.episode_length == 0) and not info["times_up"]
        if done:
            obs = env.reset()
        po = packed_obs()
        assert np.array_equal(po & 0x7FFF,
                              (obs.astype(np.uint32) << np.arange(15)).sum(-1).astype(np.uint16))
        g = env0.game
        rec["action"].append(a)
        rec["reward"].append(float(r))
        rec["done"].append(bool(done))
        rec["times_up"].append(bool(info["times_up"]))
        rec["game_over"].append(game_over)
        rec["episode_length"].append(int(info["episode"]["length"]))
        rec["agent_loc"].append(tuple(g.agent_loc))
        rec["orientation"].append(int(g.orientation))
        rec["points"].append(int(env0._old_game_value))
        rec["perf"].append(tuple(g.performance_ratio()))
        rec["side_effect"].append(int(pen_wrapper.last_side_effect))
        rec["board"].append(g.board.copy())
        rec["goals"].append(g.goals.copy())
        rec["obs"].append(po)
    out = {k: np.array(v) for k, v in rec.items()}
    out["obs0"] = rec_obs0
    for k in ("board", "goals", "agent_loc", "orientation", "spawn_prob", "min_performance"):
        out["level_" + k] = np.asarray(level_data[k])
    out["cfg"] = np.array([penalty, min_perf, seed, view[0], view[1], time_limit], np.float64)
    path = os.path.join(HERE, "traj_%s.npz" % name)
    np.savez_compressed(path, **out)
    print("traj", name, "steps", steps, "dones", int(out["done"].sum()),
          "game_overs", int(out["game_over"].sum()), "->", os.path.basename(path))


# G7 (round 5): the reference's PPO rollout loop itself (training/ppo.py:436-452) --
# np.random.choice per env from the global numpy stream, env.step, env.reset on done --
# over 16 envs, so the action draws and the spawn buffer's refills (random.c:14-26,
# 47-52) interleave in one stream.  A fixed table policy stands in for the network.
G7_SPECS = [
    ("ppo_loop_spawn", ("archive", "benchmarks/v1.0/append-spawn.npz", 3),
     dict(num_env=16, steps=40, seed=31, time_limit=15, penalty=1.0, min_perf=0.01)),
    ("ppo_loop_nav128", ("pool", "pools/c5_navigation_128.npz", 1),
     dict(num_env=16, steps=40, seed=32, time_limit=15, penalty=1.0, min_perf=0.01)),
]


def g7_table(num_env, steps, seed):
    """The table policy: float32 action probabilities [steps, num_env, 9], as a
    network's softmax would hand them to np.random.choice."""
    t = np.random.RandomState(seed + 7000).dirichlet(np.ones(9) * 0.7, size=(steps, num_env))
    t = t.astype(np.float32)
    return t / t.sum(-1, keepdims=True)


def run_ppo_loop(name, src, num_env, steps, seed, time_limit, penalty, min_perf):
    from safelife import speedups
    from safelife.safelife_env import SafeLifeEnv
    from safelife.safelife_game import SafeLifeGame
    from safelife import env_wrappers as ew
    level_data = dict(load_level_data(src))

    def level_iter():
        while True:
            yield SafeLifeGame.loaddata(level_data)

    envs = []
    for _ in range(num_env):
        e0 = SafeLifeEnv(level_iter(), view_shape=(33, 33), time_limit=time_limit)
        e = ew.MovementBonusWrapper(e0)
        e = ew.SimpleSideEffectPenalty(e, penalty_coef=penalty, min_performance=min_perf)
        envs.append((e0, ew.ContinuingEnv(e)))
    table = g7_table(num_env, steps, seed)
    speedups.seed(seed)
    for e0, env in envs:                      # run_agents' first call (ppo.py:429-434)
        env._ppo_last_obs = env.reset()
    rec = {k: [] for k in ("action", "reward", "done", "board", "goals")}
    for t in range(steps):                    # ppo.py:436-452
        policies = table[t]
        for (e0, env), policy in zip(envs, policies):
            action = np.random.choice(len(policy), p=policy)
            new_obs, reward, done, info = env.step(action)
            if done:
                new_obs = env.reset()
            env._ppo_last_obs = new_obs
            rec["action"].append(int(action))
            rec["reward"].append(float(reward))
            rec["done"].append(bool(done))
            rec["board"].append(e0.game.board.copy())
            rec["goals"].append(e0.game.goals.copy())
    out = {k: np.array(v).reshape((steps, num_env) + np.array(v[0]).shape)
           for k, v in rec.items()}
    # boards and goals of every env at every 10th step (and the last) for 128x128
    # levels (every step otherwise): rewards cover the steps in between
    keep = np.arange(steps) if level_data["board"].size <= 4096 else \
        np.unique(np.r_[np.arange(9, steps, 10), steps - 1])
    out["board"], out["goals"], out["board_steps"] = out["board"][keep], out["goals"][keep], keep
    out["table"] = table
    out["after"] = np.random.random(4)        # where the global stream ended
    for k in ("board", "goals", "agent_loc", "orientation", "spawn_prob", "min_performance"):
        out["level_" + k] = np.asarray(level_data[k])
    out["cfg"] = np.array([penalty, min_perf, seed, 33, 33, time_limit], np.float64)
    path = os.path.join(HERE, "g7_%s.npz" % name)
    np.savez_compressed(path, **out)
    print("G7", name, "dones", int(out["done"].sum()), "->", os.path.basename(path))


def gen_dens(out):
    """G5: the rollout + density half of side_effect_score (side_effects.py:131-143)."""
    from safelife import speedups
    from safelife.side_effects import _add_cell_distribution, _norm_cell_distribution
    rec = {}
    for j, src in enumerate([("archive", "benchmarks/v1.0/prune-dynamic.npz", 0),
                             ("archive", "benchmarks/v1.0/append-spawn.npz", 0)]):
        d = load_level_data(src)
        speedups.seed(11 + j)
        b0 = d["board"].copy()
        b1 = np.roll(d["board"], 1, axis=1)      # a perturbed "actual" board
        num_steps = 7
        inaction, action = {"n": 0}, {"n": 0}
        for _ in range(num_steps):
            b0 = speedups.advance_board(b0, float(d["spawn_prob"]))
        for _ in range(20):
            b0 = speedups.advance_board(b0, float(d["spawn_prob"]))
            b1 = speedups.advance_board(b1, float(d["spawn_prob"]))
            _add_cell_distribution(b0, inaction)
            _add_cell_distribution(b1, action)
        _norm_cell_distribution(inaction)
        _norm_cell_distribution(action)
        rec["l%d_board" % j] = d["board"]
        rec["l%d_spawn" % j] = float(d["spawn_prob"])
        for nm, dist in (("inaction", inaction), ("action", action)):
            keys = sorted(int(k) for k in dist)
            rec["l%d_%s_keys" % (j, nm)] = np.array(keys, np.int64)
            rec["l%d_%s_dens" % (j, nm)] = np.array([dist[np.uint16(k)] if np.uint16(k) in dist
                                                     else dist[k] for k in keys])
    np.savez_compressed(out, **rec)
    print("G5 ->", out)


# ----------------------------------------------------------------------------
POOL_SPECS = {
    # name: (yaml, board_shape, K)
    "c2_append_still_25": ("append-still", (25, 25), 64),
    "c3_prune_still_64": ("prune-still", (64, 64), 32),
    "c4_append_still_64": ("append-still", (64, 64), 32),
    "c5_navigation_128": ("navigation", (128, 128), 4),
}


def _gen_one(args):
    yaml_name, shape, k = args
    setup_reference(build=False)
    import yaml
    from safelife import speedups
    from safelife.proc_gen import gen_game
    from safelife import file_finder
    params = yaml.safe_load(open(os.path.join(REF, "safelife/levels/random/%s.yaml" % yaml_name)))
    named = file_finder._default_params["named_regions"].copy()
    named.update(params.get("named_regions", {}))
    data = file_finder._default_params.copy()
    data.update(**params)
    data["named_regions"] = named
    data["board_shape"] = list(shape)
    np.random.seed(k)
    speedups.seed(k)
    g = gen_game(**data)
    return (g.board.copy(), g.goals.copy(), np.array(g.agent_loc), int(g.orientation),
            float(g.spawn_prob), float(g.min_performance))


def gen_pool(name):
    from multiprocessing import Pool
    yaml_name, shape, K = POOL_SPECS[name]
    t0 = time.time()
    with Pool(min(8, K)) as pool:
        res = pool.map(_gen_one, [(yaml_name, shape, k) for k in range(K)])
    out = os.path.join(HERE, "pools", name + ".npz")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez_compressed(out, board=np.array([r[0] for r in res]),
                        goals=np.array([r[1] for r in res]),
                        agent_loc=np.array([r[2] for r in res]),
                        orientation=np.array([r[3] for r in res]),
                        spawn_prob=np.array([r[4] for r in res]),
                        min_performance=np.array([r[5] for r in res]),
                        seeds=np.arange(K))
    print("pool", name, K, "levels in %.1fs ->" % (time.time() - t0), out)


def copy_levels():
    """Benchmark level files the tests load (data, not source)."""
    dst = os.path.join(HERE, "levels")
    os.makedirs(dst, exist_ok=True)
    for i in range(1, 5):
        d = np.load(os.path.join(REF, "safelife/levels/benchmarks/v0.1/append-still-%d.npz" % i))
        np.savez_compressed(os.path.join(dst, "append-still-%d.npz" % i),
                            **{k: d[k] for k in d.files})
    print("levels ->", dst)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="g1,g2,levels,pools,traj,dens,g1_128,g2_128,traj128,g7")
    args = ap.parse_args()
    only = set(args.only.split(","))
    setup_reference()
    if "g1" in only:
        gen_g1(os.path.join(HERE, "advance_known_answers.npz"))
    if "g2" in only:
        gen_g2(os.path.join(HERE, "advance_stream.npz"))
    if "levels" in only:
        copy_levels()
    if "pools" in only:
        for name in ("c2_append_still_25", "c3_prune_still_64", "c4_append_still_64"):
            gen_pool(name)
    if "pool128" in only:
        gen_pool("c5_navigation_128")
    if "traj" in only:
        for name, src, kw in TRAJ_SPECS:
            run_traj(name, src, **kw)
    if "dens" in only:
        gen_dens(os.path.join(HERE, "densities.npz"))
    if "g1_128" in only:
        gen_g1_128(os.path.join(HERE, "advance_known_answers_128.npz"))
    if "g2_128" in only:
        gen_g2_128(os.path.join(HERE, "advance_stream_128.npz"))
    if "traj128" in only:
        for name, src, kw in TRAJ128_SPECS:
            run_traj(name, src, **kw)
    if "g7" in only:
        for name, src, kw in G7_SPECS:
            run_ppo_loop(name, src, **kw)


if __name__ == "__main__":
    main()
