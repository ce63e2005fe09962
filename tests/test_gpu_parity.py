"""Parity of the HIP path (through the C ABI) with the oracle and the golden vectors.

All tests here need the MI355X.  Integer/board results must be bit-exact; rewards
are float64 and are required to be bit-exact too (the kernel evaluates the same
IEEE operations in the same order; the tolerance the north star allows is 1e-6).
"""
import glob
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu
REWARD_TOL = 1e-6   # north_star bound; the checks below are stricter (==)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    import safelife_amd  # noqa: F401
    return torch, torch.device("cuda:0")


# --------------------------------------------------------------------- board
def test_advance_known_answers(torch_dev):
    torch, dev = torch_dev
    from safelife_amd import speedups
    d = np.load(os.path.join(GOLDEN, "advance_known_answers.npz"))
    groups = {}
    off = 0
    for (H, W), p in zip(d["shapes"], d["spawn_prob"]):
        n = H * W
        groups.setdefault((int(H), int(W), float(p)), []).append(
            (d["boards_in"][off:off + n].reshape(H, W), d["boards_out"][off:off + n].reshape(H, W)))
        off += n
    for (H, W, p), items in groups.items():
        bi = torch.from_numpy(np.stack([x[0] for x in items])).to(dev)
        out = speedups.advance_boards(bi, p, rng="stream")
        assert np.array_equal(out.cpu().numpy(), np.stack([x[1] for x in items])), (H, W, p)


def test_speedups_dropin_reference_stream(torch_dev):
    from safelife_amd import speedups
    d = np.load(os.path.join(GOLDEN, "advance_stream.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    for key in keys:
        s = int(key.split("_")[0][1:])
        speedups.seed(s)
        b, g = d[key + "_board0"], d[key + "_goals0"]
        for t in range(d[key + "_boards"].shape[0]):
            b = speedups.advance_board(b, 0.3)
            g = speedups.advance_board(g, 0.3)
            assert b.dtype == np.uint16
            assert np.array_equal(b, d[key + "_boards"][t]), (key, t)
            assert np.array_equal(g, d[key + "_goals"][t]), (key, t)


def _random_boards(rng, B, H, W, spawners=True):
    b = np.where(rng.rand(B, H, W) < 0.3, 9, 0).astype(np.uint16)
    b |= (rng.randint(0, 8, size=(B, H, W)) << 9).astype(np.uint16) * (b > 0)
    if spawners:
        b[rng.rand(B, H, W) < 0.03] = 152
        b[rng.rand(B, H, W) < 0.01] = 144 | (2 << 9)
    b[rng.rand(B, H, W) < 0.01] = 64
    b[rng.rand(B, H, W) < 0.01] = 32 | 16
    b[rng.rand(B, H, W) < 0.01] = 0x8000 | 4 | 16
    return b


@pytest.mark.parametrize("shape", [(2, 2), (3, 5), (25, 25), (26, 26), (64, 64), (17, 128),
                                   (128, 128)])
def test_advance_philox_vs_oracle(torch_dev, shape):
    torch, dev = torch_dev
    from safelife_amd import speedups
    H, W = shape
    rng = np.random.RandomState(H * 1000 + W)
    B = 24
    b = _random_boards(rng, B, H, W)
    p = np.float32(0.3)
    out = speedups.advance_boards(torch.from_numpy(b).to(dev), float(p), rng="philox", seed=77,
                                  env0=5, step=9, tensor=1).cpu().numpy()
    for i in range(B):
        ref, _ = oracle.advance(b[i], p, rng=oracle.RNG_PHILOX, seed=77, env_id=5 + i, step=9,
                                tensor=1)
        assert np.array_equal(out[i], ref), i


def test_advance_stream_batched_vs_oracle(torch_dev):
    torch, dev = torch_dev
    from safelife_amd import speedups
    rng = np.random.RandomState(4)
    B, H, W = 40, 26, 26
    b = _random_boards(rng, B, H, W)
    tb = torch.from_numpy(b).to(dev)
    counts = speedups.count_eligible(tb).cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    stream = rng.random_sample(int(counts.sum()) + 1)
    out = speedups.advance_boards(tb, 0.3, rng="stream", draws=torch.from_numpy(stream).to(dev),
                                  draw_offsets=torch.from_numpy(offs).to(dev)).cpu().numpy()
    for i in range(B):
        assert oracle.count_eligible(b[i]) == counts[i]
        ref, pos = oracle.advance(b[i], 0.3, stream, offs[i])
        assert pos == offs[i] + counts[i]
        assert np.array_equal(out[i], ref), i


# ----------------------------------------------------------------------- env
def _traj_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "traj_*.npz")))


def _vec_env_from_traj(d, B=1, **kw):
    from safelife_amd import SafeLifeVecEnv, LevelPool
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    pool = LevelPool.from_levels([{
        "board": d["level_board"], "goals": d["level_goals"], "agent_loc": d["level_agent_loc"],
        "orientation": d["level_orientation"], "spawn_prob": d["level_spawn_prob"],
        "min_performance": d["level_min_performance"]}])
    stream = np.random.RandomState(int(seed)).random_sample(400000)
    args = dict(time_limit=int(time_limit), view_shape=(int(vh), int(vw)), output_channels=None,
                penalty_coef=float(penalty), min_performance=float(min_perf), rng="stream",
                spawn_stream=stream)
    args.update(kw)
    return SafeLifeVecEnv(pool, B, "cuda:0", **args)


@pytest.mark.parametrize("kernel", ["fast", "generic"])
@pytest.mark.parametrize("path", _traj_files(), ids=lambda p: os.path.basename(p)[5:-4])
def test_env_golden_trajectory(torch_dev, path, kernel):
    """The reference-captured trajectories (reference-order spawn stream) through the
    bit-sliced kernels (replay prologue + SPAWN_STREAM step) and the per-cell kernel."""
    torch, dev = torch_dev
    d = np.load(path)
    env = _vec_env_from_traj(d, kernel=kernel)
    obs = env.reset().cpu().numpy()
    assert np.array_equal(obs[0], d["obs0"])
    T = len(d["action"])
    actions = torch.from_numpy(d["action"].astype(np.int32)).to(dev)
    for t in range(T):
        obs, r, done, info = env.step(actions[t:t + 1])
        ctx = (os.path.basename(path), t)
        assert r.item() == d["reward"][t], (ctx, r.item(), d["reward"][t])
        assert bool(done.item()) == bool(d["done"][t]), ctx
        assert bool(info["times_up"].item()) == bool(d["times_up"][t]), ctx
        if not (d["done"][t] or d["game_over"][t]):
            st = env.state
            assert (st["agent_x"].item(), st["agent_y"].item()) == tuple(d["agent_loc"][t]), ctx
            assert st["orientation"].item() == d["orientation"][t], ctx
            assert st["old_points"].item() == d["points"][t], ctx
            assert st["side_effect"].item() == d["side_effect"][t], ctx
        assert np.array_equal(env.board[0].cpu().numpy(), d["board"][t]), ctx
        assert np.array_equal(env.goals[0].cpu().numpy(), d["goals"][t]), ctx
        assert np.array_equal(obs[0].cpu().numpy(), d["obs"][t]), ctx
    assert not env.stream_error()


def _oracle_envs(pool_levels, B, **kw):
    envs = []
    for e in range(B):
        envs.append(oracle.OracleEnv(lambda ep, e=e: pool_levels[(e + ep * B) % len(pool_levels)],
                                     env_id=e, **kw))
    return envs


def _levels_from_pool(path):
    d = np.load(path)
    return [oracle.Level(d["board"][k], d["goals"][k], d["agent_loc"][k], d["orientation"][k],
                         d["spawn_prob"][k], d["min_performance"][k])
            for k in range(d["board"].shape[0])]


@pytest.mark.parametrize("pool_name,rng_mode", [("c2_append_still_25", "philox"),
                                                ("c3_prune_still_64", "philox"),
                                                ("c2_append_still_25", "stream")])
def test_env_batch_vs_oracle(torch_dev, pool_name, rng_mode):
    """B envs with mixed levels, random actions, short time limit (exercises resets)."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", pool_name + ".npz")
    levels = _levels_from_pool(path)
    B, T = 24, 90
    kw = dict(time_limit=40, view_shape=(15, 15), output_channels=None, penalty_coef=0.7,
              min_performance=-1.0)
    rng = np.random.RandomState(7)
    stream = rng.random_sample(300000)
    if rng_mode == "stream":
        venv = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", rng="stream",
                              spawn_stream=stream, **kw)
        shared = _SharedStream(stream)
        oenvs = _oracle_envs(levels, B, rng="stream", stream=shared, **kw)
    else:
        venv = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", rng="philox", seed=123, **kw)
        oenvs = _oracle_envs(levels, B, rng="philox", seed=123, **kw)
    vo = venv.reset().cpu().numpy()
    for e in range(B):
        assert np.array_equal(vo[e], oenvs[e].reset()), e
    for t in range(T):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        vo, vr, vd, info = venv.step(torch.from_numpy(acts).to(dev))
        vo, vr, vd = vo.cpu().numpy(), vr.cpu().numpy(), vd.cpu().numpy()
        vb, vg = venv.board.cpu().numpy(), venv.goals.cpu().numpy()
        for e in range(B):
            o, r, dn, _ = oenvs[e].step(int(acts[e]))
            ctx = (t, e)
            assert vr[e] == r, (ctx, vr[e], r)
            assert bool(vd[e]) == dn, ctx
            assert np.array_equal(vb[e], oenvs[e].board), ctx
            assert np.array_equal(vg[e], oenvs[e].goals), ctx
            assert np.array_equal(vo[e], o), ctx


class _SharedStream:
    """One uniform stream consumed env after env, board then goals (replay order)."""

    def __init__(self, s):
        self.s, self.pos = s, 0

    def take(self, n):
        out = self.s[self.pos:self.pos + n]
        self.pos += n
        return out


def test_obs_channels_vs_packed(torch_dev):
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    pool = LevelPool.load(os.path.join(GOLDEN, "pools", "c2_append_still_25.npz"))
    kw = dict(view_shape=(33, 33), rng="philox", seed=3)
    e1 = SafeLifeVecEnv(pool, 16, "cuda:0", output_channels=None, **kw)
    e2 = SafeLifeVecEnv(pool, 16, "cuda:0", output_channels=tuple(range(15)), **kw)
    e3 = SafeLifeVecEnv(pool, 16, "cuda:0", output_channels=(0, 9, 12, 15), obs_dtype="uint8",
                        **kw)
    for e in (e1, e2, e3):
        e.reset()
    rng = np.random.RandomState(0)
    for t in range(20):
        a = torch.from_numpy(rng.randint(0, 9, 16).astype(np.int32)).to(dev)
        p = e1.step(a)[0].cpu().numpy().astype(np.int64)
        c = e2.step(a)[0].cpu().numpy().astype(np.int64)
        u = e3.step(a)[0].cpu().numpy().astype(np.int64)
        assert np.array_equal((c << np.arange(15)).sum(-1), p & 0x7FFF)
        for k, ch in enumerate((0, 9, 12, 15)):
            assert np.array_equal(u[..., k], (p >> ch) & 1)


def test_reset_roll_augmentation_vs_oracle(torch_dev):
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    levels = _levels_from_pool(path)
    B, seed = 16, 99
    venv = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", rng="philox", seed=seed,
                          augment_roll=True, level_order="random", view_shape=(9, 9),
                          output_channels=None)
    venv.reset()
    K = len(levels)
    for e in range(B):
        idx = min(int(oracle.philox_uniform(e, 0, 0x5EED, 2, seed) * K), K - 1)
        dy = min(int(oracle.philox_uniform(e, 0, 0x0011, 3, seed) * 64), 63)
        dx = min(int(oracle.philox_uniform(e, 0, 0x0022, 3, seed) * 64), 63)
        lv = levels[idx].rolled(dy, dx)
        assert venv.state["level_index"][e].item() == idx
        assert np.array_equal(venv.start_board[e].cpu().numpy(), lv.board)
        assert np.array_equal(venv.goals[e].cpu().numpy(), lv.goals)
        assert (venv.state["agent_x"][e].item(), venv.state["agent_y"][e].item()) == lv.agent_loc


# ------------------------------------------------------- fast vs generic kernel
def _sprinkled_pool(path, rng, spawn_frac=0.004):
    """64x64 pool levels with extra spawners in empty cells (exercise spawning)."""
    from safelife_amd import LevelPool
    p = LevelPool.load(path)
    board = p.board.copy()
    goals = p.goals.copy()
    for k in range(p.K):
        empty = (board[k] == 0) & (rng.rand(p.H, p.W) < spawn_frac)
        empty[p.agent_y[k], p.agent_x[k]] = False
        board[k][empty] = 152 | (rng.randint(0, 8, size=empty.sum()) << 9).astype(np.uint16)
        ge = (goals[k] == 0) & (rng.rand(p.H, p.W) < spawn_frac / 2)
        goals[k][ge] = 144
    al = np.stack([p.agent_x, p.agent_y], 1)
    return LevelPool(board, goals, al, p.orientation, p.spawn_prob, p.min_performance)


def _compare_state(e1, e2, ctx):
    assert np.array_equal(e1.board.cpu().numpy(), e2.board.cpu().numpy()), ctx
    assert np.array_equal(e1.goals.cpu().numpy(), e2.goals.cpu().numpy()), ctx
    for k in e1.st_t:
        assert np.array_equal(e1.st_t[k].cpu().numpy(), e2.st_t[k].cpu().numpy()), (ctx, k)


@pytest.mark.parametrize("spawners", [False, True])
def test_fast_kernel_vs_generic(torch_dev, spawners):
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    rng = np.random.RandomState(11)
    pool = _sprinkled_pool(path, rng) if spawners else LevelPool.load(path)
    B, T = 768, 260
    kw = dict(time_limit=70, view_shape=(33, 33), output_channels=None, penalty_coef=0.7,
              min_performance=0.01, rng="philox", seed=42, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    o1, o2 = fast.reset(), gen.reset()
    assert torch.equal(o1, o2)
    for t in range(T):
        # bias towards toggles so boards fill with life and change every step
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        o1, r1, d1, i1 = fast.step(a)
        o2, r2, d2, i2 = gen.step(a)
        assert torch.equal(r1, r2), (t, (r1 - r2).abs().max().item())
        assert torch.equal(d1, d2), t
        assert torch.equal(fast.flags, gen.flags), t
        assert torch.equal(o1, o2), t
        if t % 13 == 0 or t == T - 1:
            _compare_state(fast, gen, t)


@pytest.mark.parametrize("view,remove_white,auto_reset,hi_bits", [((33, 33), True, True, False),
                                                                  ((1, 1), False, True, False),
                                                                  ((70, 9), True, False, False),
                                                                  ((7, 64), False, True, False),
                                                                  ((64, 64), True, True, False),
                                                                  ((33, 33), True, True, True)])
def test_fast_kernel_fused_obs(torch_dev, view, remove_white, auto_reset, hi_bits):
    """The 64x64 kernel writes packed views from the board it holds on chip (views of
    envs reset after the step are rewritten by a list kernel): every step they equal
    the stand-alone observation kernel's view of the state left behind (views wider
    than the board wrap; white goals kept or removed; with and without resets; boards
    using the otherwise unused cell bits 12-14)."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    pool = _sprinkled_pool(path, np.random.RandomState(4), spawn_frac=0.006)
    pool.goals[:, 5:9, 5:9] = 0x0E00 | 0x10     # white goal patch in every level
    if hi_bits:     # unused cell bits 12-14 set on walls: the kernel's bit-sliced add path
        walls = (pool.board & 0x10) != 0
        pool.board[walls] |= np.uint16(0x7000)
    B, T = 130, 50
    venv = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", view_shape=view,
                          output_channels=None, remove_white_goals=remove_white,
                          time_limit=17, auto_reset=auto_reset, rng="philox", seed=31,
                          level_order="random", augment_roll=True, min_performance=0.01)
    venv.reset()
    rng = np.random.RandomState(8)
    resets = 0
    for t in range(T):
        a = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        o, _, _, info = venv.step(a)
        fused = o.clone()
        resets += int(info["reset"].sum().item()) if auto_reset else 0
        ref = venv.observe().clone()
        assert torch.equal(fused, ref), (t, (fused != ref).nonzero()[:5].tolist())
    assert resets > 0 or not auto_reset


@pytest.mark.parametrize("view,channels,dtype,auto_reset,hi_bits", [
    ((33, 33), tuple(range(15)), "uint16", True, False),
    ((33, 33), tuple(range(15)), "bfloat16", True, False),
    ((15, 15), tuple(range(15)), "uint8", True, False),
    ((33, 33), tuple(range(15)), "float32", True, True),
    ((33, 33), (0, 3, 5, 9, 10, 11), "uint16", False, False),
    ((7, 64), (1, 4, 2, 12, 13, 14, 15, 0), "bfloat16", True, False),
    ((1, 1), tuple(range(16)), "uint8", True, False),
    ((40, 40), tuple(range(15)), "uint16", True, False)])      # > kFusedChanCells: unfused
def test_fast_kernel_fused_channel_obs(torch_dev, view, channels, dtype, auto_reset, hi_bits):
    """Channel views (the reference's default output_channels=range(15), other channel
    lists, u16 / u8 / f32 / bf16 elements) written by the 64x64 step kernel from the
    board it holds on chip, and by the reset-list kernel for envs reset after the step,
    equal every step what the stand-alone observation kernel computes from the state
    left behind; boards using cell bits 12-14 take the kernel's from-HBM fallback."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    pool = _sprinkled_pool(path, np.random.RandomState(4), spawn_frac=0.006)
    pool.goals[:, 5:9, 5:9] = 0x0E00 | 0x10
    if hi_bits:
        walls = (pool.board & 0x10) != 0
        pool.board[walls] |= np.uint16(0x7000)
    B, T = 130, 40
    venv = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", view_shape=view,
                          output_channels=channels, obs_dtype=dtype, time_limit=17,
                          auto_reset=auto_reset, rng="philox", seed=31, level_order="random",
                          augment_roll=True, min_performance=0.01)
    venv.reset()
    rng = np.random.RandomState(8)
    resets = 0
    for t in range(T):
        a = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        o, _, _, info = venv.step(a)
        fused = o.clone()
        resets += int(info["reset"].sum().item()) if auto_reset else 0
        ref = venv.observe().clone()
        assert torch.equal(fused.view(torch.uint8), ref.view(torch.uint8)), t
    assert resets > 0 or not auto_reset


def test_fast_kernel_spawners_vs_oracle(torch_dev):
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    pool = _sprinkled_pool(path, np.random.RandomState(5), spawn_frac=0.01)
    levels = [oracle.Level(pool.board[k], pool.goals[k], (pool.agent_x[k], pool.agent_y[k]),
                           pool.orientation[k], pool.spawn_prob[k], pool.min_performance[k])
              for k in range(pool.K)]
    B, T = 12, 40
    kw = dict(time_limit=1000, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01)
    venv = SafeLifeVecEnv(pool, B, "cuda:0", rng="philox", seed=9, kernel="fast", **kw)
    oenvs = _oracle_envs(levels, B, rng="philox", seed=9, **kw)
    venv.reset()
    for e in range(B):
        oenvs[e].reset()
    rng = np.random.RandomState(2)
    for t in range(T):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        _, vr, _, _ = venv.step(torch.from_numpy(acts).to(dev))
        vr, vb = vr.cpu().numpy(), venv.board.cpu().numpy()
        for e in range(B):
            _, r, _, _ = oenvs[e].step(int(acts[e]))
            assert vr[e] == r, (t, e)
            assert np.array_equal(vb[e], oenvs[e].board), (t, e)


def test_full_batch_sampled_vs_oracle(torch_dev):
    """The headline configuration at full size (B = 65 536 envs of 64x64, fast kernel,
    PPO chain, Philox, 33x33 packed views written by the step kernel): every step, a
    sample of envs spread over the batch matches the oracle run of the same global env
    ids bit for bit (board, goals, observation, reward, done), and
    the batch-wide episode counters agree with the reset flags."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    levels = _levels_from_pool(path)
    B, T = 65536, 36
    kw = dict(time_limit=15, view_shape=(33, 33), output_channels=None, penalty_coef=1.0,
              min_performance=0.01)
    venv = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", rng="philox", seed=2024,
                          compute_obs=True, kernel="fast", **kw)    # views fused in the kernel
    sample = [0, 1, 63, 4097, 32767, 40000, 65534, 65535]
    oenvs = {e: oracle.OracleEnv(lambda ep, e=e: levels[(e + ep * B) % len(levels)],
                                 env_id=e, rng="philox", seed=2024, **kw) for e in sample}
    venv.reset()
    for e in sample:
        oenvs[e].reset()
        assert np.array_equal(venv.board[e].cpu().numpy(), oenvs[e].board), e
    rng = np.random.RandomState(5)
    n_done = 0
    for t in range(T):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        vo, vr, vd, info = venv.step(torch.from_numpy(acts).to(dev))
        n_done += int(info["reset"].sum().item())     # times_up and game_over resets
        vo, vr, vd = vo.cpu().numpy(), vr.cpu().numpy(), vd.cpu().numpy()
        for e in sample:
            o, r, dn, _ = oenvs[e].step(int(acts[e]))
            ctx = (t, e)
            assert np.array_equal(vo[e], o), ctx
            assert vr[e] == r, (ctx, vr[e], r)
            assert bool(vd[e]) == dn, ctx
            assert np.array_equal(venv.board[e].cpu().numpy(), oenvs[e].board), ctx
            assert np.array_equal(venv.goals[e].cpu().numpy(), oenvs[e].goals), ctx
    assert n_done > 0
    assert int(venv.state["episodes"].sum().item()) == B + n_done


def test_fast_kernel_state_overwrite(torch_dev):
    """set_state mid-run (board/goals/start written by the caller) invalidates the fast
    kernel's bit-plane mirrors and pool start-board source, and so does set_pool (a new
    level pool while episodes run): the run continues bit-exact with the generic kernel
    given the same overwrite."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    B, T = 256, 60
    kw = dict(time_limit=40, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01, rng="philox", seed=9, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", kernel="generic", **kw)
    fast.reset()
    gen.reset()
    rng = np.random.RandomState(3)
    for t in range(T):
        a = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        if t == 25:
            # swap every env's state with its neighbour's (a state neither kernel's
            # caches have seen), identically in both envs
            perm = np.roll(np.arange(B), 1)
            bd, gl, sb = (x.cpu().numpy()[perm] for x in (fast.board, fast.goals,
                                                          fast.start_board))
            sc = {k: v.cpu().numpy()[perm] for k, v in fast.st_t.items()
                  if k != "start_roll"}
            fast.set_state(bd, gl, sb, **sc)
            gen.set_state(bd, gl, sb, **sc)
        if t == 45:
            # a new level pool mid-episode: running episodes keep their start boards
            newpool = LevelPool.load(path).subset(np.arange(31, -1, -1) % 32)
            fast.set_pool(newpool)
            gen.set_pool(newpool)
        _, r1, d1, _ = fast.step(a)
        _, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), t
        assert torch.equal(d1, d2), t
        _compare_state(fast, gen, t)


# ------------------------------------------- small-board bit-sliced kernel (C2)
def _synthetic_pool(rng, K, H, W):
    """K random levels of any shape: life of random colours, walls, crates, spawners,
    an agent and an exit, colour goals (some live)."""
    from safelife_amd import LevelPool
    board = _random_boards(rng, K, H, W)
    goals = np.where(rng.rand(K, H, W) < 0.3, rng.randint(1, 8, size=(K, H, W)) << 9, 0)
    goals = (goals | np.where(rng.rand(K, H, W) < 0.05, 9, 0)).astype(np.uint16)
    al = np.zeros((K, 2), np.int64)
    for k in range(K):
        ax, ay = rng.randint(0, W), rng.randint(0, H)
        ex, ey = (ax + W // 2) % W, (ay + H // 2) % H
        board[k, ay, ax] = 122
        if (ex, ey) != (ax, ay):
            board[k, ey, ex] = 272
        al[k] = (ax, ay)
    return LevelPool(board, goals, al, rng.randint(0, 4, size=K), np.full(K, 0.3),
                     np.full(K, 0.01))


@pytest.mark.parametrize("shape", [(25, 25), (26, 26), (2, 2), (3, 5), (32, 63), (17, 64),
                                   (31, 2), (9, 31), (32, 32), (25, 33), (7, 29), (20, 28)])
def test_small_kernel_vs_generic(torch_dev, shape):
    """Boards up to 32x64 take the bit-sliced small kernels (column pairs over all rows,
    ds_bpermute wrap at W, odd W via a column-0 copy; up to 32 wide four envs share a
    wave, and batches that are no multiple of 4 leave segments empty): bit-exact with
    the generic kernel through actions, spawns, exits and resets."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    H, W = shape
    rng = np.random.RandomState(H * 100 + W)
    if shape == (25, 25):
        pool = _sprinkled_pool(os.path.join(GOLDEN, "pools", "c2_append_still_25.npz"), rng,
                               spawn_frac=0.01)
    else:
        pool = _synthetic_pool(rng, 8, H, W)
    B, T = 94 + (H + W) % 4, 70
    kw = dict(time_limit=23, view_shape=(9, 9), output_channels=None, penalty_coef=0.7,
              min_performance=0.01, rng="philox", seed=5, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    o1, o2 = fast.reset(), gen.reset()
    assert torch.equal(o1, o2)
    for t in range(T):
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        o1, r1, d1, _ = fast.step(a)
        o2, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), (t, (r1 - r2).abs().max().item())
        assert torch.equal(d1, d2), t
        assert torch.equal(fast.flags, gen.flags), t
        assert torch.equal(o1, o2), t
        _compare_state(fast, gen, t)


@pytest.mark.parametrize("B", [1, 3, 5])
def test_bitsliced_kernels_tiny_batches(torch_dev, B):
    """Batches that fill no workgroup: the 64x64 kernel (with fused views and its reset
    list), the small-board and 128x128 kernels agree with the generic kernel."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    rng = np.random.RandomState(B)
    pools = [LevelPool.load(os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")),
             LevelPool.load(os.path.join(GOLDEN, "pools", "c2_append_still_25.npz")),
             LevelPool.load(C5_POOL)]
    for pool in pools:
        kw = dict(time_limit=9, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
                  min_performance=0.01, rng="philox", seed=77, level_order="random",
                  augment_roll=True)
        fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
        gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
        assert torch.equal(fast.reset(), gen.reset())
        for t in range(25):
            a = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
            o1, r1, d1, _ = fast.step(a)
            o2, r2, d2, _ = gen.step(a)
            ctx = (pool.H, t)
            assert torch.equal(r1, r2) and torch.equal(d1, d2), ctx
            assert torch.equal(o1, o2), ctx
            _compare_state(fast, gen, ctx)


def test_c_abi_rejects_bad_arguments(torch_dev):
    """The C ABI returns SL_EINVAL (no launch) for bad view shapes, observation modes,
    channel lists and movement-bonus periods, and SL_ETOOBIG when a bit-sliced kernel
    is required for a shape none takes."""
    import ctypes
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool, _lib
    L = _lib.lib()
    pool = LevelPool.load(os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz"))
    env = SafeLifeVecEnv(pool, 4, "cuda:0", output_channels=None, view_shape=(15, 15))
    env.reset()
    st, sp = ctypes.byref(env._state), _lib.stream_ptr(dev)
    out = torch.zeros(4 * 70 * 70 * 16, dtype=torch.int32, device=dev)
    chans = (ctypes.c_int32 * 2)(0, 16)
    assert L.sl_env_obs(st, 0, 5, 1, _lib.SL_OBS_PACKED, None, 0, out.data_ptr(), sp) == _lib.SL_EINVAL
    assert L.sl_env_obs(st, 5, 5, 1, 99, None, 0, out.data_ptr(), sp) == _lib.SL_EINVAL
    assert L.sl_env_obs(st, 5, 5, 1, _lib.SL_OBS_CHANNELS, chans, 2, out.data_ptr(), sp) == _lib.SL_EINVAL
    assert L.sl_env_obs(st, 5, 5, 1, _lib.SL_OBS_CHANNELS, None, 0, out.data_ptr(), sp) == _lib.SL_EINVAL
    a = torch.zeros(4, dtype=torch.int32, device=dev)
    cfg = env._fill_cfg()
    env._fill_obs_cfg(cfg, None)
    args = (st, ctypes.byref(env._pool_dev["struct"]), a.data_ptr(), ctypes.byref(cfg),
            env.reward.data_ptr(), env.done.data_ptr(), env.flags.data_ptr(),
            env.ep_len.data_ptr(), env.ep_rew.data_ptr(), sp)
    cfg.bonus_period = 17
    assert L.sl_env_step(*args) == _lib.SL_EINVAL
    cfg.bonus_period = env.movement_bonus_period
    cfg.obs_out = out.data_ptr()
    cfg.obs_mode, cfg.obs_vh, cfg.obs_vw = _lib.SL_OBS_PACKED, 0, 15     # empty view
    assert L.sl_env_step(*args) == _lib.SL_EINVAL
    cfg.obs_mode, cfg.obs_vh = 42, 15                                      # no such mode
    assert L.sl_env_step(*args) == _lib.SL_EINVAL
    torch.cuda.synchronize()
    odd = LevelPool(np.zeros((1, 40, 70), np.uint16), np.zeros((1, 40, 70), np.uint16),
                    [(0, 0)], [1], [0.3], [0.01])
    with pytest.raises(RuntimeError):
        SafeLifeVecEnv(odd, 2, "cuda:0", kernel="fast", output_channels=None).step(
            torch.zeros(2, dtype=torch.int32, device=dev))


# ------------------------------------------------ 128x128 bit-sliced kernel (C5)
C5_POOL = os.path.join(GOLDEN, "pools", "c5_navigation_128.npz")


@pytest.mark.parametrize("goal_bits", [False, True])
def test_fast128_vs_generic(torch_dev, goal_bits):
    """The 128x128 banded bit-sliced kernel against the per-cell generic kernel on the
    C5 navigation levels (spawners everywhere, oscillating goals in level 3): rewards,
    done, flags, observations every step, all state every few steps, across resets.
    goal_bits: two levels' goals also carry preserve / inhibit cells (outside the goal
    plane mirror: spawn_flags bit 3, their goals are read as cells), the other two use
    the mirror's six planes."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    pool = LevelPool.load(C5_POOL)
    rng = np.random.RandomState(17)
    if goal_bits:
        for k in (1, 3):
            g = pool.goals[k]
            life = (g & 0x1) != 0
            g[life & (rng.rand(*g.shape) < 0.1)] |= np.uint16(0x20)
            g[(g == 0) & (rng.rand(*g.shape) < 0.01)] = np.uint16(0x40 | 0x10)
    B, T = 160, 90
    kw = dict(time_limit=35, view_shape=(33, 33), output_channels=None, penalty_coef=0.7,
              min_performance=0.01, rng="philox", seed=77, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    o1, o2 = fast.reset(), gen.reset()
    assert torch.equal(o1, o2)
    for t in range(T):
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        o1, r1, d1, _ = fast.step(a)
        o2, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), (t, (r1 - r2).abs().max().item())
        assert torch.equal(d1, d2), t
        assert torch.equal(fast.flags, gen.flags), t
        assert torch.equal(o1, o2), t
        if t % 7 == 0 or t == T - 1:
            _compare_state(fast, gen, t)


def test_fast128_vs_oracle(torch_dev):
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    levels = _levels_from_pool(C5_POOL)
    B, T = 6, 24
    kw = dict(time_limit=1000, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01)
    venv = SafeLifeVecEnv(LevelPool.load(C5_POOL), B, "cuda:0", rng="philox", seed=3,
                          kernel="fast", **kw)
    oenvs = _oracle_envs(levels, B, rng="philox", seed=3, **kw)
    venv.reset()
    for e in range(B):
        oenvs[e].reset()
    rng = np.random.RandomState(4)
    for t in range(T):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        _, vr, vd, _ = venv.step(torch.from_numpy(acts).to(dev))
        vr, vd = vr.cpu().numpy(), vd.cpu().numpy()
        vb, vg = venv.board.cpu().numpy(), venv.goals.cpu().numpy()
        for e in range(B):
            _, r, dn, _ = oenvs[e].step(int(acts[e]))
            assert vr[e] == r, (t, e, vr[e], r)
            assert bool(vd[e]) == dn, (t, e)
            assert np.array_equal(vb[e], oenvs[e].board), (t, e)
            assert np.array_equal(vg[e], oenvs[e].goals), (t, e)


def test_fast128_state_overwrite(torch_dev):
    """set_state mid-run invalidates the 128x128 kernel's goals mirror."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    B, T = 64, 30
    kw = dict(time_limit=25, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01, rng="philox", seed=5, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(LevelPool.load(C5_POOL), B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(LevelPool.load(C5_POOL), B, "cuda:0", kernel="generic", **kw)
    fast.reset()
    gen.reset()
    rng = np.random.RandomState(8)
    for t in range(T):
        a = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        if t == 12:
            perm = np.roll(np.arange(B), 3)
            bd, gl, sb = (x.cpu().numpy()[perm] for x in (fast.board, fast.goals,
                                                          fast.start_board))
            sc = {k: v.cpu().numpy()[perm] for k, v in fast.st_t.items()
                  if k != "start_roll"}
            fast.set_state(bd, gl, sb, **sc)
            gen.set_state(bd, gl, sb, **sc)
        _, r1, d1, _ = fast.step(a)
        _, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), t
        assert torch.equal(d1, d2), t
        _compare_state(fast, gen, t)


@pytest.mark.parametrize("where", ["pool", "set_state"])
def test_fast128_hi_bits_vs_generic(torch_dev, where):
    """Cell bits 12-14 (no cell type uses them) on 128x128 boards: the kernel's 8-plane
    start-board spool leaves them out, and envs whose start board may carry them
    (spawn_flags bit 2) get the exact side-effect term from a second pass.  From pool
    levels (the resets set the flag; start boards from the pool planes) and from boards
    loaded by set_state (the host sets it; start boards from HBM), with the bits also
    on board cells whose start cells lack them, against the per-cell generic kernel."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    rng = np.random.RandomState(23)
    pool = LevelPool.load(C5_POOL)
    if where == "pool":
        walls = (pool.board & 0x10) != 0
        pool.board[walls & (rng.rand(*pool.board.shape) < 0.3)] |= np.uint16(0x5000)
        pool.board[walls & (rng.rand(*pool.board.shape) < 0.2)] |= np.uint16(0x2000)
    B, T = 96, 40
    kw = dict(time_limit=25, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01, rng="philox", seed=6, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    fast.reset()
    gen.reset()
    if where == "pool":
        assert (fast.st_t["spawn_flags"].cpu().numpy() & 4).any()
    for t in range(T):
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        if t == 6 and where == "set_state":
            bd, gl, sb = (x.cpu().numpy().copy() for x in (fast.board, fast.goals,
                                                          fast.start_board))
            walls = (sb & 0x10) != 0
            sb[walls & (rng.rand(*sb.shape) < 0.3)] |= np.uint16(0x3000)
            sb[: B // 3] &= np.uint16(0x8FFF)             # a third without them
            wb = (bd & 0x10) != 0
            bd[wb & (rng.rand(*bd.shape) < 0.2)] |= np.uint16(0x4000)   # board side only
            fast.set_state(bd, gl, sb)
            gen.set_state(bd, gl, sb)
            fl = fast.st_t["spawn_flags"].cpu().numpy()
            assert not (fl[: B // 3] & 4).any() and (fl[B // 3:] & 4).any()
        _, r1, d1, _ = fast.step(a)
        _, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), (t, (r1 - r2).abs().max().item())
        assert torch.equal(d1, d2), t
        assert torch.equal(fast.flags, gen.flags), t
        if t % 5 == 0 or t == T - 1:
            _compare_state(fast, gen, t)


def test_fast128_pool_swap_vs_generic(torch_dev):
    """A pool swap mid-run on 128x128 boards: running episodes stop reading their start
    planes and pristine goal colours from the pool (start_roll = -1: start boards and
    the goals mirror from HBM) until they are reset from the new pool, against the
    per-cell generic kernel, across the swap and the resets after it."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    pool = LevelPool.load(C5_POOL)
    perm = [2, 0, 3, 1]
    al = np.stack([pool.agent_x, pool.agent_y], 1)
    pool2 = LevelPool(np.roll(pool.board[perm], 5, axis=2), np.roll(pool.goals[perm], 5, axis=2),
                      (al[perm] + [5, 0]) % 128, pool.orientation[perm], pool.spawn_prob[perm],
                      pool.min_performance[perm])
    rng = np.random.RandomState(31)
    B, T = 96, 50
    kw = dict(time_limit=20, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01, rng="philox", seed=9, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    fast.reset()
    gen.reset()
    for t in range(T):
        if t == 13:
            fast.set_pool(pool2)
            gen.set_pool(pool2)
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        _, r1, d1, _ = fast.step(a)
        _, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), (t, (r1 - r2).abs().max().item())
        assert torch.equal(d1, d2), t
        assert torch.equal(fast.flags, gen.flags), t
        if t % 4 == 0 or t == T - 1:
            _compare_state(fast, gen, t)


# ------------------------------------------------------- side-effect densities (A15)
def test_side_effect_densities_reference_fixture(torch_dev):
    """sl_side_effect_densities in replay mode reproduces the reference's density maps
    (densities.npz, captured from side_effects.py with speedups.seed(11 + j))."""
    from safelife_amd.side_effects import side_effect_densities
    d = np.load(os.path.join(GOLDEN, "densities.npz"))
    for j in range(2):
        board = d["l%d_board" % j]
        stream = np.random.RandomState(11 + j).random_sample(200000)
        (ina, act), = side_effect_densities(board[None], np.roll(board, 1, axis=1)[None], [7],
                                            float(d["l%d_spawn" % j]), 20, rng="stream",
                                            spawn_stream=stream)
        for nm, got in (("inaction", ina), ("action", act)):
            keys = d["l%d_%s_keys" % (j, nm)].tolist()
            assert sorted(got) == keys, (j, nm)
            for k, ref in zip(keys, d["l%d_%s_dens" % (j, nm)]):
                assert np.array_equal(got[k], ref), (j, nm, k)


@pytest.mark.parametrize("pool_name", ["c2_append_still_25", "c3_prune_still_64"])
def test_side_effect_densities_philox_batch_vs_oracle(torch_dev, pool_name):
    """A batch of episodes with different num_steps (Philox) equals the oracle run of
    each episode keyed by its index."""
    from safelife_amd.side_effects import side_effect_densities
    p = np.load(os.path.join(GOLDEN, "pools", pool_name + ".npz"))
    E = 5
    init = p["board"][:E]
    rng = np.random.RandomState(4)
    final = np.stack([np.roll(b, (rng.randint(3), rng.randint(3)), (0, 1)) for b in init])
    steps = [0, 3, 11, 1, 6]
    sp = 0.3
    got = side_effect_densities(init, final, steps, sp, 9, rng="philox", seed=77, env0=0)
    for e in range(E):
        ina, act = oracle.side_effect_densities(init[e], final[e], steps[e], sp, 9,
                                                rng="philox", seed=77, env_id=e)
        for nm, g, r in (("inaction", got[e][0], ina), ("action", got[e][1], act)):
            assert sorted(g) == sorted(r), (e, nm)
            for k in r:
                assert np.array_equal(g[k], r[k]), (e, nm, k)


# ------------------------------------------------------- B=1 drop-in views
@pytest.mark.parametrize("path", _traj_files()[:6], ids=lambda p: os.path.basename(p)[5:-4])
def test_single_env_dropin_golden(torch_dev, path):
    """safelife_amd.SafeLifeEnv (B = 1, reference RNG through the global numpy stream)
    reproduces a reference trajectory's boards, goals, agent state, points and
    observations up to the first episode end (the wrappers only change the reward
    and restart episodes), and leaves numpy's global RNG where the reference would."""
    from safelife_amd import SafeLifeEnv
    d = np.load(path)
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    level = {"board": d["level_board"], "goals": d["level_goals"],
             "agent_loc": d["level_agent_loc"], "orientation": d["level_orientation"],
             "spawn_prob": d["level_spawn_prob"],
             "min_performance": d["level_min_performance"]}
    env = SafeLifeEnv(iter([level]), view_shape=(int(vh), int(vw)), output_channels=None,
                      time_limit=int(time_limit), seed=int(seed))
    obs0 = env.reset()
    env.game.min_performance = float(min_perf)     # what SimpleSideEffectPenalty.reset does
    assert np.array_equal(obs0, d["obs0"])
    for t in range(len(d["action"])):
        obs, r, done, info = env.step(int(d["action"][t]))
        if d["done"][t] or d["game_over"][t] or d["episode_length"][t] == 0:
            break
        g = env.game
        assert np.array_equal(g.board, d["board"][t]), t
        assert np.array_equal(g.goals, d["goals"][t]), t
        assert tuple(g.agent_loc) == tuple(d["agent_loc"][t]), t
        assert g.orientation == d["orientation"][t], t
        assert g.current_points() == d["points"][t], t
        assert np.array_equal(obs, d["obs"][t]), t
    # the global stream advanced exactly as the reference's draws did
    ref = oracle.RefStreamRNG()
    ref.seed(int(seed))
    env2 = oracle.OracleEnv(lambda ep: oracle.Level(**{k: v for k, v in level.items()}),
                            time_limit=int(time_limit), view_shape=(int(vh), int(vw)),
                            output_channels=None, penalty_coef=0.0,
                            min_performance=float(min_perf), rng="stream", stream=ref)
    env2.reset()
    for s in range(t + 1):
        env2.step(int(d["action"][s]))
    from safelife_amd import speedups
    assert speedups._buffer.pos == ref.pos
    assert np.array_equal(speedups._buffer.buf, ref.buf)
