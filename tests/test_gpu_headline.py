"""The headline kernel (k_env_step_bits64, C3) and the C4 / multi-GPU configs pinned
directly: against reference-captured arrays, against the oracle in the benchmark's
own regime, across shard layouts, and through checkpoint / restore.

All tests need the MI355X and run the product through the C ABI.  Boards, goals,
observations and flags are compared bit for bit; rewards with ``==`` (the north star
allows 1e-6, REWARD_TOL).
"""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
POOLS = os.path.join(GOLDEN, "pools")
C3 = os.path.join(POOLS, "c3_prune_still_64.npz")
C4 = os.path.join(POOLS, "c4_append_still_64.npz")
pytestmark = pytest.mark.gpu
REWARD_TOL = 1e-6


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    import safelife_amd  # noqa: F401
    return torch, torch.device("cuda:0")


def _levels(*paths):
    out = []
    for path in paths:
        d = np.load(path)
        out += [oracle.Level(d["board"][k], d["goals"][k], d["agent_loc"][k], d["orientation"][k],
                             d["spawn_prob"][k], d["min_performance"][k])
                for k in range(d["board"].shape[0])]
    return out


def _env_state(venv, e):
    """Env e's per-env state as host values (the fields OracleEnv.load_state reads)."""
    s = {"board": venv.board[e].cpu().numpy(), "goals": venv.goals[e].cpu().numpy(),
         "start_board": venv.start_board[e].cpu().numpy()}
    for k, t in venv.st_t.items():
        s[k] = t[e].cpu().numpy()
    return s


# ------------------------------------------------- (a) reference-captured golden
def test_bits64_reference_golden_prune_still_64(torch_dev):
    """traj_prune_still_64.npz was captured from the reference itself (SafeLifeEnv +
    the PPO wrapper chain, 1 100 steps, crossing time_limit).  Its level holds no
    spawning cell in board or goals, so no draw is ever made and the Philox-mode
    bit-sliced kernel must reproduce the reference's boards, goals, rewards, flags
    and packed 33x33 views (fused into the kernel) at every step."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    d = np.load(os.path.join(GOLDEN, "traj_prune_still_64.npz"))
    assert not ((d["level_board"] & 0x80).any() or (d["level_goals"] & 0x80).any())
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    pool = LevelPool.from_levels([{
        "board": d["level_board"], "goals": d["level_goals"], "agent_loc": d["level_agent_loc"],
        "orientation": d["level_orientation"], "spawn_prob": d["level_spawn_prob"],
        "min_performance": d["level_min_performance"]}])
    assert (pool.H, pool.W) == (64, 64)
    env = SafeLifeVecEnv(pool, 1, "cuda:0", time_limit=int(time_limit),
                         view_shape=(int(vh), int(vw)), output_channels=None,
                         penalty_coef=float(penalty), min_performance=float(min_perf),
                         rng="philox", seed=12345, kernel="fast")
    obs = env.reset().cpu().numpy()
    assert np.array_equal(obs[0], d["obs0"])
    actions = torch.from_numpy(d["action"].astype(np.int32)).to(dev)
    T = len(d["action"])
    assert T > int(time_limit)
    n_reset = 0
    for t in range(T):
        obs, r, done, info = env.step(actions[t:t + 1])
        ctx = t
        assert abs(r.item() - d["reward"][t]) <= REWARD_TOL
        assert r.item() == d["reward"][t], (ctx, r.item(), d["reward"][t])
        assert bool(done.item()) == bool(d["done"][t]), ctx
        assert bool(info["times_up"].item()) == bool(d["times_up"][t]), ctx
        n_reset += int(info["reset"].item())
        assert np.array_equal(env.board[0].cpu().numpy(), d["board"][t]), ctx
        assert np.array_equal(env.goals[0].cpu().numpy(), d["goals"][t]), ctx
        assert np.array_equal(obs[0].cpu().numpy(), d["obs"][t]), ctx
    assert n_reset >= 1


# ------------------------------------------------------------ (b) C4 mixed pool
def test_c4_mixed_pool_vs_oracle(torch_dev):
    """BASELINE config C4's levels (64x64 append-still + prune-still, both pools in one
    device pool) on the bit-sliced kernel with the PPO chain, 300 steps across a
    time_limit boundary and game-over resets, every env bit-exact with the oracle."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    levels = _levels(C4, C3)
    pool = LevelPool.load(C4, C3)
    assert pool.K == len(levels) == 64
    B, T = 64, 300
    kw = dict(time_limit=120, view_shape=(33, 33), output_channels=None, penalty_coef=1.0,
              min_performance=0.01)
    venv = SafeLifeVecEnv(pool, B, "cuda:0", rng="philox", seed=404, kernel="fast", **kw)
    oenvs = [oracle.OracleEnv(oracle.pool_level_fn(levels, e, n_total=B), env_id=e,
                              rng="philox", seed=404, **kw) for e in range(B)]
    vo = venv.reset().cpu().numpy()
    for e in range(B):
        assert np.array_equal(vo[e], oenvs[e].reset()), e
    rng = np.random.RandomState(31)
    n_reset = 0
    for t in range(T):
        acts = rng.choice(9, size=B, p=[.04] + [.12] * 4 + [.12] * 4).astype(np.int32)
        vo, vr, vd, info = venv.step(torch.from_numpy(acts).to(dev))
        n_reset += int(info["reset"].sum().item())
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
    assert n_reset >= B       # every env crossed time_limit at least once
    # the episode counters the PPO logger reads (global_counter) agree with the oracle
    gc = venv.sync_counters()
    assert gc.episodes_started == sum(o.episodes for o in oenvs)
    assert gc.episodes_completed == sum(o.completed for o in oenvs)


# ------------------------------------------------------ (c) the benchmark regime
@pytest.mark.parametrize("pool_paths,obs", [((C3,), "none"), ((C3,), "packed"),
                                            ((C3,), "channels"), ((C3,), "bfloat16"),
                                            ((C4, C3), "none")])
def test_bench_regime_sampled_vs_oracle(torch_dev, pool_paths, obs):
    """bench.py's regime at full size: 65 536 envs (32 768 for the C4 mix), random
    level order with toroidal rolls, episode clocks staggered over [0, 1000) and a
    400-step burn-in of random actions (boards full of toggled life, resets spread
    over every step), time_limit 1000.  Sampled envs' state is then handed to the
    oracle, and both run 60 more steps (crossing resets) bit-exact.  obs "channels":
    the reference's default 15-channel u16 views (safelife_env.py:79, what its PPO
    consumes), fused into the step kernel; "bfloat16": the same bits as 0.0 / 1.0."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    levels = _levels(*pool_paths)
    B = 65536 if len(pool_paths) == 1 else 32768
    seed = 1234
    chans = obs in ("channels", "bfloat16")
    kw = dict(time_limit=1000, view_shape=(33, 33),
              output_channels=tuple(range(15)) if chans else None, penalty_coef=1.0,
              min_performance=0.01)
    venv = SafeLifeVecEnv(LevelPool.load(*pool_paths), B, dev, rng="philox", seed=seed,
                          level_order="random", augment_roll=True, kernel="fast",
                          compute_obs=obs != "none",
                          obs_dtype="bfloat16" if obs == "bfloat16" else "uint16", **kw)
    venv.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    venv.st_t["episode_length"].copy_(torch.randint(0, 1000, (B,), device=dev, generator=g,
                                                    dtype=torch.int32))
    for _ in range(400):
        venv.step_async(torch.randint(0, 9, (B,), dtype=torch.int32, device=dev, generator=g))
    torch.cuda.synchronize()
    lens = venv.st_t["episode_length"].cpu().numpy()
    # envs about to time out (resets inside the compared window) and arbitrary others
    order = np.argsort(-lens, kind="stable")
    sample = sorted(set(order[:6].tolist() + [0, 1, 4097, B // 2 + 3, B - 2, B - 1]))
    oenvs = {}
    for e in sample:
        o = oracle.OracleEnv(oracle.pool_level_fn(levels, e, seed=seed, random_order=True,
                                                  augment=True),
                             env_id=e, rng="philox", seed=seed, **kw)
        o.load_state(_env_state(venv, e), venv._step_index)
        oenvs[e] = o
    rng = np.random.RandomState(6)
    n_reset = 0
    for t in range(60):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        vo, vr, vd, info = venv.step(torch.from_numpy(acts).to(dev))
        rs = info["reset"].cpu().numpy()
        vr, vd = vr.cpu().numpy(), vd.cpu().numpy()
        for e in sample:
            o, r, dn, _ = oenvs[e].step(int(acts[e]))
            ctx = (t, e)
            n_reset += int(rs[e])
            assert vr[e] == r, (ctx, vr[e], r)
            assert bool(vd[e]) == dn, ctx
            assert np.array_equal(venv.board[e].cpu().numpy(), oenvs[e].board), ctx
            assert np.array_equal(venv.goals[e].cpu().numpy(), oenvs[e].goals), ctx
            if obs == "bfloat16":
                assert np.array_equal(vo[e].float().cpu().numpy(), o.astype(np.float32)), ctx
            elif obs != "none":
                assert np.array_equal(vo[e].cpu().numpy(), o), ctx
    assert n_reset >= 6


@pytest.mark.parametrize("obs", ["none", "channels"])
def test_mass_reset_on_one_step(torch_dev, obs):
    """Every env finishes on the same step: 8 192 resets in one reset-list launch (512
    workgroups, each looping over list entries).  Sampled envs bit-exact with the
    oracle over the reset and the steps after it; every env's episode counter
    advanced."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    levels = _levels(C3)
    B, seed, T = 8192, 77, 6
    kw = dict(time_limit=T, view_shape=(33, 33),
              output_channels=tuple(range(15)) if obs == "channels" else None,
              penalty_coef=1.0, min_performance=0.01)
    venv = SafeLifeVecEnv(LevelPool.load(C3), B, dev, rng="philox", seed=seed,
                          level_order="random", augment_roll=True, kernel="fast",
                          compute_obs=obs != "none", **kw)
    venv.reset()
    sample = [0, 1, 63, 64, 4095, B - 1]
    oenvs = {}
    for e in sample:
        o = oracle.OracleEnv(oracle.pool_level_fn(levels, e, seed=seed, random_order=True,
                                                  augment=True),
                             env_id=e, rng="philox", seed=seed, **kw)
        o.load_state(_env_state(venv, e), venv._step_index)
        oenvs[e] = o
    rng = np.random.RandomState(3)
    ep0 = venv.st_t["episodes"].clone()
    most = 0
    for t in range(T + 3):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        vo, vr, vd, info = venv.step(torch.from_numpy(acts).to(dev))
        vr, vd = vr.cpu().numpy(), vd.cpu().numpy()
        for e in sample:
            o, r, dn, _ = oenvs[e].step(int(acts[e]))
            ctx = (t, e)
            assert vr[e] == r, (ctx, vr[e], r)
            assert bool(vd[e]) == dn, ctx
            assert np.array_equal(venv.board[e].cpu().numpy(), oenvs[e].board), ctx
            assert np.array_equal(venv.goals[e].cpu().numpy(), oenvs[e].goals), ctx
            if obs != "none":
                assert np.array_equal(vo[e].cpu().numpy(), o), ctx
        most = max(most, int(vd.sum()))
    assert most >= B * 9 // 10, most        # (nearly) every env timed out on one step
    n_ep = (venv.st_t["episodes"] - ep0).cpu().numpy()
    assert n_ep.min() >= 1 and n_ep.max() <= 2


C5 = os.path.join(POOLS, "c5_navigation_128.npz")


@pytest.mark.parametrize("pools,B,T,tl", [((C3,), 65536, 60, 25), ((C4, C3), 32768, 60, 25),
                                          ((C5,), 4096, 30, 12), ((C5,), 65536, 16, 6)])
def test_full_batch_every_env_vs_c_oracle(torch_dev, pools, B, T, tl):
    """Every env of a full C3 batch (65 536; the C4 mix at 32 768; C5's 128x128 levels
    with spawners and per-step side effects at 4 096 over 30 steps, and at the full
    65 536 over 16 steps of 6-step episodes, the C restatement being slower there),
    every step: rewards and dones of the GPU batch against the C restatement of the
    chain (oracle/sl_cpu_step.c, itself bit-exact with the oracle env,
    tests/test_cpu_step.py) stepping the same batch on the host's cores, from reset
    over two rounds of resets; then the boards and goals of every 16th env."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    levels = _levels(*pools)
    seed = 4321
    kw = dict(time_limit=tl, view_shape=(33, 33), penalty_coef=1.0, min_performance=0.01)
    venv = SafeLifeVecEnv(LevelPool.load(*pools), B, dev, rng="philox", seed=seed,
                          level_order="random", augment_roll=True, kernel="fast",
                          compute_obs=False, output_channels=None, **kw)
    venv.reset()
    cb = oracle.CpuBatch(levels, B, seed=seed, level_order="random", augment_roll=True, **kw)
    cb.reset()
    threads = min(16, os.cpu_count() or 1)
    rng = np.random.RandomState(12)
    n_done = 0
    for t in range(T):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        _, vr, vd, _ = venv.step(torch.from_numpy(acts).to(dev))
        _, cr, cd = cb.step(acts, threads)
        vr, vd = vr.cpu().numpy(), vd.cpu().numpy().astype(np.uint8)
        bad = np.nonzero((vr != cr) | (vd != cd))[0]
        assert bad.size == 0, (t, bad[:8], vr[bad[:4]], cr[bad[:4]])
        n_done += int(cd.sum())
    assert n_done >= B                      # every env crossed an episode end
    vb, vg = venv.board.cpu().numpy(), venv.goals.cpu().numpy()
    for e in range(0, B, 16):
        assert np.array_equal(vb[e], cb.board(e, 0)), e
        assert np.array_equal(vg[e], cb.board(e, 1)), e


# ------------------------------------------------------------- (e) shard layouts
@pytest.mark.parametrize("level_order,augment", [("random", True), ("sequential", False)])
def test_two_shards_reproduce_one_run(torch_dev, level_order, augment):
    """rank r owns global env ids [r*B/2, (r+1)*B/2).  Two shard envs
    (env0 = 0 and env0 = B/2, n_total_envs = B) reproduce one B-env run bit for bit:
    Philox draws, level choice and rolls key on the global env id, so trajectories
    do not depend on how the batch is spread over GPUs."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    from safelife_amd import dist as sdist
    pool = LevelPool.load(C4, C3)
    B, T = 512, 120
    kw = dict(time_limit=50, view_shape=(33, 33), output_channels=None, penalty_coef=1.0,
              min_performance=0.01, rng="philox", seed=8, level_order=level_order,
              augment_roll=augment, kernel="fast")
    whole = SafeLifeVecEnv(pool, B, dev, **kw)
    shards = []
    for r in range(2):
        sh = sdist.env_shard(r, 2, B // 2)
        shards.append(SafeLifeVecEnv(pool, sh.n_envs, dev, env0=sh.env0,
                                     n_total_envs=sh.n_total, **kw))
    o = whole.reset()
    assert torch.equal(o, torch.cat([s.reset() for s in shards]))
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    for t in range(T):
        a = torch.randint(0, 9, (B,), dtype=torch.int32, device=dev, generator=g)
        o, r, d, info = whole.step(a)
        outs = [s.step(a[i * (B // 2):(i + 1) * (B // 2)]) for i, s in enumerate(shards)]
        assert torch.equal(o, torch.cat([x[0] for x in outs])), t
        assert torch.equal(r, torch.cat([x[1] for x in outs])), t
        assert torch.equal(d, torch.cat([x[2] for x in outs])), t
        assert torch.equal(info["reset"], torch.cat([x[3]["reset"] for x in outs])), t
        if t % 20 == 0 or t == T - 1:
            assert torch.equal(whole.board, torch.cat([s.board for s in shards])), t
            assert torch.equal(whole.goals, torch.cat([s.goals for s in shards])), t


# ------------------------------------------------------- checkpoint and restore
@pytest.mark.parametrize("pool_path", [C3, os.path.join(POOLS, "c5_navigation_128.npz"),
                                       os.path.join(POOLS, "c2_append_still_25.npz")])
def test_state_dict_replay(torch_dev, pool_path):
    """state_dict() mid-run, N more steps, load_state_dict(), the same N steps again:
    bit-identical results, including auto-resets (the per-parity reset lists are
    cleared on restore) and with auto_reset switched off and on in between."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    pool = LevelPool.load(pool_path)
    B = 96
    env = SafeLifeVecEnv(pool, B, dev, time_limit=13, view_shape=(15, 15),
                         output_channels=None, penalty_coef=1.0, min_performance=0.01,
                         rng="philox", seed=3, level_order="random", augment_roll=True,
                         kernel="fast")
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    acts = torch.randint(0, 9, (80, B), dtype=torch.int32, device=dev, generator=g)
    for t in range(21):          # odd: the saved step index has the other parity
        env.step(acts[t])
    sd = env.state_dict()

    def run():
        outs = []
        for t in range(21, 60):
            if t == 30:
                env.auto_reset = False
            if t == 33:
                env.auto_reset = True
            o, r, d, info = env.step(acts[t])
            outs.append((o.clone(), r.clone(), d.clone(), env.flags.clone(), env.board.clone()))
        return outs

    first = run()
    env.load_state_dict(sd)
    second = run()
    for t, (x, y) in enumerate(zip(first, second)):
        for a, b in zip(x, y):
            assert torch.equal(a, b), t
    assert any(bool((f[3] & 4).any()) for f in first)       # resets happened


def test_sl_env_step_rejects_mismatched_pool(torch_dev):
    """sl_env_step with auto_reset validates the pool like sl_env_reset does."""
    import ctypes
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool, _lib
    L = _lib.lib()
    env = SafeLifeVecEnv(LevelPool.load(C3), 4, dev, output_channels=None)
    env.reset()
    other = LevelPool.load(os.path.join(POOLS, "c2_append_still_25.npz")).to_device(dev)
    a = torch.zeros(4, dtype=torch.int32, device=dev)
    cfg = env._fill_cfg()
    env._fill_obs_cfg(cfg, None)
    rc = L.sl_env_step(ctypes.byref(env._state), ctypes.byref(other["struct"]), a.data_ptr(),
                       ctypes.byref(cfg), env.reward.data_ptr(), env.done.data_ptr(),
                       env.flags.data_ptr(), env.ep_len.data_ptr(), env.ep_rew.data_ptr(),
                       _lib.stream_ptr(dev))
    assert rc == _lib.SL_EINVAL
    empty = _lib.LevelPool()
    empty.K, empty.H, empty.W = 0, 64, 64
    rc = L.sl_env_step(ctypes.byref(env._state), ctypes.byref(empty), a.data_ptr(),
                       ctypes.byref(cfg), env.reward.data_ptr(), env.done.data_ptr(),
                       env.flags.data_ptr(), env.ep_len.data_ptr(), env.ep_rew.data_ptr(),
                       _lib.stream_ptr(dev))
    assert rc == _lib.SL_EINVAL
