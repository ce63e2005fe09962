"""GPU parity of the device PPO caller (safelife_amd.rollout, sl_sample_actions,
sl_gae) and of the float observation modes, against the oracle.

Bit-exact throughout: action indices and boards are integers; returns and
advantages are float64 evaluated in the reference's order (north_star allows 1e-6).
"""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    import safelife_amd  # noqa: F401
    return torch, torch.device("cuda:0")


def _probs(rng, B, A, dtype):
    p = rng.rand(B, A) ** 3
    p[rng.rand(B, A) < 0.3] = 0.0
    p[p.sum(1) == 0, 0] = 1.0
    return (p / p.sum(1, keepdims=True)).astype(dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_sample_actions_stream_vs_oracle(torch_dev, dtype):
    torch, dev = torch_dev
    from safelife_amd.rollout import sample_actions
    rng = np.random.RandomState(11)
    for A in (1, 2, 9, 17):
        B = 5000
        p = _probs(rng, B, A, dtype)
        u = rng.random_sample(B)
        u[:4] = [0.0, np.nextafter(1.0, 0), 0.5, 0.25]
        got = sample_actions(torch.from_numpy(p).to(dev), uniforms=u).cpu().numpy()
        want = [oracle.sample_action(p[b], u[b])[0] for b in range(B)]
        assert np.array_equal(got, want), A


def test_sample_actions_philox_vs_oracle(torch_dev):
    torch, dev = torch_dev
    from safelife_amd.rollout import sample_actions
    rng = np.random.RandomState(12)
    B, A, seed, step, env0 = 3000, 9, 77, 123, 4096
    p = _probs(rng, B, A, np.float32)
    got = sample_actions(torch.from_numpy(p).to(dev), seed=seed, step=step,
                         env0=env0).cpu().numpy()
    want = [oracle.sample_action(p[b], oracle.philox_uniform(0, env0 + b, step, 2, seed))[0]
            for b in range(B)]
    assert np.array_equal(got, want)
    # non-contiguous rows (a [B, 2A] buffer's left half) read through the row stride
    wide = torch.zeros((B, 2 * A), dtype=torch.float32, device=dev)
    wide[:, :A] = torch.from_numpy(p).to(dev)
    got2 = sample_actions(wide[:, :A], seed=seed, step=step, env0=env0).cpu().numpy()
    assert np.array_equal(got2, want)


def test_sample_actions_errors(torch_dev):
    torch, dev = torch_dev
    from safelife_amd.rollout import sample_actions
    ok = np.full((8, 4), 0.25)
    for val, msg in ((-0.1, "non-negative"), (0.55, "sum to 1")):
        p = ok.copy()
        p[5, 1] = val
        with pytest.raises(ValueError, match=msg):
            sample_actions(torch.from_numpy(p).to(dev))
        with pytest.raises(ValueError, match=msg):
            np.random.choice(4, p=p[5])


@pytest.mark.parametrize("G,clip", [(1, 0.0), (3, 0.0), (2, 0.5)])
def test_gae_vs_oracle(torch_dev, G, clip):
    torch, dev = torch_dev
    from safelife_amd.rollout import returns_advantages
    rng = np.random.RandomState(G)
    T, N = 37, 1000
    gamma = np.array([0.99, 0.9, 0.5][:G], np.float32)
    rewards = rng.randn(T, N) * 0.7
    done = rng.rand(T, N) < 0.08
    values = rng.randn(T + 1, N, G).astype(np.float32)
    ret, adv = returns_advantages(torch.from_numpy(rewards).to(dev),
                                  torch.from_numpy(done).to(dev),
                                  torch.from_numpy(values).to(dev), gamma, 0.95, clip)
    wr, wa = oracle.gae(rewards, done, values, gamma, 0.95, clip)
    assert np.array_equal(ret.cpu().numpy(), wr)
    assert np.array_equal(adv.cpu().numpy(), wa)


def _levels(path):
    d = np.load(path)
    return [oracle.Level(d["board"][k], d["goals"][k], d["agent_loc"][k], d["orientation"][k],
                         d["spawn_prob"][k], d["min_performance"][k])
            for k in range(d["board"].shape[0])]


@pytest.mark.parametrize("pool_name", ["c2_append_still_25", "c3_prune_still_64"])
def test_run_agents_vs_oracle(torch_dev, pool_name):
    """Two consecutive device rollouts with an observation-dependent policy, against
    the oracle env chain driven by the oracle sampler with the same Philox draws."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    from safelife_amd.rollout import run_agents, training_batch
    path = os.path.join(GOLDEN, "pools", pool_name + ".npz")
    levels = _levels(path)
    B, T, seed = 12, 25, 31
    kw = dict(time_limit=30, view_shape=(15, 15), output_channels=None, penalty_coef=0.5,
              min_performance=0.01)
    venv = SafeLifeVecEnv(LevelPool.load(path), B, "cuda:0", rng="philox", seed=seed, **kw)
    oenvs = [oracle.OracleEnv(lambda ep, e=e: levels[(e + ep * B) % len(levels)], env_id=e,
                              rng="philox", seed=seed, **kw) for e in range(B)]
    # the policy reads the packed cell ahead of the view centre: exact integer
    # features on both sides, then a fixed probability table
    table = np.random.RandomState(5).rand(16, 9).astype(np.float32)
    table /= table.sum(1, keepdims=True)
    table_t = torch.from_numpy(table).to(dev)
    cy, cx = 7, 7

    def policy(obs, rnn):
        key = (obs[:, cy - 1, cx].to(torch.int32) + obs[:, cy, cx + 1].to(torch.int32)) & 15
        return table_t[key.long()], rnn

    o_obs = np.stack([e.reset() for e in oenvs])
    step = 0
    for chunk in range(2):
        ro = run_agents(venv, policy, T)
        states = ro.states.cpu().numpy()
        assert np.array_equal(states[0], o_obs), chunk
        acts = ro.actions.cpu().numpy()
        rew, dn = ro.rewards.cpu().numpy(), ro.end_episode.cpu().numpy()
        for t in range(T):
            for e in range(B):
                o = o_obs[e]
                key = (int(o[cy - 1, cx]) + int(o[cy, cx + 1])) & 15
                u = oracle.philox_uniform(0, e, step, 2, seed)
                a, err = oracle.sample_action(table[key], u)
                assert err == 0 and acts[t, e] == a, (chunk, t, e)
                ob, r, d, _ = oenvs[e].step(a)
                assert rew[t, e] == r and bool(dn[t, e]) == d, (chunk, t, e)
                assert np.array_equal(states[t + 1, e], ob), (chunk, t, e)
                o_obs[e] = ob
            step += 1
        for e in range(B):
            assert np.array_equal(venv.board[e].cpu().numpy(), oenvs[e].board), (chunk, e)
        assert int(ro.info["reset"].sum()) > 0 or chunk == 0
        values = torch.from_numpy(np.random.RandomState(chunk).randn(T + 1, B, 1)
                                  .astype(np.float32)).to(dev)
        policies = table_t[torch.zeros((T + 1, B), dtype=torch.long, device=dev)]
        tb = training_batch(ro, policies, values)
        wr, wa = oracle.gae(rew, dn, values.cpu().numpy(), (0.99,), 0.95)
        assert np.array_equal(tb["G"].cpu().numpy(), wr)
        assert np.array_equal(tb["A"].cpu().numpy(), wa)
        assert np.array_equal(tb["pi"].cpu().numpy(), table[0][acts])


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_obs_float_channels(torch_dev, dtype):
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    kw = dict(view_shape=(33, 33), rng="philox", seed=3)
    a = SafeLifeVecEnv(LevelPool.load(path), 16, "cuda:0", output_channels=tuple(range(15)), **kw)
    f = SafeLifeVecEnv(LevelPool.load(path), 16, "cuda:0", output_channels=tuple(range(15)),
                       obs_dtype=dtype, **kw)
    oa, of = a.reset(), f.reset()
    assert of.dtype == getattr(torch, dtype)
    acts = torch.from_numpy(np.random.RandomState(0).randint(0, 9, (20, 16))).to(dev)
    for t in range(20):
        oa, *_ = a.step(acts[t])
        of, *_ = f.step(acts[t])
        assert torch.equal(of.float(), oa.float()), t


@pytest.mark.parametrize("dtype,ch", [("uint8", tuple(range(15))), ("uint16", (3, 0, 9, 14)),
                                      ("float32", (8, 1, 2))])
def test_obs_flat_tail_and_unaligned(torch_dev, dtype, ch):
    """Channel obs through the 16-byte-chunk kernel with a ragged tail (odd B, odd
    cell count), against the packed obs; the same into a 1-element-offset buffer
    (unaligned: the LDS-staged fallback kernel)."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    pool = LevelPool.load(os.path.join(GOLDEN, "pools", "c2_append_still_25.npz"))
    kw = dict(view_shape=(33, 31), rng="philox", seed=9, time_limit=15)
    B = 7
    ep = SafeLifeVecEnv(pool, B, "cuda:0", output_channels=None, **kw)
    ec = SafeLifeVecEnv(pool, B, "cuda:0", output_channels=ch, obs_dtype=dtype, **kw)
    ep.reset()
    ec.reset()
    n = ec.obs.numel()
    raw = torch.zeros(n + 1, dtype=ec.obs.dtype, device=dev)
    un = raw[1:].view(ec.obs.shape)
    rng = np.random.RandomState(4)
    for t in range(25):
        a = torch.from_numpy(rng.randint(0, 9, B).astype(np.int32)).to(dev)
        p = ep.step(a)[0].cpu().numpy().astype(np.int64)
        c = ec.step(a)[0].float().cpu().numpy().astype(np.int64)
        ec.observe(out=un)
        assert np.array_equal(un.float().cpu().numpy().astype(np.int64), c), t
        for k, bit in enumerate(ch):
            assert np.array_equal(c[..., k], (p >> bit) & 1), (t, k)


@pytest.mark.parametrize("name", ["ppo_loop_spawn", "ppo_loop_nav128"])
def test_run_agents_reference_order_g7(torch_dev, name):
    """G7 (the reference's PPO loop, training/ppo.py:436-452, captured from the
    reference: 16 envs, np.random.choice per env from the global stream that also
    refills the spawn buffer) through run_agents(rng="reference") after
    speedups.seed(s): actions, rewards, done flags, boards and goals bit-exact, and the
    global numpy stream ends where the reference's did."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool, speedups
    from safelife_amd.rollout import run_agents
    d = np.load(os.path.join(GOLDEN, "g7_%s.npz" % name))
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    table = torch.from_numpy(d["table"]).to(dev)
    T, N, A = table.shape
    pool = LevelPool.from_levels([{
        "board": d["level_board"], "goals": d["level_goals"], "agent_loc": d["level_agent_loc"],
        "orientation": d["level_orientation"], "spawn_prob": d["level_spawn_prob"],
        "min_performance": d["level_min_performance"]}])
    venv = SafeLifeVecEnv(pool, N, dev, time_limit=int(time_limit), view_shape=(int(vh), int(vw)),
                          output_channels=None, penalty_coef=float(penalty),
                          min_performance=float(min_perf), rng="stream",
                          spawn_stream=np.zeros(1))
    step = [0]

    def policy(obs, rnn):
        p = table[step[0]]
        step[0] += 1
        return p, rnn

    speedups.seed(int(seed))
    boards, goals = [], []
    keep = set(int(s) for s in d["board_steps"])
    ro = None
    for t in range(T):                 # one slot per call, boards read at the kept steps
        ro = run_agents(venv, policy, 1, rng="reference")
        assert np.array_equal(ro.actions[0].cpu().numpy(), d["action"][t]), t
        assert np.array_equal(ro.rewards[0].cpu().numpy(), d["reward"][t]), t
        assert np.array_equal(ro.end_episode[0].cpu().numpy(), d["done"][t]), t
        if t in keep:
            boards.append(venv.board.cpu().numpy())
            goals.append(venv.goals.cpu().numpy())
    assert np.array_equal(np.array(boards), d["board"])
    assert np.array_equal(np.array(goals), d["goals"])
    assert np.array_equal(np.random.random(4), d["after"])
    # the whole loop in one call: the same rollout
    venv2 = SafeLifeVecEnv(pool, N, dev, time_limit=int(time_limit),
                           view_shape=(int(vh), int(vw)), output_channels=None,
                           penalty_coef=float(penalty), min_performance=float(min_perf),
                           rng="stream", spawn_stream=np.zeros(1))
    step[0] = 0
    speedups.seed(int(seed))
    ro2 = run_agents(venv2, policy, T, rng="reference")
    assert np.array_equal(ro2.actions.cpu().numpy(), d["action"])
    assert np.array_equal(ro2.rewards.cpu().numpy(), d["reward"])
    assert np.array_equal(venv2.board.cpu().numpy(), d["board"][-1])


def test_step_env_reference_without_obs_keeps_board_g7_nav128(torch_dev):
    """step_env_reference on a 128x128 batch with compute_obs=False runs the replay
    kernels in plane mode (the board lives in sl_env_state.board_planes); venv.board
    read afterwards -- with no step with views in between -- must be the reference's
    board (G7, captured from the reference's own loop, training/ppo.py:436-452).
    VERDICT r05 weak 1 / ADVICE r05: this read used to skip the sync."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool, speedups
    d = np.load(os.path.join(GOLDEN, "g7_ppo_loop_nav128.npz"))
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    table = d["table"]
    T, N, A = table.shape
    pool = LevelPool.from_levels([{
        "board": d["level_board"], "goals": d["level_goals"], "agent_loc": d["level_agent_loc"],
        "orientation": d["level_orientation"], "spawn_prob": d["level_spawn_prob"],
        "min_performance": d["level_min_performance"]}])
    venv = SafeLifeVecEnv(pool, N, dev, time_limit=int(time_limit), view_shape=(int(vh), int(vw)),
                          output_channels=None, penalty_coef=float(penalty),
                          min_performance=float(min_perf), rng="stream",
                          spawn_stream=np.zeros(1), compute_obs=False)
    assert venv.board_planes is not None
    speedups.seed(int(seed))
    venv.reset()
    keep = {int(s): k for k, s in enumerate(d["board_steps"])}
    in_planes = 0
    for t in range(T):
        for e in range(N):
            a = int(np.random.choice(A, p=table[t, e]))
            assert a == d["action"][t, e], (t, e)
            venv.step_env_reference(e, a)
        venv.end_reference_step()
        assert np.array_equal(venv.reward.cpu().numpy(), d["reward"][t]), t
        assert np.array_equal(venv.done.cpu().numpy(), d["done"][t]), t
        if t in keep:
            in_planes += int(((venv.planes_ok & 64) != 0).sum().item())
            assert np.array_equal(venv.board.cpu().numpy(), d["board"][keep[t]]), t
            assert np.array_equal(venv.goals.cpu().numpy(), d["goals"][keep[t]]), t
    assert in_planes > 0          # the reads did follow plane-mode steps
    assert np.array_equal(np.random.random(4), d["after"])
