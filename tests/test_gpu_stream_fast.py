"""Reference-order replay (rng="stream") on the bit-sliced kernels.

The fast kernels replay the supplied uniform stream in the reference's order: board
then goals, env after env, row-major within a tensor, one uniform per eligible cell
(random.c:47-52 as consumed by advance_board.c:109-113).  A replay prologue kernel
runs the action and counts each tensor's eligible cells, k_scan_i64 turns the counts
into stream offsets, and the step kernel ranks its eligible cells by wave ballots.
These tests pin that path against the oracle (itself pinned by the reference-captured
goldens, tests/test_oracle.py) on boards dense with spawners at every shape class,
and against the per-cell generic kernel on long mixed runs.  The golden trajectories
themselves run through both kernels in test_gpu_parity.test_env_golden_trajectory.
"""
import os

import numpy as np
import pytest

import oracle
from test_gpu_parity import (GOLDEN, _SharedStream, _compare_state, _levels_from_pool,
                             _sprinkled_pool, torch_dev)  # noqa: F401

pytestmark = pytest.mark.gpu
C5_POOL = os.path.join(GOLDEN, "pools", "c5_navigation_128.npz")


def _pool_levels(pool):
    return [oracle.Level(pool.board[k], pool.goals[k], (pool.agent_x[k], pool.agent_y[k]),
                         pool.orientation[k], pool.spawn_prob[k], pool.min_performance[k])
            for k in range(pool.K)]


def _sprinkled(path, seed, frac):
    from safelife_amd import LevelPool
    p = LevelPool.load(path)
    if p.H == 64:
        return _sprinkled_pool(path, np.random.RandomState(seed), spawn_frac=frac)
    rng = np.random.RandomState(seed)
    board, goals = p.board.copy(), p.goals.copy()
    for k in range(p.K):
        e = (board[k] == 0) & (rng.rand(p.H, p.W) < frac)
        e[p.agent_y[k], p.agent_x[k]] = False
        board[k][e] = 152 | (rng.randint(0, 8, size=e.sum()) << 9).astype(np.uint16)
        goals[k][(goals[k] == 0) & (rng.rand(p.H, p.W) < frac / 2)] = 144
    al = np.stack([p.agent_x, p.agent_y], 1)
    return LevelPool(board, goals, al, p.orientation, p.spawn_prob, p.min_performance)


@pytest.mark.parametrize("pool_name,frac,B,T", [("c2_append_still_25", 0.02, 12, 60),
                                                ("c3_prune_still_64", 0.01, 8, 45),
                                                ("c5_navigation_128", 0.0, 4, 24)])
def test_fast_stream_vs_oracle(torch_dev, pool_name, frac, B, T):
    """B envs, one shared stream, random actions, a time limit inside the run: board,
    goals, reward, done and the stream position match the oracle every step."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    path = os.path.join(GOLDEN, "pools", pool_name + ".npz")
    pool = _sprinkled(path, 3, frac)
    levels = _pool_levels(pool)
    kw = dict(time_limit=T // 2, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01)
    stream = np.random.RandomState(17).random_sample(4_000_000 if pool.H == 128 else 600_000)
    venv = SafeLifeVecEnv(pool, B, "cuda:0", rng="stream", spawn_stream=stream, kernel="fast",
                          **kw)
    shared = _SharedStream(stream)
    oenvs = [oracle.OracleEnv(lambda ep, e=e: levels[(e + ep * B) % len(levels)], env_id=e,
                              rng="stream", stream=shared, **kw) for e in range(B)]
    vo = venv.reset().cpu().numpy()
    for e in range(B):
        assert np.array_equal(vo[e], oenvs[e].reset()), e
    rng = np.random.RandomState(4)
    for t in range(T):
        acts = rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4).astype(np.int32)
        vo, vr, vd, _ = venv.step(torch.from_numpy(acts).to(dev))
        vo, vr, vd = vo.cpu().numpy(), vr.cpu().numpy(), vd.cpu().numpy()
        vb, vg = venv.board.cpu().numpy(), venv.goals.cpu().numpy()
        for e in range(B):
            o, r, dn, _ = oenvs[e].step(int(acts[e]))
            ctx = (pool_name, t, e)
            assert vr[e] == r, (ctx, vr[e], r)
            assert bool(vd[e]) == dn, ctx
            assert np.array_equal(vb[e], oenvs[e].board), ctx
            assert np.array_equal(vg[e], oenvs[e].goals), ctx
            assert np.array_equal(vo[e], o), ctx
        assert int(venv.stream_pos.item()) == shared.pos, (ctx, venv.stream_pos.item(), shared.pos)
    assert shared.pos > 0
    assert not venv.stream_error()


@pytest.mark.parametrize("pool_name,frac,B,T", [("c2_append_still_25", 0.02, 256, 150),
                                                ("c3_prune_still_64", 0.01, 256, 150),
                                                ("c5_navigation_128", 0.0, 64, 60)])
def test_fast_stream_vs_generic_stream(torch_dev, pool_name, frac, B, T):
    """Longer mixed runs (rolls, random level order, resets): the bit-sliced replay and
    the per-cell replay consume the same uniforms and produce the same state."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    pool = _sprinkled(os.path.join(GOLDEN, "pools", pool_name + ".npz"), 8, frac)
    stream = np.random.RandomState(23).random_sample(40_000_000)
    kw = dict(time_limit=T // 3, view_shape=(33, 33), output_channels=None, penalty_coef=0.7,
              min_performance=0.01, rng="stream", spawn_stream=stream, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    assert torch.equal(fast.reset(), gen.reset())
    rng = np.random.RandomState(6)
    for t in range(T):
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        o1, r1, d1, _ = fast.step(a)
        o2, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), t
        assert torch.equal(d1, d2), t
        assert torch.equal(o1, o2), t
        assert fast.stream_pos.item() == gen.stream_pos.item(), t
        if t % 10 == 9:
            _compare_state(fast, gen, (pool_name, t))
    assert not fast.stream_error()


def test_fast_stream_exhaustion_flagged(torch_dev):
    """A stream shorter than the draws flags the error word (no out-of-range reads)."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    pool = _sprinkled(os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz"), 1, 0.02)
    venv = SafeLifeVecEnv(pool, 8, "cuda:0", rng="stream", spawn_stream=np.full(5, 0.5),
                          kernel="fast", time_limit=100, output_channels=None)
    venv.reset()
    for _ in range(3):
        venv.step(torch.zeros(8, dtype=torch.int32, device=dev))
    assert venv.stream_error()


@pytest.mark.parametrize("n", [0, 1, 2, 1023, 1024, 1025, 4097, 131072, 262147])
def test_exclusive_scan_i64(torch_dev, n):
    """sl_exclusive_scan_i64 (the replay offsets): exclusive prefix sums plus a base,
    the total written to a word that may alias the base (the stream position)."""
    torch, dev = torch_dev
    from safelife_amd import _lib
    rng = np.random.RandomState(n)
    counts = rng.randint(0, 3000, size=n).astype(np.int64)
    src = torch.from_numpy(counts).to(dev)
    out = torch.full((max(n, 1),), -7, dtype=torch.int64, device=dev)
    pos = torch.tensor([123456789], dtype=torch.int64, device=dev)
    _lib.check(_lib.lib().sl_exclusive_scan_i64(_lib.ptr(src), _lib.ptr(out), n, _lib.ptr(pos),
                                                _lib.ptr(pos), _lib.stream_ptr(dev)),
               "sl_exclusive_scan_i64")
    torch.cuda.synchronize()
    want = 123456789 + np.concatenate([[0], np.cumsum(counts)])
    assert np.array_equal(out.cpu().numpy()[:n], want[:n])
    assert int(pos.item()) == int(want[n])


@pytest.mark.parametrize("shape", [(3, 5), (7, 29), (9, 31), (20, 28), (17, 40)])
def test_small_shapes_stream_vs_generic(torch_dev, shape):
    """Replay on the small-board kernels at the shapes that exercise their corners: the
    four-env waves with DPP neighbours (spare lanes holding wrap copies, odd W's
    column-0 copy), the nl = 15 ds_bpermute form (W = 29), full 16-lane segments
    (W = 31) and the one-env kernel (W = 40); batches that leave segments empty."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv
    from test_gpu_parity import _synthetic_pool
    H, W = shape
    rng = np.random.RandomState(H * 97 + W)
    pool = _synthetic_pool(rng, 6, H, W)
    B, T = 37, 60
    stream = np.random.RandomState(H + W).random_sample(3_000_000)
    kw = dict(time_limit=21, view_shape=(9, 9), output_channels=None, penalty_coef=0.7,
              min_performance=0.01, rng="stream", spawn_stream=stream, level_order="random",
              augment_roll=True)
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    assert torch.equal(fast.reset(), gen.reset())
    for t in range(T):
        a = torch.from_numpy(rng.choice(9, size=B, p=[.05] + [.1] * 4 + [.1375] * 4)
                             .astype(np.int32)).to(dev)
        o1, r1, d1, _ = fast.step(a)
        o2, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), t
        assert torch.equal(d1, d2), t
        assert torch.equal(o1, o2), t
        assert fast.stream_pos.item() == gen.stream_pos.item(), t
        _compare_state(fast, gen, (shape, t))
    assert fast.stream_pos.item() > 0
    assert not fast.stream_error()


@pytest.mark.parametrize("case", ["toggle_powers", "p1", "p0", "wrap_rows"])
def test_decided_replay128_edges_vs_generic(torch_dev, case):
    """The 128x128 replay path's own state (sl_env_state.elig_planes: the eligibility
    the step leaves, patched around the action's rows; the draw pass's decisions)
    against the per-cell replay, which keeps none of it, on the cases that path
    special-cases: actions that create and destroy spawners (can_toggle_powers: the
    spawn flags are forced and the patch window must see new spawners), spawn
    probability 1 and 0 (draws consumed, never compared), and agents on the rows
    around the 127/0 wrap (the patch window straddles it)."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    pool = _sprinkled(C5_POOL, 5, 0.0)
    al = np.stack([pool.agent_x, pool.agent_y], 1)
    sp = pool.spawn_prob.copy()
    if case == "p1":
        sp[:] = 1.0
    elif case == "p0":
        sp[:] = 0.0
    if case == "wrap_rows":        # levels rolled so the agents start on rows 126, 127, 0, 1
        board, goals = pool.board.copy(), pool.goals.copy()
        for k in range(pool.K):
            sh = (126 + k - int(pool.agent_y[k])) % 128
            board[k] = np.roll(pool.board[k], sh, 0)
            goals[k] = np.roll(pool.goals[k], sh, 0)
            al[k, 1] = (int(pool.agent_y[k]) + sh) % 128
        pool = LevelPool(board, goals, al, pool.orientation, sp, pool.min_performance)
    else:
        pool = LevelPool(pool.board, pool.goals, al, pool.orientation, sp, pool.min_performance)
    B, T = 48, 40
    stream = np.random.RandomState(29).random_sample(60_000_000)
    kw = dict(time_limit=25, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
              min_performance=0.01, rng="stream", spawn_stream=stream, level_order="random",
              augment_roll=(case != "wrap_rows"),
              can_toggle_powers=(case == "toggle_powers"),
              can_toggle_colors=(case == "toggle_powers"))
    fast = SafeLifeVecEnv(pool, B, "cuda:0", kernel="fast", **kw)
    gen = SafeLifeVecEnv(pool, B, "cuda:0", kernel="generic", **kw)
    assert fast.elig_planes is not None
    assert torch.equal(fast.reset(), gen.reset())
    rng = np.random.RandomState(8)
    moves = 0
    for t in range(T):
        a = torch.from_numpy(rng.choice(9, size=B, p=[.04] + [.12] * 4 + [.12] * 4)
                             .astype(np.int32)).to(dev)
        o1, r1, d1, _ = fast.step(a)
        o2, r2, d2, _ = gen.step(a)
        assert torch.equal(r1, r2), (case, t)
        assert torch.equal(d1, d2), (case, t)
        assert torch.equal(o1, o2), (case, t)
        assert fast.stream_pos.item() == gen.stream_pos.item(), (case, t)
        _compare_state(fast, gen, (case, t))
        moves += int((a > 0).sum().item())
    assert moves > 0 and fast.stream_pos.item() > 0
    assert not fast.stream_error()
