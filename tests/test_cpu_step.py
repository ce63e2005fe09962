"""The compiled env chain (oracle/sl_cpu_step.c, bench.py's CPU baseline) against
oracle.OracleEnv, bit for bit, and its OpenMP batch against a one-thread run.

CPU only: test infrastructure checking test infrastructure, so that the CPU
baseline bench.py reports runs the same per-env computation as the GPU path."""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _levels(name):
    d = np.load(os.path.join(GOLDEN, "pools", name + ".npz"))
    return [oracle.Level(d["board"][k], d["goals"][k], d["agent_loc"][k], d["orientation"][k],
                         d["spawn_prob"][k], d["min_performance"][k])
            for k in range(d["board"].shape[0])]


def _sprinkle(levels, rng, frac=0.01):
    """extra (coloured) spawners so the Philox spawn path is exercised"""
    out = []
    for lv in levels:
        b = lv.board.copy()
        m = (b == 0) & (rng.rand(*b.shape) < frac)
        b[m] = 152 | (rng.randint(0, 8, size=m.sum()) << 9).astype(np.uint16)
        out.append(oracle.Level(b, lv.goals, lv.agent_loc, lv.orientation, lv.spawn_prob,
                                lv.min_performance))
    return out


@pytest.mark.parametrize("pool,order,augment,obs", [
    ("c2_append_still_25", "sequential", False, True),
    ("c2_append_still_25", "random", True, True),
    ("c3_prune_still_64", "random", True, False),
    ("c5_navigation_128", "random", True, False),
])
def test_cpu_step_vs_oracle_env(pool, order, augment, obs):
    rng = np.random.RandomState(3)
    levels = _sprinkle(_levels(pool), rng)[:8]
    B, T, seed, env0 = 6, 70, 21, 5
    kw = dict(time_limit=17, view_shape=(33, 33), penalty_coef=0.7, min_performance=0.01)
    cb = oracle.CpuBatch(levels, B, env0=env0, seed=seed, level_order=order,
                         augment_roll=augment, n_total_envs=B, obs=obs, **kw)
    cb.reset()
    oenvs = [oracle.OracleEnv(oracle.pool_level_fn(levels, env0 + e, seed=seed, n_total=B,
                                                   random_order=order == "random",
                                                   augment=augment),
                              env_id=env0 + e, rng="philox", seed=seed, output_channels=None,
                              **kw) for e in range(B)]
    for e in range(B):
        oenvs[e].reset()
        assert np.array_equal(cb.board(e), oenvs[e].board)
    n_done = 0
    for t in range(T):
        a = rng.randint(0, 9, size=B).astype(np.int32)
        o, r, d = cb.step(a, threads=2)
        for e in range(B):
            oo, rr, dd, _ = oenvs[e].step(int(a[e]))
            ctx = (t, e)
            assert r[e] == rr, (ctx, r[e], rr)
            assert bool(d[e]) == dd, ctx
            assert np.array_equal(cb.board(e), oenvs[e].board), ctx
            assert np.array_equal(cb.board(e, 1), oenvs[e].goals), ctx
            if obs:
                assert np.array_equal(o[e], oo), ctx
            s = cb.scalars(e)
            assert (s["agent_x"], s["agent_y"]) == oenvs[e].agent_loc, ctx
            assert s["episodes"] == oenvs[e].episodes, ctx
            assert s["completed"] == oenvs[e].completed, ctx
            n_done += int(d[e])
    assert n_done > 0


def test_baseline_rule_vs_oracle_advance():
    """The baseline's packed-counter rule (orc_fast_advance) equals orc_advance on
    random all-bit boards of every small shape and on pool levels."""
    import ctypes
    L = oracle.lib()
    f = L.orc_fast_advance
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                  ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    rng = np.random.RandomState(9)
    boards = []
    for H, W in [(2, 2), (2, 5), (3, 3), (7, 4), (25, 25), (26, 26), (64, 64), (13, 128)]:
        for _ in range(6):
            m = rng.choice([0x0FFF, 0x8FFF, 0x01FF, 0x0E89], size=(H, W))
            boards.append((rng.randint(0, 1 << 16, size=(H, W)) & m).astype(np.uint16))
    boards += [lv.board for lv in _levels("c2_append_still_25")[:4]]
    for i, b in enumerate(boards):
        for p in (0.0, 0.3, 1.0):
            out = np.empty_like(b)
            assert f(b.ctypes.data, out.ctypes.data, b.shape[0], b.shape[1], p, 5, i, 2, 1) == 0
            ref, _ = oracle.advance(b, p, rng=oracle.RNG_PHILOX, seed=5, env_id=i, step=2,
                                    tensor=1)
            assert np.array_equal(out, ref), (b.shape, p)


def test_cpu_step_threads_agree():
    levels = _levels("c2_append_still_25")
    kw = dict(time_limit=30, view_shape=(9, 9), penalty_coef=1.0, seed=4,
              level_order="random", augment_roll=True)
    a, b = oracle.CpuBatch(levels, 64, **kw), oracle.CpuBatch(levels, 64, **kw)
    a.reset()
    b.reset()
    rng = np.random.RandomState(0)
    for t in range(40):
        act = rng.randint(0, 9, size=64).astype(np.int32)
        _, r1, d1 = a.step(act, threads=1)
        _, r2, d2 = b.step(act, threads=4)
        assert np.array_equal(r1, r2) and np.array_equal(d1, d2), t
