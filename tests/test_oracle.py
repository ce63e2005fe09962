"""Pin the CPU oracle (oracle/) against golden vectors captured from the reference.

CPU-only.  These tests are what makes the oracle trustworthy as the checker of
the HIP path (tests/test_gpu_*.py).
"""
import glob
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_g1_advance_known_answers():
    d = np.load(os.path.join(GOLDEN, "advance_known_answers.npz"))
    off = 0
    for (H, W), p in zip(d["shapes"], d["spawn_prob"]):
        n = H * W
        bi = d["boards_in"][off:off + n].reshape(H, W)
        bo = d["boards_out"][off:off + n].reshape(H, W)
        off += n
        out, _ = oracle.advance(bi, p)
        assert np.array_equal(out, bo), (H, W, p)


def test_g2_reference_stream():
    d = np.load(os.path.join(GOLDEN, "advance_stream.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    assert len(keys) >= 12
    for key in keys:
        s = int(key.split("_")[0][1:])
        rng = oracle.RefStreamRNG()
        rng.seed(s)
        b, g = d[key + "_board0"], d[key + "_goals0"]
        for t in range(d[key + "_boards"].shape[0]):
            nb, ng = d[key + "_counts"][t]
            assert oracle.count_eligible(b) == nb
            b, _ = oracle.advance(b, 0.3, rng.take(nb))
            assert oracle.count_eligible(g) == ng
            g, _ = oracle.advance(g, 0.3, rng.take(ng))
            assert np.array_equal(b, d[key + "_boards"][t]), (key, t)
            assert np.array_equal(g, d[key + "_goals"][t]), (key, t)


def test_g1_128_known_answers():
    """G1 at 128x128 (C5's board size), captured from the reference."""
    d = np.load(os.path.join(GOLDEN, "advance_known_answers_128.npz"))
    assert len(d["boards_in"]) >= 50
    for b, want, p in zip(d["boards_in"], d["boards_out"], d["spawn_prob"]):
        got, _ = oracle.advance(b, p, np.zeros(b.size), 0)
        assert np.array_equal(got, want), p


def test_g2_128_reference_stream():
    """G2 at 128x128: C5 navigation levels advanced 30 times after speedups.seed(s)."""
    d = np.load(os.path.join(GOLDEN, "advance_stream_128.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    assert len(keys) >= 2
    for key in keys:
        rng = oracle.RefStreamRNG()
        rng.seed(int(key.split("_")[0][1:]))
        p = float(d[key + "_p"])
        b, g = d[key + "_board0"], d[key + "_goals0"]
        for t in range(d[key + "_boards"].shape[0]):
            b, _ = oracle.advance(b, p, rng.take(oracle.count_eligible(b)))
            g, _ = oracle.advance(g, p, rng.take(oracle.count_eligible(g)))
            assert np.array_equal(b, d[key + "_boards"][t]), (key, t)
            assert np.array_equal(g, d[key + "_goals"][t]), (key, t)


def _traj_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "traj_*.npz")))


def make_oracle_env(d, rng=None):
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    lvl = oracle.Level(d["level_board"], d["level_goals"], d["level_agent_loc"],
                       d["level_orientation"], d["level_spawn_prob"],
                       d["level_min_performance"])
    if rng is None:
        rng = oracle.RefStreamRNG()
        rng.seed(int(seed))
    return oracle.OracleEnv(lambda ep: lvl, time_limit=int(time_limit),
                            view_shape=(int(vh), int(vw)), output_channels=None,
                            penalty_coef=float(penalty), min_performance=float(min_perf),
                            rng="stream", stream=rng)


@pytest.mark.parametrize("path", _traj_files(), ids=lambda p: os.path.basename(p)[5:-4])
def test_g3_trajectory(path):
    d = np.load(path)
    env = make_oracle_env(d)
    obs = env.reset()
    assert np.array_equal(obs, d["obs0"])
    T = len(d["action"])
    for t in range(T):
        obs, r, done, info = env.step(int(d["action"][t]))
        ctx = (os.path.basename(path), t)
        assert r == d["reward"][t], ctx          # bit-exact float64
        assert done == d["done"][t], ctx
        assert info["times_up"] == d["times_up"][t], ctx
        assert tuple(env.agent_loc) == tuple(d["agent_loc"][t]), ctx
        assert env.orientation == d["orientation"][t], ctx
        assert np.array_equal(env.board, d["board"][t]), ctx
        assert np.array_equal(env.goals, d["goals"][t]), ctx
        assert np.array_equal(obs, d["obs"][t]), ctx
        assert env.old_points == d["points"][t], ctx
        assert tuple(env._perf_ratio()) == tuple(d["perf"][t]), ctx
        assert env.last_side_effect == d["side_effect"][t], ctx


def test_obs_channels_match_packed():
    d = np.load(_traj_files()[0])
    env = make_oracle_env(d)
    env.output_channels = tuple(range(15))
    o = env.reset()
    packed = (o.astype(np.uint32) << np.arange(15)).sum(-1)
    assert np.array_equal(packed, d["obs0"] & 0x7FFF)


def test_philox_known_values():
    # Philox4x32-10 published known-answer vectors (Random123 kat_vectors):
    # counter 0, key 0 -> 6627e8d5 e169c58d bc57ac4c 9b00dbd8
    import ctypes
    out = (ctypes.c_uint32 * 4)()
    oracle.lib().orc_philox4x32.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 4 + [ctypes.c_uint64]
    oracle.lib().orc_philox4x32(out, 0, 0, 0, 0, 0)
    assert [hex(v) for v in out] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    oracle.lib().orc_philox4x32(out, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF,
                                0xFFFFFFFFFFFFFFFF)
    assert [hex(v) for v in out] == ["0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]


def test_symmetry_deterministic():
    """The rule commutes with toroidal roll / transpose / flips (p in {0,1})."""
    rng = np.random.RandomState(3)
    for _ in range(40):
        H, W = rng.randint(3, 20, size=2)
        b = rng.randint(0, 1 << 16, size=(H, W)).astype(np.uint16)
        b = (b * (rng.rand(H, W) < 0.5)).astype(np.uint16)
        for p in (0.0, 1.0):
            out, _ = oracle.advance(b, p)
            dy, dx = rng.randint(0, H), rng.randint(0, W)
            r, _ = oracle.advance(np.roll(b, (dy, dx), (0, 1)), p)
            assert np.array_equal(r, np.roll(out, (dy, dx), (0, 1)))
            t, _ = oracle.advance(np.ascontiguousarray(b.T), p)
            assert np.array_equal(t, out.T)
            f, _ = oracle.advance(np.ascontiguousarray(b[::-1]), p)
            assert np.array_equal(f, out[::-1])


def test_g5_side_effect_densities():
    """The oracle's rollout + density restatement reproduces the reference's
    _add_cell_distribution maps captured in densities.npz (replay RNG)."""
    d = np.load(os.path.join(GOLDEN, "densities.npz"))
    for j in range(2):
        stream = oracle.RefStreamRNG()
        stream.seed(11 + j)
        board = d["l%d_board" % j]
        ina, act = oracle.side_effect_densities(board, np.roll(board, 1, axis=1), 7,
                                                float(d["l%d_spawn" % j]), 20, rng="stream",
                                                stream=stream)
        for nm, got in (("inaction", ina), ("action", act)):
            keys = d["l%d_%s_keys" % (j, nm)].tolist()
            assert sorted(got) == keys, (j, nm)
            for k, ref in zip(keys, d["l%d_%s_dens" % (j, nm)]):
                assert np.array_equal(got[k], ref), (j, nm, k)
