"""C5's board size pinned to the reference itself (round 5): the 128x128 fixtures
captured from the reference (tests/golden/make_golden.py g1_128 / g2_128 / traj128)
through the banded bit-sliced kernels (k_env_step_bits128, csrc/sl_bits128.hip).

  G1-128   54 random 128x128 boards (all used bits, life-like soups, every bit
           pattern) advanced once at p in {0, 1}: pair k is env k's board and goals,
           one NULL-action step (advance_board.c:34-120, both tensors).
  G2-128   two C5 navigation levels advanced 30 times after speedups.seed(s): one
           env, NULL actions, the spawn stream generated on the device from s alone
           (csrc/sl_mt.hip) and, separately, supplied from numpy.
  G4-128   PPO-chain trajectories on C5 levels (traj_nav128_*.npz) run through the
           trajectory tests of test_gpu_parity.py / test_gpu_mt.py (they glob
           traj_*.npz), here once more from the seed alone with every state field.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu

_KW = dict(time_limit=100000, view_shape=(15, 15), output_channels=None, penalty_coef=1.0,
           min_performance=0.01, compute_obs=False)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    import safelife_amd  # noqa: F401
    return torch, torch.device("cuda:0")


def _bare_env(torch, dev, boards, goals, spawn_prob, **kw):
    """B 128x128 envs holding the given boards and goals, no exits to recolour (the
    fixtures advance bare boards), agents at (0, 0), NULL actions."""
    from safelife_amd import SafeLifeVecEnv, LevelPool
    B = len(boards)
    z = np.zeros((128, 128), np.uint16)
    pool = LevelPool.from_levels([{"board": z, "goals": z}])
    env = SafeLifeVecEnv(pool, B, dev, kernel=kw.pop("kernel", "fast"), **dict(_KW, **kw))
    env.reset()
    env.set_state(np.asarray(boards), np.asarray(goals), np.asarray(boards),
                  spawn_prob=np.asarray(spawn_prob, np.float32), exit_count=np.zeros(B),
                  episode_length=np.zeros(B), game_over=np.zeros(B),
                  agent_x=np.zeros(B), agent_y=np.zeros(B))
    return env


def test_g1_128_known_answers(torch_dev):
    """Through the 128x128 step kernel (board and goals both advanced by the banded
    rule), and through the batched per-cell advance (speedups.advance_boards).  (The
    per-cell env step takes exits from the start board -- level exits are frozen and
    recoloured every step -- so it is not a bare advance of all-bit boards.)"""
    torch, dev = torch_dev
    from safelife_amd import speedups
    d = np.load(os.path.join(GOLDEN, "advance_known_answers_128.npz"))
    bi, bo, p = d["boards_in"], d["boards_out"], d["spawn_prob"]
    assert len(bi) >= 50 and np.array_equal(p[0::2], p[1::2])
    out = speedups.advance_boards(torch.from_numpy(bi).to(dev),
                                  torch.from_numpy(p.astype(np.float32)).to(dev)).cpu().numpy()
    assert np.array_equal(out, bo)
    env = _bare_env(torch, dev, bi[0::2], bi[1::2], p[0::2], rng="philox", seed=1)
    env.step(torch.zeros(env.B, dtype=torch.int32, device=dev))
    got_b, got_g = env.board.cpu().numpy(), env.goals.cpu().numpy()
    for k in range(env.B):
        assert np.array_equal(got_b[k], bo[2 * k]), (k, p[2 * k])
        assert np.array_equal(got_g[k], bo[2 * k + 1]), (k, p[2 * k])


@pytest.mark.parametrize("source", ["device_generator", "numpy_stream"])
def test_g2_128_seeded_stream(torch_dev, source):
    """speedups.seed(s) then board, goals advanced in turn: the replay kernels (count
    prologue, scan, draw pass, SPAWN_DECIDED step) with the stream from the seed."""
    torch, dev = torch_dev
    d = np.load(os.path.join(GOLDEN, "advance_stream_128.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    assert len(keys) >= 2
    for key in keys:
        s = int(key.split("_")[0][1:])
        stream = (None if source == "device_generator"
                  else np.random.RandomState(s).random_sample(2_000_000))
        env = _bare_env(torch, dev, [d[key + "_board0"]], [d[key + "_goals0"]],
                        [float(d[key + "_p"])], rng="stream", spawn_stream=stream, seed=s)
        assert (env.mt is not None) == (stream is None)
        a = torch.zeros(1, dtype=torch.int32, device=dev)
        for t in range(d[key + "_boards"].shape[0]):
            env.step(a)
            assert np.array_equal(env.board[0].cpu().numpy(), d[key + "_boards"][t]), (key, t)
            assert np.array_equal(env.goals[0].cpu().numpy(), d[key + "_goals"][t]), (key, t)
        assert int(env.stream_pos.item()) > 1000 and not env.stream_error()


@pytest.mark.parametrize("name", ["nav128_c5", "nav128_seek"])
def test_g4_128_trajectory_from_seed_state(torch_dev, name):
    """The 128x128 PPO-chain trajectories from their seed alone (no host stream),
    every recorded field: reward, done, times_up, agent, orientation, points, the
    performance terms, the side-effect count, boards, goals, packed views."""
    from test_gpu_parity import _vec_env_from_traj
    torch, dev = torch_dev
    d = np.load(os.path.join(GOLDEN, "traj_%s.npz" % name))
    env = _vec_env_from_traj(d, kernel="fast", spawn_stream=None, seed=int(d["cfg"][2]))
    assert env.mt is not None and env.H == env.W == 128
    obs = env.reset().cpu().numpy()
    assert np.array_equal(obs[0], d["obs0"])
    actions = torch.from_numpy(d["action"].astype(np.int32)).to(dev)
    st = env.state
    for t in range(len(d["action"])):
        obs, r, done, info = env.step(actions[t:t + 1])
        ctx = (name, t)
        assert r.item() == d["reward"][t], ctx
        assert bool(done.item()) == bool(d["done"][t]), ctx
        assert bool(info["times_up"][0].item()) == bool(d["times_up"][t]), ctx
        assert np.array_equal(env.board[0].cpu().numpy(), d["board"][t]), ctx
        assert np.array_equal(env.goals[0].cpu().numpy(), d["goals"][t]), ctx
        assert np.array_equal(obs[0].cpu().numpy(), d["obs"][t]), ctx
        if not (d["done"][t] or d["game_over"][t]):
            assert (st["agent_x"][0].item(), st["agent_y"][0].item()) == \
                tuple(d["agent_loc"][t]), ctx
            assert st["orientation"][0].item() == d["orientation"][t], ctx
            assert st["old_points"][0].item() == d["points"][t], ctx
            assert st["side_effect"][0].item() == d["side_effect"][t], ctx
    assert int(d["done"].sum()) >= 2 and not env.stream_error()
