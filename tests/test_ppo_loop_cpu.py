"""G7: the reference's PPO rollout loop (training/ppo.py:436-452), captured from the
reference (tests/golden/make_golden.py g7): 16 envs stepped in turn, each action
drawn by np.random.choice from the global numpy stream that also refills the spawn
buffer 10 000 doubles at a time (speedups_src/random.c:14-26,47-52).  The oracle env
(oracle/oracle.py, the PPO wrapper chain) run the same way -- one RefStreamRNG shared
by all envs, as the reference's buffer is global -- pins the interleave on the CPU;
the device replays it in tests/test_gpu_rollout.py (run_agents(rng="reference"))."""
import glob
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
G7 = sorted(glob.glob(os.path.join(GOLDEN, "g7_*.npz")))


def oracle_level(d):
    return oracle.Level(d["level_board"], d["level_goals"], d["level_agent_loc"],
                        d["level_orientation"], d["level_spawn_prob"],
                        d["level_min_performance"])


@pytest.mark.parametrize("path", G7, ids=lambda p: os.path.basename(p)[3:-4])
def test_g7_ppo_loop_oracle(path):
    d = np.load(path)
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    table = d["table"]
    T, N, A = table.shape
    assert N == 16 and int(d["done"].sum()) > 0
    lvl = oracle_level(d)
    rng = oracle.RefStreamRNG()
    rng.seed(int(seed))
    envs = [oracle.OracleEnv(lambda ep: lvl, time_limit=int(time_limit),
                             view_shape=(int(vh), int(vw)), output_channels=None,
                             penalty_coef=float(penalty), min_performance=float(min_perf),
                             rng="stream", stream=rng) for _ in range(N)]
    for env in envs:
        env.reset()
    keep = {int(s): k for k, s in enumerate(d["board_steps"])}
    for t in range(T):
        for e, env in enumerate(envs):
            a = int(np.random.choice(A, p=table[t, e]))
            assert a == d["action"][t, e], (t, e)
            _, r, done, _ = env.step(a)
            assert r == d["reward"][t, e], (t, e)
            assert done == d["done"][t, e], (t, e)
            if t in keep:
                assert np.array_equal(env.board, d["board"][keep[t], e]), (t, e)
                assert np.array_equal(env.goals, d["goals"][keep[t], e]), (t, e)
    assert np.array_equal(np.random.random(4), d["after"])
