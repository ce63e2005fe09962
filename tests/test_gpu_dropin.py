"""The Python drop-in surface north_star names (SafeLifeEnv.step()/reset() and
SafeLifeGame.advance_board()), driven the way the reference's callers drive it, on
the device.

- A reference-captured trajectory (tests/golden/traj_*.npz, captured from
  SafeLifeEnv under the PPO wrapper chain) is replayed through the game methods
  alone -- ``execute_action``, ``advance_board``, ``current_points``,
  ``update_exit_colors``, and ``revert`` at every episode end, as SafeLifeEnv.step /
  reset call them (safelife_env.py:157-198) -- with the spawn draws taken from
  numpy's global stream (speedups.seed), bit-exact at every step.
- The relative actions and the remaining state methods (MOVE FORWARD / BACKWARD,
  TURN, FACE, bare TOGGLE, serialize / deserialize / revert / save / load) are
  checked against the oracle's restatement of move_agent (safelife_game.py:308-393).
- get_obs(board, goals, agent_loc) against the oracle's get_obs restatement.
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


def _level(d):
    return {"board": d["level_board"], "goals": d["level_goals"],
            "agent_loc": d["level_agent_loc"], "orientation": d["level_orientation"],
            "spawn_prob": d["level_spawn_prob"], "min_performance": d["level_min_performance"]}


@pytest.mark.parametrize("name", ["append_still_v01", "append_spawn_v10", "prune_spawn_v10",
                                  "append_still_seek", "prune_still_seek", "nav128_c5"])
def test_game_methods_replay_golden(torch_dev, name):
    """SafeLifeEnv.step's game calls one by one (execute_action -> advance_board ->
    current_points -> update_exit_colors; revert + update_exit_colors where the
    reference env reset), on SafeLifeGame.loaddata(level) with the reference RNG:
    boards, goals, agent, orientation, points and performance ratio equal the
    reference's at every step; numpy's global stream ends where the reference's
    did."""
    from safelife_amd import SafeLifeGame, speedups, ACTION_NAMES
    d = np.load(os.path.join(GOLDEN, "traj_%s.npz" % name))
    penalty, min_perf, seed, vh, vw, time_limit = d["cfg"]
    speedups.seed(int(seed))
    game = SafeLifeGame.loaddata(_level(d))
    # SafeLifeEnv.reset colours the exits with the level's own min_performance, then
    # SimpleSideEffectPenalty.reset replaces it (env_wrappers.py:313-317)
    game.update_exit_colors()
    old = game.current_points()
    game.min_performance = float(min_perf)
    ep_len = 0
    n_ends = 0
    for t in range(len(d["action"])):
        r = game.execute_action(ACTION_NAMES[int(d["action"][t])])
        game.advance_board()
        pts = game.current_points()
        game.update_exit_colors()
        ep_len += 1
        over = game.game_over
        assert over == bool(d["game_over"][t]), t
        assert r == (1 if d["game_over"][t] else 0), t        # points_on_level_exit
        if d["game_over"][t] or ep_len > int(time_limit):
            # SafeLifeEnv.reset (safelife_env.py:188-198) through ContinuingEnv / the
            # caller: revert, exit colours, old value
            assert game.revert()
            game.update_exit_colors()
            old = game.current_points()
            game.min_performance = float(min_perf)
            ep_len = 0
            n_ends += 1
            assert game.num_steps == 0 and not game.game_over
        else:
            assert tuple(game.agent_loc) == tuple(d["agent_loc"][t]), t
            assert game.orientation == d["orientation"][t], t
            assert pts == d["points"][t], t
            assert tuple(game.performance_ratio()) == tuple(d["perf"][t]), t
            assert game.num_steps == ep_len, t
            old = pts
        assert np.array_equal(game.board, d["board"][t]), t
        assert np.array_equal(game.goals, d["goals"][t]), t
    assert n_ends == int((d["game_over"] | d["times_up"]).sum())
    # the global stream advanced exactly as the reference's draws did
    lvl = _level(d)
    ref = oracle.RefStreamRNG()
    ref.seed(int(seed))
    o = oracle.OracleEnv(lambda ep: oracle.Level(**lvl), time_limit=int(time_limit),
                         view_shape=(int(vh), int(vw)), output_channels=None, penalty_coef=0.0,
                         min_performance=float(min_perf), rng="stream", stream=ref)
    o.reset()
    for s in range(len(d["action"])):
        o.step(int(d["action"][s]))
    assert speedups._buffer.pos == ref.pos
    assert np.array_equal(speedups._buffer.buf, ref.buf)


def _oracle_at(game):
    """An OracleEnv holding the game's current state (for single-method checks)."""
    lv = oracle.Level(game.board, game.goals, tuple(game.agent_loc), game.orientation,
                      game.spawn_prob, game.min_performance)
    o = oracle.OracleEnv(lambda ep: lv, rng="philox", output_channels=None)
    o.reset()
    o.board = game.board.copy()        # exits as they are (reset recoloured them)
    o.baseline = game._st("baseline")
    o.min_performance = game.min_performance
    return o


def test_game_relative_actions_vs_oracle(torch_dev):
    """MOVE FORWARD / BACKWARD (move_agent(+-1), orientation kept), TURN LEFT / RIGHT,
    FACE, bare TOGGLE and NULL on a 26x26 sokoban-style level with crates, against
    the oracle's move_agent / toggle restatement, over a long random sequence."""
    from safelife_amd import SafeLifeGame
    d = np.load(os.path.join(GOLDEN, "traj_sokoban_example.npz"))
    game = SafeLifeGame.loaddata(_level(d), rng="philox")
    o = _oracle_at(game)
    names = ["MOVE FORWARD", "MOVE BACKWARD", "TURN LEFT", "TURN RIGHT", "FACE UP",
             "FACE DOWN", "FACE LEFT", "FACE RIGHT", "TOGGLE", "NULL", "MOVE UP",
             "TOGGLE LEFT"]
    rng = np.random.RandomState(3)
    for t in range(400):
        nm = names[rng.randint(len(names))]
        r = game.execute_action(nm)
        # the oracle, as GameState.execute_action (safelife_game.py:347-393) runs it
        if nm == "MOVE FORWARD":
            ro = o._move_agent(1)
        elif nm == "MOVE BACKWARD":
            ro = o._move_agent(-1)
        elif nm.startswith("TURN "):
            o.orientation = (o.orientation + 2 - {"LEFT": 3, "RIGHT": 1}[nm[5:]]) % 4
            ro = 0
        elif nm.startswith("FACE "):
            o.orientation = ("UP", "RIGHT", "DOWN", "LEFT").index(nm[5:])
            ro = 0
        elif nm == "TOGGLE":
            ro = o._execute_action("TOGGLE " + ("UP", "RIGHT", "DOWN", "LEFT")[o.orientation])
        else:
            ro = o._execute_action(nm)
        assert r == ro, (t, nm)
        assert np.array_equal(game.board, o.board), (t, nm)
        assert tuple(game.agent_loc) == tuple(o.agent_loc), (t, nm)
        assert game.orientation == o.orientation, (t, nm)
        assert game.relative_loc(2, -1) == o._relative_loc(2, -1), t


def test_game_state_roundtrips(torch_dev, tmp_path):
    """serialize / deserialize / revert / save / load on the device game: a game
    stepped for a while and reverted equals the freshly loaded level; deserialize of
    a serialized mid-game state restores it exactly (the env-level counters
    untouched); save + load round-trips through npz; a view into a larger batch
    changes only its own env."""
    import torch
    from safelife_amd import SafeLifeGame, SafeLifeVecEnv, LevelPool, speedups
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    pool = LevelPool.load(path)
    lvl = {"board": pool.board[3], "goals": pool.goals[3],
           "agent_loc": (pool.agent_x[3], pool.agent_y[3]), "orientation": pool.orientation[3],
           "spawn_prob": pool.spawn_prob[3], "min_performance": pool.min_performance[3]}
    speedups.seed(5)
    game = SafeLifeGame.loaddata(lvl)
    b0, g0, a0 = game.board, game.goals, tuple(game.agent_loc)
    rng = np.random.RandomState(0)
    for _ in range(25):
        game.execute_action("TOGGLE RIGHT" if rng.rand() < .5 else "MOVE UP")
        game.advance_board()
    assert game.num_steps == 25
    mid = game.serialize()
    assert set(mid) == {"spawn_prob", "orientation", "agent_loc", "board", "class",
                        "min_performance", "goals"}
    game.revert()
    assert np.array_equal(game.board, b0) and np.array_equal(game.goals, g0)
    assert tuple(game.agent_loc) == a0 and game.num_steps == 0 and not game.game_over
    game.deserialize(mid)
    assert np.array_equal(game.board, mid["board"]) and np.array_equal(game.goals, mid["goals"])
    assert tuple(game.agent_loc) == tuple(mid["agent_loc"])
    assert game.orientation == mid["orientation"]
    f = str(tmp_path / "saved")
    game.save(f)
    g2 = SafeLifeGame.load(f + ".npz")
    assert np.array_equal(g2.board, game.board) and np.array_equal(g2.goals, game.goals)
    assert g2.title == "saved"
    # a view of env 5 of a batch: its methods touch env 5 only
    v = SafeLifeVecEnv(pool, 8, "cuda:0", rng="philox", seed=1, output_channels=None)
    v.reset()
    before = v.board.clone(), v.goals.clone()
    gv = SafeLifeGame(v, 5)
    gv.execute_action("TOGGLE UP")
    gv.advance_board()
    gv.update_exit_colors()
    for i in range(8):
        if i != 5:
            assert torch.equal(v.board[i], before[0][i]) and torch.equal(v.goals[i], before[1][i])
    assert not torch.equal(v.board[5], before[0][5])
    assert v.state["num_steps"][5].item() == 1 and v.state["num_steps"][0].item() == 0


def test_get_obs_arguments_vs_oracle(torch_dev):
    """SafeLifeEnv.get_obs(board, goals, agent_loc) (safelife_env.py:125-155) for
    caller-supplied arrays, packed and 15-channel, against the oracle's make_obs."""
    from safelife_amd import SafeLifeEnv
    d = np.load(os.path.join(GOLDEN, "traj_append_still_v01.npz"))
    rng = np.random.RandomState(9)
    for channels in (None, tuple(range(15))):
        env = SafeLifeEnv(iter([_level(d)] * 2), view_shape=(33, 33), output_channels=channels,
                          seed=1)
        env.reset()
        ex = list(zip(*env.game.exit_locs))
        for k in range(4):
            b = d["board"][100 * k + 7]
            g = d["goals"][100 * k + 3]
            al = (rng.randint(25), rng.randint(25))
            want = oracle.make_obs(b, g, al[0], al[1], ex, (33, 33), channels, True)
            assert np.array_equal(env.get_obs(b, g, al), want), (channels, k)
            gl = tuple(env.game.agent_loc)
            want = oracle.make_obs(b, env.game.goals, gl[0], gl[1], ex, (33, 33), channels, True)
            assert np.array_equal(env.get_obs(board=b), want), (channels, k)


def test_save_rebases_performance(torch_dev, tmp_path):
    """save() makes the saved state the game's _init_data (safelife_game.py:225):
    performance_ratio then scores against it (completed 0) and the side-effect start
    board is the saved board."""
    from safelife_amd import SafeLifeGame, speedups
    path = os.path.join(GOLDEN, "pools", "c3_prune_still_64.npz")
    d = np.load(path)
    lvl = {k: d[k][2] for k in ("board", "goals", "agent_loc", "orientation", "spawn_prob",
                                 "min_performance")}
    speedups.seed(9)
    game = SafeLifeGame.loaddata(lvl)
    for a in ["TOGGLE RIGHT", "MOVE UP", "TOGGLE LEFT", "TOGGLE UP"] * 5:
        game.execute_action(a)
        game.advance_board()
    done0, total0 = game.performance_ratio()
    game.save(str(tmp_path / "mid"))
    done1, total1 = game.performance_ratio()
    assert done1 == 0 and total1 == total0 - done0
    assert np.array_equal(game._venv.start_board[0].cpu().numpy(), game.board)
    assert np.array_equal(game._init_data["board"], game.board)


def test_batch_view_advance_leaves_other_envs(torch_dev):
    """advance_board on a view of a Philox batch keys its draws on the game's own
    counter: the batch's step index, and so every other env's later steps, are those
    of a twin batch whose env was never advanced by hand."""
    import torch
    from safelife_amd import SafeLifeGame, SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c5_navigation_128.npz")
    pool = LevelPool.load(path)
    kw = dict(rng="philox", seed=3, output_channels=None, time_limit=50)
    v, twin = SafeLifeVecEnv(pool, 6, "cuda:0", **kw), SafeLifeVecEnv(pool, 6, "cuda:0", **kw)
    v.reset()
    twin.reset()
    gv = SafeLifeGame(v, 2)
    for _ in range(3):
        gv.advance_board()
    assert v._step_index == twin._step_index == 0
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    for t in range(12):
        a = torch.randint(0, 9, (6,), dtype=torch.int32, device="cuda:0", generator=g)
        v.step(a)
        twin.step(a)
        for i in (0, 1, 3, 4, 5):
            assert torch.equal(v.board[i], twin.board[i]), (t, i)
            assert torch.equal(v.goals[i], twin.goals[i]), (t, i)


def test_view_advances_differ_across_game_objects(torch_dev):
    """SafeLifeEnv.reset makes a new SafeLifeGame for the same env each episode; in
    rng='philox' mode the advance counter lives on the batch, so a new game object's
    advances do not repeat the draws of the last one's."""
    import torch
    from safelife_amd import SafeLifeGame, SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c5_navigation_128.npz")
    v = SafeLifeVecEnv(LevelPool.load(path), 3, "cuda:0", rng="philox", seed=4,
                       output_channels=None)
    v.reset()
    b0, g0 = v.board[1].clone(), v.goals[1].clone()
    outs = []
    for _ in range(2):
        v.board[1].copy_(b0)
        v.goals[1].copy_(g0)
        v.planes_ok.zero_()
        gv = SafeLifeGame(v, 1)
        for _ in range(4):
            gv.advance_board()
        outs.append(v.board[1].clone())
    assert int(((b0.to(torch.int32) & 128) != 0).sum().item()) > 0   # spawners
    assert not torch.equal(outs[0], outs[1])


def test_board_setter_on_128_replay_matches_generic(torch_dev):
    """Assigning game.board on a 128x128 replay env drops the draw planes the last
    step left (planes_ok bit 3), so the next replay steps count the new board's
    eligible cells: the bit-sliced replay equals the per-cell kernel's, draw for draw,
    after the assignment."""
    import torch
    from safelife_amd import SafeLifeGame, SafeLifeVecEnv, LevelPool
    path = os.path.join(GOLDEN, "pools", "c5_navigation_128.npz")
    pool = LevelPool.load(path)
    stream = np.random.RandomState(12).random_sample(3_000_000)
    envs = [SafeLifeVecEnv(pool, 4, "cuda:0", rng="stream", spawn_stream=stream, kernel=k,
                           output_channels=None, time_limit=200) for k in ("fast", "generic")]
    g = torch.Generator(device="cuda:0")
    g.manual_seed(2)
    acts = [torch.randint(0, 9, (4,), dtype=torch.int32, device="cuda:0", generator=g)
            for _ in range(20)]
    for e in envs:
        e.reset()
        for t in range(5):
            e.step(acts[t])
    new = envs[0].board[1].cpu().numpy().copy()
    new[40:60, 40:60] = 152                  # a block of spawners
    for e in envs:
        SafeLifeGame(e, 1).board = new
    for t in range(5, 20):
        for e in envs:
            e.step(acts[t])
        assert torch.equal(envs[0].board, envs[1].board), t
        assert torch.equal(envs[0].goals, envs[1].goals), t
        assert torch.equal(envs[0].stream_pos, envs[1].stream_pos), t
    assert not envs[0].stream_error()


def test_state_dict_keeps_exchange_position(torch_dev):
    """With a StreamExchange (parity mode over shards) the global stream position is
    saved and restored with the env."""
    import torch
    from safelife_amd import SafeLifeVecEnv, LevelPool
    from safelife_amd import dist as sdist
    path = os.path.join(GOLDEN, "pools", "c5_navigation_128.npz")
    pool = LevelPool.load(path)
    ex = sdist.StreamExchange(device="cuda:0")
    v = SafeLifeVecEnv(pool, 4, "cuda:0", rng="stream",
                       spawn_stream=np.random.RandomState(1).random_sample(2_000_000),
                       stream_exchange=ex, output_channels=None)
    v.reset()
    for _ in range(4):
        v.step(torch.zeros(4, dtype=torch.int32, device="cuda:0"))
    sd = v.state_dict()
    p = int(ex.pos.item())
    assert p > 0 and int(sd["exchange_pos"].item()) == p
    ex.pos.zero_()
    v.load_state_dict(sd)
    assert int(ex.pos.item()) == p
