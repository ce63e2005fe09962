"""World-size-2 gloo tests of the multi-GPU layout, on CPU.

Each rank owns a contiguous shard of global env ids (safelife_amd.dist.env_shard)
and steps its envs with the CPU oracle in Philox mode, keyed by GLOBAL id, with the
device reset's sequential level order (idx = (gid + episode * n_total) mod K,
sl_env.hip reset_one).  The episode records gathered over gloo must equal a
single-process run of all envs: trajectories do not depend on the number of ranks,
so the data path needs no collective.  Counters are all-reduced the way bench.py
and the vec env's logging do.
"""
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POOL = os.path.join(REPO, "tests", "golden", "pools", "c2_append_still_25.npz")
ENVS_PER_RANK, WORLD, STEPS, SEED = 3, 2, 40, 77


def _paths():
    for p in (os.path.join(REPO, "safelife-k2_amd"), os.path.join(REPO, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _levels():
    _paths()
    import oracle
    d = np.load(POOL)
    return [oracle.Level(d["board"][i], d["goals"][i], d["agent_loc"][i], d["orientation"][i],
                         d["spawn_prob"][i], d["min_performance"][i])
            for i in range(d["board"].shape[0])]


def _run_envs(gids, n_total):
    """Step the given global env ids; returns [n_episodes, 4] records and counters."""
    _paths()
    import oracle
    levels = _levels()
    K = len(levels)
    recs, steps, started, completed = [], 0, 0, 0
    for gid in gids:
        env = oracle.OracleEnv(lambda ep, gid=gid: levels[(gid + ep * n_total) % K],
                               time_limit=15, view_shape=(9, 9), penalty_coef=1.0,
                               rng="philox", seed=SEED, env_id=gid)
        env.reset()
        started += 1
        acts = np.random.RandomState(1000 + gid).randint(0, 9, STEPS)
        ret = 0.0
        for t in range(STEPS):
            _, r, done, info = env.step(int(acts[t]))
            ret += r
            steps += 1
            if done:
                recs.append([gid, ret, info["episode_length"], info["side_effect"]])
                completed += 1
                started += 1
                ret = 0.0
        recs.append([gid, ret, env.episode_length, env.last_side_effect])
    return np.array(recs, dtype=np.float64), (started, completed, steps)


def _worker(rank, port, out_dir):
    _paths()
    import torch.distributed as dist
    from safelife_amd import dist as sdist
    from safelife_amd.vec_env import GlobalCounter
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=WORLD)
    sh = sdist.env_shard(rank, WORLD, ENVS_PER_RANK)
    recs, (s, c, n) = _run_envs(range(sh.env0, sh.env0 + sh.n_envs), sh.n_total)
    gc = GlobalCounter()
    gc.episodes_started, gc.episodes_completed, gc.num_steps = s, c, n
    allrec = sdist.gather_episodes(recs).numpy()
    tot = sdist.reduce_counters(gc)
    if rank == 0:
        np.savez(os.path.join(out_dir, "dist.npz"), recs=allrec,
                 counters=np.array([tot["episodes_started"], tot["episodes_completed"],
                                    tot["num_steps"]]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_env_shard_layout():
    _paths()
    from safelife_amd import dist as sdist
    shards = [sdist.env_shard(r, 4, 8) for r in range(4)]
    assert [s.env0 for s in shards] == [0, 8, 16, 24]
    assert all(s.n_total == 32 for s in shards)
    assert sdist.split_batch(262144, 8) == 32768
    with pytest.raises(ValueError):
        sdist.env_shard(4, 4, 8)
    with pytest.raises(ValueError):
        sdist.split_batch(10, 4)


def test_gather_without_process_group():
    _paths()
    from safelife_amd import dist as sdist
    r = np.arange(6, dtype=np.float64).reshape(3, 2)
    assert np.array_equal(sdist.gather_episodes(r).numpy(), r)


def test_two_rank_gloo_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    got = np.load(os.path.join(str(tmp_path), "dist.npz"))
    ref, (s, c, n) = _run_envs(range(WORLD * ENVS_PER_RANK), WORLD * ENVS_PER_RANK)
    assert np.array_equal(got["recs"], ref)
    assert got["counters"].tolist() == [s, c, n]
    assert c > 0          # episodes finished inside the window (time_limit 15)


# ------------------------------------------------ parity-mode stream exchange
def _spawner_levels():
    """The C2 pool levels with spawners sprinkled in (so every step draws)."""
    _paths()
    import oracle
    rng = np.random.RandomState(5)
    out = []
    for lv in _levels()[:6]:
        b = lv.board.copy()
        e = (b == 0) & (rng.rand(*b.shape) < 0.03)
        e[lv.agent_loc[1], lv.agent_loc[0]] = False
        b[e] = 152
        out.append(oracle.Level(b, lv.goals, lv.agent_loc, lv.orientation, 0.3,
                                lv.min_performance))
    return out


class _CountingStream:
    def __init__(self):
        self.n = 0

    def take(self, n):
        self.n += n
        return np.full(n, 0.5)


class _WindowStream:
    """A slice of the one global stream starting at `pos`."""

    def __init__(self, stream, pos):
        self.stream, self.pos = stream, pos

    def take(self, n):
        out = self.stream[self.pos:self.pos + n]
        self.pos += n
        return out


def _replay_envs(gids, n_total, exchange, steps=30):
    """Step the given global envs in reference-stream mode, one step at a time:
    the shard's draw total of the step (counted on copies), exchanged for the
    shard's base, then the real step from that base.  Returns final boards."""
    import copy
    import torch
    _paths()
    import oracle
    levels = _spawner_levels()
    stream = np.random.RandomState(3).random_sample(2_000_000)
    envs = [oracle.OracleEnv(lambda ep, gid=gid: levels[(gid + ep * n_total) % len(levels)],
                             time_limit=15, view_shape=(9, 9), penalty_coef=1.0,
                             rng="stream", stream=None, env_id=gid) for gid in gids]
    for e in envs:
        e.reset()
    for t in range(steps):
        acts = [int(np.random.RandomState(100 * t + g).randint(0, 9)) for g in gids]
        counter = _CountingStream()
        for e, a in zip(envs, acts):          # phase 1: this shard's draws
            c = copy.deepcopy(e)
            c.stream = counter
            c.step(a)
        base = int(exchange(torch.tensor([counter.n], dtype=torch.int64)).item())
        window = _WindowStream(stream, base)
        for e, a in zip(envs, acts):          # phase 2: from the shard's base
            e.stream = window
            e.step(a)
    return np.stack([e.board for e in envs]), int(exchange.pos.item())


def _replay_worker(rank, port, out_dir):
    _paths()
    import torch.distributed as dist
    from safelife_amd import dist as sdist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=WORLD)
    sh = sdist.env_shard(rank, WORLD, ENVS_PER_RANK)
    boards, pos = _replay_envs(range(sh.env0, sh.env0 + sh.n_envs), sh.n_total,
                               sdist.StreamExchange())
    np.savez(os.path.join(out_dir, "replay%d.npz" % rank), boards=boards, pos=pos)
    dist.barrier()
    dist.destroy_process_group()


def test_stream_exchange_single_rank():
    _paths()
    import torch
    from safelife_amd import dist as sdist
    ex = sdist.StreamExchange(pos=100)
    assert int(ex(torch.tensor([7])).item()) == 100
    assert int(ex(torch.tensor([5])).item()) == 107 and int(ex.pos.item()) == 112


def test_two_rank_replay_exchange_matches_one_stream(tmp_path):
    """SURVEY §8(e) collective 3 over gloo: two ranks, each placing its shard's draws
    at the base the all-gather of per-rank totals gives it, reproduce the single
    process stepping every env from one stream in global env order (the reference's
    order, training/ppo.py:436-452) -- boards and the final stream position."""
    import torch.multiprocessing as mp
    _paths()
    from safelife_amd import dist as sdist
    port = _free_port()
    mp.start_processes(_replay_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    ref, ref_pos = _replay_envs(range(WORLD * ENVS_PER_RANK), WORLD * ENVS_PER_RANK,
                                sdist.StreamExchange())
    got = [np.load(os.path.join(str(tmp_path), "replay%d.npz" % r)) for r in range(WORLD)]
    assert np.array_equal(np.concatenate([g["boards"] for g in got]), ref)
    assert all(int(g["pos"]) == ref_pos for g in got) and ref_pos > 0
