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
