"""The reference's seeded spawn stream generated on the device (csrc/sl_mt.hip,
safelife_amd.mtstream), against numpy's RandomState itself.

After speedups.seed(s) the reference draws every spawn uniform from numpy's global
RandomState(s) (speedups_src/random.c:14-52, module.c:246-253): the stream is
np.random.RandomState(s).random_sample.  Checked here:
  * the ring against numpy over consecutive fills of step-like sizes, and after seeks
    far into the stream (there against the host jump, itself checked against numpy in
    tests/test_mt_cpu.py);
  * G2 (tests/golden/advance_stream.npz, captured from the reference) and the golden
    trajectories replayed from their seed alone -- no host stream;
  * C5 at full batch (65 536 x 128x128, bench.py's regime, no rewind): the sampled envs'
    slices of the generated stream are numpy's own draws at the device's offsets, and
    the oracle fed those draws stays bit-exact.
"""
import os

import numpy as np
import pytest

import oracle
from test_gpu_bench_regime import (CONFIGS, KW, POOLS, SEED, _OffsetStream, _oracle_levels,
                                   _sample)
from test_gpu_headline import _env_state, torch_dev  # noqa: F401
from test_gpu_parity import _traj_files, _vec_env_from_traj

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


def _ring_slice(torch, mt, lo, hi):
    return mt.ring_slice(lo, hi).cpu().numpy()


@pytest.mark.parametrize("lookahead", [False, True])
@pytest.mark.parametrize("rounds,n_chains,ring,bits", [(33, 16, 1 << 21, None),
                                                       (420, 64, 1 << 24, None),
                                                       (36, 16, 1 << 21, 0.3),
                                                       (1684, 8, 1 << 24, 0.3),
                                                       (420, 64, 1 << 24, 0.30000001192092896),
                                                       (33, None, 1 << 21, None),
                                                       (36, None, 1 << 21, 0.3)])
def test_fill_matches_numpy(torch_dev, rounds, n_chains, ring, bits, lookahead):
    """Consecutive ranges, as replay steps consume the stream: empty, single draws,
    block-sized and multi-block ranges, all equal to RandomState(s).random_sample --
    also with the look-ahead generating each next range's blocks on a second stream
    while the test reads (and rewrites its range tensor for) the current one.  A bit
    ring holds draw < threshold for every draw.  n_chains None: sized by
    MT19937Stream (the chains cover the ring and a block), which with the look-ahead
    puts the chains' jumps on their own stream (sl_mt19937.jump_stream)."""
    torch, dev = torch_dev
    from safelife_amd.mtstream import MT19937Stream
    mt = MT19937Stream(2024, dev, ring_draws=ring, n_chains=n_chains, rounds=rounds,
                       lookahead=lookahead, bits_threshold=bits)
    D = mt.block
    n_chains = mt.n_chains
    ref = np.random.RandomState(2024).random_sample(6 * n_chains * D)
    if bits is not None:
        ref = ref < bits
    rng = np.random.RandomState(0)
    lohi = torch.zeros(2, dtype=torch.int64, device=dev)
    pos, n_fills = 0, 0
    sizes = [0, 1, 7, D - 1, D, D + 1, 3 * D + 17, min((n_chains - 2) * D, ring - 2 * D)]
    while pos + (n_chains - 1) * D < len(ref):
        n = int(sizes[rng.randint(len(sizes))])
        lohi[0], lohi[1] = pos, pos + n
        mt.fill(lohi[0:1], lohi[1:2])
        assert np.array_equal(_ring_slice(torch, mt, pos, pos + n), ref[pos:pos + n]), (pos, n)
        pos += n
        n_fills += 1
    assert n_fills > 10 and not mt.error()


def test_seek_far_into_the_stream(torch_dev):
    from safelife_amd.mtstream import MT19937Stream, host_window, host_jump, host_jump_poly, \
        host_draws
    torch, dev = torch_dev
    mt = MT19937Stream(77, dev, ring_draws=1 << 22, n_chains=32)
    near = 7_777_777
    mt.seek(near)
    got = mt.draws(near, 250_000).cpu().numpy()
    assert np.array_equal(got, np.random.RandomState(77).random_sample(near + 250_000)[near:])
    for far in (3 * 10 ** 9 + 12345, (1 << 36) + 3):
        mt.seek(far)
        ref = host_draws(host_jump(host_window(77), host_jump_poly(2 * far)), 200_000)
        assert np.array_equal(mt.draws(far, 200_000).cpu().numpy(), ref), far
    # a rewound position is refused (flagged), not silently served stale
    lohi = torch.tensor([0, 10], dtype=torch.int64, device=dev)
    mt.fill(lohi[0:1], lohi[1:2])
    assert mt.error()


def test_g2_reproduced_from_seed_alone(torch_dev):
    """G2 (spawner boards advanced 50 times after speedups.seed(s), captured from the
    reference): the same boards from the device generator seeded with s, each
    advance taking its draws at the running stream position (board, then goals)."""
    torch, dev = torch_dev
    from safelife_amd import speedups
    from safelife_amd.mtstream import MT19937Stream
    d = np.load(os.path.join(GOLDEN, "advance_stream.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    assert len(keys) >= 12
    n_draws = 0
    for key in keys:
        s = int(key.split("_")[0][1:])
        mt = MT19937Stream(s, dev, ring_draws=1 << 20, n_chains=4, rounds=33)
        bg = torch.from_numpy(np.stack([d[key + "_board0"], d[key + "_goals0"]])).to(dev)
        pos = 0
        for t in range(d[key + "_boards"].shape[0]):
            nb, ng = (int(c) for c in speedups.count_eligible(bg).cpu().numpy())
            draws = mt.draws(pos, max(nb + ng, 1))
            offs = torch.tensor([0, nb], dtype=torch.int64, device=dev)
            bg = speedups.advance_boards(bg, 0.3, rng="stream", draws=draws, draw_offsets=offs)
            pos += nb + ng
            out = bg.cpu().numpy()
            assert np.array_equal(out[0], d[key + "_boards"][t]), (key, t)
            assert np.array_equal(out[1], d[key + "_goals"][t]), (key, t)
        n_draws += pos
    assert n_draws > 0


@pytest.mark.parametrize("ring,kernel", [("auto", "fast"), ("doubles", "fast"),
                                         ("auto", "generic")])
@pytest.mark.parametrize("path", _traj_files(), ids=lambda p: os.path.basename(p)[5:-4])
def test_golden_trajectory_from_seed_alone(torch_dev, path, ring, kernel):
    """The reference-captured PPO-chain trajectories (speedups.seed(cfg seed), then
    1 100 env steps) through the bit-sliced (and the per-cell) kernels with the spawn
    stream generated on the device inside each step: boards, goals, rewards, views
    bit-exact.  One level, one spawn probability: a bit ring ("auto"), and a ring of
    doubles."""
    torch, dev = torch_dev
    d = np.load(path)
    seed = int(d["cfg"][2])
    env = _vec_env_from_traj(d, kernel=kernel, spawn_stream=None, seed=seed, stream_ring=ring)
    assert env.mt is not None
    assert (env.mt.bits_threshold is not None) == (ring == "auto")
    obs = env.reset().cpu().numpy()
    assert np.array_equal(obs[0], d["obs0"])
    actions = torch.from_numpy(d["action"].astype(np.int32)).to(dev)
    for t in range(len(d["action"])):
        obs, r, done, info = env.step(actions[t:t + 1])
        ctx = (os.path.basename(path), t)
        assert r.item() == d["reward"][t], ctx
        assert bool(done.item()) == bool(d["done"][t]), ctx
        assert np.array_equal(env.board[0].cpu().numpy(), d["board"][t]), ctx
        assert np.array_equal(env.goals[0].cpu().numpy(), d["goals"][t]), ctx
        assert np.array_equal(obs[0].cpu().numpy(), d["obs"][t]), ctx
    assert not env.stream_error()


@pytest.mark.parametrize("name", ["traj_nav128_c5.npz", "traj_prune_spawn_v10.npz"])
def test_bit_ring_flags_a_foreign_threshold(torch_dev, name):
    """A bit ring holds decisions for one threshold: an env that draws with another one
    (spawn_prob written behind the env's back) sets SL_STREAM_ERR_THRESHOLD -- on 128x128
    boards from the count prologue itself, elsewhere from k_bits_thr_check -- and the
    poll raises; the flag stays clear while the threshold is the ring's."""
    from safelife_amd import _lib
    torch, dev = torch_dev
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", name))
    env = _vec_env_from_traj(d, B=4, kernel="fast", spawn_stream=None, seed=int(d["cfg"][2]),
                             stream_ring="auto")
    assert env.mt is not None and env.mt.bits_threshold is not None
    env.reset()
    acts = torch.from_numpy(d["action"][:40].astype(np.int32)).to(dev)
    for t in range(20):
        env.step_async(acts[t].repeat(4))
    assert not env.stream_error()
    env.st_t["spawn_prob"][2] = 0.25          # (not through set_state: the ring is kept)
    drew = False
    for t in range(20, 40):
        env.step_async(acts[t].repeat(4))
        drew = drew or bool(env.scratch[2 * 2:2 * 2 + 2].sum().item())     # env 2's counts
    flag = int(env.scratch[8 * env.B].item())
    if drew:
        assert flag & _lib.SL_STREAM_ERR_THRESHOLD, flag
        with pytest.raises(RuntimeError, match="spawn threshold"):
            env._raise_stream_error(flag)
    else:
        assert flag == 0


class _NumpyStream:
    """RandomState(seed).random_sample, extended on demand (slices as torch tensors)."""

    def __init__(self, torch, seed):
        self.torch, self.rs, self.a = torch, np.random.RandomState(seed), np.zeros(0)

    def __getitem__(self, sl):
        if sl.stop > len(self.a):
            self.a = np.concatenate([self.a, self.rs.random_sample(sl.stop - len(self.a))])
        return self.torch.from_numpy(self.a[sl])


class _HostJumpStream:
    """RandomState(seed).random_sample at any position, from the host's own jump-ahead
    (host_window / host_jump_poly / host_jump / host_draws, checked against numpy
    itself in tests/test_mt_cpu.py): independent of the device ring.  Each request
    jumps to its start and generates a chunk, so an env's board slice and the goals
    slice after it cost one jump."""

    def __init__(self, torch, seed, chunk=16384):
        from safelife_amd.mtstream import host_window
        self.torch, self.win, self.chunk = torch, host_window(seed), chunk
        self.lo, self.a = 0, np.zeros(0)
        self.jumps = 0

    def __getitem__(self, sl):
        from safelife_amd.mtstream import host_jump, host_jump_poly, host_draws
        lo, hi = sl.start, sl.stop
        if not (self.lo <= lo and hi <= self.lo + len(self.a)):
            w = host_jump(self.win, host_jump_poly(2 * lo))
            self.lo, self.a = lo, host_draws(w, max(hi - lo, self.chunk))
            self.jumps += 1
        return self.torch.from_numpy(self.a[lo - self.lo:hi - self.lo])


def _seeded_steps(torch, dev, venv, oenvs, ostreams, sample, T, rng):
    B = venv.B
    n_reset = 0
    for t in range(T):
        acts = rng.randint(0, 9, size=B).astype(np.int32)
        _, vr, vd, info = venv.step(torch.from_numpy(acts).to(dev))
        rs = info["reset"].cpu().numpy()
        vr, vd = vr.cpu().numpy(), vd.cpu().numpy()
        offs = venv.scratch[2 * B:4 * B].cpu().numpy()
        end = int(venv.stream_pos.item())
        nxt = lambda k: int(offs[k]) if k < 2 * B else end          # noqa: E731
        for e in sample:
            ostreams[e].arm(int(offs[2 * e]), int(offs[2 * e + 1]), nxt(2 * e + 2))
        for e in sample:
            _, r, dn, _ = oenvs[e].step(int(acts[e]))
            n_reset += int(rs[e])
            assert vr[e] == r, (t, e)
            assert bool(vd[e]) == dn, (t, e)
            assert np.array_equal(venv.board[e].cpu().numpy(), oenvs[e].board), (t, e)
            assert np.array_equal(venv.goals[e].cpu().numpy(), oenvs[e].goals), (t, e)
            assert not ostreams[e].bounds, (t, e)
    return n_reset


def test_seeded_replay_c5_full_batch_vs_numpy(torch_dev):
    """C5 at full batch with the stream generated on the device (what bench.py
    --rng seeded times; no rewind, no host buffer): for the first steps the sampled
    envs' oracles draw from numpy's own RandomState(SEED).random_sample at the device's
    offsets; after 120 more steps (positions ~10^9) from the host's own jump-ahead to
    each env's offsets -- never from the device ring -- for 31 steps, so every sampled
    env's whole slice of every late step is the host's stream, and the ring's copy of
    each slice equals it too."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    fname, B = CONFIGS["c5"]
    pool = LevelPool.load(os.path.join(POOLS, fname))
    venv = SafeLifeVecEnv(pool, B, dev, rng="stream", spawn_stream=None, seed=SEED,
                          level_order="random", augment_roll=True, kernel="fast",
                          compute_obs=False, **KW)
    venv.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    venv.st_t["episode_length"].copy_(torch.randint(0, KW["time_limit"], (B,), device=dev,
                                                    generator=g, dtype=torch.int32))
    levels = _oracle_levels(pool)

    def oracles(stream):
        sample = _sample(venv)
        oenvs, ostreams = {}, {}
        for e in sample:
            ostreams[e] = _OffsetStream(stream)
            o = oracle.OracleEnv(oracle.pool_level_fn(levels, e, seed=SEED, random_order=True,
                                                      augment=True),
                                 env_id=e, rng="stream", seed=SEED, stream=ostreams[e], **KW)
            o.load_state(_env_state(venv, e), venv._step_index)
            oenvs[e] = o
        return sample, oenvs, ostreams

    rng = np.random.RandomState(6)
    sample, oenvs, ostreams = oracles(_NumpyStream(torch, SEED))
    _seeded_steps(torch, dev, venv, oenvs, ostreams, sample, 2, rng)
    for _ in range(120):
        venv.step_async(torch.randint(0, 9, (B,), dtype=torch.int32, device=dev, generator=g))
    pos0 = int(venv.stream_pos.item())
    assert pos0 > 10 ** 9
    host = _HostJumpStream(torch, SEED)
    sample, oenvs, ostreams = oracles(host)
    n_reset = 0
    n_drawn = 0
    for t in range(31):
        n_reset += _seeded_steps(torch, dev, venv, oenvs, ostreams, sample, 1, rng)
        # each sampled env's slice of this step (board then goals), as the ring holds it
        offs = venv.scratch[2 * B:4 * B].cpu().numpy()
        end = int(venv.stream_pos.item())
        for e in sample:
            lo = int(offs[2 * e])
            hi = int(offs[2 * e + 2]) if 2 * e + 2 < 2 * B else end
            if hi > lo:
                want = host[lo:hi].numpy()
                if venv.mt.bits_threshold is not None:      # C5's one p: a bit ring
                    want = want < venv.mt.bits_threshold
                assert np.array_equal(_ring_slice(torch, venv.mt, lo, hi), want), (t, e)
                n_drawn += hi - lo
    assert n_reset >= 6 and n_drawn > 10000 and host.jumps >= 31
    assert venv.mt.bits_threshold == float(np.float32(0.3))
    assert not venv.stream_error()


@pytest.mark.parametrize("ring", ["bits", "doubles"])
def test_seeded_shards_equal_one_seeded_run(torch_dev, ring):
    """Parity mode over shards with the device generator: two shard envs, each with
    its own MT19937 stream from the same seed and no look-ahead, placed by one
    StreamExchange (each rank fills only its slice [base, base + total) of the
    global stream: csrc/sl_mt.hip), reproduce one seeded 64-env C5 run bit for bit --
    rewards, done flags, boards, goals and the stream position.  C5's levels share one
    spawn probability (a bit ring); with one level's changed, rings of doubles."""
    torch, dev = torch_dev
    from safelife_amd import SafeLifeVecEnv, LevelPool
    from safelife_amd import dist as sdist
    fname, _ = CONFIGS["c5"]
    pool = LevelPool.load(os.path.join(POOLS, fname))
    if ring == "doubles":
        pool.spawn_prob[1] = 0.25
    B = 64
    kw = dict(KW, time_limit=25, level_order="random", augment_roll=True, seed=31,
              spawn_stream=None, rng="stream", kernel="fast", compute_obs=False)
    whole = SafeLifeVecEnv(pool, B, dev, **kw)
    ex = sdist.StreamExchange(device=dev)
    shards = [SafeLifeVecEnv(pool, B // 2, dev, env0=r * (B // 2), n_total_envs=B,
                             stream_exchange=ex, **kw) for r in range(2)]
    assert whole.mt is not None and all(s.mt is not None for s in shards)
    assert (whole.mt.bits_threshold is not None) == (ring == "bits")
    whole.reset()
    for s in shards:
        s.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    for t in range(60):
        a = torch.randint(0, 9, (B,), dtype=torch.int32, device=dev, generator=g)
        _, r, d, _ = whole.step(a)
        outs = [s.step(a[i * (B // 2):(i + 1) * (B // 2)]) for i, s in enumerate(shards)]
        assert torch.equal(r, torch.cat([o[1] for o in outs])), t
        assert torch.equal(d, torch.cat([o[2] for o in outs])), t
        assert int(whole.stream_pos.item()) == int(ex.pos.item()), t
        if t % 6 == 5:
            assert torch.equal(whole.board, torch.cat([s.board for s in shards])), t
            assert torch.equal(whole.goals, torch.cat([s.goals for s in shards])), t
    assert int(ex.pos.item()) > 100000
    assert not whole.stream_error() and not any(s.stream_error() for s in shards)
