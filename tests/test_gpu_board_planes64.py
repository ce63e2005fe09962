"""The 64x64 board kept in bit planes (round 6; sl_bits.hip k_env_step_bits64_planes).

A Philox step without views or capture keeps the board in half 0 of the goals
mirror, skips the planes no board of the batch can hold (sl_env_state.board_zero; on
the C3 / C4 levels cell bits 7 and 11-14), stores only the plane words that changed,
and leaves the uint16 board stale (a read completes it).  One batch in plane
mode and one in the uint16-only form run side by side from the same seed; every
output must be equal at every step, through resets, board reads between plane steps,
steps with views (back to the uint16 board), set_state, the game-level C entries and
levels whose spawners and colours make planes appear and vanish.  The C3 every-env
test (test_gpu_headline.py) and the bench-regime tests run the plane path against the
oracle at full batch.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
POOLS = os.path.join(os.path.dirname(__file__), "golden", "pools")
C3 = os.path.join(POOLS, "c3_prune_still_64.npz")
C4 = os.path.join(POOLS, "c4_append_still_64.npz")


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    import safelife_amd  # noqa: F401
    return torch, torch.device("cuda:0")


def _spawner_pool():
    """The C3 levels with spawners, blue cells and pushable / pullable blocks sprinkled in
    (planes 2, 7, 11, 15 come and go; the zero-plane mask must follow)."""
    from safelife_amd import LevelPool
    p = LevelPool.load(C3)
    rng = np.random.RandomState(4)
    b = p.board.copy()
    for k in range(p.K):
        ay, ax = p.agent_y[k], p.agent_x[k]
        free = (b[k] == 0)
        free[max(ay - 3, 0):ay + 4, max(ax - 3, 0):ax + 4] = False
        ys, xs = np.nonzero(free)
        pick = rng.choice(len(ys), size=min(40, len(ys)), replace=False)
        for n, i in enumerate(pick):
            kind = n % 4
            b[k, ys[i], xs[i]] = (152 | (3 << 9) if kind == 0 else      # spawner, blue-ish
                                  1 | 8 | (4 << 9) if kind == 1 else    # alive blue life
                                  4 if kind == 2 else 0x8000 | 16)      # pushable / pullable
    return LevelPool(b, p.goals, np.stack([p.agent_x, p.agent_y], 1), p.orientation,
                     p.spawn_prob, p.min_performance)


def _pair(torch_dev, pool, B, seed, tl, **extra):
    from safelife_amd import SafeLifeVecEnv
    torch, dev = torch_dev
    kw = dict(time_limit=tl, view_shape=(33, 33), penalty_coef=1.0, min_performance=0.01,
              rng="philox", seed=seed, level_order="random", augment_roll=True,
              kernel="fast", compute_obs=False, output_channels=None)
    kw.update(extra)
    a = SafeLifeVecEnv(pool, B, dev, board_mode="planes", **kw)
    b = SafeLifeVecEnv(pool, B, dev, **kw)
    b._state.board_planes = None         # the uint16-only form
    b.board_planes = None
    a.reset()
    b.reset()
    assert a.board_planes is not None
    return a, b


def _same_state(a, b, ctx):
    assert np.array_equal(a.board.cpu().numpy(), b.board.cpu().numpy()), ctx
    assert np.array_equal(a.goals.cpu().numpy(), b.goals.cpu().numpy()), ctx
    for k in a.st_t:
        assert np.array_equal(a.st_t[k].cpu().numpy(), b.st_t[k].cpu().numpy()), (ctx, k)


def _host_planes64(board):
    """[64, 64] uint16 -> [32, 64] uint32: word q of lane l = plane q & 15 of column
    2 (l >> 1) + (q >> 4), rows 32 (l & 1) + r at bit r."""
    bd = board.astype(np.uint64).reshape(2, 32, 32, 2)          # [h, r, j, w]
    out = np.zeros((32, 64), np.uint64)
    sh = np.arange(32, dtype=np.uint64)[:, None]
    for q in range(32):
        bits = (bd[:, :, :, q >> 4] >> np.uint64(q & 15)) & np.uint64(1)   # [h, r, j]
        words = (bits << sh[None]).sum(axis=1)                              # [h, j]
        out[q] = words.T.reshape(64)                                        # lane 2j + h
    return out.astype(np.uint32)


def _pools():
    from safelife_amd import LevelPool
    return {"c3": lambda: LevelPool.load(C3), "c4": lambda: LevelPool.load(C4),
            "spawners": _spawner_pool}


@pytest.mark.parametrize("name", ["c3", "c4", "spawners"])
def test_plane_mode64_matches_uint16_mode(torch_dev, name):
    torch, dev = torch_dev
    B, T = 512, 48
    a, b = _pair(torch_dev, _pools()[name](), B, seed=31, tl=13)
    rng = np.random.RandomState(6)
    obs_a, obs_b = torch.zeros_like(a.obs), torch.zeros_like(b.obs)
    for t in range(T):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        if t in (17, 18):          # steps with views: the uint16 board, then back
            a.step_async(acts, obs_out=obs_a)
            b.step_async(acts, obs_out=obs_b)
            assert torch.equal(obs_a, obs_b), t
        else:
            a.step_async(acts)
            b.step_async(acts)
        for x, y in ((a.reward, b.reward), (a.done, b.done), (a.flags, b.flags),
                     (a.ep_len, b.ep_len), (a.ep_rew, b.ep_rew)):
            assert torch.equal(x, y), t
        if t % 7 == 3:             # a read between plane steps
            _same_state(a, b, t)
        if t == 10:
            assert torch.equal(a.observe(), b.observe()), t
        if t == 30:                # explicit state: the next step enters plane mode again
            a.set_state(b.board.cpu().numpy(), b.goals.cpu().numpy(),
                        b.start_board.cpu().numpy())
            b.set_state(b.board.cpu().numpy(), b.goals.cpu().numpy(),
                        b.start_board.cpu().numpy())
    # the last step was a plane step: check the planes themselves, then the board
    pok = a.planes_ok.cpu().numpy()
    bp = a.planes.cpu().numpy().view(np.uint32).reshape(B, 2, 32, 64)[:, 0]
    bd = a.board.cpu().numpy()          # (completes the uint16 board; planes unchanged)
    inp = np.nonzero(pok & 64)[0]
    assert len(inp) > B // 2
    zero = a._state.board_zero
    assert zero == (0x7880 if name != "spawners" else 0x7000), hex(zero)
    keep = ((~zero) & 0xFFFF) * 0x10001        # the kept words, packed (PlaneSlots)
    for e in inp[:96]:
        hp = _host_planes64(bd[e])
        for q in range(32):
            if (zero >> (q & 15)) & 1:
                assert not hp[q].any(), (e, q)      # a plane kept zero is zero
            else:
                pos = bin(keep & ((1 << q) - 1)).count("1")
                assert np.array_equal(bp[e, pos], hp[q]), (e, q)
    _same_state(a, b, "end")


def test_plane_mode64_pool_swap_widens_zero_planes(torch_dev):
    """set_pool with levels holding cell bits the batch never had (spawners, blue) takes
    the planes out of board_zero: the envs in planes are completed and leave plane mode
    first, and everything stays equal to the uint16 form before and after."""
    from safelife_amd import LevelPool
    torch, dev = torch_dev
    B = 384
    a, b = _pair(torch_dev, LevelPool.load(C3), B, seed=23, tl=9)
    assert a._state.board_zero == 0x7880
    rng = np.random.RandomState(12)
    sp = _spawner_pool()
    for t in range(40):
        if t == 15:
            a.set_pool(sp)
            b.set_pool(sp)
            assert a._state.board_zero == 0x7000
            assert int(((a.planes_ok & 64) != 0).sum().item()) == 0
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        a.step_async(acts)
        b.step_async(acts)
        for x, y in ((a.reward, b.reward), (a.done, b.done), (a.flags, b.flags)):
            assert torch.equal(x, y), t
        if t == 35:                # (between two rounds of resets) back in planes
            assert int(((a.planes_ok & 64) != 0).sum().item()) > B // 2
    _same_state(a, b, "end")


def test_plane_mode64_full_batch_reads_only_at_end(torch_dev):
    """65 536 C3 envs, 20 plane steps with no read in between (every env crosses an
    episode end): equal to the uint16 form, outputs every step, state at the end."""
    from safelife_amd import LevelPool
    torch, dev = torch_dev
    B, T = 65536, 20
    a, b = _pair(torch_dev, LevelPool.load(C3), B, seed=7, tl=8)
    rng = np.random.RandomState(9)
    for t in range(T):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        a.step_async(acts)
        b.step_async(acts)
        assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), t
    _same_state(a, b, "end")


def test_game_entries_complete_the_board64(torch_dev):
    """The game-level C entries on a 64x64 batch in planes: sl_env_rescore's points equal
    the uint16 form's, and the entry itself completed the board (no Python-side sync)."""
    from safelife_amd import LevelPool, _lib
    torch, dev = torch_dev
    B = 64
    a, b = _pair(torch_dev, _spawner_pool(), B, seed=3, tl=50)
    rng = np.random.RandomState(2)
    for t in range(6):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        a.step_async(acts)
        b.step_async(acts)
    assert ((a.planes_ok & 64) != 0).all()
    L = _lib.lib()
    pa = torch.zeros(B, dtype=torch.int32, device=dev)
    pb = torch.zeros(B, dtype=torch.int32, device=dev)
    _lib.check(L.sl_env_rescore(ctypes.byref(a._state), pa.data_ptr(), _lib.stream_ptr(dev)),
               "sl_env_rescore")
    _lib.check(L.sl_env_rescore(ctypes.byref(b._state), pb.data_ptr(), _lib.stream_ptr(dev)),
               "sl_env_rescore")
    assert torch.equal(pa, pb)
    assert torch.equal(a._board, b.board)


def test_plane_mode64_auto_board_mode(torch_dev):
    """board_mode="auto" at 64x64: reads after every step switch to the uint16-writing
    kernel, and the batch returns to planes when they stop; equal throughout."""
    from safelife_amd import SafeLifeVecEnv, LevelPool
    torch, dev = torch_dev
    B = 256
    kw = dict(time_limit=15, view_shape=(33, 33), penalty_coef=1.0, min_performance=0.01,
              rng="philox", seed=11, level_order="random", augment_roll=True, kernel="fast",
              output_channels=None, compute_obs=False)
    a = SafeLifeVecEnv(LevelPool.load(C4), B, dev, board_mode="auto", **kw)
    b = SafeLifeVecEnv(LevelPool.load(C4), B, dev, board_mode="uint16", **kw)
    a.reset()
    b.reset()
    rng = np.random.RandomState(3)
    for t in range(30):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        a.step_async(acts)
        b.step_async(acts)
        assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), t
        inp = int(((a.planes_ok & 64) != 0).sum().item())
        if t < 8:
            assert inp > B // 2, t
        elif t < 18:
            if t >= 9:
                assert inp == 0, t
            assert torch.equal(a.board, b.board), t
        elif t >= 18 + a.BOARD_READ_WINDOW + 1:
            assert inp > B // 2, t
    _same_state(a, b, "end")
