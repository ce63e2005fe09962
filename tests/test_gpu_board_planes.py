"""The 128x128 board kept in bit planes (sl_env_state.board_planes, round 5).

A Philox step of the fast kernel without views or capture keeps the board in planes
and writes only the band-edge rows of the uint16 board; every reader completes it
first (SafeLifeVecEnv.board, sl_env_obs, the game-level entry points).  These tests
run one batch with planes and one without side by side from the same seed and require
identical outputs, through the transitions: into plane mode after resets, board reads
between plane steps (uint16 complete, planes still authoritative), observations, a
step with views (back to the uint16 board), set_state.  The planes themselves are
checked against the completed board.  The C5 every-env and bench-regime tests
(test_gpu_headline.py, test_gpu_bench_regime.py) run the plane path against the
oracle at full batch.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
POOLS = os.path.join(os.path.dirname(__file__), "golden", "pools")
C5 = os.path.join(POOLS, "c5_navigation_128.npz")


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    import safelife_amd  # noqa: F401
    return torch, torch.device("cuda:0")


def _pair(torch_dev, B, seed, tl):
    from safelife_amd import SafeLifeVecEnv, LevelPool
    torch, dev = torch_dev
    kw = dict(time_limit=tl, view_shape=(33, 33), penalty_coef=1.0, min_performance=0.01,
              rng="philox", seed=seed, level_order="random", augment_roll=True,
              kernel="fast", compute_obs=False, board_mode="planes")
    a = SafeLifeVecEnv(LevelPool.load(C5), B, dev, **kw)
    b = SafeLifeVecEnv(LevelPool.load(C5), B, dev, **kw)
    b._state.board_planes = None         # the uint16-only form
    b.board_planes = None
    a.reset()
    b.reset()
    assert a.board_planes is not None
    return a, b


def _host_planes(board):
    """[128, 128] uint16 -> [4, 32, 64] uint32 in board_planes' layout: word k of
    lane j in band t holds bit k & 15 of column 2 j + (k >> 4), rows 32 t + r at bit r."""
    b = board.astype(np.uint32).reshape(4, 32, 64, 2)          # [t, r, j, q]
    out = np.zeros((4, 32, 64), np.uint64)
    sh = np.arange(32, dtype=np.uint64)[None, :, None]
    for k in range(32):
        bits = ((b[:, :, :, k >> 4] >> (k & 15)) & 1).astype(np.uint64)
        out[:, k, :] = (bits << sh).sum(axis=1)
    return out.astype(np.uint32)


def _same_state(a, b, ctx):
    assert np.array_equal(a.board.cpu().numpy(), b.board.cpu().numpy()), ctx
    assert np.array_equal(a.goals.cpu().numpy(), b.goals.cpu().numpy()), ctx
    for k in a.st_t:
        assert np.array_equal(a.st_t[k].cpu().numpy(), b.st_t[k].cpu().numpy()), (ctx, k)


def test_plane_mode_matches_uint16_mode(torch_dev):
    torch, dev = torch_dev
    B, T = 512, 48
    a, b = _pair(torch_dev, B, seed=99, tl=12)
    rng = np.random.RandomState(5)
    obs_a = torch.zeros_like(a.obs)
    obs_b = torch.zeros_like(b.obs)
    n_done = 0
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
        n_done += int(b.done.sum().item())
        if t % 7 == 3:             # a read between plane steps
            _same_state(a, b, t)
        if t == 10:
            assert torch.equal(a.observe(), b.observe()), t
        if t == 30:                # explicit state: the next step goes into plane mode
            a.set_state(b.board.cpu().numpy(), b.goals.cpu().numpy(),
                        b.start_board.cpu().numpy())
            b.set_state(b.board.cpu().numpy(), b.goals.cpu().numpy(),
                        b.start_board.cpu().numpy())
    assert n_done >= B
    _same_state(a, b, "end")
    # the planes are the board (envs whose board lives in planes)
    pok = a.planes_ok.cpu().numpy()
    assert ((pok & 64) != 0).sum() > B // 2
    bd = a.board.cpu().numpy()
    bp = a.board_planes.cpu().numpy().view(np.uint32)
    for e in np.nonzero(pok & 64)[0][:64]:
        hp, dp = _host_planes(bd[e]), bp[e].copy()
        # an exit's colour is kept in the uint16 cell only (nothing reads it from planes)
        for y, x in zip(*np.nonzero(bd[e] & 0x100)):
            k = 9 + 16 * (x & 1)
            hp[y >> 5, k, x >> 1] &= ~np.uint32(1 << (y & 31))
            dp[y >> 5, k, x >> 1] &= ~np.uint32(1 << (y & 31))
        assert np.array_equal(dp, hp), e


def test_plane_mode_full_batch_reads_only_at_end(torch_dev):
    """65 536 envs, 20 steps of plane mode with no read in between (every env crosses
    an episode end): the same as the uint16 form, outputs every step, state at the end."""
    torch, dev = torch_dev
    B, T = 65536, 20
    a, b = _pair(torch_dev, B, seed=7, tl=8)
    rng = np.random.RandomState(9)
    for t in range(T):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        a.step_async(acts)
        b.step_async(acts)
        assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), t
    _same_state(a, b, "end")


def test_game_entries_complete_the_board(torch_dev):
    """The game-level entry points on a batch kept in planes read and write the
    completed board: sl_env_rescore's points equal the uint16 form's."""
    import ctypes
    from safelife_amd import _lib
    torch, dev = torch_dev
    B = 64
    a, b = _pair(torch_dev, B, seed=3, tl=50)
    rng = np.random.RandomState(2)
    for t in range(6):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        a.step_async(acts)
        b.step_async(acts)
    L = _lib.lib()
    pa = torch.zeros(B, dtype=torch.int32, device=dev)
    pb = torch.zeros(B, dtype=torch.int32, device=dev)
    # through the C entry directly (no Python-side sync first)
    _lib.check(L.sl_env_rescore(ctypes.byref(a._state), pa.data_ptr(), _lib.stream_ptr(dev)),
               "sl_env_rescore")
    _lib.check(L.sl_env_rescore(ctypes.byref(b._state), pb.data_ptr(), _lib.stream_ptr(dev)),
               "sl_env_rescore")
    assert torch.equal(pa, pb)
    assert torch.equal(a._board, b.board)   # (the entry completed it, before any read)


def test_plane_mode_across_pool_swaps_and_state_dict(torch_dev):
    """set_pool / PoolFeeder.swap between plane steps, then
    venv.board and state_dict() read straight after the swap (before any step), must
    be the uint16-only form's; a checkpoint taken there restores it, and both run on
    identically for 20 more steps (file_finder.py:143-201 is the reference's reset
    source; safelife_env.py:177-185 the board a caller sees after each step)."""
    torch, dev = torch_dev
    from safelife_amd import LevelPool
    from safelife_amd.pool_feed import PoolFeeder, npz_level_source
    B = 256
    a, b = _pair(torch_dev, B, seed=21, tl=15)
    full = LevelPool.load(C5)
    order2, order3 = [2, 3, 0, 1], [3, 1, 0, 2]
    lv = list(npz_level_source(C5, repeat=False))
    feeder = PoolFeeder((lv[i] for i in order2), pool_size=4, device=dev)
    rng = np.random.RandomState(13)
    try:
        for t in range(62):
            if t == 20:                # the feeder's swap vs a synchronous set_pool
                assert feeder.swap(a, block=True, timeout=60)
                b.set_pool(full.subset(order2))
                assert ((a.planes_ok & 64) != 0).any()      # boards in planes
                _same_state(a, b, "after swap")
            if t == 41:                # state_dict first, with no board read before it
                a.set_pool(full.subset(order3))
                b.set_pool(full.subset(order3))
                assert ((a.planes_ok & 64) != 0).any()
                da, db = a.state_dict(), b.state_dict()
                for k in db:
                    if k != "step_index":
                        assert torch.equal(da[k], db[k]), k
                a.load_state_dict(da)
                b.load_state_dict(db)
            acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
            a.step_async(acts)
            b.step_async(acts)
            for x, y in ((a.reward, b.reward), (a.done, b.done), (a.flags, b.flags)):
                assert torch.equal(x, y), t
        assert feeder.swaps == 1
        _same_state(a, b, "end")
    finally:
        feeder.close()


@pytest.mark.parametrize("view,rw", [((33, 33), True), ((15, 15), False), ((96, 40), True),
                                     ((1, 128), True), ((97, 33), True), ((34, 7), False)])
def test_plane_mode_views_match_uint16_views(torch_dev, view, rw):
    """Packed views written by the 128x128 step kernel from the board planes (round 6:
    views of at most 96 rows keep the batch in plane mode; get_obs,
    safelife_env.py:125-155, recenter_view, helper_utils.py:41-74) equal those of the
    uint16-only form, every step, through resets (the reset envs' views come from the
    reset list's obs kernel) and exits moved to the view's edge; a 97-row view takes
    the unfused path.  Boards and scalars stay equal too."""
    from safelife_amd import SafeLifeVecEnv, LevelPool
    torch, dev = torch_dev
    B, T = 384, 40
    kw = dict(time_limit=11, view_shape=view, penalty_coef=1.0, min_performance=0.01,
              rng="philox", seed=5, level_order="random", augment_roll=True, kernel="fast",
              output_channels=None, remove_white_goals=rw, board_mode="planes")
    a = SafeLifeVecEnv(LevelPool.load(C5), B, dev, **kw)
    b = SafeLifeVecEnv(LevelPool.load(C5), B, dev, **kw)
    b._state.board_planes = None
    b.board_planes = None
    oa, ob = a.reset(), b.reset()
    assert torch.equal(oa, ob)
    rng = np.random.RandomState(8)
    fused = view[0] <= 96
    for t in range(T):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        oa, ra, da, _ = a.step(acts)
        ob, rb, db, _ = b.step(acts)
        assert torch.equal(ra, rb) and torch.equal(da, db), t
        assert torch.equal(oa, ob), (t, int((oa != ob).flatten(1).any(1).sum()))
        if t == 20:
            _same_state(a, b, t)
        if t >= 2:      # the boards stay in planes when the view is fused (bar resets)
            inp = int(((a.planes_ok & 64) != 0).sum().item())
            nres = int(((a.flags & 4) != 0).sum().item())
            assert (inp + nres > B // 2) if fused else inp == 0, (t, inp, nres)
    _same_state(a, b, "end")


def test_board_mode_auto_follows_reads(torch_dev):
    """board_mode="auto": a batch whose board is read after every step runs the kernel
    that writes the uint16 board (no env left in planes, so a read costs no sync); once
    the reads stop it goes back into plane mode.  Every output equals the uint16-only
    form's throughout."""
    from safelife_amd import SafeLifeVecEnv, LevelPool
    torch, dev = torch_dev
    B = 256
    kw = dict(time_limit=13, view_shape=(33, 33), penalty_coef=1.0, min_performance=0.01,
              rng="philox", seed=17, level_order="random", augment_roll=True, kernel="fast",
              output_channels=None)
    a = SafeLifeVecEnv(LevelPool.load(C5), B, dev, board_mode="auto", **kw)
    b = SafeLifeVecEnv(LevelPool.load(C5), B, dev, board_mode="uint16", **kw)
    a.reset()
    b.reset()
    rng = np.random.RandomState(3)
    for t in range(36):
        acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
        oa, ra, da, _ = a.step(acts)
        ob, rb, db, _ = b.step(acts)
        assert torch.equal(ra, rb) and torch.equal(da, db) and torch.equal(oa, ob), t
        inp = int(((a.planes_ok & 64) != 0).sum().item())
        assert int(((b.planes_ok & 64) != 0).sum().item()) == 0
        if t < 12:                    # no reads yet: plane mode
            assert inp > B // 2, t
        elif t < 24:                  # reads after every step: the uint16 kernel
            if t >= 13:
                assert inp == 0, t
            assert torch.equal(a.board, b.board), t
        elif t >= 24 + a.BOARD_READ_WINDOW + 1:
            assert inp > B // 2, t    # back in planes
    _same_state(a, b, "end")
