"""npz_level_source: the static-level half of the reference's safelife_loader
(file_finder.py:78-201) -- files, globs, directories, stacked pools; repeat and
shuffle.  Host only."""
import os

import numpy as np
import pytest

from safelife_amd.pool_feed import npz_level_source
from safelife_amd.levels import LevelPool

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_single_files_glob_and_directory():
    files = sorted(os.path.join(GOLDEN, "levels", f)
                   for f in os.listdir(os.path.join(GOLDEN, "levels")))
    once = list(npz_level_source(os.path.join(GOLDEN, "levels", "append-still-*.npz"),
                                 repeat=False))
    assert len(once) == len(files) == 4
    for lv, f in zip(once, files):
        with np.load(f) as d:
            assert np.array_equal(lv["board"], d["board"])
    assert len(list(npz_level_source(os.path.join(GOLDEN, "levels"), repeat=False))) == 4
    # the extension may be omitted, as file_finder.find_files allows
    assert len(list(npz_level_source(files[0][:-4], repeat=False))) == 1
    with pytest.raises(FileNotFoundError):
        list(npz_level_source(os.path.join(GOLDEN, "nope")))


def test_stacked_pool_repeat_and_shuffle():
    path = os.path.join(GOLDEN, "pools", "c2_append_still_25.npz")
    K = np.load(path)["board"].shape[0]
    three = list(npz_level_source(path, repeat=3))
    assert len(three) == 3 * K
    assert all(np.array_equal(a["board"], b["board"]) for a, b in zip(three[:K], three[K:2 * K]))
    src = npz_level_source(path, repeat=True, shuffle=True, seed=5)
    first = [next(src)["board"] for _ in range(2 * K)]
    # every pass is a permutation of the pool, and the passes differ
    ref = sorted(np.load(path)["board"].reshape(K, -1).tolist())
    assert sorted(b.reshape(-1).tolist() for b in first[:K]) == ref
    assert any(not np.array_equal(a, b) for a, b in zip(first[:K], first[K:]))
    pool = LevelPool.from_levels(three[:K])
    assert pool.K == K


def test_levels_archive(tmp_path):
    """a structured `levels` archive (the v1.0 benchmark format, file_finder.py:89-93)"""
    path = os.path.join(GOLDEN, "pools", "c2_append_still_25.npz")
    d = np.load(path)
    K, H, W = d["board"].shape
    dt = np.dtype([("name", "U8"), ("board", np.uint16, (H, W)), ("goals", np.uint16, (H, W)),
                   ("agent_loc", np.int64, (2,)), ("orientation", np.int64),
                   ("spawn_prob", np.float64), ("min_performance", np.float64)])
    arr = np.zeros(3, dt)
    for i in range(3):
        arr[i] = ("l%d" % i, d["board"][i], d["goals"][i], d["agent_loc"][i],
                  d["orientation"][i], d["spawn_prob"][i], d["min_performance"][i])
    np.savez(tmp_path / "archive.npz", levels=arr)
    lv = list(npz_level_source(str(tmp_path / "archive.npz"), repeat=False))
    assert len(lv) == 3 and np.array_equal(lv[2]["goals"], d["goals"][2])
    assert LevelPool.from_levels(lv).K == 3


def test_level_pool_exit_cap():
    """Documented divergence: the device state keeps at most SL_MAX_EXITS exit cells
    per env (their positions for the observation and the exit recolouring); levels
    with more are rejected when the pool is built, not silently truncated (the
    reference's update_exit_colors, safelife_game.py:528-537, has no cap)."""
    from safelife_amd import _lib
    K, H, W = 1, 16, 16
    board = np.zeros((K, H, W), np.uint16)
    goals = np.zeros_like(board)
    ys, xs = np.divmod(np.arange(_lib.SL_MAX_EXITS) * 3 + 20, W)
    board[0, ys, xs] = 272                                  # level exits
    LevelPool(board, goals, [(0, 0)], [0], [0.3], [0.01])   # at the cap: accepted
    board[0, 15, 15] = 272
    with pytest.raises(ValueError, match="exits"):
        LevelPool(board, goals, [(0, 0)], [0], [0.3], [0.01])


def test_start_board_hi_bits_and_pool_cell_bits():
    """spawn_flags bit 2's host side (start boards using the unused cell bits 12-14) and
    what the 128x128 kernel's bit-2 / bit-3 paths assume of the benchmark pools: no
    level uses bits 12-14, and the C5 goals use only alive, destructible, frozen and
    colour bits (the goal plane mirror's 0x0E19) and hold no spawner."""
    import torch
    from safelife_amd.vec_env import start_board_hi_bits
    sb = torch.zeros((3, 8, 8), dtype=torch.int16)       # the uint16 boards' bits
    sb[1, 2, 3] = 0x1010
    sb[2, 7, 7] = -0x7FF0          # 0x8010: the pullable bit, not 12-14
    assert start_board_hi_bits(sb).tolist() == [False, True, False]
    pools = os.path.join(os.path.dirname(__file__), "golden", "pools")
    for name in ("c2_append_still_25", "c3_prune_still_64", "c4_append_still_64",
                 "c5_navigation_128"):
        p = LevelPool.load(os.path.join(pools, name + ".npz"))
        assert not ((p.board & 0x7000) != 0).any(), name
    c5 = LevelPool.load(os.path.join(pools, "c5_navigation_128.npz"))
    assert not (c5.goals & ~np.uint16(0x0E19)).any()
