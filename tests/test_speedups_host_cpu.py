"""speedups.advance_board on numpy boards: the host engine (csrc/sl_host.cpp through
safelife_amd/_native/_sl_host), SURVEY.md §8(b)(2)'s numpy host path.  No GPU.

Checked against the reference's own captured vectors (G1: 600 random all-bit boards,
G2: seeded spawner boards, both from tests/golden/make_golden.py) and, for what no
fixture holds -- boards up to 512 wide, spawn draws crossing the 10 000-double buffer
refill (random.c:14-26,47-52), non-uint16 input -- against the oracle's restatement
(oracle/sl_oracle.c) fed the same global numpy stream.
"""
import os

import numpy as np
import pytest

import oracle
from safelife_amd import speedups

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _oracle_seeded(boards, p, seed):
    """The oracle advancing `boards` in turn from speedups.seed(seed)'s stream."""
    rng = oracle.RefStreamRNG()
    rng.seed(seed)
    outs = []
    for b in boards:
        n = oracle.count_eligible(b)
        out, _ = oracle.advance(b, p, draws=rng.take(n), pos=0)
        outs.append(out)
    return outs


def test_g1_known_answers_through_numpy_path():
    d = np.load(os.path.join(GOLDEN, "advance_known_answers.npz"))
    o = 0
    for (H, W), p in zip(d["shapes"], d["spawn_prob"]):
        n = H * W
        b = d["boards_in"][o:o + n].reshape(H, W)
        want = d["boards_out"][o:o + n].reshape(H, W)
        o += n
        speedups.seed(0)
        got = speedups.advance_board(b, p)
        assert got.dtype == np.uint16 and got.shape == (H, W)
        assert np.array_equal(got, want), (H, W, p)


def test_g2_seeded_stream_through_numpy_path():
    d = np.load(os.path.join(GOLDEN, "advance_stream.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    assert len(keys) >= 12
    for key in keys:
        speedups.seed(int(key.split("_")[0][1:]))
        b, g = d[key + "_board0"], d[key + "_goals0"]
        for t in range(d[key + "_boards"].shape[0]):
            b = speedups.advance_board(b, 0.3)
            g = speedups.advance_board(g, 0.3)
            assert np.array_equal(b, d[key + "_boards"][t]), (key, t)
            assert np.array_equal(g, d[key + "_goals"][t]), (key, t)


def test_g1_g2_128_through_numpy_path():
    """The 128x128 fixtures (C5's board size, captured from the reference)."""
    d = np.load(os.path.join(GOLDEN, "advance_known_answers_128.npz"))
    for b, want, p in zip(d["boards_in"], d["boards_out"], d["spawn_prob"]):
        speedups.seed(1)
        assert np.array_equal(speedups.advance_board(b, p), want)
    d = np.load(os.path.join(GOLDEN, "advance_stream_128.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_board0")})
    for key in keys:
        speedups.seed(int(key.split("_")[0][1:]))
        p = float(d[key + "_p"])
        b, g = d[key + "_board0"], d[key + "_goals0"]
        for t in range(d[key + "_boards"].shape[0]):
            b = speedups.advance_board(b, p)
            g = speedups.advance_board(g, p)
            assert np.array_equal(b, d[key + "_boards"][t]), (key, t)
            assert np.array_equal(g, d[key + "_goals"][t]), (key, t)


def _spawner_soup(rng, H, W, dens=0.25):
    b = np.where(rng.rand(H, W) < dens, 9, 0).astype(np.uint16)
    b |= (rng.randint(0, 8, size=(H, W)) << 9).astype(np.uint16) * (b > 0)
    b[rng.rand(H, W) < 0.04] = 152 | (int(rng.randint(0, 8)) << 9)   # spawners
    b[rng.rand(H, W) < 0.01] = 64                                   # inhibitors
    b[rng.rand(H, W) < 0.01] = 32 | 16                              # preserving, frozen
    b[rng.rand(H, W) < 0.01] = 1 | 256                              # live exit bits
    return b


@pytest.mark.parametrize("shape", [(2, 2), (2, 7), (3, 2), (25, 25), (26, 26), (31, 63),
                                   (17, 64), (40, 65), (64, 64), (9, 127), (128, 128),
                                   (33, 200), (12, 512)])
def test_random_boards_vs_oracle_stream(shape):
    """Spawner soups of every word layout (W = 2 .. 512, one to eight 64-bit words per
    row, W = 64k and 64k + 1), several advances each from one seeded stream, so the
    draws cross the buffer refill; also all-bit boards."""
    H, W = shape
    rng = np.random.RandomState(H * 1000 + W)
    boards = [_spawner_soup(rng, H, W) for _ in range(3)]
    boards.append(rng.randint(0, 1 << 16, size=(H, W)).astype(np.uint16))
    for seed in (3, 4):
        for p in (0.3, 1.0, 0.0):
            want = _oracle_seeded(boards, p, seed)
            speedups.seed(seed)
            for b, w in zip(boards, want):
                assert np.array_equal(speedups.advance_board(b, p), w), (shape, seed, p)


def test_buffer_refill_inside_one_board():
    """A 128x128 board needing more uniforms than the buffer still holds takes the rest
    of the buffer, then a refill from the global stream -- and the global stream
    continues where the reference's would (next draw after the refill)."""
    rng = np.random.RandomState(5)
    b = _spawner_soup(rng, 128, 128, dens=0.05)
    b[::2, ::2] |= 128                      # spawners everywhere: many eligible cells
    n = oracle.count_eligible(b)
    assert n > 2000
    speedups.seed(9)
    speedups._buffer.take(10000 - n // 2)   # leave half a board's draws in the buffer
    got = speedups.advance_board(b, 0.5)
    after = np.random.random()              # the global stream past the refill
    ref = oracle.RefStreamRNG()
    ref.seed(9)
    ref.take(10000 - n // 2)
    want, _ = oracle.advance(b, 0.5, draws=ref.take(n), pos=0)
    assert np.array_equal(got, want)
    np.random.seed(9)
    np.random.random(20000)
    assert after == np.random.random()
    assert speedups._buffer.pos == ref.pos


def test_used_up_buffer_refills_only_when_a_draw_is_taken():
    """random.c:47-52 refills inside random_float, i.e. only when a draw is taken: a
    board with no eligible cell leaves a used-up buffer (and numpy's global stream)
    alone -- the first call of a process included, where the buffer starts used up
    (buffer_pos = RAND_BUFFER_SIZE, random.c:12).  Later np.random calls (proc_gen.py's,
    which share the global stream) must see the reference's state."""
    rng = np.random.RandomState(3)
    still = np.zeros((20, 30), np.uint16)
    still[5:7, 5:7] = 1                         # a block: alive, no spawner
    assert oracle.count_eligible(still) == 0
    soup = _spawner_soup(rng, 20, 30)
    n = oracle.count_eligible(soup)
    assert n > 0
    for start in ("fresh", "seeded"):
        np.random.seed(11)
        if start == "fresh":                    # a process's first call: buffer used up
            speedups._buffer.pos = 10000
        else:
            speedups.seed(11)                   # reseeds and refills: 10 000 drawn
            speedups._buffer.take(10000)        # used up again
        drawn = 0 if start == "fresh" else 10000
        for _ in range(3):
            assert np.array_equal(speedups.advance_board(still, 0.3), oracle.advance(
                still, 0.3, draws=np.zeros(0), pos=0)[0])
        assert speedups._buffer.pos == 10000    # nothing taken, nothing refilled
        probe = np.random.get_state()
        # the global stream was not touched: its next value is draw `drawn` of seed 11
        assert np.random.random() == np.random.RandomState(11).random_sample(drawn + 1)[-1]
        np.random.set_state(probe)
        # a board that draws refills now, from the global stream where it stands
        got = speedups.advance_board(soup, 0.3)
        ref_buf = np.random.RandomState(11).random_sample(drawn + 10000)[drawn:]
        want, _ = oracle.advance(soup, 0.3, draws=ref_buf[:n], pos=0)
        assert np.array_equal(got, want), start
        assert speedups._buffer.pos == n


def test_input_conversion_and_errors():
    rng = np.random.RandomState(1)
    b = _spawner_soup(rng, 20, 30)
    speedups.seed(2)
    want = speedups.advance_board(b, 0.3)
    for alt in (b.astype(np.int64), b.astype(np.int32).tolist(), np.asfortranarray(b),
                b.astype(">u2"), b.T.copy().T):
        speedups.seed(2)
        assert np.array_equal(speedups.advance_board(alt, 0.3), want)
    for bad in (np.zeros(5, np.uint16), np.zeros((0, 4), np.uint16), np.zeros((1, 4), np.uint16),
                np.zeros((2, 2, 2), np.uint16)):
        with pytest.raises(ValueError):
            speedups.advance_board(bad)
    out = speedups.advance_board(b)                 # default spawn_prob 0.3
    assert out is not b and out.flags.c_contiguous


def test_seed_wraps_like_the_reference_I_format():
    """module.c:248 parses the seed with "I": masked to 32 bits, no overflow check."""
    for s, eq in ((2 ** 32 + 7, 7), (-1, 2 ** 32 - 1), (2 ** 40 + 3, 3)):
        speedups.seed(s)
        a = np.random.random()
        np.random.seed(eq)
        np.random.random(10000)
        assert a == np.random.random(), s
    with pytest.raises(TypeError):
        speedups.seed(1.5)


def test_c_abi_host_advance_matches_module():
    """The same engine through the C ABI (sl_host_advance in libsafelife_hip.so, the
    entry an FFI integrator binds; no GPU needed): advance, the draw count, the
    too-few-draws answer and the shape check."""
    from safelife_amd import _lib
    L = _lib.lib()
    rng = np.random.RandomState(8)
    b = _spawner_soup(rng, 40, 70)
    n = oracle.count_eligible(b)
    assert n > 0
    assert L.sl_host_advance(b.ctypes.data, None, 40, 70, 0.3, None, 0) == n
    draws = rng.rand(n)
    out = np.empty_like(b)
    assert L.sl_host_advance(b.ctypes.data, out.ctypes.data, 40, 70, 0.3,
                             draws.ctypes.data, n - 1) == -(n + 1)
    assert L.sl_host_advance(b.ctypes.data, out.ctypes.data, 40, 70, 0.3,
                             draws.ctypes.data, n) == n
    want, _ = oracle.advance(b, 0.3, draws=draws, pos=0)
    assert np.array_equal(out, want)
    assert L.sl_host_advance(b.ctypes.data, out.ctypes.data, 1, 70, 0.3, None, 0) == -(1 << 63)
