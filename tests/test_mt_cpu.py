"""The host half of the device MT19937 stream (csrc/sl_mt.hip), against numpy itself.

The reference's spawn stream is np.random.RandomState(seed).random_sample
(/root/reference/safelife/speedups_src/random.c:14-52 after numpy.random.seed,
module.c:246-253); numpy is importable here, so it is the oracle: the seeded window
is RandomState(seed).get_state()'s key, the doubles are random_sample's, and a
window jumped by x^n mod phi (Berlekamp-Massey over the generator's own bits) continues
the stream exactly n raw outputs later.  No GPU: these are host functions of the C ABI.
"""
import numpy as np
import pytest

from safelife_amd import _lib, mtstream


@pytest.fixture(scope="module", autouse=True)
def built():
    _lib.build()


@pytest.mark.parametrize("seed", [0, 1, 7, 5489, 123456789, 2 ** 32 - 1])
def test_window_and_draws_are_numpys(seed):
    w = mtstream.host_window(seed)
    assert np.array_equal(w, np.random.RandomState(seed).get_state()[1])
    assert np.array_equal(mtstream.host_draws(w, 3000),
                          np.random.RandomState(seed).random_sample(3000))


@pytest.mark.parametrize("n", [2, 624, 625 * 2, 2 * 10 ** 5 + 6, 624 * 420 * 3])
def test_jump_continues_the_stream(n):
    """n raw outputs = n / 2 draws (n even keeps the draw pairs aligned)."""
    w = mtstream.host_window(42)
    wj = mtstream.host_jump(w, mtstream.host_jump_poly(n))
    got = mtstream.host_draws(wj, 500)
    ref = np.random.RandomState(42).random_sample(n // 2 + 500)[n // 2:]
    assert np.array_equal(got, ref)


def test_jumps_compose():
    """x^a * x^b = x^(a+b): two jumps equal one, far beyond what numpy checks cheaply."""
    w = mtstream.host_window(3)
    a, b = 624 * 420 * 1000, 624 * 420 * 2048
    two = mtstream.host_jump(mtstream.host_jump(w, mtstream.host_jump_poly(a)),
                             mtstream.host_jump_poly(b))
    one = mtstream.host_jump(w, mtstream.host_jump_poly(a + b))
    # word 0's low 31 bits never reach an output (only its top bit feeds the next word)
    assert np.array_equal(two[1:], one[1:]) and (two[0] >> 31) == (one[0] >> 31)
    assert np.array_equal(mtstream.host_draws(two, 200), mtstream.host_draws(one, 200))
