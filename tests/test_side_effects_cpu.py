"""Host-side EMD of side_effect_score (side_effects.py:12-56) -- known answers.

Parity with pyemd itself is unpinned (pyemd is not installed); these pin the
transport problem EMD-hat defines."""
import numpy as np

from safelife_amd.side_effects import emd_hat, earth_mover_distance


def test_emd_hat_known_answers():
    d = np.array([[0.0, 2.0], [2.0, 0.0]])
    assert emd_hat([1.0, 0.0], [1.0, 0.0], d) == 0.0
    assert abs(emd_hat([1.0, 0.0], [0.0, 1.0], d) - 2.0) < 1e-12
    # half the mass moves, half is extra (penalty 1.0)
    assert abs(emd_hat([1.0, 0.0], [0.0, 0.5], d, 1.0) - (0.5 * 2.0 + 0.5)) < 1e-12
    # negative penalty -> the largest ground distance
    assert abs(emd_hat([1.0], [0.25], np.zeros((1, 1)), -1.0) - 0.0) < 1e-12


def test_earth_mover_distance_grid():
    a = np.zeros((8, 8))
    b = np.zeros((8, 8))
    assert earth_mover_distance(a, b) == 0.0
    a[2, 2] = 1.0
    b[2, 4] = 1.0
    # manhattan distance 2, tanh(2 / 5)
    assert abs(earth_mover_distance(a, b) - np.tanh(2 / 5.0)) < 1e-9
