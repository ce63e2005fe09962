"""CPU checks of the rollout oracle (training/ppo.py's per-step arithmetic).

* ``oracle.sample_action`` is pinned against numpy itself: ppo.py:440 calls
  ``np.random.choice(len(policy), p=policy)`` on the global legacy RandomState, so
  ``RandomState(s).choice`` is the reference; the restatement must pick the same
  index from the same draw and raise for the same inputs.
* ``oracle.gae`` restates ppo.py:487-503.  The reference method cannot run here
  (training/ppo.py imports TensorFlow 1.x, absent), so this row's parity is unpinned
  beyond the restatement; it is checked against an independent float64 recursion.
"""
import numpy as np
import pytest

import oracle


def _probs(rng, A, dtype):
    p = rng.rand(A) ** 3
    p[rng.rand(A) < 0.3] = 0.0
    if p.sum() == 0:
        p[0] = 1.0
    return (p / p.sum()).astype(dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_sample_action_matches_numpy_choice(dtype):
    rng = np.random.RandomState(0)
    for trial in range(3000):
        A = int(rng.randint(1, 12))
        p = _probs(rng, A, dtype)
        if trial % 7 == 0:                       # sum off by less than numpy's atol
            p = (p * dtype(1 + 1e-5 if dtype == np.float32 else 1 + 1e-9)).astype(dtype)
        rs = np.random.RandomState(trial)
        st = rs.get_state()
        want = rs.choice(A, p=p)
        rs.set_state(st)
        u = rs.random_sample()
        got, err = oracle.sample_action(p, u)
        assert err == 0 and got == want, (trial, p, u)


def test_sample_action_edge_draws():
    p = np.array([0.25, 0.25, 0.0, 0.5])
    # u exactly on a cdf step goes right (searchsorted side='right'); zero-p skipped
    assert oracle.sample_action(p, 0.0)[0] == 0
    assert oracle.sample_action(p, 0.25)[0] == 1
    assert oracle.sample_action(p, 0.5)[0] == 3
    assert oracle.sample_action(p, np.nextafter(1.0, 0))[0] == 3


def test_sample_action_errors_match_numpy():
    cases = [np.array([0.5, -0.1, 0.6]), np.array([0.5, 0.6]), np.array([0.2, 0.2], np.float32),
             np.array([0.5, 0.5 + 1e-7])]
    for p in cases:
        with pytest.raises(ValueError) as ei:
            np.random.RandomState(0).choice(len(p), p=p)
        _, err = oracle.sample_action(p, 0.5)
        want = 1 if "non-negative" in str(ei.value) else 2
        assert err & want, (p, err, str(ei.value))
    # within tolerance: numpy accepts, err clear
    p = np.array([0.5, 0.5 + 1e-9])
    np.random.RandomState(0).choice(2, p=p)
    assert oracle.sample_action(p, 0.5)[1] == 0


def test_gae_against_float64_recursion():
    rng = np.random.RandomState(3)
    T, N = 20, 16
    gamma = np.array([0.99, 0.9], np.float32)
    rewards = rng.randn(T, N)
    done = rng.rand(T, N) < 0.1
    values = rng.randn(T + 1, N, 2).astype(np.float32)
    ret, adv = oracle.gae(rewards, done, values, gamma, 0.95)
    for g in range(2):
        gm, lm = float(gamma[g]), 0.95 * float(gamma[g])
        for n in range(N):
            R, Aa = None, 0.0
            for t in range(T - 1, -1, -1):
                m = 0.0 if done[t, n] else 1.0
                if R is None:
                    R = rewards[t, n] + m * gm * values[t + 1, n, g]
                else:
                    R = rewards[t, n] + m * gm * R
                delta = rewards[t, n] + m * gm * values[t + 1, n, g] - values[t, n, g]
                Aa = delta + (lm * m * Aa if t < T - 1 else 0.0)
                assert abs(ret[t, n, g] - R) < 1e-5 * max(1.0, abs(R))
                assert abs(adv[t, n, g] - Aa) < 1e-5 * max(1.0, abs(Aa))
    r2, _ = oracle.gae(rewards, done, values, gamma, 0.95, reward_clip=0.5)
    assert np.all(np.abs(r2[done]) <= 0.5 + 1e-12)
