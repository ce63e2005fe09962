"""The two gym spaces the reference env declares (safelife_env.py:97-109), which
PPO.build_graph reads from ``envs[0]`` (training/ppo.py:219 ``observation_space``
shape and dtype, training/safelife_ppo.py:196 ``action_space.n``).

gym itself is not a dependency of this package: when it is importable its own
``spaces.Discrete`` / ``spaces.Box`` are used, otherwise these duck types, which
carry the attributes and methods those callers use (``n``, ``shape``, ``dtype``,
``low``, ``high``, ``sample()``, ``contains()``).
"""
import numpy as np


class Discrete:
    """gym.spaces.Discrete(n): integers 0 .. n-1."""

    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)
        self._rng = np.random.RandomState()

    def seed(self, seed=None):
        self._rng = np.random.RandomState(seed)
        return [seed]

    def sample(self):
        return int(self._rng.randint(self.n))

    def contains(self, x):
        if isinstance(x, (np.generic, np.ndarray)) and np.asarray(x).shape == ():
            x = int(x)
        return isinstance(x, int) and 0 <= x < self.n

    __contains__ = contains

    def __repr__(self):
        return "Discrete(%d)" % self.n

    def __eq__(self, other):
        return isinstance(other, Discrete) and other.n == self.n


class Box:
    """gym.spaces.Box(low, high, shape, dtype) with scalar bounds broadcast."""

    def __init__(self, low, high, shape, dtype):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)
        self._rng = np.random.RandomState()

    def seed(self, seed=None):
        self._rng = np.random.RandomState(seed)
        return [seed]

    def sample(self):
        return self._rng.randint(self.low.astype(np.int64), self.high.astype(np.int64) + 1,
                                 size=self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return (x.shape == self.shape and bool(np.all(x >= self.low))
                and bool(np.all(x <= self.high)))

    __contains__ = contains

    def __repr__(self):
        return "Box(%s, %s)" % (self.shape, self.dtype)

    def __eq__(self, other):
        return (isinstance(other, Box) and other.shape == self.shape and other.dtype == self.dtype
                and np.array_equal(other.low, self.low) and np.array_equal(other.high, self.high))


try:                                  # the real classes when gym is installed
    from gym import spaces as _gym_spaces   # noqa: F401
    Discrete, Box = _gym_spaces.Discrete, _gym_spaces.Box   # noqa: F811
except ImportError:
    pass


def env_spaces(action_names, view_shape, output_channels):
    """(action_space, observation_space) exactly as SafeLifeEnv.__init__ builds them
    (safelife_env.py:97-109)."""
    action_space = Discrete(len(action_names))
    view_shape = tuple(view_shape)
    if output_channels is None:
        obs = Box(low=0, high=2 ** 15, shape=view_shape, dtype=np.uint16)
    else:
        obs = Box(low=0, high=1, shape=view_shape + (len(output_channels),), dtype=np.uint16)
    return action_space, obs
