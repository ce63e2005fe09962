"""safelife_amd -- MI355X-native batched SafeLife stepper.

Host side of the hot path of neale/safelife-k2 (SafeLifeEnv.step/reset ->
SafeLifeGame.advance_board -> the C rule engine), re-built on hand-written HIP
kernels for gfx950 behind the C ABI in include/safelife_hip.h.

    from safelife_amd import speedups          # advance_board / seed drop-in
    from safelife_amd import SafeLifeVecEnv    # B envs on the GPU (PPO chain)
    from safelife_amd import SafeLifeEnv       # single-env gym-style drop-in
"""
from .cell_types import CellTypes  # noqa: F401
from .levels import LevelPool  # noqa: F401
from .vec_env import SafeLifeVecEnv, GlobalCounter, ACTION_NAMES  # noqa: F401
from . import speedups  # noqa: F401

__version__ = "0.1.0"


def build(force=False):
    """Compile libsafelife_hip.so in-tree for gfx950."""
    from . import _lib
    _lib.build(force=force)


def __getattr__(name):
    if name in ("SafeLifeEnv", "SafeLifeGame"):
        from . import env as _env
        return getattr(_env, name)
    raise AttributeError(name)
