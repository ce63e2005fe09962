"""CPU checks of the drop-in surface: what PPO.__init__ / build_graph read from
``envs[0]`` before any step (training/ppo.py:159,219; training/safelife_ppo.py:196),
built exactly as SafeLifeEnv.__init__ builds it (safelife_env.py:87-110); no GPU is
touched (the device env is created at the first reset)."""
import numpy as np
import pytest


@pytest.mark.parametrize("view,channels", [((33, 33), None), ((15, 15), tuple(range(15))),
                                           ((9, 7), (0, 9, 12))])
def test_safelife_env_spaces_as_reference(view, channels):
    from safelife_amd import SafeLifeEnv
    env = SafeLifeEnv(iter([]), view_shape=view, output_channels=channels)
    assert env.action_space.n == 9 == len(env.action_names)
    sp = env.observation_space
    if channels is None:                       # safelife_env.py:98-103
        assert sp.shape == view and sp.dtype == np.uint16
        assert sp.low.min() == 0 and sp.high.max() == 2 ** 15
    else:                                      # safelife_env.py:104-109
        assert sp.shape == view + (len(channels),) and sp.dtype == np.uint16
        assert sp.high.max() == 1
    # PPO.build_graph: tf.placeholder(input_space.dtype, [None, None] + shape)
    shape = [None, None] + list(sp.shape)
    assert shape[2:] == list(sp.shape)
    assert sp.contains(np.zeros(sp.shape, dtype=np.uint16))
    assert env.action_space.contains(8) and not env.action_space.contains(9)


def test_safelife_env_rejects_unknown_kwargs():
    from safelife_amd import SafeLifeEnv
    with pytest.raises(ValueError):
        SafeLifeEnv(iter([]), not_a_param=3)       # safelife_env.py:90-95
    env = SafeLifeEnv(iter([]), time_limit=7, remove_white_goals=False)
    assert env.time_limit == 7 and env.remove_white_goals is False


def test_env_spaces_helper_matches_reference_shapes():
    from safelife_amd.spaces import env_spaces, Discrete, Box
    a, o = env_spaces(tuple(range(9)), (33, 33), None)
    assert isinstance(a, Discrete) and isinstance(o, Box)
    assert a == Discrete(9) and o == Box(0, 2 ** 15, (33, 33), np.uint16)
    s = o.sample()
    assert s.shape == (33, 33) and o.contains(s)
