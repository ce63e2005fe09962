"""Device-side PPO rollouts over a SafeLifeVecEnv.

Replaces the per-env Python loop of ``PPO.run_agents`` (training/ppo.py:386-464) and
the returns/advantages part of ``PPO.gen_training_batch`` (training/ppo.py:466-508):

* ``run_agents(venv, policy, steps_per_env)`` steps all envs ``steps_per_env`` times;
  per step the policy (any torch module/function) maps the observations to action
  probabilities, ``sl_sample_actions`` draws the actions exactly as
  ``np.random.choice(len(policy), p=policy)`` does (ppo.py:440), and the env-step
  kernels write rewards / dones / infos / observations straight into the rollout
  buffers -- no host round trip inside the loop.  Envs that finish are reset by the
  step (ContinuingEnv + reset-on-done, ppo.py:441-445), so slot t+1 holds the new
  episode's first observation, as in the reference.
* ``returns_advantages`` is ``sl_gae``: the discounted returns and GAE advantages
  of ppo.py:487-503 for every (env, discount) column, float64 out, in the
  reference's float32/float64 evaluation order.
* ``training_batch`` assembles gen_training_batch's named outputs
  (s, a, pi, r, G, A, v, m, c) from a rollout and the policy's outputs on it.

Action uniforms come from Philox (``rng="philox"``; key = the env's seed, counter =
(0, global env id, env-step index, 2)) or from a caller-supplied [T, N] float64
array (``uniforms``), e.g. the reference's global numpy stream.  ``rng="reference"``
replays the reference's loop itself -- envs one after another, actions and spawn
refills from the one global numpy stream -- bit for bit (tests/golden g7_*.npz).
"""
import ctypes
from typing import Any, NamedTuple

import numpy as np

from . import _lib


class Rollout(NamedTuple):
    """run_agents' named outputs (ppo.py:383-385), as device tensors."""
    states: Any          # [T+1, N, ...] observations (the env's obs layout / dtype)
    actions: Any         # int32 [T, N]
    rewards: Any         # float64 [T, N]
    end_episode: Any     # bool [T, N] (done as the caller sees it: times_up)
    rnn_states: Any      # the policy's recurrent state at the start, or None
    info: dict           # [T, N] tensors: times_up, game_over, reset (bool),
                         # episode_length, episode_reward (int32; 0 unless finished)


def _choice_atol(dtype):
    # numpy's legacy RandomState.choice: sqrt(eps) of float64, or of p's float dtype
    atol = np.sqrt(np.finfo(np.float64).eps)
    return float(max(atol, np.sqrt(np.finfo(dtype).eps)))


def sample_actions(probs, *, seed=0, step=0, env0=0, uniforms=None, out=None, err=None,
                   check=True):
    """actions[b] = np.random.choice(A, p=probs[b]) for a float32/float64 [B, A]
    device tensor.  With ``uniforms`` (float64 [B]) the draws are given; otherwise
    Philox(seed; 0, env0 + b, step, 2).  ``check`` syncs and raises numpy's
    ValueErrors (negative probabilities / sum not 1 within tolerance)."""
    torch = _torch()
    if probs.dim() != 2 or probs.dtype not in (torch.float32, torch.float64):
        raise ValueError("probs must be a float32/float64 [B, A] tensor")
    if probs.stride(1) != 1:
        probs = probs.contiguous()
    B, A = probs.shape
    dev = probs.device
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=dev)
    if check and err is None:
        err = torch.empty(B, dtype=torch.uint8, device=dev)
    mode = _lib.SL_RNG_PHILOX
    u = None
    if uniforms is not None:
        mode = _lib.SL_RNG_STREAM
        u = torch.as_tensor(uniforms, dtype=torch.float64).to(dev).reshape(B).contiguous()
    np_dtype = np.float64 if probs.dtype == torch.float64 else np.float32
    L = _lib.lib()
    _lib.check(L.sl_sample_actions(ctypes.c_void_p(probs.data_ptr()),
                                   int(probs.dtype == torch.float64), B, A, probs.stride(0),
                                   mode, _lib.ptr(u), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                   int(env0), int(step) & 0xFFFFFFFF, _choice_atol(np_dtype),
                                   ctypes.c_void_p(out.data_ptr()), _lib.ptr(err),
                                   _lib.stream_ptr(dev)), "sl_sample_actions")
    if check:
        raise_choice_errors(err)
    return out


def raise_choice_errors(err):
    """Raise numpy.random.choice's ValueError for any env whose err flag is set."""
    if not err.numel():
        return
    neg, bad_sum = ((err & 1) != 0).any(), ((err & 2) != 0).any()
    if bool(neg.item()):
        raise ValueError("probabilities are not non-negative")
    if bool(bad_sum.item()):
        raise ValueError("probabilities do not sum to 1")


def run_agents(venv, policy, steps_per_env, *, rnn_zero_state=None, uniforms=None,
               check_probs=True, rng="batch"):
    """``PPO.run_agents`` for all ``venv.B`` envs at once (training/ppo.py:386-464).

    ``policy(obs, rnn_states) -> (probs [N, A], new_rnn_states)`` (ppo.py:436); obs
    is one [N, ...] slot of the states buffer.  ``uniforms``: optional float64
    [T, N] action draws (default: Philox keyed on venv.seed).  The env keeps its
    last observation and recurrent state between calls (env._ppo_last_obs /
    _ppo_rnn_state, ppo.py:429-434).

    ``rng="reference"`` (a SafeLifeVecEnv(rng="stream")): the reference's loop order
    and its one global numpy stream, bit for bit after speedups.seed(s) -- per step
    the probabilities come to the host once, and env after env draws its action with
    np.random.choice (ppo.py:440) and then takes its step with its spawn draws from
    speedups' buffer (SafeLifeVecEnv.step_env_reference, one host sync per env), so
    the action draws and the buffer's refills interleave exactly as in the reference
    (random.c:14-26).  A parity mode: one env at a time."""
    torch = _torch()
    T, N, dev = int(steps_per_env), venv.B, venv.device
    if T < 1:
        raise ValueError("steps_per_env must be >= 1")
    if rng not in ("batch", "reference"):
        raise ValueError("rng must be 'batch' or 'reference'")
    if rng == "reference" and (uniforms is not None or venv.rng != "stream"):
        raise ValueError("rng='reference' takes its draws from the global numpy stream and "
                         "needs a SafeLifeVecEnv(rng='stream')")
    if uniforms is not None:
        uniforms = torch.as_tensor(uniforms, dtype=torch.float64).to(dev)
        if tuple(uniforms.shape) != (T, N):
            raise ValueError("uniforms must be [steps_per_env, num_envs]")
    states = torch.empty((T + 1,) + tuple(venv.obs.shape), dtype=venv.obs.dtype, device=dev)
    actions = torch.empty((T, N), dtype=torch.int32, device=dev)
    rewards = torch.empty((T, N), dtype=torch.float64, device=dev)
    dones = torch.empty((T, N), dtype=torch.uint8, device=dev)
    flags = torch.empty((T, N), dtype=torch.uint8, device=dev)
    ep_len = torch.empty((T, N), dtype=torch.int32, device=dev)
    ep_rew = torch.empty((T, N), dtype=torch.int32, device=dev)
    err = torch.zeros((T, N), dtype=torch.uint8, device=dev) if check_probs else None

    if getattr(venv, "_ppo_last_obs", None) is None:
        venv.reset()
        venv._ppo_last_obs = venv.observe().clone()
        venv._ppo_rnn_state = rnn_zero_state
    states[0].copy_(venv._ppo_last_obs)
    initial_rnn = venv._ppo_rnn_state
    rnn = initial_rnn
    for t in range(T):
        probs, rnn = policy(states[t], rnn)
        if rng == "reference":
            _reference_step(venv, probs, t, actions, rewards, dones, states, flags, ep_len,
                            ep_rew)
            continue
        sample_actions(probs, seed=venv.seed, step=venv._step_index, env0=venv.env0,
                       uniforms=None if uniforms is None else uniforms[t], out=actions[t],
                       err=None if err is None else err[t], check=False)
        venv.step_async(actions[t], reward_out=rewards[t], done_out=dones[t],
                        obs_out=states[t + 1], flags_out=flags[t], ep_len_out=ep_len[t],
                        ep_rew_out=ep_rew[t])
    if err is not None:
        raise_choice_errors(err)
    venv._ppo_last_obs.copy_(states[T])
    done_last = dones[T - 1].bool()
    if rnn_zero_state is not None and rnn is not None:
        # ppo.py:444-447: an env that ended on the last step starts its next
        # sequence from the zero state
        mask = done_last.reshape((N,) + (1,) * (rnn.dim() - 1))
        rnn = torch.where(mask, rnn_zero_state.expand_as(rnn), rnn)
    venv._ppo_rnn_state = rnn
    info = {"times_up": (flags & 1) != 0, "game_over": (flags & 2) != 0,
            "reset": (flags & 4) != 0, "episode_length": ep_len, "episode_reward": ep_rew}
    return Rollout(states, actions, rewards, dones.bool(), initial_rnn, info)


def _reference_step(venv, probs, t, actions, rewards, dones, states, flags, ep_len, ep_rew):
    """ppo.py:438-448 for slot t: env after env, np.random.choice on the host (numpy's
    own checks and draw), then that env's step on the device."""
    p = probs.detach()
    p = p.cpu().numpy()
    acts = np.empty(venv.B, np.int32)
    for e in range(venv.B):
        acts[e] = np.random.choice(len(p[e]), p=p[e])
        venv.step_env_reference(e, int(acts[e]), reward_out=rewards[t], done_out=dones[t],
                                obs_out=states[t + 1], flags_out=flags[t],
                                ep_len_out=ep_len[t], ep_rew_out=ep_rew[t])
    venv.end_reference_step()
    actions[t].copy_(_torch().from_numpy(acts))


def returns_advantages(rewards, end_episode, values, gamma=(0.99,), lmda=0.95,
                       reward_clip=0.0):
    """Discounted returns and GAE advantages (training/ppo.py:487-503) on the device.

    rewards float64 [T, N]; end_episode bool/uint8 [T, N]; values float32
    [T+1, N, G]; gamma: G discount factors (float32, ppo.py:116).  Returns
    (returns, advantages), float64 [T, N, G]."""
    torch = _torch()
    dev = rewards.device
    T, N = rewards.shape
    gamma_np = np.asarray(gamma, dtype=np.float32).reshape(-1)
    lmda_np = lmda * gamma_np                      # float32, as ppo.py:496 computes it
    G = gamma_np.size
    if tuple(values.shape) != (T + 1, N, G) or values.dtype != torch.float32:
        raise ValueError("values must be float32 [T+1, N, G] = %s" % ((T + 1, N, G),))
    r = rewards.to(torch.float64).contiguous()
    d = end_episode.to(torch.uint8).contiguous()
    v = values.contiguous()
    g_t = torch.from_numpy(gamma_np).to(dev)
    l_t = torch.from_numpy(np.asarray(lmda_np, dtype=np.float32)).to(dev)
    ret = torch.empty((T, N, G), dtype=torch.float64, device=dev)
    adv = torch.empty((T, N, G), dtype=torch.float64, device=dev)
    L = _lib.lib()
    _lib.check(L.sl_gae(ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(d.data_ptr()),
                        ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(g_t.data_ptr()),
                        ctypes.c_void_p(l_t.data_ptr()), G, T, N, float(reward_clip),
                        ctypes.c_void_p(ret.data_ptr()), ctypes.c_void_p(adv.data_ptr()),
                        _lib.stream_ptr(dev)), "sl_gae")
    return ret, adv


def training_batch(rollout, policies, values, gamma=(0.99,), lmda=0.95, reward_clip=0.0):
    """gen_training_batch's named outputs s, a, pi, r, G, A, v, m, c (ppo.py:466-508)
    from a rollout and the policy/value outputs on all T+1 states
    (policies [T+1, N, A], values float32 [T+1, N, G])."""
    torch = _torch()
    a = rollout.actions.long()
    pi = torch.gather(policies[:-1], -1, a.unsqueeze(-1)).squeeze(-1)
    G, A = returns_advantages(rollout.rewards, rollout.end_episode, values, gamma, lmda,
                              reward_clip)
    r = rollout.rewards
    if reward_clip > 0:
        r = r.clamp(-reward_clip, reward_clip)
    m = torch.roll(~rollout.end_episode, 1, dims=0)      # rnn_mask, ppo.py:492-493
    m[0] = True
    return {"s": rollout.states[:-1], "a": rollout.actions, "pi": pi, "r": r, "G": G,
            "A": A, "v": values[:-1], "m": m, "c": rollout.rnn_states}


def _torch():
    import torch
    return torch
