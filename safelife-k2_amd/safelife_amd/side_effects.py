"""Side-effect scoring (reference: safelife/side_effects.py).

``side_effect_densities`` is the rollout + density half of ``side_effect_score``
(side_effects.py:59-92, 131-139) on the GPU, batched over finished episodes through
``sl_side_effect_densities``: per episode the initial board is advanced
``num_steps`` times, then ``num_samples`` times alternately with the final board,
and every sampled board is added to its cell-type density map.  Results are the
reference's dicts ``{cell_type_key: float64 [H, W]}`` for the inaction (b0) and
action (b1) runs.

``earth_mover_distance`` / ``side_effect_score`` complete the reference API on the
host, as the reference itself does (numpy + the third-party ``pyemd``, which is
absent here).  The EMD is solved as the exact transport linear program of
EMD-hat (Pele & Werman; what ``pyemd.emd`` computes) with scipy's HiGHS solver.
Parity unpinned: no pyemd output exists in this environment to compare against.
"""
import ctypes

import numpy as np

from . import _lib


def side_effect_densities(init_boards, final_boards, num_steps, spawn_prob, num_samples=1000,
                          rng="philox", seed=0, env0=0, spawn_stream=None, stream_pos=0,
                          max_keys=64, device=None, return_stream_pos=False):
    """Density maps of E episodes' counterfactual (inaction) and actual rollouts.

    init_boards, final_boards: [E, H, W] (numpy or torch) -- game._init_data['board']
    and game.board; num_steps: [E] ints (game.num_steps); spawn_prob: scalar or [E].
    rng: 'philox' (batched) or 'stream' (E == 1: the reference's draw order from the
    uniform stream ``spawn_stream`` starting at ``stream_pos``).
    Returns a list of (inaction, action) dicts, one per episode.
    """
    import torch
    dev = _lib.require_device(device)
    L = _lib.lib()
    b0 = torch.as_tensor(np.ascontiguousarray(init_boards, dtype=np.uint16)
                         if not torch.is_tensor(init_boards) else init_boards)
    b1 = torch.as_tensor(np.ascontiguousarray(final_boards, dtype=np.uint16)
                         if not torch.is_tensor(final_boards) else final_boards)
    if b0.dim() == 2:
        b0, b1 = b0[None], b1[None]
    if b0.shape != b1.shape or b0.dim() != 3:
        raise ValueError("init_boards and final_boards must both be [E, H, W]")
    E, H, W = (int(x) for x in b0.shape)
    b0 = b0.to(dev, torch.uint16).contiguous()
    b1 = b1.to(dev, torch.uint16).contiguous()
    steps_h = np.ascontiguousarray(np.broadcast_to(np.asarray(num_steps, dtype=np.int32), (E,)))
    steps_d = torch.from_numpy(steps_h.copy()).to(dev)
    sp = torch.as_tensor(np.broadcast_to(np.asarray(spawn_prob, dtype=np.float32), (E,)).copy(),
                         device=dev)
    mode = {"philox": _lib.SL_RNG_PHILOX, "stream": _lib.SL_RNG_STREAM}[rng]
    draws = pos = None
    if mode == _lib.SL_RNG_STREAM:
        if E != 1 or spawn_stream is None:
            raise ValueError("rng='stream' replays one episode at a time from spawn_stream")
        draws = torch.as_tensor(np.ascontiguousarray(spawn_stream, dtype=np.float64), device=dev)
        pos = torch.tensor([int(stream_pos)], dtype=torch.int64, device=dev)
    keys = torch.zeros((E, max_keys), dtype=torch.uint16, device=dev)
    n_keys = torch.zeros(E, dtype=torch.int32, device=dev)
    present = torch.zeros((E, max_keys), dtype=torch.int32, device=dev)
    inaction = torch.empty((E, max_keys, H, W), dtype=torch.float64, device=dev)
    action = torch.empty_like(inaction)
    nbytes = ctypes.c_int64()
    _lib.check(L.sl_side_effect_workspace(E, H, W, ctypes.byref(nbytes)), "workspace")
    ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)
    _lib.check(L.sl_side_effect_densities(
        b0.data_ptr(), b1.data_ptr(), steps_d.data_ptr(),
        steps_h.ctypes.data_as(ctypes.c_void_p), sp.data_ptr(), E, H, W, int(num_samples),
        mode, int(seed), int(env0), _lib.ptr(draws), _lib.ptr(pos), int(max_keys),
        keys.data_ptr(), n_keys.data_ptr(), present.data_ptr(), inaction.data_ptr(),
        action.data_ptr(), ws.data_ptr(), int(nbytes.value), _lib.stream_ptr(dev)),
        "sl_side_effect_densities")
    nk = n_keys.cpu().numpy()
    if (nk > max_keys).any():
        raise ValueError("more than max_keys=%d cell types in a rollout (%d): raise max_keys"
                         % (max_keys, int(nk.max())))
    keys_h, pres_h = keys.cpu().numpy(), present.cpu().numpy()
    ina_h, act_h = inaction.cpu().numpy(), action.cpu().numpy()
    out = []
    for e in range(E):
        ina, act = {}, {}
        for k in range(int(nk[e])):
            key = int(keys_h[e, k])
            if pres_h[e, k] & 1:
                ina[key] = ina_h[e, k]
            if pres_h[e, k] & 2:
                act[key] = act_h[e, k]
        out.append((ina, act))
    if return_stream_pos:
        return out, (int(pos.item()) if pos is not None else None)
    return out


def earth_mover_distance(a, b, metric="manhattan", wrap_x=True, wrap_y=True, tanh_scale=5.0,
                         extra_mass_penalty=1.0):
    """side_effects.py:12-56: EMD between two 2-d distributions over the cells where
    they differ, with the reference's (one-sided) wrapped Manhattan/Euclidean ground
    distance.  Parity unpinned (pyemd is not installed here)."""
    from scipy.optimize import linprog
    a = np.asanyarray(a, dtype=float)
    b = np.asanyarray(b, dtype=float)
    x, y = np.meshgrid(np.arange(a.shape[1]), np.arange(a.shape[0]))
    delta = np.abs(a - b)
    changed = delta > 1e-3 * np.max(delta)
    if not changed.any():
        return 0.0
    dx = np.subtract.outer(x[changed], x[changed])
    dy = np.subtract.outer(y[changed], y[changed])
    if wrap_x:
        dx = np.minimum(dx, a.shape[1] - dx)
    if wrap_y:
        dy = np.minimum(dy, a.shape[0] - dy)
    if metric == "manhattan":
        dist = (np.abs(dx) + np.abs(dy)).astype(float)
    else:
        dist = np.sqrt(dx * dx + dy * dy)
    if tanh_scale > 0:
        dist = np.tanh(dist / tanh_scale)
    return emd_hat(a[changed], b[changed], dist, extra_mass_penalty)


def emd_hat(p, q, dist, extra_mass_penalty=-1.0):
    """EMD-hat (the quantity pyemd.emd returns): the cheapest transport of
    min(sum p, sum q) mass from p to q under ``dist`` plus |sum p - sum q| times the
    extra-mass penalty (negative: the largest ground distance).  Exact LP (HiGHS)."""
    from scipy.optimize import linprog
    p = np.asarray(p, dtype=float)
    q = np.asarray(q, dtype=float)
    n, m = len(p), len(q)
    if extra_mass_penalty < 0:
        extra_mass_penalty = float(np.max(dist)) if dist.size else 0.0
    flow = min(p.sum(), q.sum())
    a_ub = np.zeros((n + m, n * m))
    for i in range(n):
        a_ub[i, i * m:(i + 1) * m] = 1.0
    for j in range(m):
        a_ub[n + j, j::m] = 1.0
    res = linprog(np.asarray(dist, dtype=float).ravel(), A_ub=a_ub,
                  b_ub=np.concatenate([p, q]), A_eq=np.ones((1, n * m)), b_eq=[flow],
                  bounds=(0, None), method="highs")
    if not res.success:
        raise RuntimeError("EMD transport LP failed: %s" % res.message)
    return float(res.fun) + abs(p.sum() - q.sum()) * extra_mass_penalty


def side_effect_score(game, num_samples=1000, include=None, exclude=None, **kw):
    """side_effects.py:95-161 for one game-like object (``_init_data['board']``,
    ``board``, ``num_steps``, ``spawn_prob``): {key: [emd, sum(inaction density)]}.
    The rollout runs on the GPU (``side_effect_densities``); ``kw`` selects its RNG."""
    (ina, act), = side_effect_densities(game._init_data["board"][None], game.board[None],
                                        [game.num_steps], game.spawn_prob, num_samples, **kw)
    keys = set(ina) | set(act)
    if include is not None:
        keys &= set(include)
    if exclude is not None:
        keys -= set(exclude)
    zeros = np.zeros(np.shape(game.board))
    return {key: [earth_mover_distance(ina.get(key, zeros), act.get(key, zeros)),
                  np.sum(ina.get(key, zeros))] for key in keys}
