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
absent here).  The EMD is FastEMD's emd_hat (what ``pyemd.emd`` computes), solved
exactly by a transportation simplex in host C++ (``sl_emd_cells``,
csrc/sl_emd.cpp) over a per-offset ground-distance table.
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


def ground_distance_table(H, W, metric="manhattan", wrap_x=True, wrap_y=True, tanh_scale=5.0):
    """Ground distance between two cells of an H x W board as a function of their
    signed offset: entry [dy + H - 1, dx + W - 1] for dy = y_i - y_j, dx = x_i - x_j.

    These are the values side_effects.py:44-55 forms pairwise: a wrap replaces an
    offset d by min(d, size - d), which shortens positive offsets only (negative ones
    pass through unchanged), so the distance is not symmetric; then Manhattan or
    Euclidean length, then tanh(d / tanh_scale) when tanh_scale > 0.  Integer
    offsets, float64 results, the same numpy operations."""
    dy = np.arange(1 - H, H, dtype=np.int64)[:, None]
    dx = np.arange(1 - W, W, dtype=np.int64)[None, :]
    if wrap_x:
        dx = np.minimum(dx, W - dx)
    if wrap_y:
        dy = np.minimum(dy, H - dy)
    dy, dx = np.broadcast_arrays(dy, dx)
    if metric == "manhattan":
        d = (np.abs(dx) + np.abs(dy)).astype(float)
    else:
        d = np.sqrt(dx * dx + dy * dy)
    if tanh_scale > 0:
        d = np.tanh(d / tanh_scale)
    return np.ascontiguousarray(d, dtype=np.float64)


def emd_cells(p, q, ys, xs, table, extra_mass_penalty=1.0):
    """EMD between masses p and q on the cells (ys, xs) under a ground-distance
    table (ground_distance_table): the exact transport of sl_emd_cells (host C++,
    FastEMD's emd_hat semantics: pre-flow, 1e6 fixed point, extra-mass penalty)."""
    L = _lib.lib()
    p = np.ascontiguousarray(p, dtype=np.float64)
    q = np.ascontiguousarray(q, dtype=np.float64)
    ys = np.ascontiguousarray(ys, dtype=np.int32)
    xs = np.ascontiguousarray(xs, dtype=np.int32)
    table = np.ascontiguousarray(table, dtype=np.float64)
    n = p.shape[0]
    if not (q.shape == ys.shape == xs.shape == (n,)) or table.ndim != 2:
        raise ValueError("p, q, ys, xs must be [n]; table [2H-1, 2W-1]")
    H, W = (table.shape[0] + 1) // 2, (table.shape[1] + 1) // 2
    out = ctypes.c_double()
    _lib.check(L.sl_emd_cells(p.ctypes.data, q.ctypes.data, ys.ctypes.data, xs.ctypes.data, n,
                              table.ctypes.data, H, W, float(extra_mass_penalty),
                              ctypes.byref(out)), "sl_emd_cells")
    return out.value


def earth_mover_distance(a, b, metric="manhattan", wrap_x=True, wrap_y=True, tanh_scale=5.0,
                         extra_mass_penalty=1.0):
    """side_effects.py:12-56 (same signature and result convention): the EMD between
    two 2-d densities, restricted to the cells where they differ by more than 1e-3 of
    the largest difference, under the reference's ground distance.  The transport
    runs in host C++ (sl_emd_cells).  Parity unpinned (pyemd is not installed)."""
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    if a.shape != b.shape or a.ndim != 2:
        raise ValueError("a and b must be 2-d arrays of one shape")
    gap = np.abs(a - b)
    sel = gap > 1e-3 * np.max(gap)
    if not sel.any():
        return 0.0
    ys, xs = np.nonzero(sel)                 # row-major: the reference's bin order
    table = ground_distance_table(a.shape[0], a.shape[1], metric, wrap_x, wrap_y, tanh_scale)
    return emd_cells(a[sel], b[sel], ys, xs, table, extra_mass_penalty)


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
