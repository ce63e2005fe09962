"""Device-resident level pools -- the ``level_iterator`` side of SafeLifeEnv.reset.

The reference pulls one ``SafeLifeGame`` per reset from ``safelife_loader``
(/root/reference/safelife/file_finder.py:143-201), either loading a saved level
(``SafeLifeGame.loaddata``, safelife_game.py:236-251, npz schema :184-194) or
generating one on the CPU (proc_gen.gen_game).  Here a pool of K levels of one
shape lives on the GPU and the reset kernel copies level k (optionally with a
random toroidal roll, under which the dynamics are exactly equivariant) into an
env's board / goals / start board.
"""
import ctypes

import numpy as np

from . import _lib

LEVEL_KEYS = ("board", "goals", "agent_loc", "orientation", "spawn_prob", "min_performance")


def _as_level_dict(obj):
    if isinstance(obj, dict) or hasattr(obj, "files"):
        d = {k: obj[k] for k in LEVEL_KEYS if k in obj}
    elif hasattr(obj, "dtype") and obj.dtype.names:            # structured archive row
        d = {k: obj[k] for k in LEVEL_KEYS if k in obj.dtype.names}
    else:                                                      # a game-like object
        d = {k: getattr(obj, k) for k in LEVEL_KEYS if hasattr(obj, k)}
        if hasattr(obj, "_init_data"):                         # reference SafeLifeGame
            init = obj._init_data
            for k in LEVEL_KEYS:
                if k in init:
                    d[k] = init[k]
    if "board" not in d or "goals" not in d:
        raise ValueError("a level needs at least 'board' and 'goals'")
    d.setdefault("agent_loc", (0, 0))
    d.setdefault("orientation", 1)          # GameState.orientation default
    d.setdefault("spawn_prob", 0.3)         # GameState.spawn_prob default
    d.setdefault("min_performance", -1.0)   # GameState.min_performance default
    return d


class LevelPool:
    """K levels of one shape, as numpy arrays (host) and torch tensors (device)."""

    def __init__(self, board, goals, agent_loc, orientation, spawn_prob, min_performance):
        self.board = np.ascontiguousarray(board, dtype=np.uint16)
        self.goals = np.ascontiguousarray(goals, dtype=np.uint16)
        if self.board.ndim != 3 or self.board.shape != self.goals.shape:
            raise ValueError("pool boards/goals must be [K,H,W] and equal in shape")
        self.K, self.H, self.W = self.board.shape
        if self.H < 2 or self.W < 2:
            raise ValueError("boards must be at least 2x2 (the reference is undefined below)")
        al = np.asarray(agent_loc, dtype=np.int64).reshape(self.K, 2)
        self.agent_x = al[:, 0].astype(np.int32) % self.W
        self.agent_y = al[:, 1].astype(np.int32) % self.H
        self.orientation = np.asarray(orientation, dtype=np.int32).reshape(self.K)
        # GameState keeps spawn_prob as a Python float; advance_board receives a C float
        self.spawn_prob = np.asarray(spawn_prob, dtype=np.float64).reshape(self.K)
        self.min_performance = np.asarray(min_performance, dtype=np.float64).reshape(self.K)
        n_exit = ((self.board & 0x100) != 0).reshape(self.K, -1).sum(1)
        if (n_exit > _lib.SL_MAX_EXITS).any():
            raise ValueError("level with %d exits: the kernels track at most %d per env"
                             % (int(n_exit.max()), _lib.SL_MAX_EXITS))
        self._dev = None

    # -- constructors ---------------------------------------------------------
    @classmethod
    def from_levels(cls, levels):
        ds = [_as_level_dict(x) for x in levels]
        if not ds:
            raise ValueError("empty level list")
        return cls(np.stack([d["board"] for d in ds]), np.stack([d["goals"] for d in ds]),
                   np.stack([np.asarray(d["agent_loc"]) for d in ds]),
                   [int(d["orientation"]) for d in ds], [float(d["spawn_prob"]) for d in ds],
                   [float(d["min_performance"]) for d in ds])

    @classmethod
    def load(cls, *paths):
        """Pool npz (stacked arrays), single-level npz, or a `levels` archive npz."""
        levels = []
        for p in paths:
            with np.load(p, allow_pickle=False) as d:
                if "levels" in d.files:
                    levels.extend(list(d["levels"]))
                elif d["board"].ndim == 3:
                    K = d["board"].shape[0]
                    levels.extend({k: d[k][i] for k in LEVEL_KEYS if k in d.files}
                                  for i in range(K))
                else:
                    levels.append({k: d[k] for k in LEVEL_KEYS if k in d.files})
        return cls.from_levels(levels)

    def has_spawners(self):
        """Does any level's board or goals hold a spawning cell (CellTypes.spawning)?"""
        return bool(((self.board | self.goals) & 0x80).any())

    def subset(self, idx):
        idx = np.asarray(idx)
        al = np.stack([self.agent_x[idx], self.agent_y[idx]], 1)
        return LevelPool(self.board[idx], self.goals[idx], al, self.orientation[idx],
                         self.spawn_prob[idx], self.min_performance[idx])

    # -- device ---------------------------------------------------------------
    def to_device(self, device, pin=False, non_blocking=False):
        """Upload on the current stream (``pin``: through page-locked host buffers,
        so ``non_blocking`` copies do not wait for the host)."""
        import torch
        if self._dev is not None and self._dev["device"] == device:
            return self._dev

        def up(a):
            h = torch.from_numpy(np.ascontiguousarray(a))
            if pin:
                h = h.pin_memory()
            return h.to(device, non_blocking=non_blocking)
        t = {
            "device": device,
            "board": up(self.board),
            "goals": up(self.goals),
            "agent_x": up(self.agent_x),
            "agent_y": up(self.agent_y),
            "orientation": up(self.orientation),
            "spawn_prob": up(self.spawn_prob.astype(np.float32)),
            "min_performance": up(self.min_performance),
        }
        s = _lib.LevelPool()
        s.K, s.H, s.W = self.K, self.H, self.W
        for k in ("board", "goals", "agent_x", "agent_y", "orientation", "spawn_prob",
                  "min_performance"):
            setattr(s, k, t[k].data_ptr())
        if self.H in (64, 128):
            # derived: per-level bit planes (the bit-sliced kernels' start-board source),
            # uint64 [K,16,W] for 64 rows, uint32 [K,16,4,W] for 128
            t["board_planes"] = torch.empty((self.K, 16, self.H // 32, self.W),
                                            dtype=torch.int32, device=device)
            s.board_planes = t["board_planes"].data_ptr()
            if self.H == 128:      # the goals' colour planes, uint32 [K,3,4,W]
                t["goal_planes"] = torch.empty((self.K, 3, self.H // 32, self.W),
                                               dtype=torch.int32, device=device)
                s.goal_planes = t["goal_planes"].data_ptr()
            L = _lib.lib()
            _lib.check(L.sl_level_pool_prepare(ctypes.byref(s), _lib.stream_ptr(device)),
                       "sl_level_pool_prepare")
        t["struct"] = s
        self._dev = t
        return t
