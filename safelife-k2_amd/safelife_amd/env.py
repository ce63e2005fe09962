"""Single-env drop-ins: ``SafeLifeEnv`` (safelife_env.py:16-198) and ``SafeLifeGame``
(safelife_game.py:123-664), both over device state of :class:`SafeLifeVecEnv`.

``SafeLifeGame`` is the game state of one env of a vector env (B = 1 for the
drop-ins, or env ``idx`` of a larger batch).  Every method runs on the GPU through
the C ABI on that env alone (``SafeLifeVecEnv.state_slice``): ``execute_action``
(sl_env_action), ``advance_board`` (sl_env_advance), ``current_points`` /
``performance_ratio`` (sl_env_rescore), ``update_exit_colors`` (sl_env_exit_colors),
``revert`` / ``deserialize`` (a reset of the env from a one-level pool).  Reads of
``board``, ``goals``, ``agent_loc`` ... return host copies of the device values.

The spawn RNG defaults to the reference's: every draw comes from the global numpy
RNG through the 10 000-double buffer of ``safelife_amd.speedups`` (random.c), in the
order the reference consumes it (board, then goals, row-major).  Before an advance
the next ``2*H*W`` buffered draws are staged on the device without consuming them;
the advance reports how many it used and exactly that many are then taken, so
numpy's global state moves as the reference's does.  ``rng='philox'`` uses the
counter-based stream instead.

``SafeLifeEnv.step`` runs the whole env-step as one fused ``sl_env_step`` (the same
kernels as the batch); the game methods are for code that drives the game itself
(wrappers, UI, tests: SURVEY.md §3.4's callers).  Throughput comes from the batched
env.
"""
import ctypes

import numpy as np

from . import _lib, speedups
from .cell_types import CellTypes
from .levels import LevelPool
from .spaces import env_spaces
from .vec_env import ACTION_NAMES, GlobalCounter, SafeLifeVecEnv, start_board_hi_bits

# safelife_game.py:27-34
ORIENTATION = {"UP": 0, "RIGHT": 1, "DOWN": 2, "LEFT": 3, "FORWARD": 4, "BACKWARD": 6}
GAME_CLASS = "safelife.safelife_game.SafeLifeGame"
# env-level fields a game-level revert / deserialize leaves alone (they belong to
# SafeLifeEnv and its wrappers, not to the game)
_ENV_FIELDS = ("episode_length", "episode_reward", "old_points", "side_effect", "prior_x",
               "prior_y", "prior_len", "prior_head", "episodes")


def _single_venv(level, device, rng="reference", seed=0, **kw):
    """A one-env SafeLifeVecEnv over a one-level pool: no wrappers (no movement bonus,
    no side-effect penalty, the level's own min_performance), no automatic reset."""
    pool = LevelPool.from_levels([level])
    common = dict(movement_bonus=0.0, penalty_coef=0.0, min_performance=None,
                  auto_reset=False, output_channels=None, compute_obs=False,
                  global_counter=GlobalCounter())
    common.update(kw)
    if rng == "reference":
        v = SafeLifeVecEnv(pool, 1, device, rng="stream", spawn_stream=np.zeros(1), **common)
    else:
        v = SafeLifeVecEnv(pool, 1, device, rng="philox", seed=seed, **common)
    v._dropin = True      # draws from the global speedups stream (rng='reference')
    return v


class SafeLifeGame:
    """SafeLifeGame (safelife_game.py:650-664 with GameWithGoals :540-647 and GameState
    :123-537) as a view of env ``idx`` of a SafeLifeVecEnv."""
    points_on_level_exit = +1
    point_table = np.array([
        # k   r   g   y   b   m   c   w        (safelife_game.py:554-564, the table the
        [+0, -1, +0, +0, +0, +0, +0, +0],    #  kernels' cell_scores evaluate)
        [-3, +3, -3, +0, -3, +0, -3, -3],
        [+0, -3, +5, +0, +0, +0, +3, +0],
        [-3, +0, +0, +3, +0, +0, +0, +0],
        [+3, -3, +3, +0, +5, +3, +3, +3],
        [-3, +3, -3, +0, -3, +5, -3, -3],
        [+3, -3, +3, +0, +3, +0, +5, +3],
        [+0, -1, +0, +0, +0, +0, +0, +0],
    ])
    point_table.setflags(write=False)

    def __init__(self, venv, idx=0):
        self._venv = venv
        self._idx = int(idx)
        self._init = None            # level dict of the episode when not a pool level
        self.file_name = None
        torch = venv.torch
        self._act = torch.zeros(4, dtype=torch.int64, device=venv.device)
        self._pts = torch.zeros(1, dtype=torch.int32, device=venv.device)
        self._scratch = torch.zeros(8 + 16, dtype=torch.int64, device=venv.device)
        self._pos = torch.zeros(1, dtype=torch.int64, device=venv.device)

    # ------------------------------------------------------------ construction
    @classmethod
    def loaddata(cls, data, auto_cls=True, device=None, rng="reference", seed=0):
        """GameState.loaddata (safelife_game.py:236-251): a game in the initial state
        of ``data`` (a level dict / npz / reference game), on its own device env."""
        venv = _single_venv(data, device, rng=rng, seed=seed)
        venv.reset()
        game = cls(venv, 0)
        # deserialize leaves the level's own exit cells (the env reset coloured them)
        _lib.check(_lib.lib().sl_env_exit_colors(ctypes.byref(game._slice()), 1, game._stream()),
                   "sl_env_exit_colors")
        game.rescore()
        return game

    @classmethod
    def load(cls, file_name, auto_cls=True, device=None, rng="reference", seed=0):
        """GameState.load (safelife_game.py:253-260)."""
        import os
        path = os.path.abspath(os.path.expanduser(file_name))
        with np.load(path, allow_pickle=False) as d:
            game = cls.loaddata({k: d[k] for k in d.files}, auto_cls, device, rng, seed)
        game.file_name = path
        return game

    # ---------------------------------------------------------------- helpers
    def _slice(self):
        return self._venv.state_slice(self._idx, 1)

    def _stream(self):
        return _lib.stream_ptr(self._venv.device)

    def _st(self, k):
        return self._venv.state[k][self._idx].item()

    def _set(self, k, v):
        self._venv.state[k][self._idx] = v

    # --------------------------------------------------------------- attributes
    @property
    def board(self):
        return self._venv.board[self._idx].cpu().numpy()

    @board.setter
    def board(self, value):
        v = self._upload(value)
        self._venv._allow_board_bits(self._venv._device_board_bits(v))
        self._venv.board[self._idx].copy_(v)
        self._set("spawn_flags", self._st("spawn_flags") | 1)   # may now hold a spawner
        self._venv._may_spawn = True
        # bit 3: the board's draw planes (128x128 replay) described the old board;
        # bits 6-7: the board's bit planes (sl_env_state.board_planes) are stale
        self._venv.planes_ok[self._idx].bitwise_and_(~(8 | 64 | 128))
        self.rescore()

    @property
    def goals(self):
        return self._venv.goals[self._idx].cpu().numpy()

    @goals.setter
    def goals(self, value):
        self._venv.goals[self._idx].copy_(self._upload(value))
        self._set("spawn_flags", self._st("spawn_flags") | 2)
        self._venv._may_spawn = True
        self._venv.planes_ok[self._idx].zero_()        # the goals mirror is stale
        self.rescore()

    def _upload(self, a):
        torch = self._venv.torch
        a = np.ascontiguousarray(a, dtype=np.uint16)
        if a.shape != (self.height, self.width):
            raise ValueError("board must be %dx%d" % (self.height, self.width))
        return torch.from_numpy(a).to(self._venv.device)

    @property
    def agent_loc(self):
        return np.array([self._st("agent_x"), self._st("agent_y")])

    @agent_loc.setter
    def agent_loc(self, loc):
        self._set("agent_x", int(loc[0]) % self.width)
        self._set("agent_y", int(loc[1]) % self.height)

    @property
    def orientation(self):
        return self._st("orientation")

    @orientation.setter
    def orientation(self, v):
        self._set("orientation", int(v) % 4)

    @property
    def num_steps(self):
        return self._st("num_steps")

    @num_steps.setter
    def num_steps(self, v):
        self._set("num_steps", int(v))

    @property
    def game_over(self):
        return bool(self._st("game_over"))

    @game_over.setter
    def game_over(self, v):
        self._set("game_over", 1 if v else 0)

    @property
    def spawn_prob(self):
        return float(self._venv.state["spawn_prob"][self._idx].item())

    @spawn_prob.setter
    def spawn_prob(self, v):
        self._set("spawn_prob", float(v))
        self._venv._check_ring_threshold([float(v)])

    @property
    def min_performance(self):
        return float(self._venv.state["min_performance"][self._idx].item())

    @min_performance.setter
    def min_performance(self, value):
        # wrappers assign it (SimpleSideEffectPenalty.reset, env_wrappers.py:313-317)
        self._set("min_performance", float(value))

    @property
    def can_toggle_powers(self):
        return self._venv.can_toggle_powers

    @property
    def can_toggle_colors(self):
        return self._venv.can_toggle_colors

    @property
    def width(self):
        return self._venv.W

    @property
    def height(self):
        return self._venv.H

    @property
    def title(self):
        import os
        if self.file_name is None:
            return None
        return ".".join(os.path.split(self.file_name)[-1].split(".")[:-1])

    @property
    def exit_locs(self):
        """np.nonzero(board & exit) of the episode's start (update_exit_locs,
        safelife_game.py:528-529): exits never move during play."""
        n = min(self._st("exit_count"), _lib.SL_MAX_EXITS)
        ey = self._venv.state["exit_y"][self._idx, :n].cpu().numpy().astype(np.int64)
        ex = self._venv.state["exit_x"][self._idx, :n].cpu().numpy().astype(np.int64)
        return (ey, ex)

    @property
    def is_stochastic(self):
        """(board & spawning).any() (safelife_game.py:662-664)."""
        return bool((self.board & CellTypes.spawning).any())

    @property
    def _init_data(self):
        """The initial state of the episode (what deserialize stored): the level it
        was reset from, rolled as the reset rolled it."""
        if self._init is not None:
            return dict(self._init)
        v, i = self._venv, self._idx
        roll = int(v.state["start_roll"][i].item())
        if roll < 0:
            raise RuntimeError("this env's start state was written by the caller "
                               "(set_state): its initial goals are unknown")
        pool, k = v.pool, int(v.state["level_index"][i].item())
        dy, dx = roll >> 16, roll & 0xFFFF
        return {"board": v.start_board[i].cpu().numpy(),
                "goals": np.roll(pool.goals[k], (dy, dx), (0, 1)),
                "agent_loc": ((int(pool.agent_x[k]) + dx) % pool.W,
                              (int(pool.agent_y[k]) + dy) % pool.H),
                "orientation": int(pool.orientation[k]),
                "spawn_prob": float(pool.spawn_prob[k]),
                "min_performance": float(pool.min_performance[k]),
                "class": GAME_CLASS}

    # ------------------------------------------------------------------ scoring
    def rescore(self, goals=None):
        """sl_env_rescore on this env: refresh the stored perf terms (what can_exit
        and update_exit_colors read) and return current_points()."""
        s = self._slice()
        if goals is not None:
            # current_points(goals=...) scores the board against other goals; the
            # env's stored terms are left alone
            g = self._upload(goals)
            tmp = self._venv.torch.zeros(2, dtype=self._venv.torch.int32, device=self._venv.device)
            s.goals = g.data_ptr()
            s.score, s.possible = tmp.data_ptr(), tmp.data_ptr() + 4
        _lib.check(_lib.lib().sl_env_rescore(ctypes.byref(s), _lib.ptr(self._pts), self._stream()),
                   "sl_env_rescore")
        return int(self._pts.item())

    def current_points(self, board=None, goals=None):
        """safelife_game.py:590-599 (the cell colours and liveness always come from
        the game's own board, as in the reference: ``board`` is not read)."""
        return self.rescore(goals)

    def performance_ratio(self, unit_rewards=True):
        """safelife_game.py:601-631 -> (completed, possible) against the episode's
        baseline.  Only the unit-reward form (the one every reference caller uses:
        can_exit, env_wrappers.py:181) is evaluated on the device."""
        if not unit_rewards:
            raise ValueError("performance_ratio(unit_rewards=False) is not kept on the "
                             "device; every reference caller uses unit rewards")
        self.rescore()
        base = self._st("baseline")
        return self._st("score") - base, self._st("possible") - base

    def can_exit(self):
        """safelife_game.py:522-526."""
        if self.min_performance < 0:
            return True
        completed, total = self.performance_ratio()
        return completed >= self.min_performance * total

    def update_exit_locs(self):
        """Exit cells are tracked from the episode's start (safelife_game.py:528-529);
        they are frozen and never created or moved by the rule or the actions."""
        return self.exit_locs

    def update_exit_colors(self):
        """safelife_game.py:531-537 on the device (sl_env_exit_colors)."""
        self.rescore()
        _lib.check(_lib.lib().sl_env_exit_colors(ctypes.byref(self._slice()), 0, self._stream()),
                   "sl_env_exit_colors")

    # ------------------------------------------------------------------ actions
    def relative_loc(self, n_forward, n_right=0):
        """safelife_game.py:294-306 (the board is a torus)."""
        dx, dy = n_right, -n_forward
        for _ in range(self.orientation):
            dx, dy = -dy, dx
        x0, y0 = self.agent_loc
        return (x0 + dx) % self.width, (y0 + dy) % self.height

    def _device_action(self, a):
        torch = self._venv.torch
        acts = torch.tensor([a], dtype=torch.int32, device=self._venv.device)
        v = self._venv
        _lib.check(_lib.lib().sl_env_action(ctypes.byref(self._slice()), acts.data_ptr(),
                                            int(v.can_toggle_powers), int(v.can_toggle_colors),
                                            self._act.data_ptr(), self._stream()),
                   "sl_env_action")
        self.rescore()
        return int(self._act[0].item())

    def move_agent(self, dy, dx=0):
        """safelife_game.py:308-345 for the moves the game makes: one cell forward
        (dy = 1) or backward (dy = -1) without turning."""
        if dx != 0 or dy not in (1, -1):
            raise ValueError("move_agent supports dy = +-1, dx = 0 (the game's moves)")
        o = self.orientation
        if self.game_over:
            return 0
        # MOVE <d> sets orientation d and moves one cell along it: facing the
        # opposite way and moving forward touches exactly the cells of a backward
        # move (front / behind / two ahead swap roles), then the facing is restored
        d = o if dy == 1 else (o + 2) % 4
        reward = self._device_action(1 + d)
        self.orientation = o
        return reward

    def execute_action(self, action):
        """safelife_game.py:347-393: MOVE/TOGGLE <dir> on the device; the relative
        forms (MOVE FORWARD/BACKWARD, TURN, FACE, bare TOGGLE) and RESTART as there."""
        if self.game_over:
            return 0
        if action in ACTION_NAMES:
            return self._device_action(ACTION_NAMES.index(action))
        if action.startswith("MOVE "):
            direction = ORIENTATION[action[5:]]
            return self.move_agent(5 - direction)     # FORWARD: 1, BACKWARD: -1
        if action.startswith("TURN "):
            self.orientation = (self.orientation + 2 - ORIENTATION[action[5:]]) % 4
        elif action.startswith("FACE "):
            self.orientation = ORIENTATION[action[5:]]
        elif action == "TOGGLE":
            return self._device_action(5 + self.orientation)
        elif action == "RESTART":
            self.game_over = True
        return 0

    def advance_board(self):
        """safelife_game.py:657-660 (num_steps += 1; board, then goals) on the
        device.  Draws: the drop-in game (loaddata / SafeLifeEnv) replaying the
        reference takes them from the global numpy stream (speedups); a view of a
        batch with rng='stream' from the batch's own stream at its position (the
        batch's replay order is its own business); Philox from this game's own
        advance counter, which leaves the batch's step index -- and so every other
        env's keys -- alone."""
        v = self._venv
        cfg = v._fill_cfg()
        cfg.scratch = self._scratch.data_ptr()
        ref = v.rng == "stream" and getattr(v, "_dropin", False)
        if ref:
            draws = v.torch.from_numpy(speedups._buffer.peek(2 * v.H * v.W)).to(v.device)
            self._pos.zero_()
            cfg.draws, cfg.n_draws, cfg.stream_pos = draws.data_ptr(), draws.numel(), \
                self._pos.data_ptr()
            cfg.mt = None
        elif v.rng != "stream":
            cfg.env0 = v.env0 + self._idx
            # (the top bit keeps these counters apart from the batch's step indices)
            # the counter lives on the batch, per env, so that a SafeLifeGame made anew
            # for the same env (every SafeLifeEnv.reset) does not repeat its draws
            counts = v.__dict__.setdefault("_game_advances", {})
            n = counts.get(self._idx, 0)
            cfg.step = (0x80000000 | n) & 0xFFFFFFFF
            counts[self._idx] = n + 1
        _lib.check(_lib.lib().sl_env_advance(ctypes.byref(self._slice()), ctypes.byref(cfg),
                                             self._stream()), "sl_env_advance")
        if ref:
            speedups._buffer.take(int(self._pos.item()))
        self.rescore()

    # ---------------------------------------------------------------- save/load
    def serialize(self):
        """safelife_game.py:184-194 + GameWithGoals.serialize (:571-574)."""
        return {"spawn_prob": self.spawn_prob, "orientation": self.orientation,
                "agent_loc": tuple(int(x) for x in self.agent_loc), "board": self.board,
                "class": GAME_CLASS, "min_performance": self.min_performance,
                "goals": self.goals}

    def deserialize(self, data, as_initial_state=True):
        """safelife_game.py:196-212 + :576-578: the env is reset from ``data`` (a
        one-level pool on the device), so board, goals, agent, exits, game_over and
        num_steps are the level's; the env-level counters are kept."""
        from .levels import _as_level_dict
        v, i = self._venv, self._idx
        lvl = _as_level_dict(data)
        keep = {k: v.state[k][i].clone() for k in _ENV_FIELDS}
        if not as_initial_state:
            keep_start = (v.start_board[i].clone(), v.state["baseline"][i].clone())
        pool = LevelPool.from_levels([lvl])
        pdev = pool.to_device(v.device)
        v._may_spawn = v._may_spawn or pool.has_spawners()
        v._allow_board_bits(v._pool_bits(pool))      # (64x64 planes kept zero)
        cfg = v._fill_cfg()
        cfg.level_mode, cfg.augment_roll, cfg.env0, cfg.n_total_envs = 0, 0, 0, 1
        cfg.wrapper_min_performance = float("nan")
        _lib.check(_lib.lib().sl_env_reset(ctypes.byref(self._slice()), ctypes.byref(pdev["struct"]),
                                           None, ctypes.byref(cfg), self._stream()),
                   "sl_env_reset")
        # the start board is not a level of the env's pool: kernels read it from HBM
        v.state["start_roll"][i] = -1
        if as_initial_state:
            self._init = dict(lvl, **{"class": GAME_CLASS})
            for k in ("board", "goals"):
                self._init[k] = np.array(lvl[k], dtype=np.uint16)
        else:
            v.start_board[i].copy_(keep_start[0])
            v.state["baseline"][i] = keep_start[1]
            # spawn_flags bit 2 follows the start board kept (cell bits 12-14)
            hi = 4 if ((v.H, v.W) == (128, 128)
                       and bool(start_board_hi_bits(v.start_board[i:i + 1])[0])) else 0
            self._set("spawn_flags", (self._st("spawn_flags") & ~4) | hi)
        # the raw level cells (the reset coloured the exits by can_exit)
        _lib.check(_lib.lib().sl_env_exit_colors(ctypes.byref(self._slice()), 1, self._stream()),
                   "sl_env_exit_colors")
        for k, t in keep.items():
            v.state[k][i].copy_(t)
        self.rescore()

    def revert(self):
        """safelife_game.py:229-234: back to the episode's initial state."""
        self.deserialize(self._init_data)
        return True

    def save(self, file_name=None):
        """safelife_game.py:214-227."""
        import os
        if file_name is None:
            file_name = self.file_name
        if file_name is None:
            raise ValueError("Must specify a file name")
        file_name = os.path.abspath(os.path.expanduser(file_name))
        if not file_name.endswith(".npz"):
            file_name += ".npz"
        self.file_name = file_name
        data = self.serialize()
        self._init = dict(data)
        self.num_steps = 0
        # _init_data is now the saved state (safelife_game.py:225): performance_ratio,
        # can_exit and the exit colours score against it, and the side-effect start
        # board is it
        v, i = self._venv, self._idx
        self.rescore()
        v.state["baseline"][i] = v.state["score"][i]
        v.start_board[i].copy_(v.board[i])
        v.state["start_roll"][i] = -1
        hi = 4 if ((v.H, v.W) == (128, 128)
                   and bool(start_board_hi_bits(v.start_board[i:i + 1])[0])) else 0
        self._set("spawn_flags", (self._st("spawn_flags") & ~4) | hi)
        np.savez_compressed(file_name, **data)


class SafeLifeEnv:
    """Drop-in for safelife_env.SafeLifeEnv on one device env.

    ``level_iterator`` yields levels: reference ``SafeLifeGame`` objects, level
    dicts / npz files with the schema of safelife_game.py:184-194, or anything
    ``LevelPool.from_levels`` accepts.
    """
    metadata = {"render.modes": ["ansi", "rgb_array"], "video.frames_per_second": 30}
    action_names = ACTION_NAMES
    time_limit = 1000
    remove_white_goals = True
    view_shape = (15, 15)
    output_channels = tuple(range(15))
    global_counter = GlobalCounter()

    def __init__(self, level_iterator, device=None, rng="reference", seed=None, **kwargs):
        self.level_iterator = level_iterator
        for key, val in kwargs.items():
            if (not key.startswith("_") and hasattr(self, key) and
                    not callable(getattr(self, key))):
                setattr(self, key, val)
            else:
                raise ValueError("Unrecognized parameter: '%s'" % (key,))
        if rng not in ("reference", "philox"):
            raise ValueError("rng must be 'reference' or 'philox'")
        # safelife_env.py:97-109
        self.action_space, self.observation_space = env_spaces(
            self.action_names, self.view_shape, self.output_channels)
        self.rng = rng
        self.device = device
        self._venv = None
        self.game = None
        self._philox_seed = 0 if seed is None else int(seed)
        if seed is not None:
            self.seed(seed)

    def seed(self, seed=None):
        """speedups.seed (the reference seeds the global spawn stream here)."""
        seed = int(np.random.randint(2 ** 31)) if seed is None else int(seed)
        speedups.seed(seed)
        self._philox_seed = seed
        return [seed]

    def _env_for(self, level):
        pool = LevelPool.from_levels([level])
        if self._venv is None or (self._venv.H, self._venv.W) != (pool.H, pool.W):
            self._venv = _single_venv(
                level, self.device, rng=self.rng, seed=self._philox_seed,
                time_limit=self.time_limit, view_shape=tuple(self.view_shape),
                output_channels=(tuple(self.output_channels) if self.output_channels else None),
                remove_white_goals=self.remove_white_goals, compute_obs=True)
        else:
            self._venv.set_pool(pool)
        return self._venv

    def get_obs(self, board=None, goals=None, agent_loc=None):
        """safelife_env.py:125-155; ``board`` / ``goals`` / ``agent_loc`` replace the
        game's own for this one observation (exits stay the game's exit_locs)."""
        v = self._venv
        if board is None and goals is None and agent_loc is None:
            return v.observe()[0].cpu().numpy()
        torch = v.torch
        s = v.state_slice(0, 1)
        keep = []
        if board is not None:
            t = torch.from_numpy(np.ascontiguousarray(board, dtype=np.uint16)).to(v.device)
            keep.append(t)
            s.board = t.data_ptr()
            s.board_planes = None       # (the env's own planes describe its own board)
        if goals is not None:
            t = torch.from_numpy(np.ascontiguousarray(goals, dtype=np.uint16)).to(v.device)
            keep.append(t)
            s.goals = t.data_ptr()
        if agent_loc is not None:
            t = torch.tensor([int(agent_loc[0]) % v.W, int(agent_loc[1]) % v.H],
                             dtype=torch.int32, device=v.device)
            keep.append(t)
            s.agent_x, s.agent_y = t.data_ptr(), t.data_ptr() + 4
        out = torch.empty_like(v.obs[:1])
        vh, vw = v.view_shape
        ch = v._channels if v.obs_mode != _lib.SL_OBS_PACKED else None
        nch = len(v.output_channels) if v.output_channels else 0
        _lib.check(_lib.lib().sl_env_obs(ctypes.byref(s), vh, vw, int(v.remove_white_goals),
                                         v.obs_mode, ch, nch, out.data_ptr(),
                                         _lib.stream_ptr(v.device)), "sl_env_obs")
        return out[0].cpu().numpy()

    def reset(self):
        venv = self._env_for(next(self.level_iterator))
        venv.reset()
        self._frame()
        venv.stream_pos.zero_()
        self._stream_at = 0
        self.game = SafeLifeGame(venv)
        self.episode_length = 0
        self.episode_reward = 0
        self.episode_completed = False
        if self.global_counter is not None:
            self.global_counter.episodes_started += 1
        return self.get_obs()

    def _frame(self):
        """Per-env staging for step(): pinned host buffers and one device frame, so a
        step is one upload (action, staged draws), the step kernels, one gather kernel
        into the frame (obs, reward, flags, stream position, board, goals, agent) and
        one download -- a single host sync."""
        v = self._venv
        if getattr(self, "_frame_env", None) is v:
            return self._frame_data
        torch = v.torch
        parts = [v.obs[0:1], v.reward, v.flags, v.stream_pos, v.board[0:1], v.goals[0:1],
                 v.st_t["agent_x"], v.st_t["agent_y"]]
        views = [p.reshape(-1).view(torch.uint8) for p in parts]
        offs = np.cumsum([0] + [x.numel() for x in views])
        n2 = 2 * v.H * v.W
        fr = {"views": views, "offs": offs,
              "dev": torch.empty(int(offs[-1]), dtype=torch.uint8, device=v.device),
              "host": torch.empty(int(offs[-1]), dtype=torch.uint8, pin_memory=True),
              "act_h": torch.empty(1, dtype=torch.int32, pin_memory=True),
              "draws_h": torch.empty(n2, dtype=torch.float64, pin_memory=True),
              "draws_d": torch.empty(n2, dtype=torch.float64, device=v.device)}
        fr["host_np"] = fr["host"].numpy()
        # (bfloat16 views come back as their raw 16-bit words: numpy has no bfloat16)
        fr["obs_dtype"] = {torch.uint16: np.uint16, torch.uint8: np.uint8,
                           torch.float32: np.float32}.get(v.obs.dtype, np.uint16)
        if self.rng == "reference":
            v.spawn_stream = fr["draws_d"]
            v.mt = None
        self._frame_env, self._frame_data = v, fr
        return fr

    def step(self, action):
        assert self.game is not None, "Game state is not initialized."
        venv = self._venv
        torch = venv.torch
        fr = self._frame()
        o = fr["offs"]
        p0 = 0
        if self.rng == "reference":
            # stage the next draws the step can consume (<= one per cell per tensor);
            # the buffer is addressed from the running stream position, so nothing on
            # the device needs rewinding
            p0 = self._stream_at
            fr["draws_h"].numpy()[:] = speedups._buffer.peek(2 * venv.H * venv.W)
            fr["draws_d"].copy_(fr["draws_h"], non_blocking=True)
            venv._draw_base = p0
        fr["act_h"][0] = int(action)
        venv.actions_dev.copy_(fr["act_h"], non_blocking=True)
        venv.step_async(venv.actions_dev)
        torch.cat(fr["views"], out=fr["dev"])
        fr["host"].copy_(fr["dev"], non_blocking=True)
        torch.cuda.current_stream(venv.device).synchronize()
        h = fr["host_np"]
        reward = float(h[o[1]:o[2]].view(np.float64)[0])
        flags = int(h[o[2]])
        if self.rng == "reference":
            self._stream_at = int(h[o[3]:o[4]].view(np.int64)[0])
            speedups._buffer.take(self._stream_at - p0)
        obs = h[o[0]:o[1]].view(fr["obs_dtype"]).reshape(venv.obs.shape[1:]).copy()
        H, W = venv.H, venv.W
        board = h[o[4]:o[5]].view(np.uint16).reshape(H, W).copy()
        goals = h[o[5]:o[6]].view(np.uint16).reshape(H, W).copy()
        agent_loc = np.array([int(h[o[6]:o[7]].view(np.int32)[0]),
                              int(h[o[7]:o[8]].view(np.int32)[0])])
        self.episode_length += 1
        self.episode_reward += reward
        times_up = bool(flags & 1)
        already_completed = self.episode_completed
        self.episode_completed = times_up or bool(flags & 2)
        if not already_completed and self.global_counter is not None:
            self.global_counter.episodes_completed += self.episode_completed
            self.global_counter.num_steps += 1
        return obs, reward, self.episode_completed, {
            "board": board,
            "goals": goals,
            "agent_loc": agent_loc,
            "times_up": times_up,
            "episode": {"length": self.episode_length, "reward": self.episode_reward},
        }

    def render(self, mode="ansi"):
        raise ValueError("rendering (safelife_env.py:200-206) is out of scope: UI")

    def close(self):
        pass


__all__ = ["SafeLifeEnv", "SafeLifeGame", "CellTypes", "ORIENTATION"]
