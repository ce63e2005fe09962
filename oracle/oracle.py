"""
CPU oracle for the SafeLife hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker.  The product path
(``safelife-k2_amd/safelife_amd``) never imports it and fails loudly without its
HIP library.

Contents
--------
* ctypes binding of ``sl_oracle.c`` (per-cell rule engine, Philox, stream replay);
* ``RefStreamRNG``: the reference's spawn RNG model -- a 10 000-double buffer
  refilled from the *global* numpy legacy MT19937
  (/root/reference/safelife/speedups_src/random.c:8-26,47-52; seed: random.c:28-45);
* ``OracleEnv``: a per-env numpy restatement of the PPO training chain
  ``ContinuingEnv(SimpleSideEffectPenalty(MovementBonusWrapper(SafeLifeEnv)))``
  plus the caller's reset-on-done (/root/reference/training/ppo.py:441-445):

  - actions ....... safelife_game.py:294-393, safelife_env.py:61-71
  - advance ....... safelife_game.py:657-660
  - points ........ safelife_game.py:554-565,590-599
  - performance ... safelife_game.py:601-631, can_exit :522-526
  - exit colours .. safelife_game.py:528-537
  - env step ...... safelife_env.py:157-186, reset :188-198, obs :125-155
  - view .......... helper_utils.py:41-74
  - bonus ......... env_wrappers.py:67-94
  - penalty ....... env_wrappers.py:313-346
  - continuing .... env_wrappers.py:295-303

Pinning: the rule engine against tests/golden/advance_*.npz and the env chain against
tests/golden/traj_*.npz, all captured from the reference itself by
tests/golden/make_golden.py.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libsl_oracle.so")
_lib = None

RNG_STREAM = 0
RNG_PHILOX = 1


def build():
    """Compile the C restatement (and the reference ext when its sources exist)."""
    subprocess.check_call(["make", "-s", "-C", _HERE, "all"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i64, u64, u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32
        L.orc_advance.restype = ctypes.c_int
        L.orc_advance.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                  ctypes.c_int, vp, i64, vp, u64, u32, u32, u32]
        L.orc_count_eligible.restype = i64
        L.orc_count_eligible.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.orc_philox_uniform.restype = ctypes.c_double
        L.orc_philox_uniform.argtypes = [u32, u32, u32, u32, u64]
        L.orc_batch_create.restype = vp
        L.orc_batch_create.argtypes = [i64, ctypes.c_int, ctypes.c_int, i64]
        L.orc_batch_free.argtypes = [vp]
        L.orc_batch_reset.argtypes = [vp, vp, vp]
        L.orc_batch_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.orc_batch_board.restype = ctypes.POINTER(ctypes.c_uint16)
        L.orc_batch_board.argtypes = [vp, i64, ctypes.c_int]
        L.orc_batch_scalars.argtypes = [vp, i64, vp]
        L.orc_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


# --------------------------------------------------------------------------
# rule engine
# --------------------------------------------------------------------------

def advance(board, spawn_prob=0.3, draws=None, pos=0, rng=RNG_STREAM,
            seed=0, env_id=0, step=0, tensor=0):
    """One CA step of a 2-d uint16 board.  Returns (new_board, new_pos)."""
    b = np.ascontiguousarray(board, dtype=np.uint16)
    assert b.ndim == 2
    out = np.empty_like(b)
    p = ctypes.c_int64(pos)
    d = None
    nd = 0
    if draws is not None:
        draws = np.ascontiguousarray(draws, dtype=np.float64)
        d, nd = draws.ctypes.data, len(draws)
    rc = lib().orc_advance(b.ctypes.data, out.ctypes.data, b.shape[0], b.shape[1],
                           float(spawn_prob), rng, d, nd, ctypes.byref(p),
                           seed, env_id, step, tensor)
    if rc:
        raise ValueError("oracle advance failed (shape < 2 or stream exhausted)")
    return out, p.value


def count_eligible(board):
    b = np.ascontiguousarray(board, dtype=np.uint16)
    return int(lib().orc_count_eligible(b.ctypes.data, b.shape[0], b.shape[1]))


def philox_uniform(cell, env, step, tensor, seed):
    return lib().orc_philox_uniform(cell, env, step, tensor, seed)


class RefStreamRNG:
    """The reference's spawn-draw buffer (random.c) driven by numpy's global RNG."""
    SIZE = 10000

    def __init__(self):
        self.buf = None
        self.pos = self.SIZE

    def seed(self, s):
        np.random.seed(s)
        self._refill()

    def _refill(self):
        self.buf = np.random.random(self.SIZE)
        self.pos = 0

    def take(self, n):
        parts = []
        while n > 0:
            if self.pos >= self.SIZE:
                self._refill()
            k = min(n, self.SIZE - self.pos)
            parts.append(self.buf[self.pos:self.pos + k])
            self.pos += k
            n -= k
        return np.concatenate(parts) if parts else np.empty(0)


# --------------------------------------------------------------------------
# cell types and tables
# --------------------------------------------------------------------------
ALIVE, AGENT, PUSHABLE, DESTRUCTIBLE, FROZEN = 1, 2, 4, 8, 16
PRESERVING, INHIBITING, SPAWNING, EXIT = 32, 64, 128, 256
COLOR_R, COLOR_G, COLOR_B = 512, 1024, 2048
PULLABLE = 1 << 15
RAINBOW = COLOR_R | COLOR_G | COLOR_B
PLAYER = AGENT | INHIBITING | PRESERVING | FROZEN | DESTRUCTIBLE
LEVEL_EXIT = FROZEN | EXIT
LIFE = ALIVE | DESTRUCTIBLE
MOVABLE = PUSHABLE | PULLABLE

POINT_TABLE = np.array([
    [+0, -1, +0, +0, +0, +0, +0, +0],
    [-3, +3, -3, +0, -3, +0, -3, -3],
    [+0, -3, +5, +0, +0, +0, +3, +0],
    [-3, +0, +0, +3, +0, +0, +0, +0],
    [+3, -3, +3, +0, +5, +3, +3, +3],
    [-3, +3, -3, +0, -3, +5, -3, -3],
    [+3, -3, +3, +0, +3, +0, +5, +3],
    [+0, -1, +0, +0, +0, +0, +0, +0],
], dtype=np.int64)
SIGN_TABLE = np.sign(POINT_TABLE).astype(np.int64)

ACTIONS = ("NULL", "MOVE UP", "MOVE RIGHT", "MOVE DOWN", "MOVE LEFT",
           "TOGGLE UP", "TOGGLE RIGHT", "TOGGLE DOWN", "TOGGLE LEFT")


def points(board, goals):
    g = (goals & RAINBOW) >> 9
    c = (board & RAINBOW) >> 9
    return int(np.sum(POINT_TABLE[g, c] * ((board & ALIVE) > 0)))


def perf_terms(board, goals):
    """(score, possible) of performance_ratio with unit rewards."""
    g = (goals & RAINBOW) >> 9
    c = (board & RAINBOW) >> 9
    m = ((board & ALIVE) > 0) & ((board & (FROZEN | MOVABLE)) != FROZEN)
    score = int(np.sum(SIGN_TABLE[g, c] * m))
    possible = int(np.sum(np.max(SIGN_TABLE, axis=1)[g]))
    return score, possible


def side_effect_count(board, start, goals, exit_mask):
    b = board & np.uint16(~PLAYER & 0xFFFF)
    s = start & np.uint16(~PLAYER & 0xFFFF)
    b = np.where(exit_mask, s, b)
    red_life = ALIVE | COLOR_R
    start_red = (s & red_life) == red_life
    end_red = (b & red_life) == red_life
    goal_cell = (goals & RAINBOW) == COLOR_B
    end_alive = (b & red_life) == ALIVE
    unchanged = b == s
    non_effects = unchanged | (start_red & ~end_red) | (goal_cell & end_alive)
    return int(np.sum(~non_effects))


# --------------------------------------------------------------------------
# side-effect rollout + densities (side_effects.py:59-92, 131-139)
# --------------------------------------------------------------------------

def density_key_board(board):
    """Per-cell density key of _add_cell_distribution (side_effects.py:60-79):
    0 = not counted; else the masked cell type (destructible restored for alive and
    hard-spawner bases)."""
    b = np.asarray(board, dtype=np.int64)
    FROZEN_, DESTR_, MOVABLE_, AGENT_, COLORS_ = 0x10, 0x8, 0x4 | 0x8000, 0x2, 0xE00
    unchanging = (b & (FROZEN_ | DESTR_ | MOVABLE_)) == FROZEN_       # side_effects.py:62
    m = (b & ~DESTR_ & 0xFFFF) * ~unchanging                           # :63
    skip = (m == 0) | ((m & AGENT_) != 0)                              # :69-71
    base = m & ~COLORS_
    key = np.where((base == 0x1) | (base == 0x90), m | DESTR_, m)      # :72-76
    return np.where(skip, 0, key)


def add_cell_distribution(board, dist):
    """_add_cell_distribution (side_effects.py:59-86) on a {key: counts, 'n': n} dict."""
    dist["n"] += 1
    k = density_key_board(board)
    for key in np.unique(k):
        if key == 0:
            continue
        key = int(key)
        if key not in dist:
            dist[key] = np.zeros(k.shape)
        dist[key] += k == key
    return dist


def norm_cell_distribution(dist):
    """_norm_cell_distribution (side_effects.py:89-92)."""
    n = dist.pop("n")
    for x in dist.values():
        x /= n


def side_effect_densities(init_board, final_board, num_steps, spawn_prob, num_samples,
                          rng="stream", stream=None, seed=0, env_id=0):
    """The rollout of side_effect_score (side_effects.py:131-139): b0 from the initial
    board advanced num_steps times, then num_samples x (b0, b1) advances, each pair
    added to its density map.  rng 'stream' draws from stream.take() in the
    reference's order; 'philox' keys a draw on (2x2 block of the cell, env_id, advance
    index of that board, 4 + board) -- orc_spawn_uniform."""
    b0 = np.array(init_board, dtype=np.uint16)
    b1 = np.array(final_board, dtype=np.uint16)
    inaction, action = {"n": 0}, {"n": 0}

    def adv(b, which, t):
        if rng == "stream":
            d = stream.take(count_eligible(b))
            return advance(b, spawn_prob, d, 0, RNG_STREAM)[0]
        return advance(b, spawn_prob, None, 0, RNG_PHILOX, seed, env_id, t, 4 + which)[0]

    for t in range(num_steps):
        b0 = adv(b0, 0, t)
    for sidx in range(num_samples):
        b0 = adv(b0, 0, num_steps + sidx)
        b1 = adv(b1, 1, sidx)
        add_cell_distribution(b0, inaction)
        add_cell_distribution(b1, action)
    norm_cell_distribution(inaction)
    norm_cell_distribution(action)
    return inaction, action


def movement_bonus_table(n_max, bonus=0.1, power=0.01, period=4):
    """reward increment for each integer Manhattan distance (computed exactly as Python does)."""
    return np.array([bonus * (d / period) ** power for d in range(n_max + 1)],
                    dtype=np.float64)


def make_obs(board, goals, ax, ay, exits, view_shape, output_channels,
             remove_white_goals=True):
    b = board.astype(np.uint16).copy()
    g = goals & np.uint16(RAINBOW)
    if remove_white_goals:
        g = g * (g != RAINBOW)
    b = (b + (g << 3).astype(np.uint16)).astype(np.uint16)
    h, w = view_shape
    bh, bw = b.shape
    y0, x0 = ay, ax
    rows = (np.arange(h) + y0 - h // 2) % bh
    cols = (np.arange(w) + x0 - w // 2) % bw
    v = b[rows[:, None], cols[None, :]]
    for iy, ix in exits:  # numpy fancy assignment: last write wins
        jy = (iy - y0 + bh // 2) % bh - bh // 2
        jx = (ix - x0 + bw // 2) % bw - bw // 2
        jy = min(max(jy + h // 2, 0), h - 1)
        jx = min(max(jx + w // 2, 0), w - 1)
        v[jy, jx] = b[iy, ix]
    if output_channels:
        sh = np.array(list(output_channels), dtype=np.uint16)
        v = (v[..., None] & (np.uint16(1) << sh)) >> sh
    return v


# --------------------------------------------------------------------------
# one env of the PPO chain
# --------------------------------------------------------------------------
class Level:
    """A static level (the npz schema of safelife_game.py:184-194)."""

    def __init__(self, board, goals, agent_loc, orientation=1, spawn_prob=0.3,
                 min_performance=-1.0):
        self.board = np.asarray(board, dtype=np.uint16)
        self.goals = np.asarray(goals, dtype=np.uint16)
        self.agent_loc = (int(agent_loc[0]), int(agent_loc[1]))
        self.orientation = int(orientation)
        self.spawn_prob = float(spawn_prob)
        self.min_performance = float(min_performance)

    @classmethod
    def from_npz(cls, d):
        return cls(d['board'], d['goals'], d['agent_loc'], d['orientation'],
                   d['spawn_prob'], d['min_performance'])

    def rolled(self, dy, dx):
        """Toroidal roll of the whole level (dynamics commute with it)."""
        H, W = self.board.shape
        ax, ay = self.agent_loc
        return Level(np.roll(self.board, (dy, dx), (0, 1)),
                     np.roll(self.goals, (dy, dx), (0, 1)),
                     ((ax + dx) % W, (ay + dy) % H), self.orientation,
                     self.spawn_prob, self.min_performance)


def pool_level_fn(levels, gid, seed=0, n_total=1, random_order=False, augment=False):
    """The level (and toroidal roll) of global env ``gid``'s episode ``ep`` as the
    device level pool hands it out (sl_env_common.h choose_level): in pool order
    (gid + ep * n_total) mod K, or Philox-random; rolled by Philox offsets when
    ``augment``.  This replaces the reference's level iterator
    (file_finder.py:143-201) with a deterministic per-env choice, so the oracle must
    make the same choice to follow an env across resets."""
    K = len(levels)

    def fn(ep):
        if random_order:
            idx = int(philox_uniform(gid, ep, 0x5EED, 2, seed) * K)
        else:
            idx = (gid + ep * n_total) % K
        lv = levels[min(max(idx, 0), K - 1)]
        if augment:
            H, W = lv.board.shape
            dy = min(int(philox_uniform(gid, ep, 0x0011, 3, seed) * H), H - 1)
            dx = min(int(philox_uniform(gid, ep, 0x0022, 3, seed) * W), W - 1)
            lv = lv.rolled(dy, dx)
        return lv
    return fn


class OracleEnv:
    """Per-env restatement of the PPO wrapper chain (see module docstring)."""

    def __init__(self, level_fn, time_limit=1000, view_shape=(15, 15),
                 output_channels=tuple(range(15)), remove_white_goals=True,
                 movement_bonus=0.1, movement_bonus_power=0.01,
                 movement_bonus_period=4, penalty_coef=0.0, min_performance=0.01,
                 rng="stream", stream=None, seed=0, env_id=0,
                 can_toggle_powers=False, can_toggle_colors=False):
        self.level_fn = level_fn            # callable(episode_index) -> Level
        self.time_limit = time_limit
        self.view_shape = tuple(view_shape)
        self.output_channels = output_channels
        self.remove_white_goals = remove_white_goals
        self.mb = (movement_bonus, movement_bonus_power, movement_bonus_period)
        self.penalty_coef = penalty_coef
        self.wrapper_min_performance = min_performance
        self.rng = rng
        self.stream = stream                # RefStreamRNG for rng == "stream"
        self.seed = seed
        self.env_id = env_id
        self.step_counter = 0               # global batched-step index (philox)
        self.can_toggle_powers = can_toggle_powers
        self.can_toggle_colors = can_toggle_colors
        self.episodes = 0                   # global_counter.episodes_started (this env)
        self.completed = 0                  # global_counter.episodes_completed

    # ---- game-level pieces -------------------------------------------------
    def _relative_loc(self, n_forward, n_right=0):
        dx, dy = n_right, -n_forward
        for _ in range(self.orientation):
            dx, dy = -dy, dx
        H, W = self.board.shape
        x0, y0 = self.agent_loc
        return (x0 + dx) % W, (y0 + dy) % H

    def _can_exit(self):
        if self.min_performance < 0:
            return True
        completed, total = self._perf_ratio()
        return completed >= self.min_performance * total

    def _perf_ratio(self):
        cur, possible = perf_terms(self.board, self.goals)
        return int(cur - self.baseline), int(possible - self.baseline)

    def _move_agent(self, dy, dx=0):
        b = self.board
        x0, y0 = self.agent_loc
        x1, y1 = self._relative_loc(dy, dx)
        x2, y2 = self._relative_loc(-dy, -dx)
        can_push = (abs(dy), dx) == (1, 0)
        reward = 0
        if b[y1, x1] == 0:
            b[y1, x1] = b[y0, x0]
            b[y0, x0] = 0
            self.agent_loc = (x1, y1)
        elif (b[y1, x1] & EXIT) and self._can_exit():
            self.game_over = True
            reward += 1
        elif can_push and b[y1, x1] & PUSHABLE:
            x3, y3 = self._relative_loc(dy * 2)
            if b[y3, x3] == 0:
                b[y3, x3] = b[y1, x1]
                b[y1, x1] = b[y0, x0]
                b[y0, x0] = 0
                self.agent_loc = (x1, y1)
            elif b[y3, x3] & EXIT:
                b[y1, x1] = b[y0, x0]
                b[y0, x0] = 0
                self.agent_loc = (x1, y1)
        did_move = self.agent_loc == (x1, y1) and (x0, y0) != (x1, y1)
        if can_push and b[y2, x2] & PULLABLE and did_move:
            b[y0, x0] = b[y2, x2]
            b[y2, x2] = 0
        return reward

    def _execute_action(self, name):
        reward = 0
        if self.game_over:
            pass
        elif name.startswith("MOVE "):
            self.orientation = ("UP", "RIGHT", "DOWN", "LEFT").index(name[5:])
            reward = self._move_agent(1)
        elif name.startswith("TOGGLE"):
            self.orientation = ("UP", "RIGHT", "DOWN", "LEFT").index(name[7:])
            b = self.board
            x0, y0 = self.agent_loc
            x1, y1 = self._relative_loc(1)
            player_color = b[y0, x0] & RAINBOW
            target = b[y1, x1]
            if target == 0:
                b[y1, x1] = LIFE | player_color
            elif target & DESTRUCTIBLE:
                b[y1, x1] = 0
            else:
                toggle = (ALIVE | INHIBITING | PRESERVING | SPAWNING) * self.can_toggle_powers
                toggle |= RAINBOW * self.can_toggle_colors
                b[y0, x0] ^= np.uint16(target & toggle)
        return reward

    def _advance(self, x, tensor):
        p = self.spawn_prob
        if self.rng == "stream":
            n = count_eligible(x)
            draws = self.stream.take(n)
            out, _ = advance(x, p, draws, 0, RNG_STREAM)
        else:
            out, _ = advance(x, p, None, 0, RNG_PHILOX, self.seed, self.env_id,
                             self.step_counter, tensor)
        return out

    def _update_exit_colors(self):
        v = LEVEL_EXIT | COLOR_R if self._can_exit() else LEVEL_EXIT
        for (iy, ix) in self.exits:
            self.board[iy, ix] = v

    def obs(self):
        return make_obs(self.board, self.goals, self.agent_loc[0], self.agent_loc[1],
                        self.exits, self.view_shape, self.output_channels,
                        self.remove_white_goals)

    # ---- chain -------------------------------------------------------------
    def reset(self):
        lvl = self.level_fn(self.episodes)
        self.episodes += 1
        self.init_board = lvl.board.copy()
        self.init_goals = lvl.goals.copy()
        self.board = lvl.board.copy()
        self.goals = lvl.goals.copy()
        self.spawn_prob = lvl.spawn_prob
        self.orientation = lvl.orientation
        self.agent_loc = lvl.agent_loc
        self.min_performance = lvl.min_performance
        ey, ex = np.nonzero(self.init_board & EXIT)
        self.exits = list(zip(ey.tolist(), ex.tolist()))
        self.exit_mask = (self.init_board & EXIT) > 0
        self.game_over = False
        self.num_steps = 0
        self.baseline, _ = perf_terms(self.init_board, self.init_goals)
        self._update_exit_colors()
        self.old_points = points(self.board, self.goals)
        self.episode_length = 0
        self.episode_reward = 0
        self.episode_completed = False
        o = self.obs()
        self.prior = [self.agent_loc]
        self.last_side_effect = 0
        self.min_performance = self.wrapper_min_performance
        return o

    def step(self, action):
        """Returns (obs, reward, done, info); obs is the post-reset obs on done."""
        reward = self._execute_action(ACTIONS[action])
        self.num_steps += 1
        self.board = self._advance(self.board, 0)
        self.goals = self._advance(self.goals, 1)
        new_points = points(self.board, self.goals)
        reward = np.int64(reward) + np.int64(new_points - self.old_points)
        self.old_points = new_points
        self.episode_length += 1
        self.episode_reward += reward
        self._update_exit_colors()
        times_up = self.episode_length > self.time_limit
        already_completed = self.episode_completed
        self.episode_completed = times_up or self.game_over
        if not already_completed:           # safelife_env.py:169-175
            self.completed += int(self.episode_completed)
        info = {"times_up": times_up, "episode_length": self.episode_length,
                "episode_reward": int(self.episode_reward),
                "game_over": bool(self.game_over)}
        obs = self.obs()
        # MovementBonusWrapper
        bonus, power, n = self.mb
        x0, y0 = self.agent_loc
        if len(self.prior) >= n:
            p1 = self.prior[-n]
            dist = abs(x0 - p1[0]) + abs(y0 - p1[1])
        elif len(self.prior) > 0:
            p1 = self.prior[0]
            dist = abs(x0 - p1[0]) + abs(y0 - p1[1]) + n - len(self.prior)
        else:
            dist = n
        speed = dist / n
        reward = reward + bonus * speed ** power
        self.prior.append(self.agent_loc)
        if len(self.prior) > n:
            self.prior.pop(0)
        # SimpleSideEffectPenalty
        side = side_effect_count(self.board, self.init_board, self.goals, self.exit_mask)
        reward = reward - (side - self.last_side_effect) * self.penalty_coef
        self.last_side_effect = side
        info["side_effect"] = side
        done = bool(self.episode_completed)
        # the state SafeLifeRecorder.capture_frame sees after env.step, before any reset
        # (env_wrappers.py:118-126)
        self.last_frame = (self.orientation, self.board.copy(), self.goals.copy(),
                           bool(self.game_over))
        # ContinuingEnv + caller's reset-on-done
        if done and not times_up:
            done = False
            obs = self.reset()
        elif done:
            obs = self.reset()
        self.step_counter += 1
        return obs, float(reward), done, info


    def load_state(self, s, step_counter):
        """Continue from a mid-episode state taken from a batched env: ``s`` maps the
        per-env fields of SafeLifeVecEnv (board, goals, start_board, agent_x, ...,
        prior ring, exits) to this env's values; ``step_counter`` is the batched
        step index of the next step (the Philox counter)."""
        self.board = np.array(s["board"], dtype=np.uint16)
        self.goals = np.array(s["goals"], dtype=np.uint16)
        self.init_board = np.array(s["start_board"], dtype=np.uint16)
        self.init_goals = None              # only the reset reads it (baseline below)
        self.agent_loc = (int(s["agent_x"]), int(s["agent_y"]))
        self.orientation = int(s["orientation"])
        self.game_over = bool(s["game_over"])
        self.num_steps = int(s["num_steps"])
        self.episode_length = int(s["episode_length"])
        self.episode_reward = int(s["episode_reward"])
        self.episode_completed = bool(self.game_over or
                                      self.episode_length > self.time_limit)
        self.old_points = int(s["old_points"])
        self.baseline = int(s["baseline"])
        self.spawn_prob = float(s["spawn_prob"])
        self.min_performance = float(s["min_performance"])
        self.last_side_effect = int(s["side_effect"])
        n = int(s["exit_count"])
        self.exits = [(int(s["exit_y"][k]), int(s["exit_x"][k])) for k in range(n)]
        self.exit_mask = (self.init_board & EXIT) > 0
        period = self.mb[2]
        ln, hd = int(s["prior_len"]), int(s["prior_head"])
        self.prior = [(int(s["prior_x"][(hd + k) % period]), int(s["prior_y"][(hd + k) % period]))
                      for k in range(ln)]
        self.episodes = int(s["episodes"])
        self.step_counter = int(step_counter)


# ---------------------------------------------------------------------------
# The same chain compiled (sl_cpu_step.c): bench.py's CPU baseline
# ---------------------------------------------------------------------------
class _Pool(ctypes.Structure):
    _fields_ = [("K", ctypes.c_int32), ("H", ctypes.c_int32), ("W", ctypes.c_int32),
                ("board", ctypes.c_void_p), ("goals", ctypes.c_void_p),
                ("agent_x", ctypes.c_void_p), ("agent_y", ctypes.c_void_p),
                ("orientation", ctypes.c_void_p), ("spawn_prob", ctypes.c_void_p),
                ("min_performance", ctypes.c_void_p)]


class _Cfg(ctypes.Structure):
    _fields_ = [("time_limit", ctypes.c_int32), ("view_h", ctypes.c_int32),
                ("view_w", ctypes.c_int32), ("remove_white", ctypes.c_int32),
                ("obs", ctypes.c_int32), ("bonus_period", ctypes.c_int32),
                ("level_random", ctypes.c_int32), ("augment", ctypes.c_int32),
                ("n_total", ctypes.c_int32), ("penalty_coef", ctypes.c_double),
                ("wrapper_min_perf", ctypes.c_double), ("bonus", ctypes.c_double),
                ("bonus_power", ctypes.c_double), ("seed", ctypes.c_uint64)]


class CpuBatch:
    """B envs of the PPO chain stepped by sl_cpu_step.c (Philox spawns; levels from a
    pool as pool_level_fn picks them).  Same results as B OracleEnv's."""

    SCALARS = ("agent_x", "agent_y", "orientation", "game_over", "episode_length",
               "episode_reward", "old_points", "baseline", "side_effect", "episodes",
               "completed", "exit_count")

    def __init__(self, levels, num_envs, env0=0, time_limit=1000, view_shape=(15, 15),
                 remove_white_goals=True, movement_bonus=0.1, movement_bonus_power=0.01,
                 movement_bonus_period=4, penalty_coef=0.0, min_performance=0.01, seed=0,
                 level_order="sequential", augment_roll=False, n_total_envs=None, obs=False):
        L = lib()
        self.B = int(num_envs)
        self.H, self.W = levels[0].board.shape
        self._arr = dict(
            board=np.ascontiguousarray(np.stack([lv.board for lv in levels]), np.uint16),
            goals=np.ascontiguousarray(np.stack([lv.goals for lv in levels]), np.uint16),
            agent_x=np.array([lv.agent_loc[0] for lv in levels], np.int32),
            agent_y=np.array([lv.agent_loc[1] for lv in levels], np.int32),
            orientation=np.array([lv.orientation for lv in levels], np.int32),
            spawn_prob=np.array([lv.spawn_prob for lv in levels], np.float64),
            min_performance=np.array([lv.min_performance for lv in levels], np.float64))
        p = _Pool()
        p.K, p.H, p.W = len(levels), self.H, self.W
        for k, v in self._arr.items():
            setattr(p, k, v.ctypes.data)
        self._pool = p
        c = _Cfg()
        c.time_limit = int(time_limit)
        c.view_h, c.view_w = (int(v) for v in view_shape)
        c.remove_white = int(bool(remove_white_goals))
        c.obs = int(bool(obs))
        c.bonus_period = int(movement_bonus_period)
        c.level_random = int(level_order == "random")
        c.augment = int(bool(augment_roll))
        c.n_total = int(n_total_envs or self.B)
        c.penalty_coef = float(penalty_coef)
        c.wrapper_min_perf = float(min_performance)
        c.bonus = float(movement_bonus)
        c.bonus_power = float(movement_bonus_power)
        c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self._cfg = c
        self._h = L.orc_batch_create(self.B, self.H, self.W, int(env0))
        if not self._h:
            raise MemoryError("orc_batch_create")
        self.reward = np.zeros(self.B, np.float64)
        self.done = np.zeros(self.B, np.uint8)
        self.obs = np.zeros((self.B,) + tuple(view_shape), np.uint16) if obs else None

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.orc_batch_free(h)

    def reset(self):
        if lib().orc_batch_reset(self._h, ctypes.byref(self._pool), ctypes.byref(self._cfg)):
            raise ValueError("orc_batch_reset: bad pool or config")

    def step(self, actions, threads=0):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        assert a.shape == (self.B,)
        lib().orc_batch_step(self._h, a.ctypes.data, ctypes.byref(self._pool),
                             ctypes.byref(self._cfg), self.reward.ctypes.data,
                             self.done.ctypes.data,
                             self.obs.ctypes.data if self.obs is not None else None, int(threads))
        return self.obs, self.reward, self.done

    def board(self, i, which=0):
        ptr = lib().orc_batch_board(self._h, int(i), int(which))
        return np.ctypeslib.as_array(ptr, shape=(self.H, self.W)).copy()

    def scalars(self, i):
        out = np.zeros(12, np.int64)
        lib().orc_batch_scalars(self._h, int(i), out.ctypes.data)
        return dict(zip(self.SCALARS, out.tolist()))


def max_threads():
    return int(lib().orc_max_threads())


# ---------------------------------------------------------------------------
# The PPO caller's per-step arithmetic (training/ppo.py), restated in numpy.
# ---------------------------------------------------------------------------
def choice_atol(p_dtype):
    """The tolerance numpy's legacy RandomState.choice allows on sum(p) - 1."""
    atol = np.sqrt(np.finfo(np.float64).eps)
    if np.issubdtype(p_dtype, np.floating):
        atol = max(atol, np.sqrt(np.finfo(p_dtype).eps))
    return float(atol)


def sample_action(p, u):
    """``np.random.choice(len(p), p=p)`` given its uniform draw ``u`` (ppo.py:440).

    Restates numpy's legacy ``RandomState.choice`` for a 1-d ``p`` and ``size=None``:
    p as float64, cdf = cumsum(p) / cdf[-1], index = cdf.searchsorted(u, 'right').
    Returns (index, err) with err bit0 = some p < 0, bit1 = |kahan_sum(p) - 1| > atol
    (the two ValueErrors numpy raises).  Pinned against RandomState.choice itself by
    tests/test_rollout_cpu.py."""
    atol = choice_atol(np.asarray(p).dtype)
    pd = np.asarray(p, dtype=np.float64)
    s, c = pd[0], 0.0
    for v in pd[1:]:
        y = v - c
        t = s + y
        c = (t - s) - y
        s = t
    err = (1 if np.any(pd < 0) else 0) | (2 if abs(s - 1.0) > atol else 0)
    cdf = pd.cumsum()
    cdf /= cdf[-1]
    return int(cdf.searchsorted(u, side="right")), err


def gae(rewards, end_episode, values, gamma=(0.99,), lmda=0.95, reward_clip=0.0):
    """Discounted returns and GAE advantages of ``PPO.gen_training_batch``
    (training/ppo.py:487-503), with the reference's dtypes: rewards float64 [T,N],
    end_episode bool [T,N], values float32 [T+1,N,G], gamma float32 [G]
    (ppo.py:116-117).  Returns (returns, advantages), float64 [T,N,G]."""
    rewards = np.asarray(rewards, dtype=np.float64)
    end_episode = np.asarray(end_episode, dtype=bool)
    values = np.asarray(values, dtype=np.float32)
    gamma = np.asarray(gamma, dtype=np.float32)
    steps_per_env = rewards.shape[0]
    if reward_clip > 0:
        rewards = np.clip(rewards, -reward_clip, reward_clip)
    reward_mask = ~end_episode[..., np.newaxis]
    rewards = rewards[..., np.newaxis]
    lmda = lmda * gamma
    n_gamma = len(gamma)
    advantages = rewards + gamma * reward_mask * values[1:] - values[:-1]
    returns = np.broadcast_to(rewards, rewards.shape[:-1] + (n_gamma,)).copy()
    returns[-1] += reward_mask[-1] * gamma * values[-1]
    for i in range(steps_per_env - 2, -1, -1):
        returns[i] += gamma * reward_mask[i] * returns[i + 1]
        advantages[i] += lmda * reward_mask[i] * advantages[i + 1]
    return returns, advantages
