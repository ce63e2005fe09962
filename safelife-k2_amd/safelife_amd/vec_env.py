"""SafeLifeVecEnv: B SafeLife episodes stepped together on one MI355X.

Semantics are those of the reference's PPO training chain, stepped env by env:

    env = SafeLifeEnv(level_iterator, view_shape=...)          safelife_env.py:87-198
    env = MovementBonusWrapper(env)                            env_wrappers.py:39-94
    env = SimpleSideEffectPenalty(env, penalty_coef=..., min_performance=...)
                                                               env_wrappers.py:306-346
    env = ContinuingEnv(env)                                   env_wrappers.py:289-303
    ... and PPO.run_agents resets an env whenever done         training/ppo.py:441-445
(wiring: training/safelife_ppo.py:128-139; the logging-only RecordingSafeLifeWrapper
is not part of the stepped path).

Everything per step runs in HIP kernels through the C ABI (include/safelife_hip.h);
the host only fills scalar arguments.  There is no CPU fallback.

RNG: ``rng="philox"`` (default) draws each spawn uniform from Philox4x32-10 keyed by
(seed; cell, global env id, step, tensor), so results do not depend on how the
batch is sharded.  ``rng="stream"`` replays the reference's stream in the reference's
order (env by env, board then goals, row-major eligible cells), which is how the
reference's global-numpy buffer (speedups_src/random.c) is matched: either a supplied
uniform buffer (``spawn_stream``), or, with ``spawn_stream=None``, the stream of
``speedups.seed(seed)`` -- np.random.RandomState(seed).random_sample -- generated on the
device inside each step (:class:`safelife_amd.mtstream.MT19937Stream`).
"""
import ctypes
import math

import numpy as np

from . import _lib
from .levels import LevelPool
from .spaces import Box, env_spaces

ACTION_NAMES = ("NULL", "MOVE UP", "MOVE RIGHT", "MOVE DOWN", "MOVE LEFT",
                "TOGGLE UP", "TOGGLE RIGHT", "TOGGLE DOWN", "TOGGLE LEFT")


class GlobalCounter:
    """Host mirror of SafeLifeEnv.global_counter (safelife_env.py:81-85).

    ``num_steps`` is added on the host at every step (it drives the wrapper
    schedules, env_wrappers.py:29-36).  Episode starts and completions happen inside
    the step kernels (auto-reset), so a vector env folds them in from its device
    counters at logging cadence: :meth:`SafeLifeVecEnv.sync_counters` (one sync).
    One counter may be shared by several envs, like the reference's class-level one.
    """

    def __init__(self):
        self.episodes_started = 0
        self.episodes_completed = 0
        self.num_steps = 0


def _sched(val, counter):
    # BaseWrapper.scheduled (env_wrappers.py:29-36)
    return val(counter.num_steps) if callable(val) else val


def zero_planes(bits, can_toggle_powers=False, can_toggle_colors=False):
    """sl_env_state.board_zero for boards holding cell bits `bits`: the bits none of them
    can ever hold -- not set by a birth or a spawn (LIFE; colours only where present), an
    exit (COLOR_R) or a toggle (powers / colours when those can be toggled)."""
    can = bits | 0x0009 | 0x0200
    if can_toggle_powers:
        can |= 0x00E1
    if can_toggle_colors:
        can |= 0x0E00
    return (~can) & 0xFFFF


def start_board_hi_bits(start_board):
    """Per env: does any start-board cell use bits 12-14 (used by no cell type)?"""
    import torch
    return ((start_board.view(torch.int16) & 0x7000) != 0).flatten(1).any(1)


class SafeLifeVecEnv:
    action_names = ACTION_NAMES

    def __init__(self, levels, num_envs, device=None, *, time_limit=1000,
                 view_shape=(15, 15), output_channels=tuple(range(15)),
                 remove_white_goals=True, movement_bonus=0.1, movement_bonus_power=0.01,
                 movement_bonus_period=4, penalty_coef=0.0, min_performance=0.01,
                 auto_reset=True, rng="philox", seed=0, spawn_stream=None,
                 level_order="sequential", augment_roll=False, env0=0, n_total_envs=None,
                 can_toggle_powers=False, can_toggle_colors=False, obs_dtype="uint16",
                 compute_obs=True, global_counter=None, kernel="auto", stream_exchange=None,
                 stream_ring="auto", board_mode="auto"):
        import torch
        self.torch = torch
        self.device = _lib.require_device(device)
        self.pool = levels if isinstance(levels, LevelPool) else LevelPool.from_levels(levels)
        self.B = int(num_envs)
        self.H, self.W = self.pool.H, self.pool.W
        self.time_limit = int(time_limit)
        self.view_shape = tuple(int(v) for v in view_shape)
        self.output_channels = tuple(output_channels) if output_channels else None
        self.remove_white_goals = bool(remove_white_goals)
        self.movement_bonus = movement_bonus
        self.movement_bonus_power = movement_bonus_power
        self.movement_bonus_period = int(movement_bonus_period)
        if not 0 <= self.movement_bonus_period <= _lib.SL_BONUS_PERIOD_MAX:
            raise ValueError("movement_bonus_period must be in [0, %d]" % _lib.SL_BONUS_PERIOD_MAX)
        self.penalty_coef = penalty_coef
        self.min_performance = min_performance
        self.auto_reset = bool(auto_reset)
        self.rng = rng
        self.seed = int(seed)
        self.level_order = level_order
        self.augment_roll = bool(augment_roll)
        self.env0 = int(env0)
        self.n_total_envs = int(n_total_envs) if n_total_envs else self.B
        self.can_toggle_powers = bool(can_toggle_powers)
        self.can_toggle_colors = bool(can_toggle_colors)
        self.compute_obs = bool(compute_obs)
        self.kernel = {"auto": _lib.SL_KERNEL_AUTO, "generic": _lib.SL_KERNEL_GENERIC,
                       "fast": _lib.SL_KERNEL_FAST}[kernel]
        self.global_counter = global_counter if global_counter is not None else GlobalCounter()
        # rng="stream" over shards: dist.StreamExchange (or any callable of the same
        # contract) places this shard's draws in the global stream every step
        self.stream_exchange = stream_exchange
        # the device generator's ring (rng='stream', spawn_stream=None): "auto" = a bit
        # ring when every level spawns with one threshold, else doubles; "doubles"
        if stream_ring not in ("auto", "doubles"):
            raise ValueError("stream_ring must be 'auto' or 'doubles'")
        self.stream_ring = stream_ring
        # where a 128x128 step leaves the board (sl_env_cfg.board_mode): "planes" keeps
        # it in bit planes whenever the kernel can (a `board` read then completes the
        # uint16 tensor first); "uint16" has every step write the changed rows; "auto"
        # is "planes" unless `board` was read within the last BOARD_READ_WINDOW steps --
        # a caller reading the board after every step (info['board'],
        # safelife_env.py:177-178) gets the kernel that writes it, not a sync per read
        if board_mode not in ("auto", "planes", "uint16"):
            raise ValueError("board_mode must be 'auto', 'planes' or 'uint16'")
        self.board_mode = board_mode
        self._board_read_at = None   # step index of the last `board` read
        self._step_index = 0
        # step index and auto_reset flag of the last launched step: the 64x64 and
        # 128x128 kernels queue finished envs in per-parity lists (sl_env_cfg.scratch)
        # that are valid only for consecutive auto-reset steps
        self._last_step = None
        self._abandoned = 0          # explicit resets of episodes that had not ended
        self._synced = (0, 0)        # (started, completed) already in global_counter
        self._recorder = None        # TrajectoryRecorder attached to this env
        self._draw_base = 0          # stream position of spawn_stream[0]
        self._last_mode = None       # "batch" / "reference": how the last step ran
        self._alloc(obs_dtype)
        # may any env's board or goals hold a spawning cell (bit 7)?  Spawners come only
        # from levels (no rule or action creates one) unless powers can be toggled; when
        # none can exist no uniform is ever drawn, and replay runs the Philox-form
        # kernels (identical results, no count prologue / offsets scan)
        self._may_spawn = self.pool.has_spawners()
        # the spaces of one env, as SafeLifeEnv declares them (safelife_env.py:97-109);
        # PPO reads them from envs[0] (training/ppo.py:219, safelife_ppo.py:196)
        self.action_space, self.observation_space = env_spaces(
            ACTION_NAMES, self.view_shape, self.output_channels)
        if self.output_channels is not None and obs_dtype != "uint16":
            self.observation_space = Box(0, 1, self.observation_space.shape,
                                         np.uint8 if obs_dtype == "uint8" else np.float32)
        self.mt = None
        if rng == "stream":
            if spawn_stream is None:
                # the reference's seeded stream, generated on the device: the ring holds
                # a quarter of a cell per env (C5's steady state draws 1/12), and one
                # fill can generate a whole ring.  A step drawing more (at most 2 per
                # cell: every board and goal cell eligible) sets the error flag, which
                # step_async polls (_poll_stream_error) and stream_error() reads
                self.spawn_stream = None
                self.mt = self._make_mt(0, self._pool_threshold(self.pool)
                                        if stream_ring == "auto" else None)
            else:
                self.set_spawn_stream(spawn_stream)
        elif rng != "philox":
            raise ValueError("rng must be 'philox' or 'stream'")
        self._bonus_key = None

    # ------------------------------------------------------------------ setup
    def _alloc(self, obs_dtype):
        torch, dev, B, H, W = self.torch, self.device, self.B, self.H, self.W
        z = lambda *s, dt=torch.int32: torch.zeros(s, dtype=dt, device=dev)
        self._board = z(B, H, W, dt=torch.uint16)
        self.goals = z(B, H, W, dt=torch.uint16)
        self.start_board = z(B, H, W, dt=torch.uint16)
        self.st_t = {
            "agent_x": z(B), "agent_y": z(B), "orientation": z(B), "game_over": z(B),
            "episode_length": z(B), "episode_reward": z(B), "old_points": z(B),
            "baseline": z(B), "score": z(B), "possible": z(B), "side_effect": z(B),
            "spawn_prob": z(B, dt=torch.float32), "min_performance": z(B, dt=torch.float64),
            "prior_x": z(B, _lib.SL_BONUS_PERIOD_MAX), "prior_y": z(B, _lib.SL_BONUS_PERIOD_MAX),
            "prior_len": z(B), "prior_head": z(B), "exit_count": z(B),
            "exit_y": z(B, _lib.SL_MAX_EXITS, dt=torch.int16),
            "exit_x": z(B, _lib.SL_MAX_EXITS, dt=torch.int16),
            "level_index": z(B), "episodes": z(B), "num_steps": z(B), "spawn_flags": z(B),
            # (dy << 16) | dx of the pool roll the start board came from; -1 = set by caller
            "start_roll": z(B) - 1,
        }
        s = _lib.EnvState()
        s.B, s.H, s.W = B, H, W
        s.board, s.goals, s.start_board = (self._board.data_ptr(), self.goals.data_ptr(),
                                           self.start_board.data_ptr())
        for k, t in self.st_t.items():
            setattr(s, k, t.data_ptr())
        # bit-plane mirror of the goals kept by the bit-sliced kernels (derived data):
        # 64x64 [B, 2, 32, 64] (half 1 = goals), 128x128 [B, 4 bands, 32, 64]
        self.planes_ok = z(B)
        if (H, W) in ((64, 64), (128, 128)):
            self.planes = z(B, H // 32, 32, 64)
            s.planes = self.planes.data_ptr()
            s.planes_ok = self.planes_ok.data_ptr()
        self.board_planes = None
        if (H, W) == (64, 64):
            # the 64x64 board's planes share the goals mirror's tensor (half 0; the goals
            # use half 1): board_planes == planes selects plane mode (sl_bits.hip)
            self.board_planes = self.planes
            s.board_planes = self.planes.data_ptr()
            s.board_zero = self._zero_planes(self._pool_bits(self.pool))
        if (H, W) == (128, 128):
            # the 128x128 board in bit planes, kept there by steps without observations
            # or with packed views (sl_env_state.board_planes); `board` completes the
            # uint16 tensor when it is read
            self.board_planes = z(B, H // 32, 32, 64)
            s.board_planes = self.board_planes.data_ptr()
            s.board_zero = self._zero_planes(self._pool_bits(self.pool))
        if (H, W) == (128, 128) and self.rng == "stream":
            # replay's draw planes: each tensor's eligible cells, then its decided
            # spawns (4 KiB per env)
            self.elig_planes = z(B, 1024)
            s.elig_planes = self.elig_planes.data_ptr()
        self._state = s
        self.actions_dev = z(B)
        self.reward = z(B, dt=torch.float64)
        self.done = z(B, dt=torch.uint8)
        self.flags = z(B, dt=torch.uint8)
        self.ep_len = z(B)
        self.ep_rew = z(B)
        self.scratch = z(8 * B + 16, dt=torch.int64)
        self.stream_pos = z(1, dt=torch.int64)
        vh, vw = self.view_shape
        if self.output_channels is None:
            self.obs_mode = _lib.SL_OBS_PACKED
            self.obs = z(B, vh, vw, dt=torch.uint16)
        else:
            nch = len(self.output_channels)
            modes = {"uint16": (_lib.SL_OBS_CHANNELS, torch.uint16),
                     "uint8": (_lib.SL_OBS_CHANNELS_U8, torch.uint8),
                     "float32": (_lib.SL_OBS_CHANNELS_F32, torch.float32),
                     "bfloat16": (_lib.SL_OBS_CHANNELS_BF16, torch.bfloat16)}
            if obs_dtype not in modes:
                raise ValueError("obs_dtype must be one of %s" % sorted(modes))
            self.obs_mode, dt = modes[obs_dtype]
            self.obs = z(B, vh, vw, nch, dt=dt)
            self._channels = (ctypes.c_int32 * nch)(*self.output_channels)
        self._pool_dev = self.pool.to_device(self.device)
        self._cfg = _lib.EnvCfg()

    # ------------------------------------------------- 64x64 planes that stay zero
    @staticmethod
    def _pool_bits(pool):
        return int(np.bitwise_or.reduce(pool.board.reshape(-1))) if pool.board.size else 0

    def _zero_planes(self, bits):
        """sl_env_state.board_zero of this batch for boards with cell bits `bits`."""
        return zero_planes(bits, self.can_toggle_powers, self.can_toggle_colors)

    def _allow_board_bits(self, bits):
        """Boards with cell bits `bits` are about to enter the batch: planes that must now
        be loaded and stored leave board_zero.  Envs kept in planes under the old mask are
        completed and taken out of plane mode first (their planes in the new mask's
        complement were never written)."""
        s = self._state
        if not s.board_zero:
            return
        new = s.board_zero & self._zero_planes(bits)
        if new != s.board_zero:
            self.sync_board()
            self.planes_ok.bitwise_and_(~(64 | 128))
            s.board_zero = new
            s.planes_live = 0

    def _device_board_bits(self, boards):
        """OR of every cell of a uint16 device tensor (16 reductions; rare events only)."""
        v = boards.view(self.torch.int16)
        return sum(1 << k for k in range(16) if bool(((v >> k) & 1).any().item()))

    def set_pool(self, levels, pool_dev=None):
        """Replace the level pool the next resets draw from (same board shape).

        ``pool_dev`` is an already uploaded ``levels.to_device(...)`` (see
        :class:`safelife_amd.pool_feed.PoolFeeder`, which uploads on a side stream);
        the swap itself is stream-ordered and does not synchronise the host."""
        pool = levels if isinstance(levels, LevelPool) else LevelPool.from_levels(levels)
        if (pool.H, pool.W) != (self.H, self.W):
            raise ValueError("pool boards are %dx%d, the env's %dx%d"
                             % (pool.H, pool.W, self.H, self.W))
        if pool.K < 1:
            raise ValueError("empty level pool")
        self._allow_board_bits(self._pool_bits(pool))
        self.pool = pool
        self._pool_dev = pool_dev if pool_dev is not None else pool.to_device(self.device)
        self._check_ring_threshold(pool.spawn_prob)
        # running envs keep their old-pool boards: the flag only grows here
        self._may_spawn = self._may_spawn or pool.has_spawners()
        # running episodes' start boards are no longer levels of the pool: the
        # kernels read them from HBM until those envs are reset from the new pool
        self.st_t["start_roll"].fill_(-1)

    # ------------------------------------------------- the device generator's ring
    @staticmethod
    def _pool_threshold(pool):
        """The one spawn threshold (double)(float)p of every level of the pool, or
        None when they differ."""
        t = set(float(np.float32(p)) for p in np.asarray(pool.spawn_prob).reshape(-1))
        return t.pop() if len(t) == 1 else None

    def _make_mt(self, first_draw, bits_threshold):
        """The reference's seeded stream on the device (rng='stream', no spawn_stream):
        a ring of a quarter of a cell per env (C5's steady state draws 1/12), one fill
        able to generate a whole ring; a bit ring (decisions, not doubles) when every
        env spawns with one threshold.  A step drawing more (at most 2 per cell) sets
        the error flag, which step_async polls (_poll_stream_error)."""
        from .mtstream import MT19937Stream
        import os
        # blocks: longer ones mean fewer chain jumps (one per block, the dominant cost
        # once the ring holds bits and generation no longer writes HBM)
        rounds = int(os.environ.get("SAFELIFE_MT_ROUNDS",
                                    self.MT_ROUNDS_BITS if bits_threshold is not None else 420))
        return MT19937Stream(self.seed, self.device, first_draw=first_draw,
                             ring_draws=max(1 << 22, self.n_total_envs * self.H * self.W // 4),
                             lookahead=self.stream_exchange is None,
                             bits_threshold=bits_threshold, rounds=rounds)

    MT_ROUNDS_BITS = 840         # (C5 seeded, 128-thread generator blocks: 840 48.4 M,
                                 # 1680 32.2; 256 threads: 420 44.9, 840 47.5-47.8, 1680 47.2-48.6)

    def _check_ring_threshold(self, probs=None):
        """A bit ring serves only envs with its threshold: when spawn_prob may have
        changed (set_state, load_state_dict, set_pool, a game's setter) and some env or
        pool level no longer has it, the generator is rebuilt as a ring of doubles at
        the current stream position."""
        mt = self.mt
        if mt is None or mt.bits_threshold is None:
            return
        if probs is None:
            cur = self.st_t["spawn_prob"].to(self.torch.float64)
            same = bool((cur == mt.bits_threshold).all().item())
            same = same and self._pool_threshold(self.pool) == mt.bits_threshold
        else:
            same = all(float(np.float32(p)) == mt.bits_threshold
                       for p in np.asarray(probs).reshape(-1))
        if not same:
            self.mt = None
            self.torch.cuda.synchronize(self.device)
            pos = getattr(self.stream_exchange, "pos", None)
            self.mt = self._make_mt(int((pos if pos is not None else self.stream_pos).item()),
                                    None)

    def set_spawn_stream(self, stream, pos=0):
        """Uniform doubles consumed in reference order (rng='stream'): a numpy array,
        or a float64 tensor (used in place when it is already on this device)."""
        torch = self.torch
        if isinstance(stream, torch.Tensor):
            s = stream.to(device=self.device, dtype=torch.float64).contiguous()
        else:
            s = torch.as_tensor(np.ascontiguousarray(stream, dtype=np.float64)).to(self.device)
        self.spawn_stream = s
        self.mt = None
        self._draw_base = 0
        self.stream_pos.fill_(int(pos))

    def seek_stream(self, pos):
        """Move the replay stream to draw `pos` (the device generator re-seeds there)."""
        self.stream_pos.fill_(int(pos))
        if self.mt is not None:
            self.mt.seek(int(pos))

    def _bonus_table(self):
        key = (self.movement_bonus, self.movement_bonus_power, self.movement_bonus_period)
        if self._bonus_key != key:
            n = self.movement_bonus_period
            dmax = self.H + self.W + n + 2
            # evaluated in Python exactly as MovementBonusWrapper.step does
            vals = [self.movement_bonus * (d / n) ** self.movement_bonus_power if n else 0.0
                    for d in range(dmax)]
            self._bonus_t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.device)
            self._bonus_key = key
        return self._bonus_t

    def _fill_cfg(self):
        c = self._cfg
        gc = self.global_counter
        c.time_limit = self.time_limit
        c.auto_reset = int(self.auto_reset)
        c.can_toggle_powers = int(self.can_toggle_powers)
        c.can_toggle_colors = int(self.can_toggle_colors)
        c.penalty_coef = float(_sched(self.penalty_coef, gc))
        mp = _sched(self.min_performance, gc)
        c.wrapper_min_performance = float("nan") if mp is None else float(mp)
        bt = self._bonus_table()
        c.bonus_table = bt.data_ptr()
        c.bonus_len = bt.numel()
        c.bonus_period = self.movement_bonus_period
        if self.can_toggle_powers:      # a power toggle can make a spawner: sticky
            self._may_spawn = True
        # (shards exchange totals every step whether or not they can draw, so every
        # rank makes the same collective calls)
        replay = self.rng == "stream" and (self._may_spawn or self.stream_exchange is not None)
        c.rng_mode = _lib.SL_RNG_STREAM if replay else _lib.SL_RNG_PHILOX
        c.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        c.step = self._step_index & 0xFFFFFFFF
        c.env0 = self.env0
        c.mt = None
        if self.rng == "stream" and self.mt is not None:
            c.draws = None
            c.n_draws = 0
            c.mt = ctypes.addressof(self.mt.struct)
        elif self.rng == "stream":
            # _draw_base: the supplied buffer starts at this stream position (a window
            # of the stream staged per step by the single-env drop-in)
            c.draws = self.spawn_stream.data_ptr() - 8 * self._draw_base
            c.n_draws = self.spawn_stream.numel() + self._draw_base
        else:
            c.draws = None
            c.n_draws = 0
        c.stream_pos = self.stream_pos.data_ptr()
        c.stream_phase = 0
        c.stream_base = None
        c.scratch = self.scratch.data_ptr()
        c.level_mode = 1 if self.level_order == "random" else 0
        c.n_total_envs = self.n_total_envs
        c.augment_roll = int(self.augment_roll)
        c.kernel = self.kernel
        c.board_mode = _lib.SL_BOARD_UINT16 if self._wants_uint16_board() else _lib.SL_BOARD_AUTO
        return c

    BOARD_READ_WINDOW = 4

    def _wants_uint16_board(self):
        if self.board_mode != "auto":
            return self.board_mode == "uint16"
        return (self._board_read_at is not None
                and self._step_index - self._board_read_at <= self.BOARD_READ_WINDOW)

    # -------------------------------------------------------------- gym-ish API
    def reset(self, mask=None):
        """Reset all envs (or those with mask[b] != 0); returns observations."""
        L = _lib.lib()
        cfg = self._fill_cfg()
        m = None
        if mask is not None:
            m = self.torch.as_tensor(mask, device=self.device).to(self.torch.uint8).contiguous()
            if m.numel() != self.B:
                raise ValueError("reset mask must have %d entries" % self.B)
        # episodes cut short by this reset were started but never completed
        # (SafeLifeEnv.step counts a completion only when an episode ends)
        running = self._running_mask()
        if m is not None:
            running = running & (m.reshape(self.B) != 0)
        self._abandoned += int(running.sum().item())
        if m is None:           # every env starts from the pool: only its levels count
            self._may_spawn = self.pool.has_spawners()
        _lib.check(L.sl_env_reset(ctypes.byref(self._state), ctypes.byref(self._pool_dev["struct"]),
                                  _lib.ptr(m), ctypes.byref(cfg), _lib.stream_ptr(self.device)),
                   "sl_env_reset")
        self.sync_counters()
        if self._recorder is not None:
            self._recorder.on_reset(None if m is None else m.cpu().numpy())
        return self.observe() if self.compute_obs else None

    def _running_mask(self):
        """Envs inside an episode that has not ended (started, neither game over nor
        past the time limit: safelife_env.py:167-168)."""
        st = self.st_t
        ended = (st["game_over"] != 0) | (st["episode_length"] > self.time_limit)
        return (st["episodes"] > 0) & ~ended

    def sync_counters(self):
        """Fold the episodes started / completed since the last call into
        ``global_counter`` (one device sync; call at logging cadence).

        Every reset, explicit or automatic, bumps the env's device episode count;
        an episode is completed unless it is still running or was cut short by an
        explicit reset."""
        started = int(self.st_t["episodes"].sum().item())
        completed = started - int(self._running_mask().sum().item()) - self._abandoned
        s0, c0 = self._synced
        self.global_counter.episodes_started += started - s0
        self.global_counter.episodes_completed += completed - c0
        self._synced = (started, completed)
        return self.global_counter

    def observe(self, out=None):
        """Write the observations into `out` (a tensor shaped and typed like
        self.obs, e.g. one slot of a rollout buffer) or self.obs; returns it."""
        L = _lib.lib()
        vh, vw = self.view_shape
        ch = self._channels if self.obs_mode != _lib.SL_OBS_PACKED else None
        nch = len(self.output_channels) if self.output_channels else 0
        out = self.obs if out is None else self._obs_target(out)
        _lib.check(L.sl_env_obs(ctypes.byref(self._state), vh, vw, int(self.remove_white_goals),
                                self.obs_mode, ch, nch, out.data_ptr(),
                                _lib.stream_ptr(self.device)), "sl_env_obs")
        return out

    def step(self, actions):
        """One env-step for every env.  `actions`: int [B] (torch or numpy), 0..8.

        Returns (obs, reward float64 [B], done bool [B], info) as device tensors.
        Envs that finished are already reset (ContinuingEnv + run_agents semantics);
        their obs are those of the new episode.
        """
        self.step_async(actions)
        return self.step_wait()

    def step_async(self, actions, reward_out=None, done_out=None, obs_out=None,
                   flags_out=None, ep_len_out=None, ep_rew_out=None):
        """Launch one env-step (stream-ordered, no host sync).  reward_out (float64
        [B]), done_out / flags_out (uint8 [B]), ep_len_out / ep_rew_out (int32 [B])
        and obs_out (like self.obs) optionally redirect the outputs, e.g. into one
        time slot of a rollout buffer; the env's own tensors are then left as they
        were."""
        torch = self.torch
        a = torch.as_tensor(actions)
        if a.device != self.device or a.dtype != torch.int32:
            a = a.to(device=self.device, dtype=torch.int32)
        a = a.reshape(self.B)
        if not a.is_contiguous():
            a = a.contiguous()
        # the kernel reads the caller's int32 device tensor in place (stream-ordered);
        # keep a reference until the next step
        self._actions_in_flight = a
        L = _lib.lib()
        if self._last_mode == "reference" and self.planes_ok is not None:
            self.planes_ok.bitwise_and_(~8)     # (see step_env_reference)
        self._last_mode = "batch"
        cfg = self._fill_cfg()
        self._check_reset_lists()
        cfg.capture = self._recorder._next_capture() if self._recorder is not None else None
        # the observation is written by sl_env_step itself (from the on-chip board
        # where the kernel allows it)
        obs = None
        if self.compute_obs or obs_out is not None:
            obs = self.obs if obs_out is None else self._obs_target(obs_out)
        self._fill_obs_cfg(cfg, obs)
        outs = [self._out(reward_out, self.reward), self._out(done_out, self.done),
                self._out(flags_out, self.flags), self._out(ep_len_out, self.ep_len),
                self._out(ep_rew_out, self.ep_rew)]

        def launch():
            _lib.check(L.sl_env_step(ctypes.byref(self._state),
                                     ctypes.byref(self._pool_dev["struct"]), a.data_ptr(),
                                     ctypes.byref(cfg), *[o.data_ptr() for o in outs],
                                     _lib.stream_ptr(self.device)), "sl_env_step")
        if cfg.rng_mode == _lib.SL_RNG_STREAM and self.stream_exchange is not None:
            # parity mode over shards: counts -> totals exchanged -> this shard's base
            cfg.stream_phase = 1
            launch()
            self._stream_base = self.stream_exchange(self.stream_pos)
            cfg.stream_phase = 2
            cfg.stream_base = self._stream_base.data_ptr()
        launch()
        self._step_index += 1
        self.global_counter.num_steps += self.B
        if self.mt is not None and self._step_index % self.STREAM_CHECK_EVERY == 0:
            self._poll_stream_error()

    # the device generator's error flag is polled every this many steps, without a sync
    STREAM_CHECK_EVERY = 16

    def _poll_stream_error(self):
        """rng='stream' with the device generator: a step whose range the ring cannot
        serve (a fill wider than the ring, or rewound below it) sets the error flag
        and the replay would read stale draws.  The flag is copied to pinned host
        memory behind the step (no sync) and the copy of the last poll is read, so a
        failure raises at most 2 * STREAM_CHECK_EVERY steps late."""
        torch = self.torch
        if getattr(self, "_err_h", None) is None:
            self._err_h = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._err_ev = None
        if self._err_ev is not None and self._err_ev.query():
            self._raise_stream_error(int(self._err_h[0]))
        self._err_h.copy_(self.scratch[8 * self.B:8 * self.B + 1], non_blocking=True)
        self._err_ev = torch.cuda.Event()
        self._err_ev.record(torch.cuda.current_stream(self.device))

    @staticmethod
    def _raise_stream_error(flag):
        if flag & _lib.SL_STREAM_ERR_THRESHOLD:
            raise RuntimeError("rng='stream': an env drew with a spawn threshold other than "
                               "the device generator's bit ring holds (spawn_prob changed "
                               "outside set_state / load_state_dict / set_pool, e.g. by "
                               "writing st_t['spawn_prob'] directly); rebuild the ring with "
                               "stream_ring='doubles' or through set_state")
        if flag & _lib.SL_STREAM_ERR_RANGE:
            raise RuntimeError("rng='stream': the device generator could not serve a step's "
                               "draw range (ring too small for the draws per step, or a "
                               "rewind); re-seed with seek_stream / a larger ring")

    # ------------------------------------------------- the reference's PPO loop order
    def step_env_reference(self, e, action, *, reward_out=None, done_out=None, obs_out=None,
                           flags_out=None, ep_len_out=None, ep_rew_out=None):
        """One env-step of env ``e`` alone, its spawn draws taken from the reference's
        global numpy stream: speedups' emulated 10 000-double buffer, refilled from
        np.random when it runs out (random.c:14-26,47-52).  The reference's PPO loop
        steps its envs one after another (training/ppo.py:438-448), so env e's draws
        follow the previous envs' draws and the np.random.choice calls in between in
        one stream; rollout.run_agents(rng="reference") drives this.  The outputs
        (full [B] tensors, like step_async's) get env e's entry.  The step runs the
        replay kernels on the one-env slice (state_slice) with the next 2 H W draws
        staged; one host sync reads how many it consumed, which the buffer then
        gives up."""
        from . import speedups
        torch = self.torch
        if self.rng != "stream":
            raise ValueError("step_env_reference needs rng='stream'")
        if self._recorder is not None:
            raise ValueError("step_env_reference does not record (detach the recorder)")
        if not 0 <= e < self.B:
            raise IndexError("env %d outside [0, %d)" % (e, self.B))
        fr = self._ref_frame()
        if self._last_mode != "reference" and self.planes_ok is not None:
            # the 128x128 replay keeps each env's next-step eligible count in the scratch
            # (act[2B + b]); the reference steps keep theirs per env in fr["scratch"],
            # so the draw planes are recounted from the board once on a switch
            self.planes_ok.bitwise_and_(~8)
        self._last_mode = "reference"
        n2 = 2 * self.H * self.W
        fr["draws_h"].numpy()[:] = speedups._buffer.peek(n2)
        fr["draws_d"].copy_(fr["draws_h"], non_blocking=True)
        fr["act_h"][0] = int(action)
        fr["act_d"].copy_(fr["act_h"], non_blocking=True)
        fr["pos"].zero_()
        sc = fr["scratch"][e]
        sc[8 + 2:8 + 4].zero_()
        cfg = _lib.EnvCfg.from_buffer_copy(self._fill_cfg())
        cfg.rng_mode = _lib.SL_RNG_STREAM
        cfg.draws, cfg.n_draws = fr["draws_d"].data_ptr(), n2
        cfg.stream_pos, cfg.mt = fr["pos"].data_ptr(), None
        cfg.stream_phase, cfg.stream_base = 0, None
        cfg.scratch = sc.data_ptr()
        cfg.env0 = self.env0 + e
        cfg.capture = None
        obs = None
        if self.compute_obs or obs_out is not None:
            obs = (self.obs if obs_out is None else self._obs_target(obs_out))[e:e + 1]
        self._fill_obs_cfg(cfg, obs)
        outs = [self._out(o, d)[e:e + 1] for o, d in
                ((reward_out, self.reward), (done_out, self.done), (flags_out, self.flags),
                 (ep_len_out, self.ep_len), (ep_rew_out, self.ep_rew))]
        st = self.state_slice(e, 1)
        _lib.check(_lib.lib().sl_env_step(ctypes.byref(st), ctypes.byref(self._pool_dev["struct"]),
                                          fr["act_d"].data_ptr(), ctypes.byref(cfg),
                                          *[o.data_ptr() for o in outs],
                                          _lib.stream_ptr(self.device)), "sl_env_step")
        self._state.planes_live |= st.planes_live     # (the slice may have left planes)
        if self.stream_error_of(sc, 1):
            raise RuntimeError("reference step consumed more draws than staged")
        speedups._buffer.take(int(fr["pos"].item()))
        self.global_counter.num_steps += 1

    def end_reference_step(self):
        """After every env took its step_env_reference: the batch's step index moves
        on, and the batched reset lists start afresh."""
        self._step_index += 1
        self._last_step = None

    def _ref_frame(self):
        fr = getattr(self, "_ref_frame_data", None)
        if fr is None:
            torch, n2 = self.torch, 2 * self.H * self.W
            fr = {"draws_h": torch.empty(n2, dtype=torch.float64, pin_memory=True),
                  "draws_d": torch.empty(n2, dtype=torch.float64, device=self.device),
                  "act_h": torch.empty(1, dtype=torch.int32, pin_memory=True),
                  "act_d": torch.empty(1, dtype=torch.int32, device=self.device),
                  "pos": torch.zeros(1, dtype=torch.int64, device=self.device),
                  # one 1-env scratch per env: the 128x128 replay carries state in it
                  # from one step of the env to the next
                  "scratch": torch.zeros((self.B, 8 + 16), dtype=torch.int64,
                                         device=self.device)}
            self._ref_frame_data = fr
        return fr

    @staticmethod
    def stream_error_of(scratch, B):
        return bool(scratch[8 * B].item() & (_lib.SL_STREAM_ERR_RANGE | _lib.SL_STREAM_ERR_THRESHOLD))

    def _check_reset_lists(self):
        """Zero the per-parity reset-list lengths (scratch[8B+2 : 8B+4]) unless this
        step directly follows an auto-reset step: each step's reset kernel zeroes
        only the other parity's list (sl_env_common.h, Scratch)."""
        cur = (self._step_index, self.auto_reset)
        last = self._last_step
        if not (self.auto_reset and last is not None and last[1]
                and last[0] + 1 == self._step_index):
            self.scratch[8 * self.B + 2:8 * self.B + 4].zero_()
        self._last_step = cur

    def _fill_obs_cfg(self, cfg, out):
        cfg.obs_out = None if out is None else out.data_ptr()
        vh, vw = self.view_shape
        cfg.obs_mode = self.obs_mode
        cfg.obs_vh, cfg.obs_vw = vh, vw
        cfg.obs_remove_white = int(self.remove_white_goals)
        chs = self.output_channels or ()
        cfg.obs_nch = len(chs)
        for k, c in enumerate(chs):
            cfg.obs_channels[k] = c

    def _obs_target(self, out):
        if (out.shape != self.obs.shape or out.dtype != self.obs.dtype
                or out.device != self.device or not out.is_contiguous()):
            raise ValueError("obs out must be a contiguous %s %s tensor on %s"
                             % (tuple(self.obs.shape), self.obs.dtype, self.device))
        return out

    def _out(self, t, default):
        if t is None:
            return default
        if (t.shape != default.shape or t.dtype != default.dtype or t.device != self.device
                or not t.is_contiguous()):
            raise ValueError("output must be a contiguous %s %s tensor on %s"
                             % (tuple(default.shape), default.dtype, self.device))
        return t

    def step_wait(self):
        info = {"times_up": (self.flags & 1) != 0, "game_over": (self.flags & 2) != 0,
                "reset": (self.flags & 4) != 0, "episode_length": self.ep_len,
                "episode_reward": self.ep_rew}
        return (self.obs if self.compute_obs else None), self.reward, self.done.bool(), info

    # ---------------------------------------------------------------- helpers
    def state_slice(self, i0, n=1):
        """An sl_env_state addressing envs [i0, i0 + n) of this batch: every per-env
        pointer offset by i0 envs (the C ABI's slicing convention), for the
        game-level entry points (sl_env_action / _advance / _rescore /
        _exit_colors) on part of the batch."""
        if not (0 <= i0 and n >= 0 and i0 + n <= self.B):
            raise IndexError("env slice [%d, %d) outside [0, %d)" % (i0, i0 + n, self.B))
        full, s = self._state, _lib.EnvState()
        s.B, s.H, s.W = n, self.H, self.W
        for name, _ in _lib.EnvState._fields_[3:]:
            base = getattr(full, name)
            if name in ("board_zero", "planes_live"):     # (not per-env pointers)
                setattr(s, name, base)
                continue
            if not base:
                setattr(s, name, None)
                continue
            t = self._state_tensor(name)
            setattr(s, name, base + i0 * (t.stride(0) * t.element_size()))
        return s

    def _state_tensor(self, name):
        if name == "board":
            return self._board
        if name in ("goals", "start_board", "planes", "planes_ok", "elig_planes", "board_planes"):
            return getattr(self, name)
        return self.st_t[name]

    @property
    def board(self):
        """uint16 [B, H, W] boards.  A 128x128 batch keeps its boards in bit planes
        across its steps (sl_env_state.board_planes); reading this always completes the
        tensor first (sl_env_board_sync, stream-ordered).  Whether an env's uint16 board
        is complete is decided on the device, per env (planes_ok bits 6-7), never by a
        host flag: an env whose board is already complete costs its workgroup one load.
        Write boards through set_state / load_state_dict (or clear planes_ok after
        writing).  With board_mode="auto" a read also makes the next
        BOARD_READ_WINDOW steps write the uint16 board themselves."""
        self._board_read_at = self._step_index
        self.sync_board()
        return self._board

    def sync_board(self):
        """Complete the uint16 boards of envs whose board lives in planes (no-op
        otherwise; no host sync)."""
        L = _lib.lib()
        # (an A/B build of an older revision, SAFELIFE_HIP_LIB, has no board planes)
        if self.board_planes is not None and hasattr(L, "sl_env_board_sync"):
            _lib.check(L.sl_env_board_sync(ctypes.byref(self._state),
                                           _lib.stream_ptr(self.device)),
                       "sl_env_board_sync")

    @property
    def state(self):
        """Per-env scalar state tensors (agent_x, agent_y, orientation, ...)."""
        return self.st_t

    def stream_error(self):
        """True if rng='stream' ran past the end of the supplied stream (or asked the
        device generator for a range it could not serve)."""
        return bool(self.scratch[8 * self.B].item()
                    & (_lib.SL_STREAM_ERR_RANGE | _lib.SL_STREAM_ERR_THRESHOLD))

    def set_state(self, board, goals, start_board, **scalars):
        """Load explicit state (for tests / checkpoints).  Arrays are [B,...]."""
        torch = self.torch
        for dst, src in ((self._board, board), (self.goals, goals), (self.start_board, start_board)):
            dst.copy_(torch.as_tensor(np.ascontiguousarray(src, dtype=np.uint16)).to(self.device))
        for k, v in scalars.items():
            t = self.st_t[k]
            t.copy_(torch.as_tensor(np.asarray(v)).to(device=self.device, dtype=t.dtype))
        self._invalidate_caches()

    def _invalidate_caches(self):
        """After state was written from outside the kernels: the start boards no
        longer match pool levels (kernels read them from HBM), the bit-plane
        mirrors are stale and the reset lists start empty."""
        self.st_t["start_roll"].fill_(-1)
        if self._state.board_zero:      # boards written from outside: their bits count
            self._state.board_zero &= self._zero_planes(self._device_board_bits(self._board)
                                                        | self._device_board_bits(self.start_board))
        # may hold spawners (replay counts them); bit 2 (128x128 boards): the start board
        # uses cell bits 12-14, which the 128x128 kernel then compares in a second pass
        hi = start_board_hi_bits(self.start_board) & ((self.H, self.W) == (128, 128))
        self.st_t["spawn_flags"].copy_(3 | 4 * hi.to(self.st_t["spawn_flags"].dtype))
        self._may_spawn = True
        self.planes_ok.zero_()
        self.scratch[8 * self.B + 2:8 * self.B + 4].zero_()
        self._last_step = None
        self._check_ring_threshold()
        self._synced = (int(self.st_t["episodes"].sum().item()),
                        int(self.st_t["episodes"].sum().item())
                        - int(self._running_mask().sum().item()) - self._abandoned)

    def state_dict(self):
        d = {"board": self.board.clone(), "goals": self.goals.clone(),
             "start_board": self.start_board.clone(), "step_index": self._step_index,
             "stream_pos": self.stream_pos.clone()}
        pos = getattr(self.stream_exchange, "pos", None)
        if pos is not None:
            # parity mode over shards: the global stream position lives in the exchange
            d["exchange_pos"] = pos.clone()
        d.update({k: v.clone() for k, v in self.st_t.items()})
        return d

    def load_state_dict(self, d):
        """Restore a state_dict().  The start boards are restored from the dict and
        read from HBM (start_roll = -1), so level_index is informational: a snapshot
        taken before a swap to a smaller pool restores, with a warning."""
        li = d["level_index"]
        if int(li.min().item()) < 0 or int(li.max().item()) >= self.pool.K:
            import warnings
            warnings.warn("state_dict level_index outside the current pool of %d levels"
                          " (informational only)" % self.pool.K)
        self._board.copy_(d["board"])
        self.goals.copy_(d["goals"])
        self.start_board.copy_(d["start_board"])
        for k, v in self.st_t.items():
            v.copy_(d[k])
        self._step_index = int(d["step_index"])
        self.stream_pos.copy_(d["stream_pos"])
        pos = getattr(self.stream_exchange, "pos", None)
        if pos is not None and "exchange_pos" in d:
            pos.copy_(d["exchange_pos"])
        if self.mt is not None:      # the next step reads from the (global) position on
            self.mt.seek(int((pos if pos is not None else self.stream_pos).item()))
        self._invalidate_caches()
