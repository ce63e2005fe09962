"""Trajectory recording from device tensors.

The reference records chosen episodes with ``SafeLifeRecorder``
(/root/reference/safelife/env_wrappers.py:97-136), driven by
``RecordingSafeLifeWrapper`` (:139-286): a frame (orientation, board, goals) is
captured when the episode starts and after every step while the game is not over,
and the episode's frames are written with ``np.savez_compressed`` to
``<base_path>.npz`` (keys ``orientation``, ``board``, ``goals``) when the episode
ends.  Episodes are recorded when ``episode_num % video_recording_freq == 0``.

On the device, ``sl_env_step`` copies the chosen envs' state into a ring of capture
slots twice per step (``sl_capture``: after the board advance, before any reset --
the reference's post-step frame -- and after the resets: the next episode's first
frame).  Nothing is synchronised per step; the ring is copied to the host when it
fills or at :meth:`TrajectoryRecorder.flush` (logging cadence), and the episodes
are cut from the per-step flags.

Divergence, documented: the reference numbers episodes with the process-wide
``global_counter.episodes_started``; here each recorded env numbers its own
episodes (1, 2, ...), so ``video_recording_freq`` applies per env.  Videos (gym's
VideoRecorder / rendering) are out of scope; only the npz trajectory is written.
"""
import ctypes
import os

import numpy as np

from . import _lib


class TrajectoryRecorder:
    """Record episodes of the envs ``env_ids`` of a SafeLifeVecEnv.

    video_name: path template, formatted with ``env`` (global env id),
    ``episode_num`` (the env's episode number, from 1) and ``step_num`` (the
    batched step index at the episode's start); ``.npz`` is appended, and
    " (k)" before it when the file exists (RecordingSafeLifeWrapper's rule).
    """

    def __init__(self, venv, video_name, env_ids=(0,), video_recording_freq=100, ring=128):
        if not venv.auto_reset:
            raise ValueError("TrajectoryRecorder needs auto_reset=True (episodes are cut "
                             "at the resets inside sl_env_step)")
        torch = venv.torch
        self.venv = venv
        self.video_name = video_name
        self.freq = max(1, int(video_recording_freq))
        self.env_ids = [int(e) for e in env_ids]
        if not self.env_ids or min(self.env_ids) < 0 or max(self.env_ids) >= venv.B:
            raise ValueError("env_ids must be env indices in [0, %d)" % venv.B)
        n, R, H, W, dev = len(self.env_ids), int(ring), venv.H, venv.W, venv.device
        self.R = R
        self._ids = torch.tensor(self.env_ids, dtype=torch.int32, device=dev)
        z = lambda *s, dt: torch.zeros(s, dtype=dt, device=dev)   # noqa: E731
        self._b0, self._g0 = z(R, n, H, W, dt=torch.uint16), z(R, n, H, W, dt=torch.uint16)
        self._b1, self._g1 = z(R, n, H, W, dt=torch.uint16), z(R, n, H, W, dt=torch.uint16)
        self._o0, self._o1 = z(R, n, dt=torch.int32), z(R, n, dt=torch.int32)
        self._f = z(R, n, dt=torch.uint8)
        self._cap = _lib.Capture()
        self._slot = 0
        self._slot_step = []
        self.files = []
        st = venv.st_t
        eps = st["episodes"][self._ids.long()].cpu().numpy()
        lens = st["episode_length"][self._ids.long()].cpu().numpy()
        self._ep = [int(x) for x in eps]
        self._rec = [None] * n
        for i, e in enumerate(self.env_ids):
            # an env at the start of an episode is recorded from its first frame;
            # otherwise from its next episode on
            if self._ep[i] > 0 and lens[i] == 0 and self._wanted(self._ep[i]):
                self._start(i, venv._step_index, self._state_frame(e))
        venv._recorder = self

    # --------------------------------------------------------------- per step
    def _wanted(self, ep):
        return ep % self.freq == 0

    def _next_capture(self):
        """The sl_capture of the coming step (called by SafeLifeVecEnv.step_async)."""
        if self._slot == self.R:
            self.flush()
        s, c = self._slot, self._cap
        hw = self.venv.H * self.venv.W
        n = len(self.env_ids)
        c.n = n
        c.env = self._ids.data_ptr()
        c.board = self._b0.data_ptr() + 2 * s * n * hw
        c.goals = self._g0.data_ptr() + 2 * s * n * hw
        c.orientation = self._o0.data_ptr() + 4 * s * n
        c.flags = self._f.data_ptr() + s * n
        c.reset_board = self._b1.data_ptr() + 2 * s * n * hw
        c.reset_goals = self._g1.data_ptr() + 2 * s * n * hw
        c.reset_orientation = self._o1.data_ptr() + 4 * s * n
        self._slot_step.append(self.venv._step_index)
        self._slot += 1
        return ctypes.addressof(c)

    # ------------------------------------------------------------- episodes
    def _state_frame(self, e):
        v = self.venv
        return (int(v.st_t["orientation"][e].item()), v.board[e].cpu().numpy(),
                v.goals[e].cpu().numpy())

    def _start(self, i, step, frame):
        self._rec[i] = {"episode_num": self._ep[i], "step_num": step,
                        "orientation": [frame[0]], "board": [frame[1]], "goals": [frame[2]]}

    def _save(self, i):
        r, self._rec[i] = self._rec[i], None
        gid = self.venv.env0 + self.env_ids[i]
        p0 = os.path.abspath(self.video_name.format(env=gid, episode_num=r["episode_num"],
                                                    step_num=r["step_num"]))
        os.makedirs(os.path.dirname(p0), exist_ok=True)
        path, k = p0, 1
        while os.path.exists(path + ".npz"):
            k += 1
            path = p0 + " ({})".format(k)
        np.savez_compressed(path + ".npz", orientation=np.array(r["orientation"]),
                            board=np.stack(r["board"]), goals=np.stack(r["goals"]))
        self.files.append(path + ".npz")

    def flush(self):
        """Copy the captured slots to the host (one synchronisation) and write the
        episodes that ended."""
        S = self._slot
        if S == 0:
            return
        b0, g0, o0 = self._b0[:S].cpu().numpy(), self._g0[:S].cpu().numpy(), self._o0[:S].cpu().numpy()
        b1, g1, o1 = self._b1[:S].cpu().numpy(), self._g1[:S].cpu().numpy(), self._o1[:S].cpu().numpy()
        fl = self._f[:S].cpu().numpy()
        for s in range(S):
            for i in range(len(self.env_ids)):
                f = int(fl[s, i])
                r = self._rec[i]
                if r is not None and not (f & 2):          # capture_frame: not game over
                    r["orientation"].append(int(o0[s, i]))
                    r["board"].append(b0[s, i].copy())
                    r["goals"].append(g0[s, i].copy())
                if f & 4:                                  # the episode ended; reset
                    if r is not None:
                        self._save(i)
                    self._ep[i] += 1
                    if self._wanted(self._ep[i]):
                        self._start(i, self._slot_step[s] + 1,
                                    (int(o1[s, i]), b1[s, i].copy(), g1[s, i].copy()))
        self._slot = 0
        self._slot_step = []

    def on_reset(self, mask=None):
        """An explicit SafeLifeVecEnv.reset: the masked envs' episodes end here."""
        self.flush()
        m = None if mask is None else np.asarray(mask).reshape(-1)
        for i, e in enumerate(self.env_ids):
            if m is not None and not m[e]:
                continue
            if self._rec[i] is not None:
                self._save(i)
            self._ep[i] = int(self.venv.st_t["episodes"][e].item())
            if self._wanted(self._ep[i]):
                self._start(i, self.venv._step_index, self._state_frame(e))

    def close(self):
        """Flush and write the episodes still being recorded (SafeLifeRecorder.close)."""
        self.flush()
        for i in range(len(self.env_ids)):
            if self._rec[i] is not None:
                self._save(i)
        if getattr(self.venv, "_recorder", None) is self:
            self.venv._recorder = None
        return self.files
