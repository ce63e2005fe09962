"""Drop-in for the reference's C extension ``safelife.speedups`` (hot entries only).

    advance_board(board, spawn_prob=0.3) -> new uint16 board      module.c:19-44
    seed(i)                                                       module.c:246-253

Spawn draws follow the reference exactly: a 10 000-double buffer refilled from the
*global* numpy RNG (``np.random.random(10000)``, random.c:14-26), one draw per
eligible cell in row-major order (random.c:47-52), compared as
``u < (double)(float)spawn_prob``.

Where a board is advanced:
  * numpy in -> numpy out: on the host, by the build's bit-sliced CPU engine
    (``csrc/sl_host.cpp`` through the CPython module ``_native/_sl_host``), reading
    its uniforms straight from the emulated buffer.  The reference's numpy callers
    (side_effects.py:136-139, proc_gen.py:382,625) advance single small boards
    thousands of times, where a device round trip would cost ~35x the reference's
    own C call.  Boards wider than 512 cells go to the GPU path below;
  * torch in -> torch out: on the GPU (libsafelife_hip.so): the draws a board needs
    are counted on the device, the host takes that many doubles from the emulated
    buffer, and the board is advanced on the device.

Deliberate divergences: a non-2-d or empty board raises ValueError (the reference
returns NULL without an exception, i.e. SystemError); H or W == 1 raises ValueError
(undefined behaviour in the reference).  ``seed`` truncates to 32 bits
as the reference's ``"I"`` format does (module.c:248).

``advance_boards`` is the batched device entry (torch uint16 [B,H,W] in and out).
"""
import ctypes
import operator
import sys

import numpy as np

from . import _lib

_RAND_BUFFER_SIZE = 10000


class _RefBuffer:
    """random.c's buffer: 10 000 doubles of np.random.random, refilled when used up.
    The position lives in a one-element int64 array, which the host engine advances
    in place."""

    def __init__(self):
        self.buf = np.zeros(_RAND_BUFFER_SIZE)
        self.posarr = np.full(1, _RAND_BUFFER_SIZE, np.int64)

    @property
    def pos(self):
        return int(self.posarr[0])

    @pos.setter
    def pos(self, v):
        self.posarr[0] = v

    def refill(self):
        self.buf = np.random.random(_RAND_BUFFER_SIZE)
        self.pos = 0

    def take(self, n):
        parts = []
        while n > 0:
            if self.pos >= _RAND_BUFFER_SIZE:
                self.refill()
            k = min(n, _RAND_BUFFER_SIZE - self.pos)
            parts.append(self.buf[self.pos:self.pos + k])
            self.pos += k
            n -= k
        return np.concatenate(parts) if parts else np.zeros(0)

    def peek(self, n):
        """The next n draws without consuming them (numpy's global state and the
        buffer are restored)."""
        state, buf, pos = np.random.get_state(), self.buf, self.pos
        try:
            return self.take(n)
        finally:
            np.random.set_state(state)
            self.buf, self.pos = buf, pos


_buffer = _RefBuffer()


def seed(i):
    """np.random.seed(i) followed by an immediate buffer refill (random.c:28-45).

    The reference parses ``i`` with PyArg_ParseTuple's "I" format (module.c:248):
    any int, wrapped to 32 bits without an overflow check (a float is a TypeError)."""
    np.random.seed(operator.index(i) & 0xFFFFFFFF)
    _buffer.refill()


def _host():
    global _HOST
    if _HOST is None:
        from ._native import _sl_host
        _HOST = _sl_host
    return _HOST


_HOST = None


def _to_device_board(board, device):
    import torch
    if isinstance(board, torch.Tensor):
        t = board
        if t.dtype != torch.uint16:
            t = t.to(torch.int64).remainder(65536).to(torch.int32).to(torch.uint16)
        return t.to(device).contiguous(), True
    a = np.asarray(board)
    if a.dtype != np.uint16:
        a = a.astype(np.uint16)           # NPY_ARRAY_FORCECAST
    return torch.from_numpy(np.ascontiguousarray(a)).to(device), False


class _Frames:
    """Pinned host + device staging for one board shape: [board u16 | draws f64] up and
    [new board u16 | draw count i64] down, so a numpy call is one copy each way and
    one host sync (the board's draws are peeked -- at most one per cell -- and only the
    count the device reports is then consumed)."""
    _cache = {}

    @classmethod
    def get(cls, H, W, device):
        key = (H, W, str(device))
        if key not in cls._cache:
            cls._cache[key] = cls(H, W, device)
        return cls._cache[key]

    def __init__(self, H, W, device):
        import torch
        n = H * W
        self.nb = (2 * n + 7) // 8 * 8                  # board bytes, padded to 8
        up, down = self.nb + 8 * n, self.nb + 8
        self.up_h = torch.empty(up, dtype=torch.uint8, pin_memory=True)
        self.up_d = torch.empty(up, dtype=torch.uint8, device=device)
        self.dn_h = torch.empty(down, dtype=torch.uint8, pin_memory=True)
        self.dn_d = torch.empty(down, dtype=torch.uint8, device=device)
        self.off = torch.zeros(1, dtype=torch.int64, device=device)
        self.up_np = self.up_h.numpy()
        self.dn_np = self.dn_h.numpy()


def _is_torch(x):
    t = sys.modules.get("torch")
    return t is not None and isinstance(x, t.Tensor)


def advance_board(board, spawn_prob=0.3):
    """Advance one board; returns a new array (numpy in -> numpy out on the host,
    torch -> torch on the GPU)."""
    b = _buffer
    r = (_HOST or _host()).advance(board, spawn_prob, b.buf, b.posarr)
    if r is not None and r is not NotImplemented:
        return r                        # the common case: one C call
    if _is_torch(board):
        return _advance_device_torch(board, float(np.float32(spawn_prob)))
    a = np.asarray(board)
    if a.dtype != np.uint16 or not a.flags.c_contiguous or a.dtype.byteorder == ">":
        a = np.ascontiguousarray(a, dtype=np.uint16)     # NPY_ARRAY_FORCECAST
    if a.ndim != 2 or a.size == 0:
        raise ValueError("advance_board expects a non-empty 2-d board")
    H, W = a.shape
    if H < 2 or W < 2:
        raise ValueError("advance_board needs H, W >= 2")
    if W > 512:
        return _advance_device_numpy(a, float(np.float32(spawn_prob)))
    r = _host().advance(a, spawn_prob, b.buf, b.posarr)
    if r is not None:
        return r
    # the board needs more uniforms than the buffer still holds: take them as the
    # reference does, refilling from the global stream only when a draw is taken and
    # the buffer is used up (random.c:47-52) -- a board with no eligible cell never
    # refills, so np.random calls after it see the reference's global state
    return _host().advance_with(a, spawn_prob, b.take(_host().count_eligible(a)))


def _advance_device_numpy(a, p):
    """A numpy board too wide for the host engine: one copy up, count + advance on
    the device, one copy down."""
    import torch
    device = _lib.require_device()
    L = _lib.lib()
    s = _lib.stream_ptr(device)
    H, W = a.shape
    f = _Frames.get(H, W, device)
    n = H * W
    f.up_np[:2 * n] = np.ascontiguousarray(a, dtype=np.uint16).reshape(-1).view(np.uint8)
    f.up_np[f.nb:] = _buffer.peek(n).view(np.uint8)
    f.up_d.copy_(f.up_h, non_blocking=True)
    bd = f.up_d.data_ptr()
    _lib.check(L.sl_count_eligible(bd, f.dn_d.data_ptr() + f.nb, 1, H, W, s),
               "sl_count_eligible")
    _lib.check(L.sl_advance(bd, f.dn_d.data_ptr(), 1, H, W, None, p, _lib.SL_RNG_STREAM,
                            0, 0, 0, 0, bd + f.nb, f.off.data_ptr(), s), "sl_advance")
    f.dn_h.copy_(f.dn_d, non_blocking=True)
    torch.cuda.current_stream(device).synchronize()
    _buffer.take(int(f.dn_np[f.nb:].view(np.int64)[0]))   # consumed whatever p is
    return f.dn_np[:2 * n].view(np.uint16).reshape(H, W).copy()


def _advance_device_torch(board, p):
    """A torch board on the device: the board's draws (at most one per cell) are
    peeked from the emulated buffer and uploaded with it, count and advance run
    back to back, and the one host sync reads the count the buffer then consumes."""
    import torch
    device = _lib.require_device()
    L = _lib.lib()
    s = _lib.stream_ptr(device)
    t, _ = _to_device_board(board, device)
    if t.dim() != 2 or t.numel() == 0:
        raise ValueError("advance_board expects a non-empty 2-d board")
    H, W = t.shape
    if H < 2 or W < 2:
        raise ValueError("advance_board needs H, W >= 2")
    f = _Frames.get(H, W, device)
    n = H * W
    f.up_np[f.nb:] = _buffer.peek(n).view(np.uint8)
    f.up_d.copy_(f.up_h, non_blocking=True)
    out = torch.empty_like(t)
    cnt = f.dn_d.data_ptr() + f.nb
    _lib.check(L.sl_count_eligible(t.data_ptr(), cnt, 1, H, W, s), "sl_count_eligible")
    _lib.check(L.sl_advance(t.data_ptr(), out.data_ptr(), 1, H, W, None, p, _lib.SL_RNG_STREAM,
                            0, 0, 0, 0, f.up_d.data_ptr() + f.nb, f.off.data_ptr(), s),
               "sl_advance")
    f.dn_h[f.nb:].copy_(f.dn_d[f.nb:], non_blocking=True)
    torch.cuda.current_stream(device).synchronize()
    _buffer.take(int(f.dn_np[f.nb:].view(np.int64)[0]))   # consumed whatever p is
    return out


def advance_boards(boards, spawn_prob=0.3, rng="philox", seed=0, env0=0, step=0, tensor=0,
                   draws=None, draw_offsets=None, out=None):
    """Batched device advance: boards uint16 [B,H,W] (torch, on the GPU).

    rng="philox": spawn uniforms from Philox(seed; cell, env0+b, step, tensor).
    rng="stream": board b takes draws[draw_offsets[b] + k] for its k-th eligible cell.
    spawn_prob: a float or a float32 tensor [B].
    """
    import torch
    device = _lib.require_device()
    if boards.dim() != 3 or boards.dtype != torch.uint16:
        raise ValueError("boards must be a uint16 [B,H,W] tensor")
    boards = boards.to(device).contiguous()
    B, H, W = boards.shape
    if out is None:
        out = torch.empty_like(boards)
    sp_ptr, sp_scalar = None, 0.3
    if isinstance(spawn_prob, torch.Tensor):
        sp = spawn_prob.to(device=device, dtype=torch.float32).contiguous()
        sp_ptr = sp.data_ptr()
    else:
        sp_scalar = float(np.float32(spawn_prob))
    mode = _lib.SL_RNG_PHILOX if rng == "philox" else _lib.SL_RNG_STREAM
    dp = draws.data_ptr() if draws is not None else None
    op = draw_offsets.data_ptr() if draw_offsets is not None else None
    _lib.check(_lib.lib().sl_advance(boards.data_ptr(), out.data_ptr(), B, H, W, sp_ptr,
                                     sp_scalar, mode, seed & 0xFFFFFFFFFFFFFFFF, env0, step,
                                     tensor, dp, op, _lib.stream_ptr(device)), "sl_advance")
    return out


def count_eligible(boards):
    """Draws each board of a uint16 [B,H,W] device tensor consumes in one advance."""
    import torch
    device = _lib.require_device()
    boards = boards.to(device).contiguous()
    B, H, W = boards.shape
    cnt = torch.zeros(B, dtype=torch.int64, device=device)
    _lib.check(_lib.lib().sl_count_eligible(boards.data_ptr(), cnt.data_ptr(), B, H, W,
                                            _lib.stream_ptr(device)), "sl_count_eligible")
    return cnt
