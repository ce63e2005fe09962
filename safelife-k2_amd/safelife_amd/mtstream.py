"""The reference's seeded spawn stream, generated on the device.

``speedups.seed(s)`` makes the reference draw every spawn uniform from numpy's global
RandomState(s), refilled 10 000 doubles at a time
(/root/reference/safelife/speedups_src/random.c:14-26,28-52, module.c:246-253), so its
spawn stream is ``np.random.RandomState(s).random_sample(n)``.  :class:`MT19937Stream`
produces exactly that stream into a device ring (``sl_mt19937_*`` in
include/safelife_hip.h, csrc/sl_mt.hip): MT19937 blocks generated side by side, each
chain jumping ahead by a polynomial in the transition matrix.  A replay env given one
(``SafeLifeVecEnv(rng="stream", spawn_stream=None, seed=s)``) fills it inside each
step, after the offsets scan has fixed the step's range, so no host buffer is involved.
"""
import ctypes

import numpy as np

from . import _lib

MT_N = 624
PREFIX = 21216            # SL_MT_PREFIX
POLY_WORDS = 640          # SL_MT_POLY_WORDS


def _pow2_at_least(n):
    return 1 << max(0, int(n - 1).bit_length())


class MT19937Stream:
    """RandomState(seed).random_sample, draw d at ``ring[d & mask]`` on ``device`` (or,
    with ``bits_threshold``, the decision draw < threshold at bit d & mask of the ring).

    ``ring_draws``: doubles the ring holds (power of two); a step may read at most
    ``ring_draws`` minus one block.  ``n_chains``: blocks one fill can generate (power of
    two); ``rounds``: a block is 624 * rounds raw outputs (312 * rounds draws).
    ``lookahead``: after each fill, generate the next fill's likely blocks (1.25x the
    last range, past it) on a second stream beside the step that reads this fill's, the
    next fill waiting for them (a single stream of consecutive ranges: one shard)."""

    def __init__(self, seed, device, *, first_draw=0, ring_draws=1 << 24, n_chains=None,
                 rounds=420, lookahead=False, bits_threshold=None):
        import torch
        self.torch = torch
        self.device = _lib.require_device(device)
        self.seed = int(seed) & 0xFFFFFFFF
        self.rounds = int(rounds)
        self.block = 312 * self.rounds
        self.ring_draws = _pow2_at_least(max(int(ring_draws), 2 * self.block))
        if n_chains is None:
            n_chains = _pow2_at_least(max(2, -(-self.ring_draws // self.block) + 1))
        self.n_chains = _pow2_at_least(int(n_chains))
        nk = (self.n_chains - 1).bit_length()
        dev = self.device
        # bits_threshold: a ring of decisions (draw < threshold) for replay batches
        # whose envs all spawn with that one threshold (double)(float)p: 1 bit per draw
        self.bits_threshold = None if bits_threshold is None else float(bits_threshold)
        if self.bits_threshold is not None:
            if self.rounds % 4:
                raise ValueError("a bit ring needs rounds % 4 == 0")
            self.ring = torch.zeros(self.ring_draws // 32, dtype=torch.int32, device=dev)
        else:
            self.ring = torch.empty(self.ring_draws, dtype=torch.float64, device=dev)
        self.chains = torch.zeros(self.n_chains, MT_N, dtype=torch.int32, device=dev)
        self.prefix = torch.zeros(self.n_chains, PREFIX, dtype=torch.int32, device=dev)
        self.polys = torch.zeros(nk + 1, POLY_WORDS, dtype=torch.int32, device=dev)
        self.ctl = torch.zeros(8, dtype=torch.int64, device=dev)
        s = _lib.MT19937()
        s.n_chains, s.rounds, s.ring_draws = self.n_chains, self.rounds, self.ring_draws
        s.ring, s.chains, s.prefix = self.ring.data_ptr(), self.chains.data_ptr(), self.prefix.data_ptr()
        s.polys, s.ctl = self.polys.data_ptr(), self.ctl.data_ptr()
        if self.bits_threshold is not None:
            s.bit_ring, s.bits_thr = 1, self.bits_threshold
        self.struct = s
        self._ahead = None
        if lookahead:
            # its kernels are latency-bound chains: a high-priority stream gets them
            # dispatched among the step's waves
            import os
            self._ahead = torch.cuda.Stream(
                device=dev, priority=int(os.environ.get("SAFELIFE_MT_AHEAD_PRIORITY", "-1")))
            _lib.check(_lib.lib().sl_mt19937_lookahead(ctypes.byref(s), self._ahead.cuda_stream),
                       "sl_mt19937_lookahead")
        self.seek(first_draw)

    def __del__(self):
        try:
            if self._ahead is not None:
                self._ahead.synchronize()       # its kernels use this object's buffers
            _lib.lib().sl_mt19937_release(ctypes.byref(self.struct))
        except Exception:
            pass

    @property
    def mask(self):
        return self.ring_draws - 1

    def seek(self, first_draw):
        """(Re-)seed so that draws from `first_draw` on can be generated (host
        polynomial work + device init; synchronises the device's current stream)."""
        L = _lib.lib()
        if self._ahead is not None:
            self._ahead.synchronize()           # a look-ahead still moving the chains
        _lib.check(L.sl_mt19937_seed(ctypes.byref(self.struct), self.seed, int(first_draw),
                                     _lib.stream_ptr(self.device)), "sl_mt19937_seed")

    def fill(self, lo, hi, err=None):
        """Generate the blocks holding draws [*lo, *hi) (int64 device tensors)."""
        L = _lib.lib()
        _lib.check(L.sl_mt19937_fill(ctypes.byref(self.struct), _lib.ptr(lo), _lib.ptr(hi),
                                     _lib.ptr(err), _lib.stream_ptr(self.device)),
                   "sl_mt19937_fill")

    def error(self):
        return bool(self.ctl[2].item() & 1)

    def draws(self, lo, n):
        """Draws [lo, lo + n) as a float64 device tensor (generating them first); a bit
        ring gives its decisions (draw < threshold) as a bool tensor."""
        torch = self.torch
        a = torch.tensor([int(lo), int(lo) + int(n)], dtype=torch.int64, device=self.device)
        self.fill(a[0:1], a[1:2])
        return self.ring_slice(lo, lo + n)

    def ring_slice(self, lo, hi):
        """What the ring holds for draws [lo, hi) (no generation): float64 draws, or a
        bit ring's decisions as bool."""
        torch = self.torch
        idx = (torch.arange(int(lo), int(hi), device=self.device) & self.mask)
        if self.bits_threshold is None:
            return self.ring[idx]
        return ((self.ring[idx >> 5] >> (idx & 31).to(torch.int32)) & 1) != 0


# ---------------------------------------------------------- host reference pieces
def host_window(seed):
    w = np.zeros(MT_N, np.uint32)
    _lib.check(_lib.lib().sl_mt19937_host_window(int(seed) & 0xFFFFFFFF,
                                                 w.ctypes.data_as(ctypes.c_void_p)),
               "sl_mt19937_host_window")
    return w


def host_jump_poly(n):
    p = np.zeros(POLY_WORDS, np.uint32)
    _lib.check(_lib.lib().sl_mt19937_host_jump_poly(int(n), p.ctypes.data_as(ctypes.c_void_p)),
               "sl_mt19937_host_jump_poly")
    return p


def host_jump(window, poly):
    out = np.zeros(MT_N, np.uint32)
    w = np.ascontiguousarray(window, np.uint32)
    p = np.ascontiguousarray(poly, np.uint32)
    _lib.check(_lib.lib().sl_mt19937_host_jump(w.ctypes.data_as(ctypes.c_void_p),
                                               p.ctypes.data_as(ctypes.c_void_p),
                                               out.ctypes.data_as(ctypes.c_void_p)),
               "sl_mt19937_host_jump")
    return out


def host_draws(window, n):
    out = np.zeros(int(n), np.float64)
    w = np.ascontiguousarray(window, np.uint32)
    _lib.check(_lib.lib().sl_mt19937_host_draws(w.ctypes.data_as(ctypes.c_void_p), int(n),
                                                out.ctypes.data_as(ctypes.c_void_p)),
               "sl_mt19937_host_draws")
    return out
