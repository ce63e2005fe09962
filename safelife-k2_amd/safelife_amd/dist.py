"""Multi-GPU layout of the batched stepper.

One process per GPU (torchrun), envs split into contiguous shards.  Every env
is addressed by its GLOBAL id (``env0 + local index``): the Philox spawn
counters, the level sequence (``level_order='sequential'`` uses ``n_total``) and
the reset roll augmentation all key on that id, so an env's trajectory does not
depend on how many ranks the batch is spread over.  The data path has no
collective.  Collectives run at logging cadence only:

* :func:`reduce_counters` -- all_reduce(SUM) of the ``global_counter`` analogues
  (episodes started / completed, env-steps; safelife_env.py:81-85);
* :func:`gather_episodes` -- all_gather of finished-episode records
  (return, length, ...), padded to the largest shard's count.

Parity mode is the exception (SURVEY.md §8(e) collective 3): the reference draws
every spawn uniform from ONE stream, env after env over the whole batch
(training/ppo.py:436-452, random.c:47-52), so a shard's draws start where the
shards before it end.  :class:`StreamExchange` is that per-step exchange: one int64
per rank (the shard's draw total of the step) all-gathered, each rank's base = the
global position plus the totals of the ranks before it (SafeLifeVecEnv's
``stream_exchange``; sl_env_cfg.stream_phase).

Works with any ``torch.distributed`` backend: ``nccl`` (RCCL over xGMI) on the
GPU box, ``gloo`` in the CPU tests.
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    env0: int          # global id of this rank's first env
    n_envs: int        # envs on this rank
    n_total: int       # envs over all ranks


def env_shard(rank, world, envs_per_rank):
    """Contiguous shard of rank ``rank``: global ids [rank*B, (rank+1)*B)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    if envs_per_rank < 0:
        raise ValueError("envs_per_rank must be >= 0")
    return Shard(rank, world, rank * envs_per_rank, envs_per_rank, world * envs_per_rank)


def split_batch(total, world):
    """Envs per rank for a fixed global batch (strong scaling): equal shards."""
    if total % world:
        raise ValueError("global batch %d not divisible by %d ranks" % (total, world))
    return total // world


def reduce_counters(counter, device=None):
    """Sum a GlobalCounter-like object's fields over ranks; returns a dict."""
    import torch
    import torch.distributed as dist
    keys = ("episodes_started", "episodes_completed", "num_steps")
    t = torch.tensor([float(getattr(counter, k)) for k in keys], dtype=torch.float64,
                     device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


def gather_episodes(records, device=None):
    """All-gather [n_i, F] float64 episode records from every rank.

    Returns the [sum n_i, F] concatenation in rank order.
    """
    import torch
    import torch.distributed as dist
    rec = torch.as_tensor(records, dtype=torch.float64, device=device)
    if rec.dim() != 2:
        raise ValueError("records must be [n, F]")
    if not (dist.is_available() and dist.is_initialized()):
        return rec
    world = dist.get_world_size()
    n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    counts = [int(x.item()) for x in ns]
    m = max(counts) if counts else 0
    pad = torch.zeros((m, rec.shape[1]), dtype=rec.dtype, device=device)
    pad[:rec.shape[0]] = rec
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return torch.cat([o[:c] for o, c in zip(outs, counts)], 0)


class StreamExchange:
    """Places each shard's reference-order draws in the one global stream.

    ``pos`` (a device int64 [1]) is the global stream position, identical on every
    rank.  Called with the shard's draw total of the step (device int64 [1], what
    the count phase leaves in the env's stream_pos), it all-gathers the totals of
    every rank (one int64 each: RCCL over xGMI on the GPU box, gloo on the CPU),
    returns this rank's base -- pos + the totals of the lower ranks -- and advances
    pos past all of them.  Stream-ordered, no host synchronisation.  Without an
    initialised process group it is the single-rank exchange (base = pos).
    """

    def __init__(self, device=None, pos=0, group=None):
        import torch
        self.group = group
        self.pos = torch.tensor([int(pos)], dtype=torch.int64, device=device)

    def _world(self):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(self.group), dist.get_rank(self.group)
        return 1, 0

    def __call__(self, local_total):
        import torch
        import torch.distributed as dist
        world, rank = self._world()
        local_total = local_total.reshape(1).to(torch.int64)
        if world == 1:
            totals = local_total
        else:
            parts = [torch.zeros_like(local_total) for _ in range(world)]
            dist.all_gather(parts, local_total, group=self.group)
            totals = torch.cat(parts)
        base = self.pos + totals[:rank].sum()
        self.pos += totals.sum()
        return base
