"""Lane sharding across GPUs: one process per GPU, torch.distributed over RCCL (backend "nccl").

Trajectories are independent, so the batch is partitioned into contiguous shards with no
data-path collective.  The only exchange is one SUM all-reduce per outer iteration of the 8
solver statistics (solver.STAT_FIELDS: active lanes, sum of J, sum of max|sigma|^2, ...), which
gives every rank the global stop condition and the global cost / descent-norm scalars.  The
message is 64 bytes, so it is latency-bound.  It is enqueued from the solver's stream (the engine
launches on torch's current stream, and RCCL's communication stream waits on it), so it orders after
the iteration's statistics kernel without a host synchronisation.

``force=True`` (every collective helper here) runs the collective even on a 1-rank group: RCCL refuses two
ranks on one device, so that is how a one-GPU box executes the device-tensor RCCL branches the 8-GPU run uses.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) lane range of ``rank`` (first ``total % world`` ranks get one more)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(int(total), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def env_rank_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from torchrun's environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def rank_world(group=None) -> tuple[int, int]:
    """(rank, world_size) of the initialised process group, or (0, 1) for a single process."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def backend_name(group=None) -> str | None:
    """The process group's backend ("nccl" = RCCL, "gloo"), or None for a single process without a group."""
    if dist.is_available() and dist.is_initialized():
        return str(dist.get_backend(group))
    return None


def local_device_index(local_rank: int) -> int:
    """This rank's GPU: local_rank, wrapped onto the visible devices (one process per GPU on a full node; a
    multi-rank rehearsal on fewer GPUs shares them)."""
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    return local_rank % n if n else 0


def init_process_group(backend: str | None = None, force: bool = False):
    """Initialise torch.distributed from the environment if WORLD_SIZE > 1 (RCCL on GPUs, gloo on CPU), or at
    any world size with ``force`` (a 1-rank group: exercises the collective path on one GPU).

    GYM_DIST_BACKEND overrides the backend (e.g. gloo to rehearse several ranks on one GPU: RCCL refuses two
    ranks on the same device)."""
    rank, local_rank, world = env_rank_world()
    if (world > 1 or force) and not dist.is_initialized():
        backend = backend or os.environ.get("GYM_DIST_BACKEND")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_device_index(local_rank))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {"device_id": torch.device("cuda", local_device_index(local_rank))} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, local_rank, world


def _collective(group, force: bool) -> bool:
    """Whether the helpers below run a collective: a process group exists and holds several ranks (or force)."""
    return dist.is_available() and dist.is_initialized() and (force or dist.get_world_size(group) > 1)


def make_reduce_stats(group=None, force: bool = False):
    """SUM all-reduce of the per-iteration statistics, or None when running a single process (unless force)."""
    if not _collective(group, force):
        return None
    backend = dist.get_backend(group)

    def reduce_stats(st):
        if isinstance(st, np.ndarray):
            st = torch.from_numpy(st.copy())
        t = st.detach().cpu().clone() if backend == "gloo" else st.detach().clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return t

    def max_of(value: float) -> float:
        """MAX over ranks of a host scalar (the straggler-tail switch's per-rank active count)."""
        return max_over_ranks(value, group=group, force=force)

    reduce_stats.max_of = max_of
    return reduce_stats


class TimedReduce:
    """A ``make_reduce_stats`` all-reduce with host-side accounting, for diagnosing a multi-GPU run: ``reduce_s``
    accumulates the host time inside the collective call (enqueue on RCCL; the whole exchange on gloo) and
    ``readback_s`` the host time of reading the reduced statistics back (it also waits for the iterations queued
    before the collective, so it bounds the collective's share from above); ``calls`` counts the collectives.  It
    returns the statistics on the host (the solver loops read them there at once), so the solve is unchanged."""

    def __init__(self, reduce):
        self.reduce = reduce
        self.max_of = getattr(reduce, "max_of", None)
        self.reduce_s = 0.0
        self.readback_s = 0.0
        self.calls = 0

    def reset(self):
        self.reduce_s = self.readback_s = 0.0
        self.calls = 0

    def __call__(self, st):
        import time
        t0 = time.perf_counter()
        r = self.reduce(st)
        t1 = time.perf_counter()
        r = r.cpu() if isinstance(r, torch.Tensor) else r
        t2 = time.perf_counter()
        self.reduce_s += t1 - t0
        self.readback_s += t2 - t1
        self.calls += 1
        return r


def allreduce_latency_us(n: int = 200, group=None, force: bool = False) -> float | None:
    """Average wall time of one 8 x fp64 SUM all-reduce (the solver's statistics message) issued back to back and
    synchronised once, in microseconds; None without a collective."""
    if not _collective(group, force):
        return None
    import time
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.zeros(8, dtype=torch.float64, device=dev)
    for _ in range(10):
        dist.all_reduce(t, group=group)
    if dev != "cpu":
        torch.cuda.synchronize()
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(n):
        dist.all_reduce(t, group=group)
    if dev != "cpu":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def gather_floats(values, group=None, force: bool = False) -> list:
    """Every rank's list of host floats, in rank order, on every rank (one all-gather)."""
    if not _collective(group, force):
        return [list(map(float, values))]
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, list(map(float, values)), group=group)
    return parts


def barrier(group=None):
    if dist.is_available() and dist.is_initialized():
        dist.barrier(group=group)


def max_over_ranks(value: float, group=None, force: bool = False) -> float:
    """Max of a host scalar over ranks (timing: the job's time is its slowest rank's)."""
    if not _collective(group, force):
        return float(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sum_over_ranks(value: float, group=None, force: bool = False) -> float:
    if not _collective(group, force):
        return float(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item())


def solve_sharded(x0_all, x_ref, u_ref, max_iters, engine=None, keep_stats: bool = False, gather: bool = False,
                  force_collectives: bool = False, **solver_kw):
    """Solve this rank's contiguous shard of ``x0_all`` (B_total,4); stop on the GLOBAL active count.

    Every rank must hold a non-empty shard (``len(x0_all) >= world``; checked on every rank before any
    collective, so all of them raise together).  The automatic schedule is chosen on the largest shard
    (``schedule_lanes``), so every rank runs the same schedule and issues its all-reduces at the same
    iterations.  Returns (lo, hi, SolveResult of the local shard); with ``gather=True`` the third item is instead
    the dict of global per-lane results (``gather_sharded`` of GATHER_FIELDS) on every rank.  Per-lane references
    (x_ref (B_total,N,4), u_ref (B_total,T,2)) are cut to the rank's shard.  ``force_collectives`` runs the
    all-reduce / all-gather even on a 1-rank group."""
    from .engine import AcrobotEngine
    from .solver import BatchedNewtonSolver
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_initialized() else 1
    total = len(x0_all)
    lo, hi = shard_range(total, rank, world)
    if total < world:
        raise ValueError(f"{total} lanes cannot be sharded over {world} ranks (every rank needs one)")
    if np.ndim(x_ref) == 3:       # per-lane references: this rank's rows only
        if len(x_ref) != total or len(u_ref) != total:
            raise ValueError(f"per-lane references must hold {total} lanes, got {len(x_ref)} / {len(u_ref)}")
        x_ref, u_ref = x_ref[lo:hi], u_ref[lo:hi]
    eng = engine or AcrobotEngine()
    solver_kw.setdefault("schedule_lanes", schedule_lanes(total, world))
    solver_kw.setdefault("world_size", world)
    solver = BatchedNewtonSolver(eng, x_ref, u_ref, hi - lo, **solver_kw)
    x0_loc = x0_all[lo:hi] if isinstance(x0_all, torch.Tensor) else np.asarray(x0_all)[lo:hi]
    res = solver.solve(x0_loc, max_iters, reduce_stats=make_reduce_stats(force=force_collectives),
                       keep_stats=keep_stats)
    if gather:
        return lo, hi, gather_sharded({f: getattr(res, f) for f in GATHER_FIELDS}, total, force=force_collectives)
    return lo, hi, res


GATHER_FIELDS = ("x", "u", "K", "sigma", "cost", "n_iter", "status", "n_rollouts", "gamma")


def gather_sharded(local: dict, total: int, group=None, force: bool = False) -> dict:
    """The global per-lane results on every rank from each rank's contiguous shard ("ship the final
    per-lane outputs with an all-gather ... only if requested"): ``local`` maps a name to this rank's
    (hi - lo, ...) tensor; returns name -> (total, ...) tensors in lane order.  Ragged shards are padded to the
    largest one for the collective (RCCL all-gather on device tensors; gloo moves them through the host)."""
    if not _collective(group, force):
        return dict(local)
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    lo, hi = shard_range(total, rank, world)
    width = -(-int(total) // world)
    gloo = dist.get_backend(group) == "gloo"
    out = {}
    for name, t in local.items():
        if t.shape[0] != hi - lo:
            raise ValueError(f"{name}: {t.shape[0]} rows for the shard [{lo}, {hi})")
        src = t.detach().cpu() if gloo else t.detach()
        pad = torch.zeros((width,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        pad[:hi - lo] = src
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        rows = [parts[r][:shard_range(total, r, world)[1] - shard_range(total, r, world)[0]] for r in range(world)]
        out[name] = torch.cat(rows).to(t.device)
    return out


def schedule_lanes(total: int, world: int) -> int:
    """The lane count every rank bases its automatic schedule choice on: the largest shard, identical on all
    ranks (ragged shards differ by one lane and could otherwise straddle a schedule threshold)."""
    return -(-int(total) // int(world))
