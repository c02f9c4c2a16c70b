"""Batched Newton / Armijo swing-up solver on the HIP engine (newton_Algorithm, batched).

Reference semantics, per lane (trajectory_generation.py:298-398):
  * u_ref trimmed to N-1 rows if it has N (:301-303); ValueError on other mismatches (:305-306);
  * u_0 = 0 and x_0 = open-loop rollout (:311-312); J_0 = total_cost (:319);
  * each iteration: backward sweep -> K, sigma, dJ (:332-338); Armijo gamma_0, gamma_0*beta, ...
    with the strict test J_new < J + c*gamma*dJ (:352-365), at most ``max_ls`` = 20 trials;
  * LS failure: stop without update (:367-369); otherwise update, then stop if max|sigma| < tol
    (:383-396).
The batch runs every lane in lock-step on the device.  Trial 1 is fused with its rollout; lanes
that reject it evaluate trials 2..max_ls *in parallel* (one thread per candidate) and re-run the
first accepted one -- the same decision the sequential search makes.

Schedules: ``serial`` launches the backward sweep and the trial of all lanes one after the other
(gym_newton_iteration); ``pipelined`` splits the lanes into two halves offset by one phase and runs
one half's (HBM-bound) sweep beside the other half's (fp64-VALU-bound) trial in a single launch
(gym_newton_phase); ``persistent`` runs every lane's iterations back to back inside one launch per
``chunk`` iterations (gym_newton_run): lanes are independent problems, so no grid-wide step separates
one iteration from the next.  Per lane the arithmetic is identical; only the overlap differs.

Streams per stage: the sweep reads x (2 pairs) + u (2 planes) and writes K row 1 (2 pairs) +
(c1, sigma1); the trial reads those + u0 and writes x_new, u_new.  When u_ref[:,0] == 0 (the headline
task-2 reference) the unactuated tau1 controls are identically zero and their planes are skipped.

Multi-GPU: one process per GPU, each owning a contiguous shard of lanes; the only cross-GPU
traffic is one all-reduce (SUM) of the 8 per-iteration statistics (see distributed.py).
"""
from __future__ import annotations

import ctypes as C
import time
import weakref
from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from .engine import AcrobotEngine, padded, F64
from .params import MAX_LINE_SEARCH_ITERS

STAT_FIELDS = ("n_active", "sum_cost", "sum_smax2", "lanes_ran", "n_retry", "n_converged", "n_failed", "n_rollouts")


@dataclass
class SolveResult:
    x: torch.Tensor          # (B,N,4)
    u: torch.Tensor          # (B,T,2)
    K: torch.Tensor          # (B,T,2,4)  gains of each lane's last iteration
    sigma: torch.Tensor      # (B,T,2)
    cost: torch.Tensor       # (B,)
    n_iter: torch.Tensor     # (B,) outer iterations executed (incl. a final failed one)
    status: torch.Tensor     # (B,) _lib.CONVERGED / LS_FAILED / MAX_ITERS
    n_rollouts: torch.Tensor # (B,)
    gamma: torch.Tensor      # (B,) last accepted step
    iterations: int          # outer loop iterations run for the whole batch
    lane_iterations: int     # sum of n_iter over lanes (the throughput numerator)
    seconds: float           # wall time of the solve loop (init + iterations + finalize)
    stats_log: list = field(default_factory=list)
    hist_cost: torch.Tensor | None = None   # (hist_len, B)
    hist_smax: torch.Tensor | None = None   # (hist_len, B)
    x_trajs: dict | None = None             # {lane: [x_0, x_1, ...]} of the captured lanes (capture_lanes)
    cost0: dict | None = None               # {lane: J_0} of the captured lanes
    sigmas: dict | None = None              # {lane: {iteration: sigma (T,2)}} of the captured lanes (capture_sigma)
    schedule: str = ""                      # "serial" | "pipelined" | "persistent"
    tail_lane_iterations: int = 0           # lane-iterations run by the straggler tail (gym_newton_tail)
    compactions: int = 0                    # lane compactions during the loop (BatchedNewtonSolver.compact)
    lowocc_lane_iterations: int = 0         # lane-iterations run in the low-occupancy regime (maybe_compact)
    tail_from_iteration: int | None = None  # the outer iteration the straggler tail took over at (None: no tail)
    tail_iterations: int = 0                # outer iterations the tail ran (its slowest lane's, up to the last one)


class PlacementPool:
    """Process-wide cache of the stream-buffer sets that placement selection chose (BatchedNewtonSolver._placement_*),
    keyed by (device index, stream shapes).  A solver that chose a set leases it; when the solver is garbage-collected
    the set comes back here, and the next solver of the same shape takes it without a probe or an allocation (the
    batched newton_Algorithm builds a solver per call, bench.py one per leg).  At most one free set per key; free sets
    beyond MAX_SHARE of the device's memory are dropped, oldest first.  ``clear()`` returns every free set to the
    device."""
    MAX_SHARE = 0.35
    _free: "OrderedDict" = OrderedDict()

    @staticmethod
    def _bytes(key) -> int:
        return 8 * sum(int(np.prod(sh)) for sh in key[1])

    @classmethod
    def take(cls, key):
        """(streams, record) of a free set for ``key``, now leased to the caller, or None."""
        return cls._free.pop(key, None)

    @classmethod
    def put(cls, key, streams, record):
        if key in cls._free:
            return
        cls._free[key] = (streams, record)
        try:
            cap = cls.MAX_SHARE * torch.cuda.get_device_properties(key[0]).total_memory
        except Exception:
            return
        while len(cls._free) > 1 and sum(cls._bytes(k) for k in cls._free) > cap:
            cls._free.popitem(last=False)

    @classmethod
    def clear(cls):
        cls._free.clear()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()

    @classmethod
    def held_bytes(cls) -> int:
        return sum(cls._bytes(k) for k in cls._free)


class BatchedNewtonSolver:
    """Owns the device buffers of a batch of ``B`` lanes that share x_ref / u_ref."""

    # The pipelined schedule pays off once the batch holds two wavefronts per SIMD: with the round-2 kernels
    # serial is ahead by 2% at 73,728 and 81,920 lanes and by 1% at 98,304, the two are level (+-1%, box
    # dependent) from 131,072 to 327,680 (same-box sweeps, profiles/r02_sched_sweep_large.log; round 1's
    # kernels crossed at ~81,920, profiles/r01_batch_sweep.log).  In lanes per compute unit (4 SIMDs x 64 x 2).
    PIPELINE_MIN_LANES_PER_CU = 512
    # The persistent schedule (one launch per solve: no per-iteration launches, statistics or host round trips)
    # is ahead while the batch is latency-bound and fits in one round of its workgroups: k_nt_run2 holds 64 lanes
    # on four wavefronts and ~98 KiB of LDS, one workgroup per CU.  Round 6, same box (profiles/r06/sched/):
    # persistent 28.95 M it/s against serial 17.16 at 16,384 lanes (64 per CU), but 22.94 / 24.60 at 24,576 and
    # 29.40 / 32.19 at 32,768, where CUs take a second workgroup (round 2's threshold of 128 per CU predates the
    # kernel's LDS ring).
    PERSISTENT_MAX_LANES_PER_CU = 64
    # The straggler tail (gym_newton_tail: one workgroup per lane, every Armijo trial at once) takes over the serial /
    # pipelined loop once at most this many lanes per CU (of all ranks) are still active: one wavefront per lane, so up
    # to one per SIMD it runs each lane's iteration at the latency of one sweep pass plus one trial chain.
    TAIL_LANES_PER_CU = 4
    # Placement selection (see PlacementPool, _arm_placement and _placement_tick): the phase kernel's speed depends on
    # where its six stream buffers land (1.89-2.08 ms per launch for sets alive at once in one process, each stable for
    # its lifetime; profiles/r05/placement/, profiles/r06/README.md).  A large pipelined solver allocates up to
    # PLACEMENT_CANDIDATES stream sets (as free memory allows), ranks them at construction with the placement probe
    # (gym_placement_probe: the phase kernel's traffic without arithmetic, ~2 ms a launch; it ranks sets as the kernel
    # does, Pearson 0.87-0.93), keeps the PLACEMENT_TRIALS best, and races those in its first solve: blocks of
    # PLACEMENT_BLOCK iterations of that solve on each (the live state copied from set to set between blocks: the same
    # bits on any set), the fastest kept.  In the zero-arithmetic probe about a third of the sets are fast (1.84-1.86
    # ms), a third middling (1.95-2.03), the rest slow: eight candidates leave one selection in ~25 without a fast set,
    # four one in 5 (profiles/r06/layout/).
    PLACEMENT_CANDIDATES = 8
    PLACEMENT_TRIALS = 3
    PLACEMENT_MEM_SHARE = 0.45
    PLACEMENT_BLOCK = 12
    # Candidate slots of the post-trial Armijo search (gym_batch.cand_scratch): 32,768 (0.79 GB at T = 500) cover
    # 1,724 backtracking lanes at max_ls = 20; a hard solve's iterations mostly have 0-30 (tools/retry_counts.py).
    CAND_SLOTS = 32768

    @staticmethod
    def pipeline_min_lanes(device) -> int:
        n_cu = torch.cuda.get_device_properties(device).multi_processor_count
        return BatchedNewtonSolver.PIPELINE_MIN_LANES_PER_CU * n_cu

    @staticmethod
    def persistent_max_lanes(device) -> int:
        n_cu = torch.cuda.get_device_properties(device).multi_processor_count
        return BatchedNewtonSolver.PERSISTENT_MAX_LANES_PER_CU * n_cu

    def __init__(self, engine: AcrobotEngine, x_ref, u_ref, B: int, tol=1e-6, beta=0.7, c=0.5, gamma_0=1.0,
                 max_ls: int = MAX_LINE_SEARCH_ITERS, hist_len: int = 0, pipeline: bool | None = None,
                 u0_zero: bool | None = None, checkpoint: bool = False, persistent: bool | None = None,
                 chunk: int = 128, reorder: bool = True, schedule_lanes: int | None = None,
                 capture_lanes=None, capture_every: int = 1, split_waves: bool = True,
                 capture_sigma=(0, 1, 2), tail_lanes: int | None = None, tail_chunk: int = 128,
                 compact: bool | None = None, world_size: int = 1, cand_slots: int | None = None,
                 arena=False, placement_trials: int | None = None):
        if B <= 0:
            raise ValueError("batch must hold at least one lane")
        # the automatic schedule choice is made on ``schedule_lanes`` (default: this batch).  Sharded solves pass
        # the largest shard of the global batch, so that every rank picks the same schedule: the schedules
        # synchronise (all-reduce) at different points, and mixed choices would pair up the wrong collectives.
        sched_B = self.B_sched = int(schedule_lanes) if schedule_lanes is not None else int(B)
        auto_schedule = pipeline is None and persistent is None
        engine.weights.require_gain_solvable()
        self.eng = engine
        self.x_ref, self.u_ref = engine.refs(x_ref, u_ref, per_lane=True)
        self.B, self.Bp = int(B), padded(int(B))
        self.N = int(self.x_ref.shape[-2])
        # per-lane references (x_ref (B,N,4), u_ref (B,T,2); GYM_FLAG_REF_LANE): every schedule, no state
        # checkpointing
        self.ref_lane = self.x_ref.ndim == 3
        if self.ref_lane:
            if self.x_ref.shape[0] != self.B:
                raise ValueError(f"per-lane references must hold {self.B} lanes, got {self.x_ref.shape[0]}")
            if checkpoint:
                raise ValueError("per-lane references do not combine with state checkpointing")
            pad = self.Bp - self.B                     # padding lanes read valid rows (the last lane's)
            self._xr_in, self._ur_in = self.x_ref, self.u_ref
            self.xr_buf = torch.cat([self.x_ref, self.x_ref[-1:].expand(pad, -1, -1)]).contiguous()
            self.ur_buf = torch.cat([self.u_ref, self.u_ref[-1:].expand(pad, -1, -1)]).contiguous()
        self.T = self.N - 1
        self.armijo = _lib.GymArmijo(float(tol), float(beta), float(c), float(gamma_0), int(max_ls),
                                     1 if hist_len > 0 else 0)
        if max_ls < 1:
            raise ValueError("max_ls must be >= 1")
        dev = engine.device
        e = lambda *s, dt=F64: torch.empty(s, dtype=dt, device=dev)  # noqa: E731
        Bp, N, T = self.Bp, self.N, self.T
        shapes = [(N, 2, Bp, 2), (N, 2, Bp, 2), (T, 2, Bp, 1), (T, 2, Bp, 1), (T, 2, Bp, 2), (T, 2, Bp, 1)]
        self.pipeline = (sched_B >= self.pipeline_min_lanes(dev)) if pipeline is None else bool(pipeline)
        # placement selection: default for the automatic schedule's pipelined solvers (the only schedule whose
        # throughput is the HBM streams'); a set chosen by an earlier solver of this shape in this process is reused
        # from the PlacementPool without a probe
        if placement_trials is None:
            placement_trials = (self.PLACEMENT_TRIALS if (auto_schedule and self.pipeline and persistent is not True
                                                          and not arena and not checkpoint) else 1)
        self.placement = None
        self._pl = None
        self._pool_key = (torch.device(dev).index, tuple(shapes))
        pooled = PlacementPool.take(self._pool_key) if int(placement_trials) > 1 and not arena else None
        if pooled is not None:
            st, rec = pooled
            self.placement = dict(rec, reused=True)
        elif arena:
            # the six streams carved from one allocation, each 2 MiB aligned, in this order (arena: True = a torch
            # allocation, or a callable n -> fp64 device tensor of n elements that provides it)
            al = (2 << 20) // 8
            offs, n = [], 0
            for sh in shapes:
                offs.append(n)
                n += -(-int(np.prod(sh)) // al) * al
            self._arena = arena(n) if callable(arena) else e(n)
            st = [self._arena[o:o + int(np.prod(sh))].view(sh) for o, sh in zip(offs, shapes)]
        else:
            st = [e(*sh) for sh in shapes]
        self._stream_shapes = shapes
        self._set_streams(st)
        self.cost, self.dJ, self.smax, self.gamma = e(Bp), e(Bp), e(Bp), e(Bp)
        i32 = torch.int32
        self.status, self.n_iter, self.res_buf, self.n_roll = (e(Bp, dt=i32) for _ in range(4))
        self.retry_list = e(Bp, dt=i32)
        self.counters = torch.zeros(4, dtype=i32, device=dev)
        self.cand_ok = torch.zeros((max(int(max_ls), 1), Bp), dtype=torch.uint8, device=dev)
        self.partials = e(256 * 8)
        self.stats = torch.zeros(24, dtype=F64, device=dev)     # [0,8) totals, [8,16) / [16,24) halves
        self.max_iters = None
        self.hist_len = int(hist_len)
        self.hist_cost = torch.full((hist_len, Bp), float("nan"), dtype=F64, device=dev) if hist_len else None
        self.hist_smax = torch.full((hist_len, Bp), float("nan"), dtype=F64, device=dev) if hist_len else None
        self.K1.zero_(); self.cs.zero_()
        b = _lib.GymBatch()
        b.B, b.Bp, b.N, b.hist_len = self.B, self.Bp, self.N, self.hist_len
        # tau1 is unactuated (dynamics.py:205); with u_ref[:,0] == 0 its controls stay exactly 0 and the
        # kernels skip their planes (GYM_FLAG_U0_ZERO) -- bit-identical results, 24 B/stage less traffic
        ref_u0_zero = bool((self.u_ref[..., 0] == 0).all().item())
        if u0_zero and not ref_u0_zero:
            raise ValueError("u0_zero=True requires u_ref[:, 0] == 0")
        self.u0_zero = ref_u0_zero if u0_zero is None else bool(u0_zero)
        # state checkpointing (GYM_FLAG_X_CKPT, opt-in): trials store x at every CKPT_INTERVAL-th knot only
        # and the sweep re-integrates the rest -- bit-identical results, 48 B/stage less traffic, but +0.75 RK4
        # per sweep stage: on MI355X the solver is as VALU- as HBM-limited and this measured 13% slower
        self.checkpoint = bool(checkpoint)
        # persistent schedule (gym_newton_run): not combined with checkpointing (its sweep re-integrates blocks)
        if persistent and self.checkpoint:
            raise ValueError("the persistent schedule does not support state checkpointing")
        if persistent is None:   # automatic only when the caller chose no schedule at all
            persistent = pipeline is None and sched_B <= self.persistent_max_lanes(dev)
        self.persistent = bool(persistent) and not self.checkpoint
        # iterations per persistent launch (0: all of max_iters in one).  128 keeps one launch to ~0.15 s at the
        # batch sizes that use the schedule (a non-converging batch at max_iters = 5000 would otherwise hold the
        # GPU in one multi-second kernel); the 3-4 launch boundaries of a headline solve cost nothing measurable.
        self.chunk = int(chunk)
        # solve() works on the lanes in the Morton order of their initial states (see morton_order)
        self.reorder = bool(reorder)
        self.lane_order = None
        # persistent schedule on two wavefronts per 64 lanes (k_nt_run2: a helper wavefront takes the Jacobians,
        # the cost and the stores off the lanes' dependency chains; same bits) unless split_waves=False
        self.split_waves = bool(split_waves)
        b.flags = ((_lib.FLAG_U0_ZERO if self.u0_zero else 0) | (_lib.FLAG_X_CKPT if self.checkpoint else 0) |
                   (0 if self.split_waves else _lib.FLAG_RUN_SINGLE) | (_lib.FLAG_REF_LANE if self.ref_lane else 0))
        for name in ("cost", "dJ", "smax", "gamma", "status", "n_iter", "res_buf", "n_roll",
                     "retry_list", "counters", "cand_ok", "partials", "stats"):
            setattr(b, name, getattr(self, name).data_ptr())
        if self.ref_lane:
            b.x_ref, b.u_ref = self.xr_buf.data_ptr(), self.ur_buf.data_ptr()
        else:
            b.x_ref, b.u_ref = self.x_ref.data_ptr(), self.u_ref.data_ptr()
        b.hist_cost = _lib.ptr(self.hist_cost)
        b.hist_smax = _lib.ptr(self.hist_smax)
        self.batch = b
        self._set_streams(st)
        self.k = 0
        self.timeline = None     # diagnostics: a list records (iterations, active lanes, host time) per sync
        self.timing = None
        self.launches = {"phase": 0, "run": 0, "tail": 0, "iteration": 0}   # launches since reset_timing()
        # selected-lane trajectory capture (the reference's history['x_trajs'], trajectory_generation.py:322-327,
        # 387-388): after every iteration the captured lanes' current iterates are gathered on the device; the
        # persistent schedule then runs one iteration per launch.  Not combined with checkpointing (the state
        # buffers hold checkpoints only).
        self.capture_lanes = None if capture_lanes is None else [int(i) for i in capture_lanes]
        if self.capture_lanes is not None:
            if self.checkpoint:
                raise ValueError("trajectory capture needs the full state store (checkpoint=False)")
            if any(not (0 <= i < self.B) for i in self.capture_lanes):
                raise ValueError(f"capture_lanes must lie in [0, {self.B})")
        self.capture_every = max(int(capture_every), 1)
        # sigma of the captured lanes at these iterations (the reference's report plots iterations 0, 1, 2 and the
        # last, trajectory_generation.py:341, 476-480; the last one is the solve's own sigma output)
        self.capture_sigma = tuple(sorted({int(i) for i in (capture_sigma or ())}))
        # straggler tail (serial / pipelined schedules; needs the full state store, whole-iteration launches: no
        # trajectory capture, at most 64 Armijo trials): switch once the global active count is <= tail_lanes.
        # Default: on with the automatic schedule choice, TAIL_LANES_PER_CU per CU of every rank (``world_size``:
        # the ranks the statistics are all-reduced over, so the switch comes at the same per-GPU occupancy at any
        # world size); a caller that picks a schedule gets it pure
        # the default also caps each rank's own active count at its per-GPU budget (tail_lanes_rank; the maximum over
        # ranks is all-reduced once the global count is under the threshold): with skewed shards one rank could
        # otherwise enter the tail with up to world x its budget of lanes, one workgroup each
        self.tail_lanes_rank = None
        if tail_lanes is None:
            per_rank = (self.TAIL_LANES_PER_CU * torch.cuda.get_device_properties(dev).multi_processor_count
                        if auto_schedule else 0)
            tail_lanes = per_rank * max(int(world_size), 1)
            self.tail_lanes_rank = per_rank or None
        # the tail kernel's limits: at most 64 trials, horizons up to its LDS staging, and that LDS within the
        # device's opt-in limit (checked here, so a device with less LDS turns the tail off instead of failing mid-solve)
        need, lds, lds_max = C.c_int64(), C.c_int64(), C.c_int64()
        tail_ok = (not self.persistent and not self.checkpoint and self.capture_lanes is None and
                   engine.lib.gym_newton_tail_scratch(self.N, 1, int(max_ls), C.byref(need)) == 0 and
                   engine.lib.gym_newton_tail_lds(self.N, C.byref(lds), C.byref(lds_max)) == 0 and
                   lds.value <= lds_max.value)
        self.tail_lanes = int(tail_lanes) if tail_ok else 0
        self.tail_chunk = max(int(tail_chunk), 1)
        # lane compaction (serial / pipelined schedules, solve(); see maybe_compact): default on with the automatic
        # schedule choice.  "force" compacts at every host synchronisation (tests)
        if compact is None:
            compact = auto_schedule
        self.compact_mode = ("force" if compact == "force" else bool(compact)) if (
            not self.persistent and not self.checkpoint and self.capture_lanes is None) else False
        self.compactions = 0
        self._compact_prev = None
        self.lane_order_live = False   # True inside solve(), whose results follow lane_order back
        self._serial_now = False
        self._run_now = False
        self.serial_switch_at = None   # the iteration the low-occupancy switch happened at
        self._its_switch, self._its_tail_start = 0, None
        self._tail_scratch = None
        # candidate scratch (gym_batch.cand_scratch, ABI 13): the post-trial Armijo candidates of the serial /
        # pipelined schedules and the low-occupancy regime record their trajectories, and the accepted one is copied
        # instead of re-run (a T-step chain per backtracking iteration).  Slots for min(lanes x (max_ls - 1),
        # cand_slots) candidates (~24 KiB each at T = 500); lanes past them are re-run.  The straggler tail borrows
        # the same buffer.  0 turns it off (the same bits either way).
        # Allocated on demand (ensure_cand_scratch): at the first host synchronisation whose iteration had lanes
        # rejecting trial 1, on entering the low-occupancy regime, or for the tail; a solve in which no lane
        # backtracks (the headline workload) never holds it.  Until then the accepted candidates are re-run (the
        # same bits).
        if cand_slots is None:
            cand_slots = self.CAND_SLOTS
        slots = min(self.Bp * max(int(max_ls) - 1, 0), int(cand_slots))
        slots = slots // 64 * 64
        self._cand_scratch = None
        ok = slots > 0 and not self.persistent and not self.checkpoint and self.split_waves
        self.cand_slots = slots if ok else 0
        self.tail_lane_its = 0
        self.tail_from, self.tail_iters = None, 0
        self._cap_pos = None
        self._cap_log = []
        self._sig_log = []
        if self.placement is not None:            # a pooled set: back to the pool when this solver goes
            self._lease_placement()
        elif int(placement_trials) > 1 and self.pipeline and not self.persistent:
            self._arm_placement(int(placement_trials))

    def _set_streams(self, st, zero: bool = True):
        """Use the stream set st = [x0, x1, u0, u1, K1, cs]; ``zero``: K1 and cs zeroed, as at construction (False: a
        set that holds the live state, copied by _move_streams)."""
        self.x = list(st[0:2])
        self.u = list(st[2:4])                         # control planes (tau1, tau2)
        self.K1 = st[4]                                # gain row 1, pairs
        self.cs = st[5]                                # planes: cg = (u1 - K1 x) + gamma0 sigma1, sigma1
        if zero:
            self.K1.zero_(); self.cs.zero_()
        b = getattr(self, "batch", None)
        if b is not None:
            b.x[0], b.x[1] = self.x[0].data_ptr(), self.x[1].data_ptr()
            b.u[0], b.u[1] = self.u[0].data_ptr(), self.u[1].data_ptr()
            b.K1, b.cs = self.K1.data_ptr(), self.cs.data_ptr()

    def _streams(self) -> list:
        return [*self.x, *self.u, self.K1, self.cs]

    def _move_streams(self, st):
        """Continue on stream set ``st``: the six streams copied into it (stream-ordered device copies, ~19 GB each way
        at 262,144 lanes), then the launches pointed at it.  Between two iterations the streams hold the whole state a
        later iteration reads (both state / control buffers, the gains and offsets of the half whose sweep already ran),
        so the solve continues bit for bit."""
        for src, dst in zip(self._streams(), st):
            dst.copy_(src)
        self._set_streams(st, zero=False)

    # --- placement selection ---------------------------------------------------------------
    # Why placements differ (profiles/r06/README.md): on a slow set the same fabric requests come back later (+13..24%
    # read latency, ~2x the L2's DRAM-credit and write stalls; no more translation misses, no channel imbalance), and
    # the slowness follows how the streams the same waves touch in lock step lie relative to each other in physical
    # memory; no allocation rule reachable from user space fixes it (contiguous VRAM at 200 layouts, record layouts),
    # so the solver measures: candidates ranked by the placement probe, the best raced in the first solve, the winner
    # pooled for the process's later solvers of the same shape.
    def _arm_placement(self, trials: int, candidates: int | None = None):
        """Allocate up to ``candidates`` - 1 further stream sets (while the free memory allows, beside the lane-major
        results a solve allocates), rank all of them with the placement probe and keep the ``trials`` best for the
        online selection of the next solve (_placement_tick); the others go back to the device."""
        dev = self.eng.device
        candidates = max(int(candidates or self.PLACEMENT_CANDIDATES), int(trials))
        set_bytes = 8 * sum(int(np.prod(sh)) for sh in self._stream_shapes)
        B, N, T = self.B, self.N, self.T
        results_bytes = 8 * B * (4 * N + 2 * T + 8 * T + 2 * T)      # finalize's x, u, K, sigma
        free, total = torch.cuda.mem_get_info(dev)
        # beside the results a solve allocates, and at most PLACEMENT_MEM_SHARE of the device for the extra sets (so
        # that processes sharing a GPU leave each other room); an allocation that fails (another process was faster)
        # just ends the candidate list
        room = min(free - results_bytes - (4 << 30), self.PLACEMENT_MEM_SHARE * total)
        k = min(candidates, 1 + max(0, int(room // max(set_bytes, 1))))
        if k < 2:
            return
        t0 = time.perf_counter()
        sets = [self._streams()]
        try:
            for _ in range(k - 1):
                sets.append([torch.empty(sh, dtype=F64, device=dev) for sh in self._stream_shapes])
        except torch.cuda.OutOfMemoryError:
            torch.cuda.empty_cache()
        k = len(sets)
        if k < 2:
            return
        screen = None
        if k > trials and self.Bp % 128 == 0:
            # rank the candidates by the placement probe (two rounds, each set's faster launch), keep the best
            ms = [float("inf")] * k
            for r in range(2):
                for i, st in enumerate(sets):
                    self._set_streams(st, zero=False)
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    ev[0].record()
                    _lib.check(self.eng.lib.gym_placement_probe(C.byref(self.batch), r & 1, self.eng.stream),
                               "gym_placement_probe")
                    ev[1].record()
                    ev[1].synchronize()
                    ms[i] = min(ms[i], ev[0].elapsed_time(ev[1]))
            keep = sorted(range(k), key=lambda i: ms[i])[:trials]
            screen = {"candidates": k, "probe_ms": ms, "kept": keep}
            sets = [sets[i] for i in keep]
            torch.cuda.empty_cache()                # the screened-out sets go back to the device
        self._set_streams(sets[0])                  # K1, cs zeroed (the probe left garbage), as at construction
        if len(sets) < 2:
            return
        self._pl = {"sets": sets, "cur": 0, "attempts": 0, "alloc_s": time.perf_counter() - t0, "screen": screen}
        self.placement = {"trials": len(sets), "state": "pending", "alloc_s": self._pl["alloc_s"], "screen": screen}

    def _placement_start(self):
        """(init) A new solve: the selection schedule restarts from the set in use, in the order c, the others, then
        the reverse (each set runs two blocks placed symmetrically, so a drift of the iterations' cost over the probe
        cancels out of the comparison)."""
        pl = self._pl
        pl["attempts"] += 1
        if pl["attempts"] > 2:                     # two solves ended before the probe did: keep the set in use
            self._placement_finish(abandon=True)
            return
        k = len(pl["sets"])
        seq = [pl["cur"]] + [i for i in range(k) if i != pl["cur"]]
        pl.update(order=seq + seq[::-1], blocks=[], open=None, copies=0)

    def _placement_tick(self):
        """(iteration, before its launches) At the block boundaries of the schedule: close the running block with an
        event, move the state to the next block's set, open the next block.  Only on the pipelined schedule while it
        runs its phases (the low-occupancy regime and the tail end the probe for this solve)."""
        pl = self._pl
        if self._serial_now or self._run_now or "order" not in pl:
            return
        k, n = self.k, self.PLACEMENT_BLOCK
        if k % n:
            return
        if pl["open"] is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            pl["blocks"].append((*pl["open"], ev))
            pl["open"] = None
        i = k // n
        if i >= len(pl["order"]):
            self._placement_finish()
            return
        target = pl["order"][i]
        if target != pl["cur"]:
            self._move_streams(pl["sets"][target])
            pl["cur"] = target
            pl["copies"] += 1
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        pl["open"] = (target, ev)

    def _placement_finish(self, abandon: bool = False):
        """Keep the fastest set (by the mean of its blocks' ms per iteration), release the others, and lease the kept
        one to this solver (back to the PlacementPool when the solver goes)."""
        pl, n = self._pl, self.PLACEMENT_BLOCK
        per = {}
        for s, e0, e1 in pl.get("blocks", []):
            e1.synchronize()
            per.setdefault(s, []).append(e0.elapsed_time(e1) / n)
        best = pl["cur"]
        if not abandon and per:
            best = min(per, key=lambda s: sum(per[s]) / len(per[s]))
            if best != pl["cur"]:
                self._move_streams(pl["sets"][best])
                pl["copies"] += 1
        self.placement = {"trials": len(pl["sets"]), "state": "abandoned" if abandon else "chosen", "chosen": best,
                          "ms_per_iteration": {int(s): v for s, v in sorted(per.items())},
                          "probe_iterations": n * len(pl.get("blocks", [])), "copies": pl.get("copies", 0),
                          "alloc_s": pl["alloc_s"], "at_iteration": int(self.k), "screen": pl.get("screen")}
        self._pl = None
        pl.clear()
        torch.cuda.empty_cache()                    # the unused sets go back to the device, not the process's cache
        self._lease_placement()

    def _lease_placement(self):
        st, rec = self._streams(), {k: v for k, v in self.placement.items() if k != "reused"}
        f = weakref.finalize(self, PlacementPool.put, self._pool_key, st, rec)
        f.atexit = False

    def ensure_cand_scratch(self) -> bool:
        """Allocate the candidate scratch (cand_slots slots, ~24 KiB each at T = 500) if this solver uses one and has
        not yet; stream-ordered, so the next launch may use it.  Returns whether it is in place."""
        if self._cand_scratch is None and self.cand_slots > 0:
            need = C.c_int64()
            _lib.check(self.eng.lib.gym_newton_cand_scratch(self.N, self.cand_slots, C.byref(need)),
                       "gym_newton_cand_scratch")
            self._cand_scratch = torch.empty(int(need.value), dtype=F64, device=self.eng.device)
            self.batch.cand_scratch, self.batch.cand_slots = self._cand_scratch.data_ptr(), self.cand_slots
        return self._cand_scratch is not None

    @property
    def schedule(self) -> str:
        return "persistent" if self.persistent else ("pipelined" if self.pipeline else "serial")

    def phase_kind(self) -> str | None:
        """The build of the phase kernel this batch's full phases launch (pipelined schedule; gym_newton_phase_kind):
        "two-wavefront" (more than 7/8 and at most two wavefronts per SIMD: compiled for two, prefetching two stages
        ahead) or "four-wavefront"; None for the other schedules.  Both builds give the same bits."""
        if self.schedule != "pipelined":
            return None
        lo = C.c_int32()
        _lib.check(self.eng.lib.gym_newton_phase_kind(C.byref(self.batch), C.byref(lo)), "gym_newton_phase_kind")
        return "two-wavefront" if lo.value else "four-wavefront"

    # --- optional per-kernel HIP-event timing (on the solver's stream) ---------------------
    def enable_timing(self):
        if self.timing is None:
            t = _lib.GymTiming()
            _lib.check(self.eng.lib.gym_timing_create(C.byref(t)), "gym_timing_create")
            self.timing = t
            self.batch.timing = C.pointer(t)
        return self

    def reset_timing(self):
        self.launches = {"phase": 0, "run": 0, "tail": 0, "iteration": 0}
        if self.timing is not None:
            torch.cuda.synchronize(self.eng.device)   # collect_timing reads completed event pairs only
            self.collect_timing()       # drains the pool (pairs of launches before the reset)
            for i in range(len(_lib.KERNEL_KINDS)):
                self.timing.ms[i] = 0.0
                self.timing.launches[i] = 0
            self.timing.pending = 0

    def collect_timing(self):
        """Accumulate recorded event pairs; the stream must have been synchronised."""
        if self.timing is not None:
            _lib.check(self.eng.lib.gym_timing_collect(C.byref(self.timing)), "gym_timing_collect")

    def kernel_times(self) -> dict:
        """{kind: (total_ms, launches)} for kinds _lib.KERNEL_KINDS."""
        if self.timing is None:
            return {}
        return {k: (float(self.timing.ms[i]), int(self.timing.launches[i])) for i, k in enumerate(_lib.KERNEL_KINDS)}

    def __del__(self):
        t = getattr(self, "timing", None)
        if t is not None:
            try:
                self.eng.lib.gym_timing_destroy(C.byref(t))
            except Exception:
                pass

    # --- the three stream-ordered phases (no host synchronisation inside) -----------------
    def init(self, x0, _ref_perm=None):
        self.lane_order = None
        x0 = self.eng.t(x0).reshape(-1, 4)
        if x0.shape[0] != self.B:
            raise ValueError(f"x0 must hold {self.B} lanes, got {x0.shape[0]}")
        if self.ref_lane:   # the references in the lanes' internal order (solve()'s Morton order, or the caller's)
            self.xr_buf[:self.B] = self._xr_in if _ref_perm is None else self._xr_in[_ref_perm]
            self.ur_buf[:self.B] = self._ur_in if _ref_perm is None else self._ur_in[_ref_perm]
        self._x0 = x0
        if self._pl is not None:
            self._placement_start()
        _lib.check(self.eng.lib.gym_newton_init(C.byref(self.eng.model), C.byref(self.eng._w), x0.data_ptr(),
                                                C.byref(self.batch), self.eng.stream), "gym_newton_init")
        self.k = 0
        self._capture_start(self.capture_lanes or [])
        self._serial_now = False   # the low-occupancy regime (maybe_compact / _enter_low_occupancy)
        self._run_now = False
        self._sigma_streamed = False
        self.batch.flags &= ~_lib.FLAG_SIGMA_STREAM
        if self.pipeline and not self.persistent and (self.max_iters is None or self.max_iters > 0):
            self._phase(0, True)                 # prologue: backward sweep of half H0, iteration 0

    def _run(self, k0: int, k1: int):
        self.launches["run"] += 1
        _lib.check(self.eng.lib.gym_newton_run(C.byref(self.eng.model), C.byref(self.eng._w), C.byref(self.armijo),
                                               C.byref(self.batch), int(k0), int(k1), self.eng.stream),
                   "gym_newton_run")

    def tail_run(self, k0: int, k1: int) -> torch.Tensor:
        """Iterations k0 .. k1-1 of every lane still active, on the straggler-tail kernel (gym_newton_tail: one
        workgroup per lane, every Armijo trial at once; the serial schedule's bits).  Every active lane must have
        done k0 iterations (the lock-step schedules' state after ``k0`` calls of iteration()).  Returns the 8
        statistics after iteration k1 - 1 (device)."""
        lanes = (self.status[:self.B] == _lib.ACTIVE).nonzero().flatten().to(torch.int32)
        n = int(lanes.numel())
        need = C.c_int64()
        _lib.check(self.eng.lib.gym_newton_tail_scratch(self.N, n, int(self.armijo.max_ls), C.byref(need)),
                   "gym_newton_tail_scratch")
        self.ensure_cand_scratch()
        if self._cand_scratch is not None and self._cand_scratch.numel() >= need.value:
            sc = self._cand_scratch          # the candidate scratch (the tail and the post-trial kernels never overlap)
        else:
            if self._tail_scratch is None or self._tail_scratch.numel() < need.value:
                self._tail_scratch = None
                self._tail_scratch = torch.empty(int(need.value), dtype=F64, device=self.eng.device)
            sc = self._tail_scratch
        self.launches["tail"] += 1
        _lib.check(self.eng.lib.gym_newton_tail(C.byref(self.eng.model), C.byref(self.eng._w), C.byref(self.armijo),
                                                C.byref(self.batch), lanes.data_ptr() if n else None, n,
                                                sc.data_ptr(), int(sc.numel()), int(k0), int(k1), self.eng.stream),
                   "gym_newton_tail")
        self.k = int(k1)
        return self.stats[:8]

    def _phase(self, p: int, do_backward: bool):
        self.launches["phase"] += 1
        _lib.check(self.eng.lib.gym_newton_phase(C.byref(self.eng.model), C.byref(self.eng._w), C.byref(self.armijo),
                                                 C.byref(self.batch), p, int(do_backward), self.eng.stream),
                   "gym_newton_phase")

    def iteration(self) -> torch.Tensor:
        """Enqueue outer iteration k for every active lane; returns the 8 total statistics (device)."""
        if self._pl is not None:
            self._placement_tick()
        k = self.k
        if self.persistent or self._run_now:
            self._run(k, k + 1)
        elif self.pipeline and not self._serial_now:
            more = self.max_iters is None or k + 1 < self.max_iters
            self._phase(2 * k + 1, True)         # sweep H1 (iteration k) beside trial H0 (iteration k)
            self._phase(2 * k + 2, more)         # sweep H0 (iteration k+1) beside trial H1 (iteration k)
        else:
            self.launches["iteration"] += 1
            _lib.check(self.eng.lib.gym_newton_iteration(C.byref(self.eng.model), C.byref(self.eng._w),
                                                         C.byref(self.armijo), C.byref(self.batch), k,
                                                         self.eng.stream), "gym_newton_iteration")
        self.k += 1
        self._capture()
        return self.stats[:8]

    # --- selected-lane trajectory capture -----------------------------------------------------
    def _capture_start(self, positions):
        """Begin capturing the lanes at internal positions ``positions`` (after init: the open-loop rollout)."""
        self._cap_log = []
        self._sig_log = []
        if self.capture_lanes is None:
            self._cap_pos = None
            return
        self._cap_pos = torch.as_tensor(positions, dtype=torch.int64, device=self.eng.device)
        self._capture(initial=True)

    def _capture(self, initial: bool = False):
        """Enqueue a gather of the captured lanes' current iterates, their iteration counts, statuses and costs.
        Device work only: no host synchronisation."""
        if self._cap_pos is None or (not initial and self.k % self.capture_every):
            return
        pos = self._cap_pos
        W = self.Bp // 64
        # wave-blocked pairs: (N, Bp/64, 2 rows, 64 lanes, 2) -> (n_cap, N, 2, 2) per buffer (the advanced
        # indices' dimension leads)
        # after k iterations a lane that accepted iteration k-1 holds its iterate in buffer k & 1 (iteration k-1
        # wrote its candidate there); the records of lanes that did not are discarded by captured_trajectories
        xb = self.x[self.k & 1]
        x = xb.view(self.N, W, 2, 64, 2)[:, pos // 64, :, pos % 64, :].reshape(-1, self.N, 4)
        self._cap_log.append((self.k, x.clone(), self.n_iter[pos].clone(), self.status[pos].clone(),
                              self.cost[pos].clone()))
        if not initial and (self.k - 1) in self.capture_sigma:
            # iteration k-1's sigma: gym_newton_sigma re-runs each lane's sweep at the iterate of its last
            # iteration (the same bits as that iteration's own sweep); it writes only the sigma1 plane, which every
            # schedule rewrites before reading it, so the solve is unchanged
            self._sig_log.append((self.k - 1, self.sigma()[pos].clone(), self.n_iter[pos].clone()))

    def captured_trajectories(self) -> dict:
        """{caller lane: [x_0, x after each accepted iteration ...]} as (N,4) numpy arrays -- the reference's
        history['x_trajs'] of each captured lane (entries only every ``capture_every`` iterations)."""
        if self.capture_lanes is None:
            return {}
        out = {lane: [] for lane in self.capture_lanes}
        for k, x, n_it, st, _ in self._cap_log:
            x, n_it, st = x.cpu().numpy(), n_it.cpu().numpy(), st.cpu().numpy()
            for j, lane in enumerate(self.capture_lanes):
                if k == 0:
                    out[lane].append(x[j])
                elif n_it[j] == k and st[j] != _lib.LS_FAILED:   # the lane ran iteration k-1 and accepted it
                    out[lane].append(x[j])
        return out

    def captured_sigmas(self) -> dict:
        """{caller lane: {iteration i: sigma (T,2)}} for the iterations of ``capture_sigma`` each captured lane ran
        (the reference's history['sigmas'][i])."""
        if self.capture_lanes is None:
            return {}
        out = {lane: {} for lane in self.capture_lanes}
        for it, sg, n_it in self._sig_log:
            sg, n_it = sg.cpu().numpy(), n_it.cpu().numpy()
            for j, lane in enumerate(self.capture_lanes):
                if n_it[j] == it + 1:                    # the lane ran iteration it
                    out[lane][it] = sg[j]
        return out

    def captured_initial_costs(self) -> dict:
        """{caller lane: J_0} of the captured lanes (the reference's history['cost'][0])."""
        if self.capture_lanes is None or not self._cap_log:
            return {}
        c0 = self._cap_log[0][4].cpu().numpy()
        return {lane: float(c0[j]) for j, lane in enumerate(self.capture_lanes)}

    def finalize(self):
        B, N, T, dev = self.B, self.N, self.T, self.eng.device
        x = torch.empty((B, N, 4), dtype=F64, device=dev)
        u = torch.empty((B, T, 2), dtype=F64, device=dev)
        K = torch.empty((B, T, 2, 4), dtype=F64, device=dev)
        s = torch.empty((B, T, 2), dtype=F64, device=dev)
        _lib.check(self.eng.lib.gym_newton_finalize(C.byref(self.eng.model), C.byref(self.eng._w), C.byref(self.batch),
                                                    self.k, x.data_ptr(),
                                                    u.data_ptr(), K.data_ptr(), s.data_ptr(), self.eng.stream),
                   "gym_newton_finalize")
        return x, u, K, s

    def states(self, buf: int) -> torch.Tensor:
        """Every knot of state buffer ``buf`` (SoA (N,2,Bp,2)), rebuilt from its checkpoints if checkpointing."""
        _lib.check(self.eng.lib.gym_newton_fill_states(C.byref(self.eng.model), C.byref(self.batch), int(buf),
                                                       self.eng.stream), "gym_newton_fill_states")
        return self.x[buf]

    def gamma_sweep(self, gammas) -> torch.Tensor:
        """Armijo line-search curve of every lane at the current iterate (the one iteration ``self.k`` starts
        from): J(gamma_g) of the trial rollout along iteration k's direction, (B, G); NaN for finished lanes.
        At the trial step sizes gamma_0 beta^i the values are the Armijo trials' costs bit for bit.  Runs
        iteration k's backward sweep, which that iteration recomputes identically, so the solve is unchanged."""
        g = self.eng.t(gammas).reshape(-1)
        G = int(g.numel())
        if G < 1:
            raise ValueError("gamma_sweep needs at least one step size")
        J = torch.empty((G, self.Bp), dtype=F64, device=self.eng.device)
        _lib.check(self.eng.lib.gym_newton_gamma_sweep(C.byref(self.eng.model), C.byref(self.eng._w),
                                                       C.byref(self.armijo), C.byref(self.batch), self.k, g.data_ptr(), G, J.data_ptr(),
                                                       self.eng.stream), "gym_newton_gamma_sweep")
        return J[:, :self.B].t()

    def gains(self) -> torch.Tensor:
        """K (B,T,2,4) of every lane's most recent backward sweep."""
        K = torch.empty((self.B, self.T, 2, 4), dtype=F64, device=self.eng.device)
        _lib.check(self.eng.lib.gym_unpack_gains(self.K1.data_ptr(), K.data_ptr(), self.B, self.Bp, self.T,
                                                 self.eng.stream), "gym_unpack_gains")
        return K

    def controls(self, buf: int) -> torch.Tensor:
        """u (B,T,2) of control buffer ``buf``."""
        return self.eng.unpack(self.u[buf], self.B)

    def stream_sigma(self):
        """Call right after init(): run every iteration as the low-occupancy regime does (one launch of the
        four-wavefront persistent kernel per iteration, its sweep storing sigma1; _enter_low_occupancy), so that
        sigma() reads each iteration's sigma from the stored plane instead of re-running every lane's sweep.  For
        callers that want every iteration's sigma of a few lanes (the drop-in newton_Algorithm's history).  The same
        bits as any schedule."""
        if self.k != 0:
            raise RuntimeError("stream_sigma() must follow init() directly")
        self.pipeline = False
        self._enter_low_occupancy()
        self._sigma_streamed = True
        return self

    def sigma(self, rerun: bool = False) -> torch.Tensor:
        """sigma (B,T,2) of every lane's last completed iteration: its sweep re-run (sigma1 is not streamed), or,
        after stream_sigma() with the tau1 channel zero (u0_zero: sigma0 = -(2R0 (u0 - ur0)) / (2R0) = -0 on every
        stage), the sigma1 plane that iteration's sweep stored -- bit for bit the re-run (``rerun`` forces it)."""
        if self._sigma_streamed and self.u0_zero and not rerun:
            s = self.eng.unpack(self.cs, self.B)      # (B, T, 2): cg, sigma1
            s[..., 0] = -0.0
            return s
        s = torch.empty((self.B, self.T, 2), dtype=F64, device=self.eng.device)
        _lib.check(self.eng.lib.gym_newton_sigma(C.byref(self.eng.model), C.byref(self.eng._w), C.byref(self.batch),
                                                 s.data_ptr(),
                                                 self.eng.stream), "gym_newton_sigma")
        return s

    # --- lane compaction ------------------------------------------------------------------
    COMPACT_MAX_SHARE = 0.25   # consider compacting once at most this share of the lanes is active ...
    COMPACT_MIN_KEEP = 0.5     # ... and the active count kept at least half its value since the last sync

    def maybe_compact(self, active: int) -> bool:
        """At a host synchronisation (iteration boundary), once at most a quarter of the lanes stay active (a stable
        population: the count kept at least half its value since the last sync), enter the low-occupancy regime:
        move the active lanes to the front (compact) and continue one iteration per launch of the persistent kernel
        with external retries (_enter_low_occupancy); later, compact again whenever the active lanes are spread over
        more than twice the wavefronts they need.  A wavefront runs its whole chains while any of its 64 lanes is
        active, so late in a hard solve (SURVEY 8(d)'s stress batch: ~22,000 of 262,144 lanes active for hundreds of
        iterations) every SIMD may still run its four wavefronts for a few lanes each; and with at most one
        wavefront per SIMD every launch is a latency-bound chain.  ``active``: this rank's count.  The trigger is
        rank-local (neither step changes a collective)."""
        if not self.compact_mode:
            return False
        prev, self._compact_prev = self._compact_prev, int(active)
        if active <= 0:
            return False
        if self.compact_mode != "force":
            if active > self.COMPACT_MAX_SHARE * self.B or prev is None or active < self.COMPACT_MIN_KEEP * prev:
                return False   # most lanes active, or a collapsing population that finishes on its own
            occupied = int((self.status.view(-1, 64) == _lib.ACTIVE).any(1).sum().item())
            if occupied < 2 * (-(-int(active) // 64) + 2) and (self._serial_now or not self.split_waves):
                if self._serial_now:
                    return False           # already dense, already switched
                self._enter_low_occupancy()
                return True
        self.compact()                     # (entering the persistent kernel's mode: always dense first)
        return True

    def _enter_low_occupancy(self):
        """Continue a pipelined or serial solve one iteration per launch of the four-wavefront persistent kernel
        (k_nt_run2: split Riccati sweep, lane-pair trial chains), its sweep storing sigma1 and the lanes that reject
        trial 1 finished by the serial schedule's parallel candidates and accepted re-run (GYM_FLAG_SIGMA_STREAM);
        with single-wavefront persistent kernels (split_waves=False), on the serial schedule (its sweep storing
        sigma1).  The same bits either way (the schedules' bitwise equality)."""
        self.ensure_cand_scratch()
        if not self._serial_now:
            self.serial_switch_at = self.k
            self._its_switch = int(self.n_iter[:self.B].sum().item())
        self._serial_now = True
        self._run_now = self.split_waves
        self.batch.flags |= _lib.FLAG_SIGMA_STREAM

    def compact(self, to_serial: bool = True):
        """Permute the lanes so that each lane range the kernels launch over (the serial schedule's batch, the
        pipelined schedule's halves H0 / H1) holds its active lanes first, in their order, and the finished ones
        behind them; waves of finished lanes then exit at once.  Every per-lane buffer moves with its lane (the
        state and trajectory buffers, gains, per-lane scalars, histories, per-lane references) and ``lane_order``
        follows, so solve() returns every lane in the caller's order: the results are the uncompacted solve's
        bit for bit (each lane's arithmetic is its own).  Only lanes that change position are moved.
        ``to_serial`` (the default): the solve then continues in the low-occupancy regime (_enter_low_occupancy;
        the next iteration re-runs H0's sweep, which the pipeline had already run: the same values), and the whole
        batch is one range.  Otherwise lanes keep their pipeline half."""
        B, Bp, dev = self.B, self.Bp, self.eng.device
        act = self.status[:B] == _lib.ACTIVE
        perm = torch.arange(Bp, device=dev)
        pipelined = self.pipeline and not self._serial_now and not to_serial
        if to_serial:
            self._enter_low_occupancy()
        if pipelined:
            Bh = C.c_int64()
            _lib.check(self.eng.lib.gym_newton_pipeline_split(C.byref(self.batch), C.byref(Bh)),
                       "gym_newton_pipeline_split")
            ranges = [(0, int(Bh.value)), (int(Bh.value), B)]
        else:
            ranges = [(0, B)]
        for lo, hi in ranges:
            if hi > lo:   # active lanes first, each group in its present order
                perm[lo:hi] = torch.argsort((~act[lo:hi]).to(torch.int8), stable=True) + lo
        moved = (perm != torch.arange(Bp, device=dev)).nonzero().flatten()
        if moved.numel() == 0:
            return
        src = perm[moved]
        gd, jd, gs, js = moved // 64, moved % 64, src // 64, src % 64
        for t in (self.x[0], self.x[1], self.K1):   # wave-blocked pairs (rows, Bp/64, 2, 64, 2)
            v = t.view(t.shape[0], Bp // 64, 2, 64, 2)
            v[:, gd, :, jd, :] = v[:, gs, :, js, :]
        for t in (self.u[0], self.u[1], self.cs):   # planes (rows, 2, Bp)
            v = t.view(t.shape[0], 2, Bp)
            v[:, :, moved] = v[:, :, src]
        for t in (self.cost, self.dJ, self.smax, self.gamma, self.status, self.n_iter, self.res_buf, self.n_roll):
            t[moved] = t[src]
        for t in (self.hist_cost, self.hist_smax):
            if t is not None:
                t[:, moved] = t[:, src]
        if self.ref_lane:
            self.xr_buf[moved] = self.xr_buf[src]
            self.ur_buf[moved] = self.ur_buf[src]
        order = self.lane_order if self.lane_order is not None else torch.arange(B, device=dev)
        self.lane_order = order[perm[:B]]
        self.compactions += 1

    # --- full solve ----------------------------------------------------------------------
    def solve(self, x0, max_iters: int, reduce_stats=None, sync_every: int = 1, log_every: int = 0,
              keep_stats: bool = False) -> SolveResult:
        """Run until every lane (of every rank, if ``reduce_stats`` all-reduces) is done or max_iters.

        With ``reorder`` (default) the lanes are solved in the Morton order of their initial states
        (``morton_order``) and the results are returned in the caller's order; the device buffers then hold
        lane ``lane_order[i]`` of the input at position i."""
        torch.cuda.synchronize(self.eng.device)
        t0 = time.perf_counter()
        self.max_iters = int(max_iters)
        perm = None
        if self.reorder and self.B > 1:
            x0 = self.eng.t(x0).reshape(-1, 4)
            perm = morton_order(x0)
            x0 = x0[perm]
        self.init(x0, _ref_perm=perm)
        self.lane_order = perm
        if perm is not None and self.capture_lanes is not None:
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(self.B, device=perm.device)
            self._capture_start(inv[torch.as_tensor(self.capture_lanes, device=perm.device)].tolist())
        self.tail_lane_its = 0
        self.tail_from, self.tail_iters = None, 0
        self.compactions = 0
        self._compact_prev = None
        self.serial_switch_at = None
        self._its_switch = 0
        self._its_tail_start = None
        if self.persistent:
            log = run_loop(self, int(max_iters), reduce_stats, log_every, keep_stats)
        else:
            self.lane_order_live = True
            try:
                log = newton_loop(self, max_iters, reduce_stats=reduce_stats, sync_every=sync_every,
                                  log_every=log_every, keep_stats=keep_stats)
            finally:
                self.lane_order_live = False
        B = self.B
        perm = self.lane_order   # the Morton order, composed with any lane compaction of the loop
        if perm is None:
            back = slice(0, B)
        else:   # internal lane i is input lane perm[i]: finalize writes row perm[i]; gather the scalars back
            back = torch.empty_like(perm)
            back[perm] = torch.arange(B, device=perm.device)
            self.batch.lane_map = perm.data_ptr()
        try:
            x, u, K, s = self.finalize()
        finally:
            self.batch.lane_map = None
        lanes = lambda t: t[:B][back]  # noqa: E731
        n_iter = lanes(self.n_iter)
        res = dict(cost=lanes(self.cost), status=lanes(self.status), n_rollouts=lanes(self.n_roll),
                   gamma=lanes(self.gamma),
                   hist_cost=None if self.hist_cost is None else self.hist_cost[:, :B][:, back],
                   hist_smax=None if self.hist_smax is None else self.hist_smax[:, :B][:, back])
        torch.cuda.synchronize(self.eng.device)
        secs = time.perf_counter() - t0
        # persistent: the lanes' own iteration counts (no lock-step outer loop); otherwise the loop's count
        iters = int(n_iter.max().item()) if self.persistent else self.k
        res["x_trajs"] = self.captured_trajectories() if self.capture_lanes is not None else None
        res["cost0"] = self.captured_initial_costs() if self.capture_lanes is not None else None
        res["sigmas"] = self.captured_sigmas() if self.capture_lanes is not None else None
        res["schedule"] = self.schedule
        res["tail_lane_iterations"] = int(self.tail_lane_its)
        res["tail_from_iteration"] = self.tail_from
        res["tail_iterations"] = int(self.tail_iters)
        res["compactions"] = int(self.compactions)
        lowocc = 0
        if self.serial_switch_at is not None:   # up to the tail switch, or the end of the solve
            end = self._its_tail_start if self._its_tail_start is not None else int(n_iter.sum().item())
            lowocc = end - self._its_switch
        res["lowocc_lane_iterations"] = int(lowocc)
        return SolveResult(x=x, u=u, K=K, sigma=s, n_iter=n_iter, iterations=iters,
                           lane_iterations=int(n_iter.sum().item()), seconds=secs, stats_log=log, **res)


def morton_order(x0: torch.Tensor, bits: int = 10) -> torch.Tensor:
    """Lane permutation along a Z-order (Morton) curve over the initial states x0 (B,4).

    A wavefront runs until the last of its 64 lanes has converged, so lanes that need different iteration
    counts waste the slots of the early finishers (on the headline workload, lanes converge after 381-404
    iterations: 97.8% of the slots do useful work in input order).  Neighbouring initial states converge in
    similar counts; grouping them along a space-filling curve raises that to 99.7% (C oracle, 8,192 lanes).
    Each coordinate is quantised to ``bits`` bits over the batch's range (non-finite values as 0) and the
    bits are interleaved; ties keep the input order."""
    x = torch.nan_to_num(x0, nan=0.0, posinf=0.0, neginf=0.0)
    lo, hi = x.min(0).values, x.max(0).values
    span = torch.where(hi > lo, hi - lo, torch.ones_like(hi))
    q = ((x - lo) / span * (2 ** bits - 1)).clamp(0, 2 ** bits - 1).to(torch.int64)
    key = torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)
    d = x.shape[1]
    for b in range(bits):
        for j in range(d):
            key |= ((q[:, j] >> b) & 1) << (b * d + j)
    return torch.argsort(key, stable=True)


def run_loop(solver: BatchedNewtonSolver, max_iters: int, reduce_stats, log_every: int, keep_stats: bool):
    """Persistent schedule: launches of ``chunk`` iterations (0: all of max_iters); after each one the
    statistics are all-reduced across ranks (``reduce_stats``) and read, and the loop stops when no lane of any
    rank is active."""
    log = []
    chunk = solver.chunk if solver.chunk > 0 else max(int(max_iters), 1)
    # trajectory capture: one iteration per launch, but the statistics are still read (and all-reduced) at the
    # same iterations as without capture, so ranks that capture and ranks that do not stay paired
    step = 1 if solver._cap_pos is not None else chunk
    k = 0
    while k < max_iters:
        k1 = min(int(max_iters), k + step)
        solver._run(k, k1)
        solver.k = k = k1
        solver._capture()
        if k % chunk and k < max_iters:
            continue
        st = solver.stats[:8]
        if reduce_stats is not None:
            st = reduce_stats(st)
        host = st.cpu().numpy()
        solver.collect_timing()
        if keep_stats:
            log.append(host.copy())
        if log_every:
            print(f"iter {k}: active={int(host[0])} sumJ={host[1]:.6e} ran={int(host[3])}", flush=True)
        if host[0] == 0:
            break
    return log


def newton_loop(stepper, max_iters: int, reduce_stats=None, sync_every: int = 1, log_every: int = 0,
                keep_stats: bool = False) -> list:
    """Outer Newton loop shared by every stepper (HIP solver; the test oracle stepper).

    ``stepper.iteration()`` enqueues one iteration for all of its lanes and returns the 8-entry
    statistics tensor (STAT_FIELDS).  Every ``sync_every`` iterations the statistics are
    all-reduced across ranks (``reduce_stats``, SUM) and read on the host; the loop stops when no
    lane of any rank is active.  Returns the list of host statistics if ``keep_stats``."""
    log = []
    tail = int(getattr(stepper, "tail_lanes", 0) or 0)
    compact = getattr(stepper, "maybe_compact", None) if getattr(stepper, "lane_order_live", False) else None
    for k in range(int(max_iters)):
        st = stepper.iteration()
        if (k + 1) % sync_every == 0 or k + 1 == max_iters:
            local = st
            if reduce_stats is not None:
                st = reduce_stats(st)
            host = st.cpu().numpy() if isinstance(st, torch.Tensor) else np.asarray(st)
            collect = getattr(stepper, "collect_timing", None)
            if collect is not None:
                collect()
            if keep_stats:
                log.append(host.copy())
            if getattr(stepper, "timeline", None) is not None:   # diagnostics: (iterations, active, host time)
                stepper.timeline.append((k + 1, int(host[0]), time.perf_counter()))
            if log_every and (k % log_every == 0):
                print(f"iter {k}: active={int(host[0])} sumJ={host[1]:.6e} ran={int(host[3])} "
                      f"retry={int(host[4])}", flush=True)
            if host[0] == 0:
                break
            if host[4] > 0:   # lanes rejected trial 1: from now on the post-trial search records its candidates
                ensure = getattr(stepper, "ensure_cand_scratch", None)
                if ensure is not None:
                    ensure()
            # the straggler tail: decided on the (all-reduced) global active count, so every rank switches at the
            # same iteration and pairs up the same collectives afterwards; with a per-rank budget (tail_lanes_rank)
            # also on the largest rank's own count, all-reduced (MAX) by every rank at the same iteration (they all
            # see the same global count)
            if tail and host[0] <= tail and k + 1 < max_iters and _tail_rank_ok(stepper, host, local, reduce_stats):
                log += tail_loop(stepper, k + 1, int(max_iters), reduce_stats, log_every, keep_stats)
                break
            if compact is not None and k + 1 < max_iters:   # rank-local: no collective depends on it
                compact(int(local[0].item()) if reduce_stats is not None else int(host[0]))
    return log


def _tail_rank_ok(stepper, host, local, reduce_stats) -> bool:
    """The per-rank part of the straggler-tail switch: the largest rank's active count within ``tail_lanes_rank``
    (None: no per-rank budget).  Sharded, the maximum is one MAX all-reduce (``reduce_stats.max_of``) that every rank
    issues at the same iteration; with a reducer that has no ``max_of`` the budget is not applied (a warning)."""
    cap = getattr(stepper, "tail_lanes_rank", None)
    if cap is None:
        return True
    if reduce_stats is None:
        return host[0] <= cap
    max_of = getattr(reduce_stats, "max_of", None)
    if max_of is None:
        # a caller-supplied reducer without a MAX: the per-rank budget cannot be checked without a collective the
        # other ranks would not pair, so the global threshold alone decides (comparing the global count with the
        # per-rank cap would delay the tail until the whole job fits one rank's budget)
        if not getattr(stepper, "_warned_no_max_of", False):
            import warnings
            warnings.warn("reduce_stats has no max_of: the straggler tail's per-rank budget is not applied")
            stepper._warned_no_max_of = True
        return True
    n = float(local[0].item()) if isinstance(local, torch.Tensor) else float(np.asarray(local)[0])
    return max_of(n) <= cap


def tail_loop(solver, k: int, max_iters: int, reduce_stats, log_every: int, keep_stats: bool) -> list:
    """The rest of a serial / pipelined solve on the straggler-tail kernel, ``tail_chunk`` iterations per launch
    (a lane stops inside a launch when it finishes; the launch ends with its last lane); the statistics are
    all-reduced and read after each launch, and the loop stops when no lane of any rank is active."""
    log = []
    k_switch = k
    its0 = int(solver.n_iter[:solver.B].sum().item())
    solver._its_tail_start = its0
    while k < max_iters:
        k1 = min(max_iters, k + solver.tail_chunk)
        st = solver.tail_run(k, k1)
        k = k1
        if reduce_stats is not None:
            st = reduce_stats(st)
        host = st.cpu().numpy()
        solver.collect_timing()
        if keep_stats:
            log.append(host.copy())
        if getattr(solver, "timeline", None) is not None:
            solver.timeline.append((k, int(host[0]), time.perf_counter()))
        if log_every:
            print(f"tail iter {k}: active={int(host[0])} sumJ={host[1]:.6e}", flush=True)
        if host[0] == 0:
            break
    solver.tail_lane_its = int(solver.n_iter[:solver.B].sum().item()) - its0
    # a launch runs up to tail_chunk iterations but ends with its last lane: report the last iteration a lane ran,
    # not the end of the chunk.  Sharded (reduce_stats): the chunk end, identical on every rank, as the lock-step loop
    # reports its global count (a rank-local maximum would differ between ranks)
    if reduce_stats is None and solver.B:
        solver.k = max(k_switch, min(solver.k, int(solver.n_iter[:solver.B].max().item())))
    solver.tail_from, solver.tail_iters = k_switch, solver.k - k_switch
    return log


def newton_solve_batch(x0, x_ref, u_ref, max_iters, tol=1e-6, beta=0.7, c=0.5, gamma_0=1.0,
                       max_ls=MAX_LINE_SEARCH_ITERS, engine: AcrobotEngine | None = None, hist_len=0,
                       reduce_stats=None, pipeline: bool | None = None,
                       persistent: bool | None = None, capture_lanes=None) -> SolveResult:
    """Batched newton_Algorithm: x0 (B,4) -> SolveResult (device tensors)."""
    eng = engine or AcrobotEngine()
    x0 = eng.t(x0).reshape(-1, 4)
    solver = BatchedNewtonSolver(eng, x_ref, u_ref, x0.shape[0], tol=tol, beta=beta, c=c, gamma_0=gamma_0,
                                 max_ls=max_ls, hist_len=hist_len, pipeline=pipeline, persistent=persistent,
                                 capture_lanes=capture_lanes)
    return solver.solve(x0, max_iters, reduce_stats=reduce_stats)
