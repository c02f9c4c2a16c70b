#!/usr/bin/env python3
"""Benchmark: batched acrobot Newton/Armijo swing-up on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B_PER_GPU]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher (WORLD_SIZE unset) and N > 1, bench.py starts its N ranks itself: the parent makes no HIP
call, spawns N child processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, and exits with the first
non-zero child status.  Under a launcher WORLD_SIZE must equal --gpus, or the run exits with status 2.

One *step* = one complete batched solve (newton_Algorithm semantics per lane, task-2 settings:
tol 1e-4, gamma_0 0.1, beta 0.7, c 0.5, <= 20 Armijo trials, max_iters 5000) of this rank's shard
of synthetic lanes, from u = 0 to every lane converged / failed, with inputs resident in HBM.
Workload (N=1): BASELINE cfg 3 -- 262,144 lanes per GPU, x0 = [th1, th2, 0, 0], th ~ U(-0.5,0.5)
(numpy default_rng(0)), lane 0 = 0 (the golden lane), T = 500 stages, fp64.  Weak scaling: every GPU
owns 262,144 lanes; ranks exchange one 64-byte all-reduce per host sync of the statistics.

value = lane-iterations executed by all ranks / max-over-ranks wall time  ("Newton iterations/s";
states/s = value * T).  Prints ONE JSON line on rank 0.  Secondary legs timed in the same process and
reported inside that line (--extra-legs): "strong_scaling_cfg4" (BASELINE cfg 4: 1,048,576 lanes
strong-scaled over the N ranks) and, at N = 1, "general_path" (the same workload on the general kernels that
stream the tau1 planes), "cfg2" (BASELINE cfg 2: 4,096 lanes) and "mpc_cfg5" (BASELINE cfg 5).  --workload cfg4
makes cfg 4 the main line; --workload mpc makes cfg 5 the main line (with its CPU baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "swing-up Newton iterations/sec (batch×T states/s) at 1/2/4/8 MI355X"
CFG4_LANES = 1048576           # BASELINE cfg 4: global lanes sharded over 8 GPUs
CFG2_LANES = 4096              # BASELINE cfg 2: one GPU
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector peak (datasheet)


def algorithmic_bytes(N: int, u0_zero: bool = True) -> dict:
    """Compulsory HBM bytes per lane for one pass of each solver kernel (fp64), see DESIGN.md section 4.

    backward sweep : read x (4N) + u (2T);         write K row 1 (4T) + cg (T)
    Armijo trial   : read K row 1 (4T) + cg (T) + u0 (T) + x_0 (4);  write x_new (4N) + u_new (2T)
    (cg = (u1 - K1 x) + gamma0 sigma1; sigma1 itself is not streamed -- the rare lanes that backtrack re-run
    their sweep for it, which the per-launch count below does not include.)
    u0_zero (u_ref[:,0] == 0, GYM_FLAG_U0_ZERO): the tau1 plane is neither read nor written (-T on
    the sweep's reads, -T / -T on the trial's reads / writes).
    A Newton iteration of one lane is one sweep + one trial (no backtracking): 92,096 B at N = 501,
    80,096 B with u0_zero.  (SURVEY.md 8(d)'s 152,096 B is the reference's data flow: K stored 2x4,
    sigma stored 2-wide and the trial re-reading x and u.)
    """
    T = N - 1
    z = T if u0_zero else 0
    bwd = 8 * (4 * N + 2 * T - z + 4 * T + T)
    trial = 8 * (4 * T + T + (T - z) + 4 + 4 * N + 2 * T - z)
    return {"backward": bwd, "trial": trial, "iteration": bwd + trial,
            "survey_per_iteration": 8 * ((4 * N + 2 * T) + 10 * T + (2 * (4 * N + 2 * T) + 10 * T))}


def load_refs():
    d = np.load(os.path.join(ROOT, "gymnast_optimalcontrol_amd", "data", "fully_actuated_trajectory.npz"))
    u_ref = np.zeros(d["u"].shape)
    u_ref[:, 1] = d["u"][:, 1]
    return d["x"], 2.0 * u_ref          # get_fully_actuated_ref (trajectory_generation.py:511-518)


def make_x0(total: int, seed: int = 0, spread: float = 0.5) -> np.ndarray:
    """x0 = [th1, th2, 0, 0], th ~ U(-spread, spread) from default_rng(seed) (spread 1.5 is its stress
    variant); lane 0 = 0."""
    x0 = np.zeros((total, 4))
    x0[:, :2] = np.random.default_rng(seed).uniform(-spread, spread, (total, 2))
    x0[0] = 0.0                          # golden lane (main.task_2, main.py:55)
    return x0


def cpu_baseline(x0, x_ref, u_ref, lanes: int, max_iters: int):
    """The plain-C oracle (OpenMP over lanes) on a bounded sample of the same workload."""
    from oracle import c_oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    os.environ["OMP_NUM_THREADS"] = str(threads)
    c_oracle.lib()
    t0 = time.perf_counter()
    r = c_oracle.newton_solve(x0[:lanes], x_ref, u_ref, max_iters=max_iters, tol=1e-4, gamma_0=0.1)
    dt = time.perf_counter() - t0
    its = int(r["n_iter"].sum())
    return {"value": its / dt, "unit": "Newton iterations/s", "cores": threads, "kind": "port",
            "sample": f"first {lanes} lanes of the bench workload solved to convergence ({its} lane-iterations, "
                      f"{dt:.1f} s) by oracle/acrobot_oracle.c (fp64, OpenMP {threads} threads)",
            "seconds": dt, "lane_iterations": its}


def numpy_baseline(x0, x_ref, u_ref, lanes: int, iters: int):
    """The NumPy restatement (oracle/acrobot_np.py: the reference's dense algorithm vectorised over lanes) on a
    bounded sample: the first ``lanes`` lanes, ``iters`` Newton iterations from u = 0."""
    from oracle import acrobot_np as an
    an._model(1)                                   # sympy model build: setup, not timed
    t0 = time.perf_counter()
    r = an.newton_solve(x0[:lanes], x_ref, u_ref, iters, tol=1e-4, gamma_0=0.1)
    dt = time.perf_counter() - t0
    its = int(np.asarray(r["n_iter"]).sum())
    return {"value": its / dt, "unit": "Newton iterations/s", "cores": 1, "kind": "port",
            "sample": f"first {lanes} lanes of the bench workload, {iters} Newton iterations from u = 0 "
                      f"({its} lane-iterations, {dt:.1f} s), oracle/acrobot_np.py (numpy, lanes vectorised, "
                      f"one Python thread)", "seconds": dt, "lane_iterations": its}


def run_mpc(a):
    """--workload mpc: the cfg 5 line (mpc_line) printed as the bench's JSON line."""
    print(json.dumps(mpc_line(a, a.batch, a.steps, a.warmup, a.cpu_lanes)), flush=True)


def mpc_line(a, B, steps, warmup, cpu_lanes):
    """BASELINE cfg 5: batched receding-horizon MPC (trajectory_tracking.py:8-69 / main.py task_4).

    One step = the whole tracking run of B disturbed initial states: the exact per-control-step QP
    solutions of all 500 windows (gym_mpc_gains; horizon a.horizon) plus the batched closed-loop RK4
    simulation under them (gym_track_rollout) and the lane-major results.  value = lanes x 500 control
    steps / seconds per step.  cpu_lanes = 0: no CPU baseline (the parity sample is then 256 lanes)."""
    import torch
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine  # noqa: F401
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))   # acrobot_optimal_trajectory
    x_ref, u_ref = g["x"], g["u"]
    N = x_ref.shape[0]
    x0 = x_ref[0] + np.random.default_rng(0).uniform(-0.1, 0.1, (B, 4))
    x0[0] = x_ref[0] + 0.1                                      # main.task_4's disturbance
    eng = tt._eng()
    x0d, xrd, urd = eng.t(x0), eng.t(x_ref), eng.t(u_ref)
    for _ in range(warmup):
        tt.solve_mpc_tracking_batch(x0d, xrd, urd, a.horizon)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        x, u, K0 = tt.solve_mpc_tracking_batch(x0d, xrd, urd, a.horizon)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ctrl_steps = B * (N - 1)
    # per-kernel times (HIP events on the engine's stream = torch's current stream).  The stream is kept busy
    # (torch.cuda._sleep) while the host enqueues the events and the two launches, so each interval is the kernel's
    # execution, not the host's Python time between two records on an idle GPU (round 3's line included it:
    # 0.111 ms for a 77 us gains kernel)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    torch.cuda._sleep(2_000_000)
    ev[0].record()
    K0, QT = tt.mpc_gains(xrd, urd, a.horizon)
    ev[1].record()
    xs, us = eng.track_rollout(x0d, xrd, urd, K0)
    ev[2].record()
    torch.cuda.synchronize()
    t_gain, t_roll = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    roll_bytes = B * (N * 32 + (N - 1) * 16 + 32)                 # x (pairs) + u (planes) written, x0 read
    out = {"metric": "receding-horizon MPC control steps/s (BASELINE cfg 5)", "value": ctrl_steps / dt,
           "unit": "control steps/s", "n_gpus": 1, "steps": steps, "warmup": warmup, "ms_per_step": 1e3 * dt,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"cfg5: {B} disturbed initial states (x_ref[0] + U(-0.1,0.1)^4) x 500 control "
                                  f"steps, horizon {a.horizon}, exact QP solution per step, RK4 plant",
                      "lanes": B, "horizon": a.horizon, "control_steps": N - 1},
           "kernels": {"mpc_gains_ms": t_gain, "track_rollout_ms": t_roll},
           "roofline": {"bound": "hbm", "kernel": "track_rollout", "achieved": roll_bytes / (t_roll * 1e-3) / 1e9,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": roll_bytes / (t_roll * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "kernel_name": "k_track_rollout_pair", "algorithmic_bytes_per_launch": roll_bytes,
                        "note": "latency-bound: B/32 wavefronts (a lane pair per trajectory) each run 500 dependent "
                                "RK4 steps; the bytes are the trajectories written and x0 read"}}
    traffic, ratio, _, src = pmc_traffic("track_rollout")
    if traffic is not None and B == 8192:
        out["roofline"].update({"traffic": traffic, "traffic_over_algorithmic": ratio, "traffic_source": src})
    from oracle import tracking_np as tr
    lanes = min(B, cpu_lanes or 256)
    t1 = time.perf_counter()
    xo, uo, K0o = tr.solve_mpc_tracking(x0[:lanes], x_ref, u_ref, a.horizon)
    tc = time.perf_counter() - t1
    if cpu_lanes:
        out["cpu_baseline"] = {"value": lanes * (N - 1) / tc, "unit": "control steps/s", "cores": 1, "kind": "port",
                               "sample": f"first {lanes} lanes, numpy restatement (oracle/tracking_np.py) with the "
                                         f"window QPs solved by the same Riccati recursion", "seconds": tc}
    xg = x[:lanes].cpu().numpy()
    out["parity"] = {"rel_l2_x_vs_oracle": float(np.linalg.norm(xg - xo) / np.linalg.norm(xo)),
                     "rel_l2_K0_vs_oracle": float(np.linalg.norm(K0.cpu().numpy() - K0o) / np.linalg.norm(K0o)),
                     "oracle_lanes": lanes, "lane0_final_state": x[0, -1].cpu().numpy().tolist(), "tolerance": 1e-9}
    return out


def process_warmup(eng, x_ref, u_ref) -> float:
    """A fresh process's one-time GPU costs (kernel code objects and torch operators loaded on first use, clocks
    ramping from idle: ~0.6 s before the first solve's fourth iteration, tools/first_solve.py) paid on a small solve
    of another shape (2,048 lanes, pipelined, 8 iterations), untimed, so that the main leg's first solve measures what
    a call of the batched solver costs in a running process.  Returns its wall time (reported as cold_start_s)."""
    import torch
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = BatchedNewtonSolver(eng, x_ref, u_ref, 2048, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, pipeline=True)
    s.solve(make_x0(2048), 8, sync_every=4)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def cfg1_line(repeats: int = 2) -> dict:
    """BASELINE cfg 1 through the drop-in: main.task_2's own call (/root/reference/main.py:52-71),
    tg.newton_Algorithm(np.zeros(4), x_ref, u_ref, max_iters=5000, tol=1e-4, gamma_0=0.1, plot_armijo_iters=7) on
    the reference-named module (one lane; the reference's history -- every iterate and sigma -- copied to the host
    after each iteration, as the reference keeps it), timed end to end after one untimed warm-up call.  The Armijo
    report figures of the first iterations are drawn when matplotlib is importable (Agg); their time is reported
    apart, since the reference's 78.3 s was measured with the plotting function stubbed."""
    os.environ.setdefault("MPLBACKEND", "Agg")
    from gymnast_optimalcontrol_amd import trajectory_generation as tg
    x_ref, u_ref, _ = tg.get_fully_actuated_ref(os.path.join(ROOT, "gymnast_optimalcontrol_amd", "data",
                                                              "fully_actuated_trajectory.npz"))
    plot_s = [0.0]
    orig = tg.plot_armijo_line_search

    def timed_plot(*args, **kw):
        t = time.perf_counter()
        try:
            return orig(*args, **kw)
        finally:
            plot_s[0] += time.perf_counter() - t
    tg.plot_armijo_line_search = timed_plot
    try:
        tg.newton_Algorithm(np.zeros(4), x_ref, u_ref, max_iters=3, tol=1e-4, gamma_0=0.1, plot_armijo_iters=7,
                            verbose=False)
        runs = []
        for _ in range(repeats):
            plot_s[0] = 0.0
            t0 = time.perf_counter()
            x, u, K, sigma, hist = tg.newton_Algorithm(np.zeros(4), x_ref, u_ref, max_iters=5000, tol=1e-4,
                                                       gamma_0=0.1, plot_armijo_iters=7, verbose=False)
            runs.append((time.perf_counter() - t0, plot_s[0]))
    finally:
        tg.plot_armijo_line_search = orig
        try:
            import matplotlib.pyplot as plt
            plt.close("all")
        except ImportError:
            pass
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))
    its = len(hist["sigma_norm"])
    sec, psec = min(runs, key=lambda r: r[0])
    return {"seconds": sec, "plot_seconds": psec, "seconds_without_plots": sec - psec, "iterations": its,
            "iterations_per_s": its / sec, "repeats": [r[0] for r in runs],
            "parity": {"rel_l2_x": float(np.linalg.norm(x - g["x"]) / np.linalg.norm(g["x"])),
                       "rel_l2_u": float(np.linalg.norm(u - g["u"]) / np.linalg.norm(g["u"])), "tolerance": 1e-8},
            "reference_seconds": 78.3, "reference_iterations": 393,
            "speedup_vs_reference_without_plots": 78.3 / (sec - psec),
            "note": "main.task_2's call on the drop-in module (one lane, host history every iteration); reference: "
                    "the same call on one core of the survey container with its plotting stubbed (SURVEY 3.1), not "
                    "re-measured on this box"}


class NewtonLeg:
    """One timed configuration of the batched solver on this rank: ``total`` global lanes of the bench workload,
    this rank's contiguous shard, the schedule chosen on the largest shard (identical on every rank)."""

    def __init__(self, a, gd, eng, x_ref, u_ref, total: int, timing: bool, u0_zero=None, spread=None, shard=None,
                 **solver_kw):
        """``shard`` = (r, W): this process solves rank r's shard of a W-rank job alone (a one-GPU rehearsal of one
        rank's workload: its lanes, and the schedule every rank of that job picks)."""
        from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
        self.rank, self.world = gd.rank_world()
        self.total = int(total)
        self.x0_all = make_x0(self.total, spread=a.spread if spread is None else spread)
        srank, sworld = shard if shard is not None else (self.rank, self.world)
        lo, hi = gd.shard_range(self.total, srank, sworld)
        sched = {"auto": None, "serial": False, "pipelined": True, "persistent": None}[a.schedule]
        import torch
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.solver = BatchedNewtonSolver(
            eng, x_ref, u_ref, hi - lo, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20, pipeline=sched,
            persistent={"auto": None, "persistent": True}.get(a.schedule, False), chunk=a.chunk,
            schedule_lanes=gd.schedule_lanes(self.total, sworld), u0_zero=u0_zero,
            split_waves=a.split_waves == "on", tail_lanes=a.tail_lanes, world_size=self.world,
            compact=None if a.compact == "auto" else a.compact == "on", **solver_kw)
        torch.cuda.synchronize()
        # construction: buffers (and, with placement selection, the further stream sets the first solve probes; a set
        # pooled by an earlier solver of this shape is taken instead)
        self.setup_s = time.perf_counter() - t0
        if timing:
            self.solver.enable_timing()
        self.x0_dev = eng.t(self.x0_all[lo:hi])          # inputs resident in HBM before the timed region
        self.first_solve = None
        base = gd.make_reduce_stats()
        self.reduce = gd.TimedReduce(base) if base is not None else None
        self.a, self.gd = a, gd

    def run(self, steps: int, warmup: int, box=None):
        import torch
        a, gd, solver = self.a, self.gd, self.solver
        for w in range(warmup):
            r = solver.solve(self.x0_dev, a.max_iters, reduce_stats=self.reduce, sync_every=a.sync_every)
            if w == 0:    # the first solve of this solver (placement selection, if any, runs inside it)
                self.first_solve = (r.seconds, r.lane_iterations)
            r = None
        solver.reset_timing()
        if self.reduce is not None:
            self.reduce.reset()
        smi0 = box.smi() if box is not None else None       # outside the timed region (an amd-smi call, ~0.3 s)
        gd.barrier()
        torch.cuda.synchronize()
        if box is not None:
            box.mark()
        t0 = time.perf_counter()
        lane_its, rolls, res, tail_its, compactions, lowocc_its = 0, 0, None, 0, 0, 0
        tail_iters_max = 0
        for _ in range(steps):
            res = None                                   # free the previous solve's outputs first
            res = solver.solve(self.x0_dev, a.max_iters, reduce_stats=self.reduce, sync_every=a.sync_every)
            lane_its += res.lane_iterations
            if self.first_solve is None:
                self.first_solve = (res.seconds, res.lane_iterations)
            rolls += int(res.n_rollouts.sum().item())   # after the solve's own final synchronisation
            tail_its += res.tail_lane_iterations
            tail_iters_max = max(tail_iters_max, res.tail_iterations)
            compactions += res.compactions
            lowocc_its += res.lowocc_lane_iterations
        torch.cuda.synchronize()
        local = time.perf_counter() - t0       # this rank's own time, before waiting for the others
        win = box.window() if box is not None else None    # sysfs samples only: no delay
        gd.barrier()
        elapsed = gd.max_over_ranks(time.perf_counter() - t0)
        self.box = box.summary(win, smi0, box.smi()) if box is not None else None
        red = self.reduce
        self.rank_records = gd.gather_floats([local, lane_its, red.reduce_s if red else 0.0,
                                              red.readback_s if red else 0.0, red.calls if red else 0,
                                              res.iterations if res is not None else 0])
        self.res, self.lane_its, self.steps, self.tail_lane_its = res, lane_its, steps, tail_its
        self.tail_iters_max = tail_iters_max
        self.compactions = compactions
        self.lowocc_lane_its = lowocc_its
        self.elapsed = elapsed
        self.lane_its_all = int(gd.sum_over_ranks(lane_its))
        self.rollouts_all = int(gd.sum_over_ranks(rolls))
        self.value = self.lane_its_all / elapsed
        if self.box is not None and self.box.get("energy_j"):
            self.box["uj_per_lane_iteration"] = round(1e6 * self.box["energy_j"] / max(lane_its, 1), 3)
        return self

    def kernel_report(self, N: int):
        """Per-kernel HIP-event times (this rank) and the dominant kernel's algorithmic GB/s."""
        solver = self.solver
        kt = solver.kernel_times()
        if not kt:
            return None, None
        ab = algorithmic_bytes(N, solver.u0_zero)
        kern = {}
        for kind, (ms, launches) in kt.items():
            if launches:
                kern[kind] = {"avg_ms": ms / launches, "launches": launches}
        lane_its = self.lane_its
        if solver.persistent:
            # persistent schedule: every lane-iteration (sweep + trial) runs inside the run launches
            dom = "run"
            per_launch = lane_its * ab["iteration"] / kern["run"]["launches"]
            kern["run"]["algorithmic_bytes_per_launch"] = per_launch
            kern["run"]["achieved_GBs"] = per_launch / (kern["run"]["avg_ms"] * 1e-3) / 1e9
            bytes_per_lane, unit_note = ab["iteration"], "sweep + trial of one lane-iteration"
        elif "phase_odd" in kern:
            # pipelined schedule: every lane-iteration = one sweep + one trial inside the phase launches (2 per
            # outer iteration + 1 per solve) -- up to the low-occupancy switch and the straggler tail, whose
            # lane-iterations are not in them
            dom = "phase"
            rec_ms = sum(kern[k]["avg_ms"] * kern[k]["launches"] for k in ("phase_odd", "phase_even") if k in kern)
            rec_n = sum(kern[k]["launches"] for k in ("phase_odd", "phase_even") if k in kern)
            total_launches = solver.launches["phase"]
            tail_its = self.tail_lane_its + self.lowocc_lane_its
            per_launch = (lane_its - tail_its) * ab["iteration"] / total_launches
            kern["phase"] = {"avg_ms": rec_ms / rec_n, "launches": total_launches, "recorded": rec_n,
                             "algorithmic_bytes_per_launch": per_launch}
            kern["phase"]["achieved_GBs"] = per_launch / (kern["phase"]["avg_ms"] * 1e-3) / 1e9
            bytes_per_lane, unit_note = ab["iteration"], "sweep + trial of one lane-iteration"
        else:
            for kind in ("backward", "trial"):
                if kind in kern:
                    per_launch = ((lane_its - self.tail_lane_its - self.lowocc_lane_its) * ab[kind] /
                                  kern[kind]["launches"])
                    kern[kind]["algorithmic_bytes_per_launch"] = per_launch
                    kern[kind]["achieved_GBs"] = per_launch / (kern[kind]["avg_ms"] * 1e-3) / 1e9
            dom = max(("backward", "trial"), key=lambda k: kern.get(k, {}).get("avg_ms", 0))
            bytes_per_lane, unit_note = ab[dom], f"one {dom} pass of one lane"
        ach = kern[dom]["achieved_GBs"]
        roof = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": ach / HBM_PEAK_GBS, "bytes_per_unit": bytes_per_lane, "unit_of_work": unit_note,
                "algorithmic_bytes_per_launch": kern[dom]["algorithmic_bytes_per_launch"],
                "u0_zero_streams_skipped": solver.u0_zero}
        return kern, roof

    def schedule(self) -> str:
        return self.res.schedule if self.res is not None else self.solver.schedule

    def setup_record(self) -> dict:
        """What a one-shot caller pays (the batched newton_Algorithm builds a solver per call): construction, and the
        first solve (placement selection included); one_shot_value = its lane-iterations over both, all ranks."""
        fs, fi = self.first_solve or (float("nan"), 0)
        setup = self.gd.max_over_ranks(self.setup_s)
        first = self.gd.max_over_ranks(fs)
        its = self.gd.sum_over_ranks(fi)
        rec = {"setup_s": setup, "first_solve_s": first, "one_shot_value": its / (setup + first),
               "steady_solve_s": self.elapsed / max(self.steps, 1)}
        if self.solver is not None and self.solver.placement:
            rec["placement"] = dict(self.solver.placement)
        return rec

    def free(self):
        import torch
        self.solver = self.res = self.x0_dev = None
        torch.cuda.empty_cache()


class BoxMonitor:
    """The box state of this rank's GPU during each timed leg (tools/box_state.py): SCLK / MCLK DPM levels, power
    against its cap, junction and memory temperatures (sysfs, sampled every 0.1 s on a background thread, mean / min /
    max over the leg's timed region), and from amd-smi's accumulated counters the share of the region spent under the
    power cap (PPT) or a thermal limit and the energy it used.  File reads and one amd-smi call outside each timed
    region; nothing touches the GPU."""

    KEYS = {"dpm_sclk_mhz": "sclk_mhz", "dpm_mclk_mhz": "mclk_mhz", "dpm_fclk_mhz": "fclk_mhz",
            "power_ppt_in_w": "power_w", "power_ppt_avg_w": "power_avg_w", "power_cap_w": "power_cap_w",
            "temp_junction_c": "temp_junction_c", "temp_hotspot_c": "temp_hotspot_c", "temp_mem_c": "temp_mem_c",
            "temp_edge_c": "temp_edge_c"}

    def __init__(self, device_index: int = 0, use_smi: bool = True):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import box_state
        self._bs = box_state
        self.use_smi = use_smi          # amd-smi's GPU matched by PCI address (tools/box_state.smi_index)
        self.s = box_state.Sampler(device_index, 0.1).start()

    def mark(self):
        self.s.mark()

    def window(self):
        return self.s.window()

    def smi(self):
        bdf = os.path.basename(self.s.dev) if self.s.dev else None
        return self._bs.smi_counters(20.0, bdf) if self.use_smi else {}

    def summary(self, win, smi0, smi1) -> dict:
        out = {self.KEYS[k]: v for k, v in win.items() if k in self.KEYS}
        if "power_cap_w" in out:
            out["power_cap_w"] = out["power_cap_w"][0]
        out.update(self._bs.smi_delta(smi0 or {}, smi1 or {}))
        out["samples"] = win.get("samples", 0)
        return out

    def stop(self):
        self.s.stop()


def stress_tail_record(leg, ks, T: int) -> dict:
    """The straggler tail of the stress leg and the bound it sets (SURVEY 8(d) stress variant).

    The tail runs every remaining lane's iterations in one workgroup per lane, so a tail launch lasts as long as its
    slowest lane: its seconds over the outer iterations it ran are one lane-iteration's latency on the critical path
    (a sweep pass and the Armijo trials, T stages each).  critical_path_s = the longest lane's iteration count x that
    latency: the solve time if every iteration of the batch's slowest lane ran at the tail's single-lane speed, i.e.
    the floor one lane running to max_iters sets with today's chains; frac_of_critical_path = critical_path_s / the
    measured seconds per solve (1 = the solve is that one lane's chain and nothing else)."""
    steps = max(leg.steps, 1)
    rec = {"launches_per_step": leg.solver.launches["tail"] / steps,
           "share_of_lane_iterations": leg.tail_lane_its / max(leg.lane_its, 1), "seconds_per_step": None}
    if not ks or "tail" not in ks or not leg.tail_iters_max:
        return rec
    tail_s = ks["tail"]["avg_ms"] * ks["tail"]["launches"] / 1e3 / steps
    lat = tail_s / leg.tail_iters_max
    n_max = int(leg.res.n_iter.max().item())
    solve_s = leg.elapsed / steps
    rec.update({"seconds_per_step": tail_s, "from_iteration": leg.res.tail_from_iteration,
                "outer_iterations_per_step": leg.tail_iters_max, "lane_iteration_latency_ms": 1e3 * lat,
                "max_lane_iterations": n_max, "critical_path_s": n_max * lat,
                "frac_of_critical_path": n_max * lat / solve_s,
                "share_of_solve": tail_s / solve_s})
    sclk = (leg.box or {}).get("sclk_mhz")
    if sclk:
        # cycles per stage of one tail lane-iteration (one sweep stage + one trial stage) at the leg's SCLK range
        rec["cycles_per_stage_at_sclk"] = {"mean": lat * sclk[0] * 1e6 / T, "max": lat * sclk[2] * 1e6 / T}
    return rec


def persistent_chain_record(leg, ks, T: int) -> dict:
    """The bound of a latency-bound persistent leg (BASELINE cfg 2): k_nt_run2 runs every lane's iterations back to
    back, so a launch lasts as long as its slowest lane's chain; the run kernel's seconds per solve over the longest
    lane's iteration count are one lane-iteration's latency (a sweep pass and a trial pass, T stages each) and, at the
    leg's SCLK, the cycles per stage of that chain.  share_of_solve = the run kernel's share of the
    measured seconds per solve (the rest: init, statistics, host synchronisation, results)."""
    steps = max(leg.steps, 1)
    if not ks or "run" not in ks or not ks["run"]["launches"]:
        return {}
    run_s = ks["run"]["avg_ms"] * ks["run"]["launches"] / 1e3 / steps
    n_max = int(leg.res.n_iter.max().item())
    lat = run_s / max(n_max, 1)
    rec = {"max_lane_iterations": n_max, "lane_iteration_latency_ms": 1e3 * lat, "run_seconds_per_step": run_s,
           "share_of_solve": run_s / (leg.elapsed / steps)}
    sclk = (leg.box or {}).get("sclk_mhz")
    if sclk:
        rec["cycles_per_stage_at_sclk"] = {"mean": lat * sclk[0] * 1e6 / T, "max": lat * sclk[2] * 1e6 / T}
    return rec


def outcome_record(res) -> dict:
    """Per-lane outcomes of a solve: statuses, iteration range, rollouts and the per-lane extra Armijo trials
    (rollouts beyond one per iteration) binned."""
    st = res.status.cpu().numpy()
    extra = (res.n_rollouts - res.n_iter).cpu().numpy()
    edges = [0, 1, 2, 4, 8, 16, 32, 1 << 30]
    return {"converged": int((st == 1).sum()), "ls_failed": int((st == 2).sum()), "max_iters": int((st == 3).sum()),
            "lane_iters_min_max": [int(res.n_iter.min().item()), int(res.n_iter.max().item())],
            "outer_iterations": int(res.iterations), "rollouts": int(res.n_rollouts.sum().item()),
            "lanes_that_backtracked": int((res.n_rollouts > res.n_iter).sum().item()),
            "extra_trials_histogram": {
                (f"{lo}" if hi == lo + 1 else f"{lo}-{hi - 1}" if hi < (1 << 30) else f">={lo}"):
                    int(((extra >= lo) & (extra < hi)).sum()) for lo, hi in zip(edges[:-1], edges[1:])}}


def pmc_traffic(dom: str):
    """The committed rocprofv3 PMC measurement of the dominant kernel (tools/profile.sh, parse_profiles.py)."""
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    traffic, ratio, valu, src = None, None, None, None
    if os.path.exists(tfile):
        try:
            d = json.load(open(tfile))
            t = d.get(dom, {})
            traffic, ratio = t.get("hbm_bytes_per_launch"), t.get("traffic_over_algorithmic")
            src = d.get("source", "profiles/pmc_traffic.json (rocprofv3 PMC)")
            if "valu_busy_upper_est" in t:
                valu = {"busy_upper_est": t["valu_busy_upper_est"],
                        "wave_instructions_per_launch": t["sq_insts_valu_per_launch"],
                        "note": "SQ_INSTS_VALU x 4 cycles (fp64 wave64 on SIMD-32) / SIMD-cycles of the launch, "
                                "rocprofv3 PMC (profiles/pmc_traffic.json)"}
        except Exception:
            traffic = None
    return traffic, ratio, valu, src


def spawn_ranks(n: int) -> int:
    """Run this script as ``n`` ranks on one node (the torch.distributed.run equivalent), from a parent that has
    made no HIP call: children are started with fork + exec of a fresh interpreter.  Returns the exit status
    (0, or the first failing rank's; the other ranks are then terminated by PID)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   GYM_BENCH_LAUNCHER="bench.py (spawned ranks)")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {procs.index(p)} exited with status {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None,
                    help="lanes per GPU (weak scaling); default 262144 (newton, cfg 3) or 8192 (mpc, cfg 5)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: this many lanes in total, sharded over the ranks (cfg4: 1048576)")
    ap.add_argument("--max-iters", type=int, default=5000)
    ap.add_argument("--cpu-lanes", type=int, default=4096,
                    help="lanes of the bounded C-oracle CPU-baseline sample (about 10 s on 16 host cores)")
    ap.add_argument("--numpy-lanes", type=int, default=256,
                    help="lanes of the bounded NumPy-restatement CPU-baseline sample (numpy-iters iterations)")
    ap.add_argument("--numpy-iters", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--no-box", action="store_true", help="skip the box-state record (sysfs clocks / power / "
                                                            "temperatures, amd-smi throttle and energy counters)")
    ap.add_argument("--sync-every", type=int, default=4,
                    help="outer iterations between host reads of the (all-reduced) statistics; iterations "
                         "enqueued after every lane has finished are no-ops")
    ap.add_argument("--workload", choices=("newton", "cfg4", "mpc", "stress"), default="newton",
                    help="newton: the north-star metric (cfg 3 per GPU, weak scaling); cfg4: 1,048,576 lanes "
                         "strong-scaled over the ranks; mpc: BASELINE cfg 5; stress: the cfg 3 batch with "
                         "th ~ U(+-1.5) (SURVEY 8(d)'s stress variant: backtracking and Armijo failures)")
    ap.add_argument("--extra-legs", default="cfg4,cfg4share,general,cfg2,mpc,stress,cfg1",
                    help="comma list of secondary timed legs reported inside the same JSON line (newton "
                         "workload): cfg4 = 1,048,576 lanes strong-scaled over the ranks; general = the same "
                         "workload on the general (tau1-streaming) kernels, N=1 only; cfg2 = BASELINE cfg 2 "
                         "(4,096 lanes, N=1 only); mpc = BASELINE cfg 5 (N=1 only); stress = SURVEY 8(d)'s "
                         "stress variant (th ~ U(+-1.5), N=1 only); cfg4share = one rank's share of cfg 4 at N = 8 "
                         "(131,072 lanes, N=1 only); cfg1 = main.task_2's call through the drop-in module (N=1 "
                         "only); '' for none")
    ap.add_argument("--extra-steps", type=int, default=2, help="timed solves of each extra leg (1 warmup)")
    ap.add_argument("--horizon", type=int, default=50, help="MPC prediction horizon T_pred (cfg 5: 50)")
    ap.add_argument("--schedule", choices=("auto", "serial", "pipelined", "persistent"), default="auto",
                    help="solver schedule (auto: the solver's choice for the batch size)")
    ap.add_argument("--chunk", type=int, default=128,
                    help="persistent schedule: iterations per launch (0: all of max_iters in one)")
    ap.add_argument("--tail-lanes", type=int, default=None,
                    help="straggler tail: hand the last lanes to gym_newton_tail once at most this many are active "
                         "(default: the solver's, 4 per CU; 0 = off)")
    ap.add_argument("--compact", choices=("auto", "on", "off"), default="auto",
                    help="lane compaction of the serial / pipelined loop (BatchedNewtonSolver.maybe_compact; auto: "
                         "the solver's default, on with the automatic schedule)")
    ap.add_argument("--split-waves", choices=("on", "off"), default="on",
                    help="persistent schedule: two wavefronts per 64 lanes (k_nt_run2, default) or one (k_nt_run)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rendezvous check only (no GPU work): every rank joins the process group and "
                         "rank 0 prints the ranks' view of it as one JSON line")
    ap.add_argument("--u0-zero", choices=("auto", "off"), default="auto",
                    help="off: force the general kernels (tau1 planes streamed) for the main leg")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))         # before any torch / HIP call in this process
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={env_world} ranks", file=sys.stderr)
        sys.exit(2)
    if a.batch is None:
        a.batch = 8192 if a.workload == "mpc" else 262144
    if a.workload == "mpc":
        if a.gpus > 1:
            print("bench.py: --workload mpc runs on one GPU (--gpus 1)", file=sys.stderr)
            sys.exit(2)
        return run_mpc(a)
    if a.workload == "cfg4" and a.global_batch is None:
        a.global_batch = CFG4_LANES
    a.spread = 1.5 if a.workload == "stress" else 0.5

    import torch
    from gymnast_optimalcontrol_amd import distributed as gd
    rank, local_rank, world = gd.init_process_group()
    if gd.rank_world()[1] != world or world != a.gpus:
        print(f"bench.py: process group holds {gd.rank_world()[1]} ranks, expected {a.gpus}", file=sys.stderr)
        sys.exit(2)
    if a.dry_run:
        seen = [rank, world, os.getpid()]
        backend = gd.backend_name()
        if world > 1:
            import torch.distributed as dist
            parts = [None] * world
            dist.all_gather_object(parts, seen)
            dist.destroy_process_group()
        else:
            parts = [seen]
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "dist": {"backend": backend,
                              "world_size": world, "launcher": os.environ.get("GYM_BENCH_LAUNCHER")},
                              "ranks": [p[0] for p in parts], "pids": [p[2] for p in parts]}), flush=True)
        return
    torch.cuda.set_device(gd.local_device_index(local_rank))
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine

    x_ref, u_ref = load_refs()
    N = x_ref.shape[0]
    T = N - 1
    strong = a.global_batch is not None
    total = a.global_batch if strong else a.batch * world
    eng = AcrobotEngine()
    cold_s = process_warmup(eng, x_ref, u_ref)
    box = None if a.no_box or rank != 0 else BoxMonitor(gd.local_device_index(local_rank))
    main_leg = NewtonLeg(a, gd, eng, x_ref, u_ref, total, not a.no_timing,
                         u0_zero=False if a.u0_zero == "off" else None).run(a.steps, a.warmup, box)
    res = main_leg.res
    value = main_leg.value

    # parity of the golden lane (rank 0 owns lane 0)
    parity = None
    if rank == 0:
        g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))
        x0l, u0l = res.x[0].cpu().numpy(), res.u[0].cpu().numpy()
        st = res.status.cpu().numpy()
        parity = {"lane0_rel_l2_x": float(np.linalg.norm(x0l - g["x"]) / np.linalg.norm(g["x"])),
                  "lane0_rel_l2_u": float(np.linalg.norm(u0l - g["u"]) / np.linalg.norm(g["u"])),
                  "lane0_iters": int(res.n_iter[0].item()), "tolerance": 1e-8,
                  "converged_frac": float((st == 1).mean()), "ls_failed": int((st == 2).sum()),
                  "outer_iterations": int(res.iterations),
                  "lane_iters_min_max": [int(res.n_iter.min().item()), int(res.n_iter.max().item())],
                  "rollouts": int(res.n_rollouts.sum().item()),
                  "lanes_that_backtracked": int((res.n_rollouts > res.n_iter).sum().item())}
        # per-lane extra Armijo trials over the solve (rollouts beyond one per iteration), binned
        extra = (res.n_rollouts - res.n_iter).cpu().numpy()
        edges = [0, 1, 2, 4, 8, 16, 32, 1 << 30]
        parity["extra_trials_histogram"] = {
            (f"{lo}" if hi == lo + 1 else f"{lo}-{hi - 1}" if hi < (1 << 30) else f">={lo}"): int(((extra >= lo) & (extra < hi)).sum())
            for lo, hi in zip(edges[:-1], edges[1:])}

    per_gpu = -(-total // world)
    if strong:
        label = (f"{'cfg4' if total == CFG4_LANES else 'custom'}: {total} randomised-theta0 acrobot swing-ups "
                 f"strong-scaled over {world} GPU(s) ({per_gpu} per GPU)")
    elif a.workload == "stress":
        label = (f"stress (SURVEY 8(d)): {a.batch} acrobot swing-ups per GPU, theta0 ~ U(+-1.5) (backtracking and "
                 f"Armijo failures)" + (f" x {world} GPUs (weak scaling)" if world > 1 else ""))
    else:
        label = (f"{ {4096: 'cfg2', 262144: 'cfg3'}.get(a.batch, 'custom') }: {a.batch} randomised-theta0 acrobot "
                 f"swing-ups per GPU" + (f" x {world} GPUs (weak scaling)" if world > 1 else ""))
    out = {"metric": METRIC, "value": value, "unit": "Newton iterations/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": 1e3 * main_leg.elapsed / a.steps, "higher_is_better": True,
           "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": label + f", T={T}, fp64, task-2 Newton/Armijo settings, solved to convergence",
                      "lanes_per_gpu": per_gpu, "global_lanes": total, "horizon_T": T,
                      "parallelism": f"lane-sharded x{world} (1 all-reduce of 8 fp64 stats per host sync)"},
           "states_per_s": value * T,
           "dist": {"backend": gd.backend_name(), "world_size": gd.rank_world()[1],
                    "launcher": os.environ.get("GYM_BENCH_LAUNCHER", "torch.distributed.run" if world > 1 else None)}}
    out["rollouts_per_s"] = main_leg.rollouts_all / main_leg.elapsed   # closed-loop Armijo rollouts, all ranks
    sv = main_leg.solver
    out["straggler_tail"] = {
        "lanes_threshold": sv.tail_lanes, "launches": sv.launches["tail"],
        "lane_iterations_per_step": main_leg.tail_lane_its // max(a.steps, 1),
        "share_of_lane_iterations": main_leg.tail_lane_its / max(main_leg.lane_its, 1),
        "note": "gym_newton_tail: once at most lanes_threshold lanes are active (all ranks), one workgroup per lane, "
                "every Armijo trial at once (bitwise the serial schedule, tests/test_gpu_tail.py)"}
    out["lane_compaction"] = {
        "enabled": bool(sv.compact_mode), "compactions_per_step": main_leg.compactions / max(a.steps, 1),
        "serial_from_iteration": sv.serial_switch_at,
        "lane_iterations_per_step": main_leg.lowocc_lane_its // max(a.steps, 1),
        "note": "once at most a quarter of the lanes stay active: the active lanes move to the front and the solve "
                "continues one iteration per launch of the persistent kernel with parallel Armijo retries "
                "(BatchedNewtonSolver.maybe_compact, GYM_FLAG_SIGMA_STREAM; bitwise invisible, tests/test_gpu_tail.py)"}

    kern, roof = main_leg.kernel_report(N)
    if kern and rank == 0:
        traffic, ratio, valu, src = pmc_traffic(roof["kernel"])
        if roof["kernel"] == "run" and ratio is not None:
            # the PMC pass profiles one 20-iteration launch; a bench launch runs up to `chunk` iterations
            traffic = ratio * roof["algorithmic_bytes_per_launch"]
            src = (src or "") + "; measured / algorithmic ratio of a 20-iteration launch, scaled to this launch"
        elif ratio is not None and roof.get("algorithmic_bytes_per_launch"):
            # the PMC passes profile launches with every lane active; this run's average launch carries fewer lanes
            # near the end of the solve, so its per-launch traffic is the measured ratio times its own bytes
            traffic = ratio * roof["algorithmic_bytes_per_launch"]
            src = (src or "") + "; measured / algorithmic ratio of full launches, times this run's bytes per launch"
        roof.update({"traffic": traffic, "traffic_over_algorithmic": ratio, "traffic_source": src,
                     "survey_bytes_per_iteration": algorithmic_bytes(N)["survey_per_iteration"], "fp64_valu": valu})
        # the ordering the contract prescribes: bound, achieved, peak, unit, frac, traffic first
        out["roofline"] = {k: roof[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")}
        out["roofline"].update({k: v for k, v in roof.items() if k not in out["roofline"]})
        out["kernels"] = kern
    out["schedule"] = main_leg.schedule()
    out["phase_kernel"] = sv.phase_kind()
    out["setup"] = dict(main_leg.setup_record(), cold_start_s=cold_s, note=(
        "setup_s: solver construction (buffers, and the extra stream sets of placement selection); first_solve_s: the "
        "first solve of the solver (warm-up; placement selection runs inside it: blocks of 12 iterations of that solve "
        "on each stream set, the live state copied between sets, the fastest kept); one_shot_value: its "
        "lane-iterations / (setup_s + first_solve_s), what one call of the batched newton_Algorithm achieves in a "
        "running process; steady_solve_s: a timed solve; cold_start_s: the process's one-time GPU start-up (kernel "
        "code objects, torch operators, clock ramp), paid before the main leg on a 2,048-lane solve (bench."
        "process_warmup).  placement.reused: the set came from the process's PlacementPool (DESIGN 6)"))
    if world > 1:
        # per-rank diagnostics of the main leg: a sub-linear scaling curve then says whether stragglers (spread of
        # the ranks' own elapsed times and lane-iterations), the statistics all-reduce or its read-back is the cause
        recs = main_leg.rank_records
        el = [r[0] for r in recs]
        out["dist"].update({
            "rank_elapsed_s": el, "rank_elapsed_min_max": [min(el), max(el)],
            "rank_lane_iterations": [int(r[1]) for r in recs],
            "rank_outer_iterations_last_step": [int(r[5]) for r in recs],
            "rank_reduce_host_s": [r[2] for r in recs], "rank_readback_host_s": [r[3] for r in recs],
            "allreduce_calls_per_step": int(recs[0][4]) // max(a.steps, 1),
            "allreduce_8xf64_us": gd.allreduce_latency_us(),
            "note": "rank_elapsed_s: each rank's own timed region before the closing barrier (max = ms_per_step x "
                    "steps); rank_reduce_host_s: host time inside the statistics all-reduce calls; "
                    "rank_readback_host_s: host time reading the reduced statistics back (includes waiting for the "
                    "queued iterations); allreduce_8xf64_us: one statistics all-reduce, measured after the run"})
    if parity is not None:
        out["parity"] = parity
    res = sv = None            # the main solver goes with main_leg.free() (its stream set back to the pool)
    main_leg.free()

    # secondary legs (same process, same JSON line)
    legs = [s for s in a.extra_legs.split(",") if s] if a.workload == "newton" else []
    box_legs = {"main": main_leg.box}
    if "cfg4" in legs and not strong:
        leg = NewtonLeg(a, gd, eng, x_ref, u_ref, CFG4_LANES, not a.no_timing).run(a.extra_steps, 1, box)
        box_legs["strong_scaling_cfg4"] = leg.box
        k4, r4 = leg.kernel_report(N)
        out["strong_scaling_cfg4"] = {
            "value": leg.value, "unit": "Newton iterations/s", "scaling": "strong", "global_lanes": CFG4_LANES,
            "lanes_per_gpu": -(-CFG4_LANES // world), "n_gpus": world, "steps": a.extra_steps, "warmup": 1,
            "ms_per_step": 1e3 * leg.elapsed / a.extra_steps, "schedule": leg.schedule(),
            "lane_iterations_per_step": leg.lane_its_all // a.extra_steps,
            "roofline_frac": None if r4 is None else r4["frac"], "setup": leg.setup_record(),
            "note": "BASELINE cfg 4: 1,048,576 lanes sharded over the ranks (one all-reduce of 8 fp64 stats per "
                    "host sync); max-over-ranks wall time"}
        leg.free()
    if "general" in legs and world == 1 and a.u0_zero == "auto":
        leg = NewtonLeg(a, gd, eng, x_ref, u_ref, total, not a.no_timing, u0_zero=False).run(a.extra_steps, 1, box)
        box_legs["general_path"] = leg.box
        kg, rg = leg.kernel_report(N)
        out["general_path"] = {
            "value": leg.value, "unit": "Newton iterations/s", "steps": a.extra_steps, "warmup": 1,
            "ms_per_step": 1e3 * leg.elapsed / a.extra_steps, "schedule": leg.schedule(),
            "roofline": None if rg is None else {k: rg[k] for k in ("kernel", "achieved", "peak", "unit", "frac",
                                                                     "bytes_per_unit")},
            "specialisation_share": 1.0 - leg.value / value,
            "serial_from_iteration": leg.solver.serial_switch_at, "compactions_per_step": leg.compactions / a.extra_steps,
            "note": "the same workload on the general kernels (u0_zero off: the tau1 planes are read and written, "
                    "as for any reference with a live tau1 channel such as task 1); bitwise-identical results "
                    "(tests/test_gpu_parity.py::test_u0_zero_stream_skipping_is_bitwise_identical)"}
        leg.free()

    if "cfg2" in legs and world == 1 and (strong or a.batch != CFG2_LANES):
        leg = NewtonLeg(a, gd, eng, x_ref, u_ref, CFG2_LANES, not a.no_timing).run(a.extra_steps, 1, box)
        box_legs["cfg2"] = leg.box
        k2, r2 = leg.kernel_report(N)
        out["cfg2"] = {
            "value": leg.value, "unit": "Newton iterations/s", "lanes": CFG2_LANES, "steps": a.extra_steps,
            "warmup": 1, "ms_per_step": 1e3 * leg.elapsed / a.extra_steps, "schedule": leg.schedule(),
            "lane_iterations_per_step": leg.lane_its_all // a.extra_steps,
            "roofline": None if r2 is None else {k: r2[k] for k in ("kernel", "achieved", "peak", "unit", "frac")},
            "chain": persistent_chain_record(leg, k2, T),
            "note": "BASELINE cfg 2: 4,096 lanes on one GPU (64 wavefronts of lanes on 1,024 SIMDs: latency-bound, "
                    "the persistent schedule); --batch 4096 makes it the main line"}
        leg.free()
    if "stress" in legs and world == 1:
        # SURVEY 8(d)'s stress variant: the cfg 3 batch with th ~ U(+-1.5): backtracking, Armijo failures and a
        # straggler tail; the automatic schedule (pipelined -> lane compaction / low-occupancy regime -> tail)
        leg = NewtonLeg(a, gd, eng, x_ref, u_ref, total, not a.no_timing, spread=1.5).run(a.extra_steps, 1, box)
        box_legs["stress"] = leg.box
        ks, rs = leg.kernel_report(N)
        sv = leg.solver
        out["stress"] = {
            "value": leg.value, "unit": "Newton iterations/s", "lanes": total, "steps": a.extra_steps, "warmup": 1,
            "ms_per_step": 1e3 * leg.elapsed / a.extra_steps, "schedule": leg.schedule(),
            "lane_iterations_per_step": leg.lane_its_all // a.extra_steps,
            "rollouts_per_s": leg.rollouts_all / leg.elapsed,
            "roofline": None if rs is None else {k: rs[k] for k in ("kernel", "achieved", "peak", "unit", "frac")},
            "straggler_tail": stress_tail_record(leg, ks, T),
            "low_occupancy": {"from_iteration": sv.serial_switch_at, "compactions_per_step":
                              leg.compactions / a.extra_steps,
                              "share_of_lane_iterations": leg.lowocc_lane_its / max(leg.lane_its, 1)},
            "outcomes": outcome_record(leg.res), "setup": leg.setup_record(),
            "note": "SURVEY 8(d) stress variant: x0 = [th1, th2, 0, 0], th ~ U(+-1.5) (default_rng(0)), task-2 "
                    "settings, solved to convergence; the roofline is the phase kernel's over the lane-iterations "
                    "the phases ran (the tail and the low-occupancy regime are reported apart); decisions pinned "
                    "lane by lane against the C oracle (tests/test_gpu_stress.py)"}
        sv = None
        leg.free()
    if "cfg4share" in legs and world == 1:
        # the per-GPU workload of cfg 4 at N = 8 (rank 0's 131,072 lanes of the 1,048,576-lane batch, the schedule
        # every rank of that job picks: exactly the pipelined threshold, 512 lanes per CU) on this one GPU
        leg = NewtonLeg(a, gd, eng, x_ref, u_ref, CFG4_LANES, not a.no_timing, shard=(0, 8)).run(a.extra_steps, 1, box)
        box_legs["cfg4_rank_share"] = leg.box
        ksh, rsh = leg.kernel_report(N)
        out["cfg4_rank_share"] = {
            "value": leg.value, "unit": "Newton iterations/s", "lanes": leg.solver.B, "steps": a.extra_steps,
            "warmup": 1, "ms_per_step": 1e3 * leg.elapsed / a.extra_steps, "schedule": leg.schedule(),
            "phase_kernel": leg.solver.phase_kind(),
            "lane_iterations_per_step": leg.lane_its_all // a.extra_steps,
            "roofline": None if rsh is None else {k: rsh[k] for k in ("kernel", "achieved", "peak", "unit", "frac")},
            "setup": leg.setup_record(),
            "note": "one rank's share of BASELINE cfg 4 at N = 8 (lanes [0, 131072) of the cfg 4 batch), solved alone "
                    "on this GPU: the per-GPU workload and schedule of the 8-GPU run, without its all-reduces"}
        leg.free()
    if "cfg1" in legs and world == 1:
        out["cfg1_drop_in"] = cfg1_line()
    if "mpc" in legs and world == 1:
        m = mpc_line(a, 8192, max(a.extra_steps, 3), 1, 0)
        out["mpc_cfg5"] = {k: m[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "kernels",
                                             "roofline", "parity")}
        out["mpc_cfg5"]["note"] = "BASELINE cfg 5 (--workload mpc makes it the main line, with its CPU baseline)"

    if box is not None:
        box.stop()
        out["box"] = {"sysfs": box.s.dev, "legs": box_legs, "note": (
            "this GPU during each leg's timed region: DPM SCLK / MCLK / FCLK (MHz), power and its cap (W), junction and "
            "HBM temperatures (C) as [mean, min, max] of sysfs samples every 0.1 s; ppt_share / *_thermal_share: share "
            "of the region the SMU spent limited by the package power cap / a thermal limit (amd-smi throttle "
            "counters), energy_j and uj_per_lane_iteration from its energy counter.  A leg at power = cap with "
            "ppt_share near 1 runs at the SCLK the cap allows (DESIGN 6)")}
    if rank == 0 and world == 1 and not a.no_cpu:
        x0_all = make_x0(total, spread=a.spread)
        out["cpu_baseline"] = cpu_baseline(x0_all, x_ref, u_ref, a.cpu_lanes, a.max_iters)
        out["cpu_baseline"]["numpy"] = numpy_baseline(x0_all, x_ref, u_ref, a.numpy_lanes, a.numpy_iters)
        out["cpu_baseline"]["reference_python_single_core"] = {
            "value": 5.0, "unit": "Newton iterations/s", "note": "reference newton_Algorithm, 1 core, build "
            "container (Intel Xeon), SURVEY.md 3.1: 0.199 s/iteration; not a same-box measurement"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
