#!/usr/bin/env python3
"""Benchmark: batched acrobot Newton/Armijo swing-up on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B_PER_GPU]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One *step* = one complete batched solve (newton_Algorithm semantics per lane, task-2 settings:
tol 1e-4, gamma_0 0.1, beta 0.7, c 0.5, <= 20 Armijo trials, max_iters 5000) of this rank's shard
of synthetic lanes, from u = 0 to every lane converged / failed, with inputs resident in HBM.
Workload (N=1): BASELINE cfg 3 -- 262,144 lanes per GPU, x0 = [th1, th2, 0, 0], th ~ U(-0.5,0.5)
(numpy default_rng(0)), lane 0 = 0 (the golden lane), T = 500 stages, fp64.  Weak scaling: every GPU
owns 262,144 lanes; ranks exchange one 64-byte all-reduce per outer iteration.

value = lane-iterations executed by all ranks / max-over-ranks wall time  ("Newton iterations/s";
states/s = value * T).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "swing-up Newton iterations/sec (batch×T states/s) at 1/2/4/8 MI355X"
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


def make_x0(total: int, seed: int = 0) -> np.ndarray:
    x0 = np.zeros((total, 4))
    x0[:, :2] = np.random.default_rng(seed).uniform(-0.5, 0.5, (total, 2))
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


def run_mpc(a):
    """BASELINE cfg 5: batched receding-horizon MPC (trajectory_tracking.py:8-69 / main.py task_4).

    One step = the whole tracking run of a.batch disturbed initial states: the exact per-control-step QP
    solutions of all 500 windows (gym_tv_lqr_gains; horizon a.horizon) plus the batched closed-loop RK4
    simulation under them (gym_track_rollout) and the lane-major results.  value = lanes x 500 control
    steps / seconds per step."""
    import torch
    from gymnast_optimalcontrol_amd import trajectory_tracking as tt
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine  # noqa: F401
    g = np.load(os.path.join(ROOT, "tests", "golden", "task2_reference_output.npz"))   # acrobot_optimal_trajectory
    x_ref, u_ref = g["x"], g["u"]
    N = x_ref.shape[0]
    B = a.batch
    x0 = x_ref[0] + np.random.default_rng(0).uniform(-0.1, 0.1, (B, 4))
    x0[0] = x_ref[0] + 0.1                                      # main.task_4's disturbance
    eng = tt._eng()
    x0d, xrd, urd = eng.t(x0), eng.t(x_ref), eng.t(u_ref)
    for _ in range(a.warmup):
        tt.solve_mpc_tracking_batch(x0d, xrd, urd, a.horizon)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        x, u, K0 = tt.solve_mpc_tracking_batch(x0d, xrd, urd, a.horizon)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    steps = B * (N - 1)
    # per-kernel times (HIP events on the engine's stream = torch's current stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    K0, QT = tt.mpc_gains(xrd, urd, a.horizon)
    ev[1].record()
    xs, us = eng.track_rollout(x0d, xrd, urd, K0)
    ev[2].record()
    torch.cuda.synchronize()
    t_gain, t_roll = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    roll_bytes = B * (N * 32 + (N - 1) * 16 + 32)                 # x (pairs) + u (planes) written, x0 read
    out = {"metric": "receding-horizon MPC control steps/s (BASELINE cfg 5)", "value": steps / dt,
           "unit": "control steps/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": 1e3 * dt,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"cfg5: {B} disturbed initial states (x_ref[0] + U(-0.1,0.1)^4) x 500 control "
                                  f"steps, horizon {a.horizon}, exact QP solution per step, RK4 plant",
                      "lanes": B, "horizon": a.horizon, "control_steps": N - 1},
           "kernels": {"mpc_gains_ms": t_gain, "track_rollout_ms": t_roll},
           "roofline": {"bound": "hbm", "kernel": "track_rollout", "achieved": roll_bytes / (t_roll * 1e-3) / 1e9,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": roll_bytes / (t_roll * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "note": "latency-bound: B/64 wavefronts each run 500 dependent RK4 steps; the bytes are "
                                "the trajectories written"}}
    from oracle import tracking_np as tr
    lanes = min(B, a.cpu_lanes)
    t1 = time.perf_counter()
    xo, uo, K0o = tr.solve_mpc_tracking(x0[:lanes], x_ref, u_ref, a.horizon)
    tc = time.perf_counter() - t1
    out["cpu_baseline"] = {"value": lanes * (N - 1) / tc, "unit": "control steps/s", "cores": 1, "kind": "port",
                           "sample": f"first {lanes} lanes, numpy restatement (oracle/tracking_np.py) with the "
                                     f"window QPs solved by the same Riccati recursion", "seconds": tc}
    xg = x[:lanes].cpu().numpy()
    out["parity"] = {"rel_l2_x_vs_oracle": float(np.linalg.norm(xg - xo) / np.linalg.norm(xo)),
                     "rel_l2_K0_vs_oracle": float(np.linalg.norm(K0.cpu().numpy() - K0o) / np.linalg.norm(K0o)),
                     "lane0_final_state": x[0, -1].cpu().numpy().tolist(), "tolerance": 1e-9}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None,
                    help="lanes per GPU (weak scaling); default 262144 (newton, cfg 3) or 8192 (mpc, cfg 5)")
    ap.add_argument("--max-iters", type=int, default=5000)
    ap.add_argument("--cpu-lanes", type=int, default=4096,
                    help="lanes of the bounded CPU-baseline sample (about 10 s on 16 host cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-kernel HIP-event timing")
    ap.add_argument("--sync-every", type=int, default=4,
                    help="outer iterations between host reads of the (all-reduced) statistics; iterations "
                         "enqueued after every lane has finished are no-ops")
    ap.add_argument("--workload", choices=("newton", "mpc"), default="newton",
                    help="newton: the north-star metric (cfg 3); mpc: BASELINE cfg 5")
    ap.add_argument("--horizon", type=int, default=50, help="MPC prediction horizon T_pred (cfg 5: 50)")
    ap.add_argument("--schedule", choices=("auto", "serial", "pipelined", "persistent"), default="auto",
                    help="solver schedule (auto: the solver's choice for the batch size)")
    ap.add_argument("--chunk", type=int, default=128,
                    help="persistent schedule: iterations per launch (0: all of max_iters in one launch)")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = 8192 if a.workload == "mpc" else 262144
    if a.workload == "mpc":
        return run_mpc(a)

    import torch
    from gymnast_optimalcontrol_amd import distributed as gd
    rank, local_rank, world = gd.init_process_group()
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(gd.local_device_index(local_rank))
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver

    x_ref, u_ref = load_refs()
    N = x_ref.shape[0]
    T = N - 1
    total = a.batch * world
    x0_all = make_x0(total)
    lo, hi = gd.shard_range(total, rank, world)
    eng = AcrobotEngine()
    solver = BatchedNewtonSolver(eng, x_ref, u_ref, hi - lo, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                                 pipeline={"auto": None, "serial": False, "pipelined": True, "persistent": None}[a.schedule],
                                 persistent={"auto": None, "persistent": True}.get(a.schedule, False), chunk=a.chunk)
    if not a.no_timing:
        solver.enable_timing()
    x0_dev = eng.t(x0_all[lo:hi])                  # inputs resident in HBM before the timed region
    reduce = gd.make_reduce_stats()

    for _ in range(a.warmup):
        solver.solve(x0_dev, a.max_iters, reduce_stats=reduce, sync_every=a.sync_every)
    solver.reset_timing()
    gd.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lane_its = 0
    res = None
    for _ in range(a.steps):
        res = solver.solve(x0_dev, a.max_iters, reduce_stats=reduce, sync_every=a.sync_every)
        lane_its += res.lane_iterations
    torch.cuda.synchronize()
    gd.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = gd.max_over_ranks(elapsed)
    lane_its_all = int(gd.sum_over_ranks(lane_its))
    kt = solver.kernel_times()
    n_iters_outer = res.iterations

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
                  "outer_iterations": int(n_iters_outer),
                  "lane_iters_min_max": [int(res.n_iter.min().item()), int(res.n_iter.max().item())],
                  "rollouts": int(res.n_rollouts.sum().item()),
                  "lanes_that_backtracked": int((res.n_rollouts > res.n_iter).sum().item())}

    value = lane_its_all / elapsed
    out = {"metric": METRIC, "value": value, "unit": "Newton iterations/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": 1e3 * elapsed / a.steps, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": f"{ {4096: 'cfg2', 262144: 'cfg3'}.get(a.batch, 'custom') }: {a.batch} randomised-theta0 acrobot swing-ups per GPU, T={T}, fp64, "
                                  "task-2 Newton/Armijo settings, solved to convergence",
                      "lanes_per_gpu": a.batch, "global_lanes": total, "horizon_T": T,
                      "parallelism": f"lane-sharded x{world} (1 all-reduce of 8 fp64 stats / iteration)"},
           "states_per_s": value * T}

    if kt and rank == 0:
        ab = algorithmic_bytes(N, solver.u0_zero)
        kern = {}
        for kind, (ms, launches) in kt.items():
            if launches:
                kern[kind] = {"avg_ms": ms / launches, "launches": launches}
        if "run" in kern:
            # persistent schedule: every lane-iteration (sweep + trial) runs inside the run launches
            dom = "run"
            per_launch = lane_its * ab["iteration"] / kern["run"]["launches"]
            kern["run"]["algorithmic_bytes_per_launch"] = per_launch
            kern["run"]["achieved_GBs"] = per_launch / (kern["run"]["avg_ms"] * 1e-3) / 1e9
            bytes_per_lane, unit_note = ab["iteration"], "sweep + trial of one lane-iteration"
        elif "phase_odd" in kern:
            # pipelined schedule: every lane-iteration = one sweep + one trial, all inside the phase launches
            # (2 * iterations + 1 per solve; a launch's time is recorded whenever its timing slot is free)
            dom = "phase"
            rec_ms = sum(kern[k]["avg_ms"] * kern[k]["launches"] for k in ("phase_odd", "phase_even") if k in kern)
            rec_n = sum(kern[k]["launches"] for k in ("phase_odd", "phase_even") if k in kern)
            total_launches = a.steps * (2 * n_iters_outer + 1)
            per_launch = lane_its * ab["iteration"] / total_launches
            kern["phase"] = {"avg_ms": rec_ms / rec_n, "launches": total_launches, "recorded": rec_n,
                             "algorithmic_bytes_per_launch": per_launch}
            kern["phase"]["achieved_GBs"] = per_launch / (kern["phase"]["avg_ms"] * 1e-3) / 1e9
            bytes_per_lane, unit_note = ab["iteration"], "sweep + trial of one lane-iteration"
        else:
            for kind in ("backward", "trial"):
                if kind in kern:
                    per_launch = lane_its * ab[kind] / kern[kind]["launches"]
                    kern[kind]["algorithmic_bytes_per_launch"] = per_launch
                    kern[kind]["achieved_GBs"] = per_launch / (kern[kind]["avg_ms"] * 1e-3) / 1e9
            dom = max(("backward", "trial"), key=lambda k: kern.get(k, {}).get("avg_ms", 0))
            bytes_per_lane, unit_note = ab[dom], f"one {dom} pass of one lane"
        traffic, traffic_ratio, valu = None, None, None
        tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tfile):      # committed rocprofv3 --pmc measurement (tools/profile.sh, parse_profiles.py)
            try:
                t = json.load(open(tfile)).get(dom, {})
                traffic, traffic_ratio = t.get("hbm_bytes_per_launch"), t.get("traffic_over_algorithmic")
                if "valu_busy_upper_est" in t:
                    valu = {"busy_upper_est": t["valu_busy_upper_est"],
                            "wave_instructions_per_launch": t["sq_insts_valu_per_launch"],
                            "note": "SQ_INSTS_VALU x 4 cycles (fp64 wave64 on SIMD-32) / SIMD-cycles of the launch, "
                                    "rocprofv3 PMC (profiles/pmc_traffic.json)"}
            except Exception:
                traffic = None
        ach = kern[dom]["achieved_GBs"]
        out["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_over_algorithmic": traffic_ratio,
                           "traffic_source": "profiles/pmc_traffic.json (rocprofv3 PMC, 20-iteration run, all lanes "
                                             "active)", "bytes_per_unit": bytes_per_lane,
                           "unit_of_work": unit_note, "algorithmic_bytes_per_launch":
                           kern[dom]["algorithmic_bytes_per_launch"], "u0_zero_streams_skipped": solver.u0_zero,
                           "survey_bytes_per_iteration": ab["survey_per_iteration"],
                           "whole_solve_GBs_at_survey_bytes": value * ab["survey_per_iteration"] / 1e9 / world,
                           "fp64_valu": valu}
        out["kernels"] = kern
        out["schedule"] = "persistent" if solver.persistent else ("pipelined" if solver.pipeline else "serial")
    if parity is not None:
        out["parity"] = parity
    if rank == 0 and world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(x0_all, x_ref, u_ref, a.cpu_lanes, a.max_iters)
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
