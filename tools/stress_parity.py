#!/usr/bin/env python3
"""Diagnostic (GPU): dump the automatic schedule's per-lane outcomes on hard lanes, for comparison with the C
oracle on the host (tests/golden/make_stress_oracle.py, tools/stress_compare.py).

  full : bench.py's stress workload (262,144 lanes, th ~ U(+-1.5), default_rng(0)), automatic schedule
         (pipelined -> lane compaction -> low-occupancy regime -> straggler tail), max_iters 5000: n_iter, status,
         n_rollouts, cost, x_N of every lane and the trajectory of every 1024th lane.
  hard : 2,048 lanes, th ~ U(+-1.5), every 4th lane with thdot ~ U(+-2) (default_rng(7)), the automatic schedule
         of a 262,144-lane shard (schedule_lanes) with the tail at 128 lanes so that compaction comes first;
         per-lane histories (cost, max|sigma|) up to each lane's last iteration.

    python tools/stress_parity.py [full] [hard] --out gpurun_out/stress
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_refs, make_x0  # noqa: E402


def hard_x0(B=2048, seed=7):
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 4))
    x0[:, :2] = rng.uniform(-1.5, 1.5, (B, 2))
    x0[::4, 2:] = rng.uniform(-2.0, 2.0, (len(x0[::4]), 2))
    return x0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="*", default=["full", "hard"])
    ap.add_argument("--out", default="gpurun_out/stress")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    xr, ur = load_refs()
    eng = AcrobotEngine()
    kw = dict(tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20)
    if "full" in a.which:
        x0 = make_x0(262144, spread=1.5)
        s = BatchedNewtonSolver(eng, xr, ur, len(x0), **kw)
        t0 = time.time()
        r = s.solve(x0, 5000, sync_every=4)
        dt = time.time() - t0
        x = r.x
        np.savez_compressed(os.path.join(a.out, "full.npz"), n_iter=r.n_iter.cpu().numpy(),
                            status=r.status.cpu().numpy(), n_rollouts=r.n_rollouts.cpu().numpy(),
                            cost=r.cost.cpu().numpy(), x_last=x[:, -1].cpu().numpy(), traj=x[::1024].cpu().numpy(),
                            schedule=r.schedule, compactions=r.compactions, tail_its=r.tail_lane_iterations,
                            lowocc_its=r.lowocc_lane_iterations, iterations=r.iterations, seconds=dt)
        print(f"full: {dt:.2f} s, schedule {r.schedule}, compactions {r.compactions}, tail its "
              f"{r.tail_lane_iterations}, low-occupancy its {r.lowocc_lane_iterations}, statuses "
              f"{np.bincount(r.status.cpu().numpy())}", flush=True)
        del r, x, s
    if "hard" in a.which:
        x0 = hard_x0()
        B = len(x0)
        s = BatchedNewtonSolver(eng, xr, ur, B, hist_len=5000, schedule_lanes=262144, tail_lanes=128, **kw)
        t0 = time.time()
        r = s.solve(x0, 5000, sync_every=4)
        dt = time.time() - t0
        n_iter = r.n_iter.cpu().numpy()
        hc, hs = r.hist_cost.cpu().numpy(), r.hist_smax.cpu().numpy()      # (hist_len, B)
        cat_c = np.concatenate([hc[:n_iter[i], i] for i in range(B)])
        cat_s = np.concatenate([hs[:n_iter[i], i] for i in range(B)])
        np.savez_compressed(os.path.join(a.out, "hard.npz"), x0=x0, n_iter=n_iter, status=r.status.cpu().numpy(),
                            n_rollouts=r.n_rollouts.cpu().numpy(), cost=r.cost.cpu().numpy(), x=r.x.cpu().numpy(),
                            hist_cost=cat_c, hist_smax=cat_s, schedule=r.schedule, compactions=r.compactions,
                            tail_its=r.tail_lane_iterations, lowocc_its=r.lowocc_lane_iterations, seconds=dt)
        print(f"hard: {dt:.2f} s, schedule {r.schedule}, compactions {r.compactions}, tail its "
              f"{r.tail_lane_iterations}, low-occupancy its {r.lowocc_lane_iterations}, statuses "
              f"{np.bincount(r.status.cpu().numpy())}", flush=True)


if __name__ == "__main__":
    main()
