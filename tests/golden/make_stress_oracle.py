"""Fixture: the C oracle's outcome for every lane of bench.py's stress workload (test infrastructure only).

SURVEY 8(d)'s stress variant, exactly as `bench.py --workload stress` builds it: 262,144 lanes, x0 = [th1, th2, 0, 0]
with th ~ U(+-1.5) from default_rng(0), lane 0 = 0, task-2 reference and settings (tol 1e-4, beta 0.7, c 0.5,
gamma_0 0.1, <= 20 Armijo trials, max_iters 5000).  oracle/acrobot_oracle.c solves every lane (OpenMP) and this
script stores per lane: n_iter, status, n_rollouts, final cost, final state x_N, plus the whole trajectory of
every 1024th lane.  tests/test_gpu_stress.py compares the GPU's automatic schedule (pipelined, lane compaction, the
low-occupancy regime, the straggler tail) with it lane by lane.  Runs for about an hour on 8 host cores.

Usage:  python tests/golden/make_stress_oracle.py [--chunk 8192]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from bench import load_refs, make_x0          # noqa: E402
from oracle import c_oracle                   # noqa: E402

LANES = 262144
TRAJ_STRIDE = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "stress_oracle.npz"))
    a = ap.parse_args()
    x_ref, u_ref = load_refs()
    x0 = make_x0(LANES, spread=1.5)
    N = x_ref.shape[0]
    n_iter = np.zeros(LANES, np.int32)
    status = np.zeros(LANES, np.int8)
    n_roll = np.zeros(LANES, np.int32)
    cost = np.zeros(LANES)
    x_last = np.zeros((LANES, 4))
    traj = np.zeros((LANES // TRAJ_STRIDE, N, 4))
    t0 = time.time()
    for lo in range(0, LANES, a.chunk):
        hi = min(LANES, lo + a.chunk)
        r = c_oracle.newton_solve(x0[lo:hi], x_ref, u_ref, max_iters=5000, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1,
                                  max_ls=20)
        n_iter[lo:hi], status[lo:hi], n_roll[lo:hi] = r["n_iter"], r["status"], r["n_rollouts"]
        cost[lo:hi], x_last[lo:hi] = r["cost"], r["x"][:, -1]
        sel = np.arange(lo, hi)[np.arange(lo, hi) % TRAJ_STRIDE == 0]
        traj[sel // TRAJ_STRIDE] = r["x"][sel - lo]
        print(f"{hi}/{LANES} lanes, {time.time() - t0:.0f} s, statuses {np.bincount(status[:hi], minlength=4)}",
              flush=True)
    np.savez_compressed(a.out, x0=x0, n_iter=n_iter, status=status, n_rollouts=n_roll, cost=cost, x_last=x_last,
                        traj_stride=TRAJ_STRIDE, traj=traj)
    print("wrote", a.out, flush=True)


if __name__ == "__main__":
    main()
