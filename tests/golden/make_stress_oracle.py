"""Fixture: the C oracle's outcome for every lane of bench.py's stress workload (test infrastructure only).

SURVEY 8(d)'s stress variant, exactly as `bench.py --workload stress` builds it: 262,144 lanes, x0 = [th1, th2, 0, 0]
with th ~ U(+-1.5) from default_rng(0) (bench.make_x0), lane 0 = 0, task-2 reference and settings (tol 1e-4, beta
0.7, c 0.5, gamma_0 0.1, <= 20 Armijo trials, max_iters 5000).  oracle/acrobot_oracle.c solves every lane (OpenMP,
with its per-iteration record) and this script stores per lane: n_iter, status, n_rollouts, final cost, and the
Armijo tie record -- k_tie, the first iteration with an Armijo test within TIE of a tie (|J_new - (J + c gamma dJ)|
< TIE |J|, oracle/c_oracle.py hist_margin; -1: none) and margin_min, the smallest such margin of the lane's run.
tests/test_gpu_stress.py compares the GPU's automatic schedule (pipelined, lane compaction, the low-occupancy regime,
the straggler tail) with it lane by lane.  About an hour on 8 host cores.
make_headline_oracle.py runs the same solve on the headline workload (spread 0.5).

Usage:  python tests/golden/make_stress_oracle.py [--chunk 4096]
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
MAX_ITERS = 5000
TIE = 1e-11          # relative Armijo margin counted as a tie (tests/test_gpu_stress.py: TIE)


def solve_all(spread: float, out: str, chunk: int = 4096, lanes: int = LANES):
    """The C oracle over bench.make_x0(lanes, spread), chunk by chunk, with its per-iteration record; writes ``out``."""
    x_ref, u_ref = load_refs()
    x0 = make_x0(lanes, spread=spread)
    n_iter = np.zeros(lanes, np.int16)
    status = np.zeros(lanes, np.int8)
    n_roll = np.zeros(lanes, np.int32)
    cost = np.zeros(lanes)
    k_tie = np.full(lanes, -1, np.int16)
    margin_min = np.full(lanes, np.inf, np.float32)
    t0 = time.time()
    for lo in range(0, lanes, chunk):
        hi = min(lanes, lo + chunk)
        r = c_oracle.newton_solve(x0[lo:hi], x_ref, u_ref, max_iters=MAX_ITERS, tol=1e-4, beta=0.7, c=0.5,
                                  gamma_0=0.1, max_ls=20, hist_len=MAX_ITERS)
        n_iter[lo:hi], status[lo:hi], n_roll[lo:hi], cost[lo:hi] = r["n_iter"], r["status"], r["n_rollouts"], r["cost"]
        m = np.where(np.isnan(r["hist_margin"]), np.inf, r["hist_margin"])   # past a lane's last iteration: none
        margin_min[lo:hi] = m.min(axis=1)
        tie = m < TIE
        k_tie[lo:hi] = np.where(tie.any(axis=1), tie.argmax(axis=1), -1)
        print(f"{hi}/{lanes} lanes, {time.time() - t0:.0f} s, statuses {np.bincount(status[:hi], minlength=4)}, "
              f"lanes with a tie {(k_tie[:hi] >= 0).sum()}", flush=True)
    np.savez_compressed(out, n_iter=n_iter, status=status, n_rollouts=n_roll, cost=cost, k_tie=k_tie,
                        margin_min=margin_min, tie=np.float64(TIE), max_iters=np.int64(MAX_ITERS),
                        spread=np.float64(spread))
    print("wrote", out, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "stress_oracle.npz"))
    a = ap.parse_args()
    solve_all(1.5, a.out, a.chunk)


if __name__ == "__main__":
    main()
