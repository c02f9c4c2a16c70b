#!/usr/bin/env python3
"""How many lanes backtrack per Newton iteration on bench.py's stress workload (measurement tool, host only): the C
oracle's per-iteration record (hist_trials >= 2: the lane rejected Armijo trial 1 and went to the post-trial
candidates) on every STRIDE-th lane of the 262,144-lane batch, scaled back by STRIDE.  Sizes the candidate scratch
(solver.CAND_SLOTS): the post-trial kernels run one chain per backtracking iteration, whatever the lane count.

    python tools/retry_counts.py [--stride 16] [--max-iters 1000]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stride", type=int, default=16)
    ap.add_argument("--max-iters", type=int, default=1000)
    a = ap.parse_args()
    from bench import load_refs, make_x0
    from oracle import c_oracle
    xr, ur = load_refs()
    x0 = make_x0(262144, spread=1.5)[::a.stride]
    t = time.time()
    o = c_oracle.newton_solve(x0, xr, ur, max_iters=a.max_iters, tol=1e-4, gamma_0=0.1, hist_len=a.max_iters)
    tr = o["hist_trials"]
    cnt = (tr >= 2).sum(axis=0) * a.stride
    act = (tr >= 1).sum(axis=0) * a.stride
    print(f"{len(x0)} lanes in {time.time() - t:.0f} s; iteration, active lanes, backtracking lanes (x{a.stride})")
    for k in list(range(0, 20)) + list(range(20, a.max_iters, 20)):
        print(k, int(act[k]), int(cnt[k]))
    for slots in (16384, 32768):
        cap = slots // 19
        print(f"{slots} slots ({cap} lanes at max_ls 20): iterations above {int((cnt > cap).sum())}, backtracking "
              f"lane-iterations within {int(np.minimum(cnt, cap).sum())} of {int(cnt.sum())}")


if __name__ == "__main__":
    main()
