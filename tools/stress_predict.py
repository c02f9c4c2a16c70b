#!/usr/bin/env python3
"""Can the stress workload's longest lanes be told early, so a concurrent straggler tail could take them?  (analysis
tool, CPU)

    python tools/stress_predict.py [--out profiles/r06/stress/oracle_sample_smax.npz]

The C oracle with per-iteration records (cost, max|sigma|, Armijo trials) on the 300 longest lanes of bench.py's stress
batch (tests/golden/stress_oracle.npz) plus 4,096 random lanes, 5,000 iterations.  For iterations K = 400 .. 650 it
ranks the lanes still active at K by a feature (cumulative extra Armijo trials, those of the last 50 iterations,
max|sigma| at K, the cost's stall over the last 50 iterations, the cost) among the random active lanes, and reports how
many lanes of the full 262,144-lane batch a tail would have to take at K to hold every lane that runs >= 3,000
iterations.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from bench import load_refs, make_x0
    from oracle import c_oracle
    o = np.load(os.path.join(ROOT, "tests", "golden", "stress_oracle.npz"))
    nall = o["n_iter"]
    x0all = make_x0(262144, spread=1.5)
    top = np.argsort(-nall)[:300]
    samp = np.unique(np.concatenate([top, np.random.default_rng(1).choice(262144, 4096, replace=False)]))
    xr, ur = load_refs()
    r = c_oracle.newton_solve(x0all[samp], xr, ur, max_iters=5000, tol=1e-4, gamma_0=0.1, hist_len=5000)
    n, tr, sm, cost = r["n_iter"], r["hist_trials"], r["hist_smax"], r["hist_cost"]
    rand = ~np.isin(samp, top)
    extra = np.cumsum(np.where(tr > 0, tr - 1, 0), axis=1)
    longm = n >= 3000
    print(f"{int(longm.sum())} lanes >= 3000 iterations in the sample: {sorted(n[longm].tolist())}")
    for K in (400, 420, 450, 480, 500, 520, 550, 600, 650):
        act = n > K
        full = (act & rand).sum() / rand.sum() * 262144
        feats = {"extra_cum": extra[:, K - 1], "extra_last50": extra[:, K - 1] - extra[:, K - 51],
                 "smax": sm[:, K - 1], "stall": -np.abs(cost[:, K - 51] - cost[:, K - 1]) / np.abs(cost[:, K - 1]),
                 "cost": cost[:, K - 1]}
        row = []
        for name, f in feats.items():
            ref = f[act & rand]
            ranks = [(ref >= f[i]).mean() for i in np.nonzero(longm & act)[0]]
            row.append(f"{name} {max(ranks) * full:7.0f}")
        print(f"K={K:4d} active ~{full:7.0f}; lanes a tail must take at K to hold every long lane, by: " + ", ".join(row))
    if a.out:
        ks = np.arange(400, 701, 20)
        np.savez_compressed(a.out, lanes=samp, n_iter=n, status=r["status"], k=ks, smax_at_k=sm[:, ks - 1])


if __name__ == "__main__":
    main()
