#!/usr/bin/env python3
"""Settle every GPU / C-oracle decision difference of bench.py's stress workload lane by lane
and write the per-lane record (tests/stress_settle.settle) to an npz, with a summary on stdout.

    python tools/stress_settle_dump.py --out gpurun_out/r05/settle/settle.npz

The full 262,144-lane stress solve on the automatic schedule (as tests/test_gpu_stress.py runs it), its decisions
against tests/golden/stress_oracle.npz, then every differing lane re-run with records on the GPU and on the C oracle.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    from stress_settle import settle
    xr, ur = load_refs()
    B = 262144
    x0 = make_x0(B, spread=1.5)
    eng = AcrobotEngine()
    t0 = time.time()
    r = BatchedNewtonSolver(eng, xr, ur, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20).solve(x0, 5000,
                                                                                                     sync_every=4)
    ng, sg, rg = (t.cpu().numpy() for t in (r.n_iter, r.status, r.n_rollouts))
    del r
    o = np.load(os.path.join(ROOT, "tests", "golden", "stress_oracle.npz"))
    same = (ng == o["n_iter"]) & (sg == o["status"]) & (rg == o["n_rollouts"])
    diff = np.nonzero(~same)[0]
    print(f"full solve {time.time() - t0:.1f} s; {len(diff)} lanes differ from the fixture", flush=True)
    t1 = time.time()
    d = settle(eng, x0, xr, ur, diff)
    print(f"settled {len(diff)} lanes in {time.time() - t1:.1f} s", flush=True)
    # the re-run reproduces the full batch's decisions lane by lane
    print("re-run == full batch:", bool((d["ng"] == ng[diff]).all() and (d["sg"] == sg[diff]).all()
                                        and (d["rg"] == rg[diff]).all()), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    np.savez_compressed(a.out, **d)
    for kind in ("trials", "cost", "length"):
        sel = d["kind"] == kind
        print(f"{kind} divergences: {int(sel.sum())}", flush=True)
        if not sel.any():
            continue
        mk = d["margin_k"][sel]
        if kind != "length":
            for thr in (1e-16, 1e-15, 1e-14, 1e-13, 1e-12, 1e-11, 1e-10):
                print(f"  margin at k < {thr:.0e}: {int((mk < thr).sum())}", flush=True)
            order = np.argsort(-np.where(np.isfinite(mk), mk, np.inf))
            print("  largest margins at k (lane, k, margin, margin before k):",
                  [(int(d['lane'][sel][i]), int(d['k'][sel][i]), float(mk[i]), float(d['margin_before'][sel][i]))
                   for i in order[:15]], flush=True)
        else:
            print("  (lane, ng, no, sg, so, smax_rel_o, smax_rel_g):",
                  [(int(d['lane'][i]), int(d['ng'][i]), int(d['no'][i]), int(d['sg'][i]), int(d['so'][i]),
                    float(d['smax_rel_o'][i]), float(d['smax_rel_g'][i])) for i in np.nonzero(sel)[0][:60]],
                  flush=True)
    print("max pre-divergence cost rel diff:", float(d["pre_rel"].max()), flush=True)

if __name__ == "__main__":
    main()
