#!/usr/bin/env python3
"""Per-wavefront timing and placement of the solver's sweep / trial launches (diagnostic tool).

    python tools/wave_trace.py build_ab/trace.so [--batch 262144] [--iters 3]

``trace.so`` is the library built with -DGYM_WAVE_TRACE (see _build.build(defines=...)): the serial
schedule's k_nt_backward / k_nt_trial record s_memrealtime (100 MHz) at wave start and end plus
HW_ID / XCC_ID.  Prints, per kernel of the last iteration: the spread of wave start / end times,
the wave-duration distribution, waves per SIMD, and the mean duration per XCD and per waves-on-SIMD.
"""
import argparse
import ctypes as C
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def decode(hw, xcc):
    # gfx9 HW_ID: wave [3:0], simd [5:4], pipe [7:6], cu [11:8], sh [12], se [15:13]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    return xcc & 15, se, sh, cu, simd


def main():
    os.environ["GYM_ALLOW_FOREIGN_BUILD"] = "1"     # a define-variant of this tree (its build id differs)
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    eng = AcrobotEngine(lib_path=os.path.abspath(a.lib))
    eng.lib.gym_debug_wave_trace.argtypes = [C.c_void_p]
    x_ref, u_ref = load_refs()
    s = BatchedNewtonSolver(eng, x_ref, u_ref, a.batch, tol=1e-4, gamma_0=0.1, pipeline=False)
    s.solve(make_x0(a.batch), a.iters)
    torch.cuda.synchronize()
    buf = np.zeros((2, 8192, 4), dtype=np.uint64)
    assert eng.lib.gym_debug_wave_trace(buf.ctypes.data) == 0
    nw = (a.batch + 63) // 64
    out = {}
    for kind, name in ((0, "backward"), (1, "trial")):
        r = buf[kind, :nw].astype(np.int64)
        t0, t1 = r[:, 0], r[:, 1]
        base = t0.min()
        start, end = (t0 - base) / 100.0, (t1 - base) / 100.0        # microseconds (100 MHz)
        dur = end - start
        place = [decode(int(h), int(x)) for h, x in zip(r[:, 2], r[:, 3])]
        simd_key = [(p[0], p[1], p[2], p[3], p[4]) for p in place]
        per_simd = defaultdict(int)
        for k in simd_key:
            per_simd[k] += 1
        occ = np.array([per_simd[k] for k in simd_key])
        by_xcc = defaultdict(list)
        for p, d in zip(place, dur):
            by_xcc[p[0]].append(d)
        by_occ = defaultdict(list)
        for o, d in zip(occ, dur):
            by_occ[int(o)].append(d)
        rank = np.zeros(len(dur), dtype=int)        # order of a wave's start among its SIMD's waves
        groups = defaultdict(list)
        for i, k in enumerate(simd_key):
            groups[k].append(i)
        for idx in groups.values():
            for j, i in enumerate(sorted(idx, key=lambda i: (t0[i], i))):
                rank[i] = j
        by_rank = {int(j): round(float(dur[rank == j].mean()), 1) for j in np.unique(rank)}
        out[name] = {
            "mean_dur_by_start_rank_on_simd": by_rank,
            "kernel_span_us": float(end.max()),
            "start_us_p50_p99_max": [float(np.percentile(start, 50)), float(np.percentile(start, 99)), float(start.max())],
            "end_us_min_p10_p50_p90_max": [float(end.min()), float(np.percentile(end, 10)), float(np.percentile(end, 50)),
                                           float(np.percentile(end, 90)), float(end.max())],
            "dur_us_min_p50_max": [float(dur.min()), float(np.percentile(dur, 50)), float(dur.max())],
            "mean_dur_over_span": float(dur.mean() / end.max()),
            "simds_used": len(per_simd),
            "waves_per_simd_hist": {int(k): int(v) for k, v in zip(*np.unique(list(per_simd.values()), return_counts=True))},
            "mean_dur_by_waves_on_simd": {k: round(float(np.mean(v)), 1) for k, v in sorted(by_occ.items())},
            "mean_dur_by_xcc": {int(k): round(float(np.mean(v)), 1) for k, v in sorted(by_xcc.items())},
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
