#!/usr/bin/env python3
"""Search the relative placement of the phase kernel's six streams inside physically contiguous VRAM (measurement
tool; profiles/r06/README.md "layout search").

    python tools/layout_search.py --layouts 200 --out gpurun_out/r06/ls/search.json

tools/layout6_probe.hip's k_sep moves the phase kernel's bytes with its access pattern and no arithmetic; on ordinary
allocations it reproduces the placement spread of the real kernel (1.90-2.13 ms per launch for four stream sets in
one process).  Here the six streams are carved from one physically contiguous allocation
(hipExtMallocWithFlags(hipDeviceMallocContiguous), tools/contig_alloc.hip), so a layout -- the order of the streams
and the gaps between them -- fixes their relative physical placement.  --layouts random layouts (a random order,
random gaps in multiples of --gran bytes) are timed (3 launches each, the median of the last two), the best ones are
re-timed, and then carved from a SECOND contiguous allocation (another physical base) to see whether a layout's speed
is a property of the relative offsets alone (then a solver could allocate for it) or of the absolute addresses too.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SIZES = [4202692608, 4202692608, 2097152000, 2097152000, 4194304000, 2097152000]   # x0 x1 u0 u1 K1 cs
NAMES = ["x0", "x1", "u0", "u1", "K1", "cs"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layouts", type=int, default=200)
    ap.add_argument("--gran", type=int, default=2 << 20)
    ap.add_argument("--arena-gb", type=float, default=40.0)
    ap.add_argument("--best", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    probe = C.CDLL(os.path.join(ROOT, "tools", "liblayout6_probe.so"))
    probe.l6_run.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.c_int64, C.c_int, C.c_int, C.c_void_p]
    ca = C.CDLL(os.path.join(ROOT, "tools", "libcontig_alloc.so"))
    stream = torch.cuda.current_stream().cuda_stream
    B, T = 262144, 500

    def arena(gb):
        p = C.c_void_p()
        n = int(gb * (1 << 30)) // (2 << 20) * (2 << 20)
        rc = ca.ca_malloc(C.c_int64(n), 4, C.byref(p))
        return (p.value, n) if rc == 0 else (None, 0)

    def time_layout(base, offs, reps=3):
        ptrs = (C.c_void_p * 6)(*[base + o for o in offs])
        ts = []
        for r in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            assert probe.l6_run(0, ptrs, B, T, r & 1, stream) == 0
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        return float(np.median(ts[1:]))

    rng = np.random.default_rng(a.seed)
    A, nA = arena(a.arena_gb)
    if A is None:
        print(json.dumps({"error": "contiguous allocation failed", "gb": a.arena_gb}), flush=True)
        sys.exit(3)
    total = sum(SIZES)
    slack = nA - total - a.gran * 8

    def random_layout():
        order = rng.permutation(6)
        cuts = np.sort(rng.integers(0, slack // a.gran, 6)) * a.gran
        gaps = np.diff(np.concatenate([[0], cuts]))
        offs, o = [0] * 6, 0
        for k, s in enumerate(order):
            o += int(gaps[k])
            offs[s] = o
            o += -(-SIZES[s] // a.gran) * a.gran
        return [int(v) for v in offs]

    # warm-up on a plain layout
    plain = list(np.cumsum([0] + [-(-s // a.gran) * a.gran for s in SIZES[:-1]]))
    for _ in range(2):
        time_layout(A, [int(v) for v in plain])
    res = {"arena_gb": nA / (1 << 30), "base_A": hex(A), "plain_ms": time_layout(A, [int(v) for v in plain]),
           "layouts": []}
    t0 = time.time()
    for i in range(a.layouts):
        offs = random_layout()
        ms = time_layout(A, offs)
        res["layouts"].append({"offs": offs, "ms": ms})
        if i % 20 == 0:
            print(json.dumps({"i": i, "ms": round(ms, 4), "elapsed_s": round(time.time() - t0, 1)}), flush=True)
    ms_all = np.array([r["ms"] for r in res["layouts"]])
    res["summary_A"] = {"min": float(ms_all.min()), "p10": float(np.percentile(ms_all, 10)),
                        "median": float(np.median(ms_all)), "max": float(ms_all.max())}
    print(json.dumps(res["summary_A"]), flush=True)
    best = np.argsort(ms_all)[:a.best]
    worst = np.argsort(-ms_all)[:2]
    res["retime_A"] = [{"i": int(i), "ms": [time_layout(A, res["layouts"][i]["offs"]) for _ in range(2)]}
                       for i in list(best) + list(worst)]
    print(json.dumps({"retime_A": res["retime_A"]}), flush=True)
    # a second contiguous allocation: another physical base
    Bp_, nB = arena(a.arena_gb)
    if Bp_ is not None:
        res["base_B"] = hex(Bp_)
        fits = [i for i in list(best) + list(worst) if max(o + s for o, s in zip(res["layouts"][i]["offs"], SIZES)) <= nB]
        res["retime_B"] = [{"i": int(i), "ms": [time_layout(Bp_, res["layouts"][i]["offs"]) for _ in range(2)]}
                           for i in fits]
        print(json.dumps({"retime_B": res["retime_B"], "arena_B_gb": nB / (1 << 30)}), flush=True)
    else:
        res["base_B"] = None
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
