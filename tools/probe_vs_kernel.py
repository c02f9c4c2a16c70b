#!/usr/bin/env python3
"""Does the zero-arithmetic stream probe rank stream-buffer sets as the phase kernel does?  (measurement tool)

    python tools/probe_vs_kernel.py --sets 8 --out gpurun_out/r06/pvk/pvk.json

Keeps --sets stream-buffer sets of the headline solver alive in one process and measures on each, interleaved over
--rounds rounds: the real phase kernel (12 iterations of the pipelined schedule from a fresh init, HIP events per
phase launch: the solver's own timing) and tools/layout6_probe.hip's k_sep run directly on the set's six buffers (the
phase kernel's access pattern without arithmetic, 3 launches).  A probe that ranks sets like the kernel can select a
placement at construction in a few ms per set, with no solver iterations.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine, F64
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver, morton_order
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    probe = C.CDLL(os.path.join(ROOT, "tools", "liblayout6_probe.so"))
    probe.l6_run.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.c_int64, C.c_int, C.c_int, C.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    x_ref, u_ref = bench.load_refs()
    eng = AcrobotEngine()
    B = 262144
    sv = BatchedNewtonSolver(eng, x_ref, u_ref, B, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                             placement_trials=1)
    sv.enable_timing()
    x0 = eng.t(bench.make_x0(B))
    x0 = x0[morton_order(x0)]
    sets = [sv._streams()] + [[torch.empty(sh, dtype=F64, device=dev) for sh in sv._stream_shapes]
                              for _ in range(a.sets - 1)]

    def kernel_ms(st):
        sv._set_streams(st)
        sv.reset_timing()
        sv.max_iters = a.iters + 1
        sv.init(x0)
        for _ in range(a.iters):
            sv.iteration()
        torch.cuda.synchronize(dev)
        sv.collect_timing()
        kt = sv.kernel_times()
        return sum(kt[k][0] for k in ("phase_odd", "phase_even")) / sum(kt[k][1] for k in ("phase_odd", "phase_even"))

    def probe_ms(st):
        ptrs = (C.c_void_p * 6)(*[t.data_ptr() for t in st])
        ts = []
        for r in range(3):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            assert probe.l6_run(0, ptrs, B, 500, r & 1, stream) == 0
            ev[1].record()
            torch.cuda.synchronize(dev)
            ts.append(ev[0].elapsed_time(ev[1]))
        return float(np.median(ts[1:]))

    kernel_ms(sets[0]); probe_ms(sets[0])   # warm-up
    recs = []
    for r in range(a.rounds):
        for i, st in enumerate(sets if r % 2 == 0 else sets[::-1]):
            i = i if r % 2 == 0 else len(sets) - 1 - i
            k, p = kernel_ms(st), probe_ms(st)
            recs.append({"round": r, "set": i, "kernel_phase_ms": k, "probe_ms": p})
            print(json.dumps(recs[-1]), flush=True)
    km = {i: min(x["kernel_phase_ms"] for x in recs if x["set"] == i) for i in range(a.sets)}
    pm = {i: min(x["probe_ms"] for x in recs if x["set"] == i) for i in range(a.sets)}
    kv, pv = np.array([km[i] for i in range(a.sets)]), np.array([pm[i] for i in range(a.sets)])
    out = {"records": recs, "kernel_ms": km, "probe_ms": pm, "pearson": float(np.corrcoef(kv, pv)[0, 1]),
           "best_by_kernel": int(np.argmin(kv)), "best_by_probe": int(np.argmin(pv)),
           "kernel_ms_of_probe_best": float(kv[np.argmin(pv)]), "kernel_ms_best": float(kv.min())}
    print(json.dumps({k: v for k, v in out.items() if k != "records"}), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
