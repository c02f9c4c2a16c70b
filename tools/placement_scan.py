#!/usr/bin/env python3
"""Phase-kernel time against the relative placement of its streams in physically contiguous VRAM (measurement tool;
VERDICT r05 item 1).

    python tools/placement_scan.py --out gpurun_out/r06/scan/scan.json

tools/placement_pmc.py found that on a slow stream set the slowness follows the (K1, cs) pair: swapping either of the
two for a fast set's copy makes the slow set fast, while x0 / x1 / u0 / u1 do not matter there, and each buffer alone
streams at the same rate wherever it lies.  Two streams the same waves touch in lock step (the sweep writes K1 row 1
and cg of stage t together, the trial reads them together) are slow together at some relative placements.  Here the
six streams are carved from ONE physically contiguous allocation (hipExtMallocWithFlags(hipDeviceMallocContiguous),
tools/contig_alloc.hip), so the relative physical offset of two streams is their virtual one, and the gap between K1
and cs (and, second, between x_b and u_b) is scanned; each layout is timed over --iters iterations of the real
pipelined schedule, --rounds interleaved rounds.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MiB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lanes", type=int, default=262144)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver, morton_order
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x_ref, u_ref = bench.load_refs()
    eng = AcrobotEngine()
    sv = BatchedNewtonSolver(eng, x_ref, u_ref, a.lanes, tol=1e-4, beta=0.7, c=0.5, gamma_0=0.1, max_ls=20,
                             placement_trials=1)
    sv.enable_timing()
    x0 = eng.t(bench.make_x0(a.lanes))
    x0 = x0[morton_order(x0)]
    sizes = [int(np.prod(sh)) * 8 for sh in sv._stream_shapes]      # x0 x1 u0 u1 K1 cs
    gaps_kc = ([0, 4096, 65536, 256 * 1024, MiB] + [2 * MiB * i for i in range(1, 33)] +
               [96 * MiB, 128 * MiB, 192 * MiB, 256 * MiB, 384 * MiB, 512 * MiB, 1024 * MiB])
    arena_bytes = sum(sizes) + max(gaps_kc) + 256 * MiB
    lib = C.CDLL(os.path.join(ROOT, "tools", "libcontig_alloc.so"))
    p = C.c_void_p()
    rc = lib.ca_malloc(C.c_int64(arena_bytes), 4, C.byref(p))
    print(json.dumps({"contiguous_alloc_bytes": arena_bytes, "rc": rc, "ptr": hex(p.value or 0)}), flush=True)
    if rc != 0:
        sys.exit(3)
    n = arena_bytes // 8

    class Blob:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (p.value, False), "version": 2,
                                    "strides": None}
    arena = torch.as_tensor(Blob(), device=dev)

    def carve(offsets):
        return [arena[o // 8:o // 8 + sz // 8].view(sh) for o, sz, sh in zip(offsets, sizes, sv._stream_shapes)]

    def layout_kc(gap):
        # [x0][x1][u0][u1][K1][gap][cs]
        o, offs = 0, []
        for i, sz in enumerate(sizes):
            if i == 5:
                o += gap
            offs.append(o)
            o += sz
        return offs

    def layout_xu(gap):
        # [K1][cs][x0][gap][u0][x1][gap][u1]: x_b / u_b separated by gap
        xs, us = sizes[0], sizes[2]
        k, c = 0, sizes[4]
        x0o = k + sizes[4] + sizes[5]
        u0o = x0o + xs + gap
        x1o = u0o + us
        u1o = x1o + xs + gap
        return [x0o, x1o, u0o, u1o, k, c]

    def timed(st):
        sv._set_streams(st)
        sv.reset_timing()
        sv.max_iters = a.iters + 1
        sv.init(x0)
        for _ in range(a.iters):
            sv.iteration()
        torch.cuda.synchronize(dev)
        sv.collect_timing()
        kt = sv.kernel_times()
        ms = sum(kt[k][0] for k in ("phase_odd", "phase_even"))
        nn = sum(kt[k][1] for k in ("phase_odd", "phase_even"))
        return ms / max(nn, 1)

    configs = [("kc", g) for g in gaps_kc] + [("xu", g) for g in (0, 2 * MiB, 4 * MiB, 6 * MiB, 8 * MiB, 12 * MiB,
                                                                  16 * MiB, 64 * MiB, 256 * MiB)]
    res = {f"{k}:{g}": [] for k, g in configs}
    for r in range(a.rounds):
        seq = configs if r % 2 == 0 else configs[::-1]
        for kind, g in seq:
            offs = layout_kc(g) if kind == "kc" else layout_xu(g)
            if max(o + sz for o, sz in zip(offs, sizes)) > arena_bytes:
                continue
            ms = timed(carve(offs))
            res[f"{kind}:{g}"].append(ms)
            print(json.dumps({"round": r, "kind": kind, "gap_bytes": g, "gap_MiB": g / MiB, "phase_ms": round(ms, 4)}),
                  flush=True)
    summary = {k: {"min": min(v), "all": v} for k, v in res.items() if v}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump({"sizes": sizes, "arena_bytes": arena_bytes, "ptr": hex(p.value), "scan": summary}, open(a.out, "w"),
              indent=1)
    sv._set_streams([torch.empty(sh, dtype=torch.float64, device=dev) for sh in sv._stream_shapes])
    arena = None
    torch.cuda.synchronize(dev)


if __name__ == "__main__":
    main()
