#!/usr/bin/env python3
"""Where the straggler-tail kernel (k_nt_tail) spends its cycles (diagnostic tool).

    python tools/tail_trace.py build_ab/tail_trace.so [--batch 64] [--iters 200] [--spread 1.5]

The library is built with -DGYM_TAIL_TRACE (_build.build(defines=["GYM_TAIL_TRACE"], out=...)).  A small batch is
handed to the tail from its first iteration; prints the mean cycles per iteration (s_memtime) in the sweep, the
trials and the rest (copy of the accepted candidate, bookkeeping), and per stage."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--spread", type=float, default=1.5)
    a = ap.parse_args()
    os.environ["GYM_ALLOW_FOREIGN_BUILD"] = "1"     # a define-variant of this tree
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    eng = AcrobotEngine(lib_path=os.path.abspath(a.lib))
    eng.lib.gym_debug_tail_trace.argtypes = [C.c_void_p, C.c_int]
    x_ref, u_ref = load_refs()
    s = BatchedNewtonSolver(eng, x_ref, u_ref, a.batch, tol=1e-4, gamma_0=0.1, pipeline=False,
                            tail_lanes=10 ** 9, tail_chunk=10 ** 6)
    x0 = make_x0(a.batch, spread=a.spread)
    s.solve(x0, a.iters)
    buf = np.zeros((4096, 4), np.uint64)
    eng.lib.gym_debug_tail_trace(buf.ctypes.data, 1)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    r = s.solve(x0, a.iters)
    t1.record(); torch.cuda.synchronize()
    eng.lib.gym_debug_tail_trace(buf.ctypes.data, 0)
    tr = buf.astype(np.float64)
    tr = tr[tr[:, 3] > 0]
    its = tr[:, 3].sum()
    T = x_ref.shape[0] - 1
    sw, tri, rest = (tr[:, i].sum() / its for i in range(3))
    print(f"B={a.batch} iters={a.iters} solve {t0.elapsed_time(t1):.2f} ms, {int(its)} tail lane-iterations "
          f"over {len(tr)} workgroups, {r.lane_iterations} lane-iterations in the solve")
    print(f"  cycles/iteration: sweep {sw:9.0f}  trials {tri:9.0f}  rest {rest:8.0f}  total {sw + tri + rest:9.0f}")
    print(f"  per stage: sweep {sw / T:.0f}  trials {tri / T:.0f} cycles")


if __name__ == "__main__":
    main()
