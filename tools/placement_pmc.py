#!/usr/bin/env python3
"""Why does the phase kernel's speed depend on where its stream buffers land?  (measurement tool)

    python tools/placement_pmc.py --sets 6 --out gpurun_out/r06/placement/run.json
    rocprofv3 --pmc <counters> --kernel-include-regex k_nt_phase -d <dir> -o run --output-format csv -- \
        python3 tools/placement_pmc.py --sets 6 --out <dir>/run.json

One process keeps ``--sets`` stream-buffer sets of the headline solver (262,144 lanes; x0/x1/u0/u1/K1/cs, ~21 GB
each) alive at once and, in this order:
  1. probe: ``--rounds`` round-robin rounds of ``--iters`` iterations of the real pipelined schedule on each set
     (HIP events on the solver's stream), which ranks the sets fast / slow in this process;
  2. swap: on each slow set (> 1.5% behind the fastest), each of its six streams replaced in turn by the fastest
     set's (and the reverse), so a placement effect that lives in one stream (or one pair) shows which;
  3. stream: a plain torch in-place pass (t.mul_(1.0): read + write, no solver) over each stream of the fastest and
     the slowest set, so a property of the memory itself (translation, channel spread) shows without the kernel.
Every block of solver iterations is recorded as a segment (set label, phase launches, ms per iteration, the phase
kernel's own average), in launch order, so that a rocprofv3 --pmc run of the same command (kernels filtered to
k_nt_phase) assigns each counter record to its segment by dispatch order (tools/placement_pmc_parse.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ("x0", "x1", "u0", "u1", "K1", "cs")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--lanes", type=int, default=262144)
    ap.add_argument("--no-swap", action="store_true")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine, F64
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
    sets = [[*sv.x, *sv.u, sv.K1, sv.cs]]
    for _ in range(a.sets - 1):
        sets.append([torch.empty(sh, dtype=F64, device=dev) for sh in sv._stream_shapes])
    segs = []

    def block(label, st, iters):
        sv._set_streams(st)
        sv.reset_timing()
        n0 = sv.launches["phase"]
        sv.max_iters = iters + 1
        sv.init(x0)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(iters):
            sv.iteration()
        ev[1].record()
        torch.cuda.synchronize(dev)
        sv.collect_timing()
        kt = sv.kernel_times()
        ph_ms = sum(kt[k][0] for k in ("phase_odd", "phase_even"))
        ph_n = sum(kt[k][1] for k in ("phase_odd", "phase_even"))
        rec = {"label": label, "phase_launches": sv.launches["phase"] - n0,
               "ms_per_iteration": ev[0].elapsed_time(ev[1]) / iters, "phase_ms": ph_ms / max(ph_n, 1)}
        segs.append(rec)
        print(json.dumps(rec), flush=True)
        return rec

    probe = {}
    for r in range(a.rounds):
        for i, st in enumerate(sets):
            rec = block(f"set{i}", st, a.iters)
            probe[i] = min(probe.get(i, float("inf")), rec["phase_ms"])
    order = sorted(probe, key=probe.get)
    fast, slow = order[0], order[-1]
    print(json.dumps({"probe_phase_ms": probe, "fast": fast, "slow": slow}), flush=True)
    swaps = []
    slows = [i for i in order if probe[i] > probe[fast] * 1.015] if not a.no_swap else []
    for s_i in slows[::-1]:          # every slow set, the slowest first
        for j, nm in enumerate(NAMES):
            hyb = list(sets[s_i])
            hyb[j] = sets[fast][j]
            r1 = block(f"slow{s_i}_with_fast_{nm}", hyb, a.iters)
            hyb = list(sets[fast])
            hyb[j] = sets[s_i][j]
            r2 = block(f"fast_with_slow{s_i}_{nm}", hyb, a.iters)
            swaps.append({"slow_set": s_i, "stream": nm, "slow_with_fast": r1["phase_ms"],
                          "fast_with_slow": r2["phase_ms"]})
        block(f"set{fast}", sets[fast], a.iters)
        block(f"set{s_i}", sets[s_i], a.iters)
    # plain torch streaming pass over each buffer of the fastest and slowest set (no solver kernel)
    stream = {}
    for tag, i in (("fast", fast), ("slow", slow)):
        for j, nm in enumerate(NAMES):
            t = sets[i][j]
            ts = []
            for _ in range(5):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                t.mul_(1.0)
                ev[1].record()
                torch.cuda.synchronize(dev)
                ts.append(ev[0].elapsed_time(ev[1]))
            gbs = 2 * t.numel() * 8 / (min(ts) * 1e-3) / 1e9
            stream[f"{tag}_{nm}"] = {"bytes": 2 * t.numel() * 8, "min_ms": min(ts), "GBs": gbs}
            print(json.dumps({"stream": f"{tag}_{nm}", "GBs": round(gbs, 1)}), flush=True)
    out = {"lanes": a.lanes, "iters": a.iters, "segments": segs, "probe_phase_ms": probe, "fast": fast,
           "slow": slow, "swaps": swaps, "torch_stream": stream,
           "set_ptrs": [[hex(t.data_ptr()) for t in st] for st in sets]}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({"swaps": swaps}), flush=True)


if __name__ == "__main__":
    main()
