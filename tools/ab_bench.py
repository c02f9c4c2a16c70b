#!/usr/bin/env python3
"""Interleaved A/B timing of library variants in ONE process on one device (measurement tool).

    python tools/ab_bench.py --batch 262144 --rounds 3 lib_a.so lib_b.so:serial lib_b.so:pipe:nou0z ...
(":serial" / ":pipe" / ":run" (persistent) select the schedule, ":nou0z" disables the tau1 = 0 stream skipping, ":ck" enables the
state checkpointing (the solver's default is off), ":noreorder" the Morton-order lane grouping of
solve(), ":notime" the HIP-event kernel timing; default:
the solver's choice)
Each round runs one full batched solve per variant on the SAME device buffers (one solver whose
kernel library is swapped), so buffer placement -- worth +-4% on its own -- is held fixed; prints
per-variant median backward / trial kernel times and whole-solve throughput.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--max-iters", type=int, default=5000)
    ap.add_argument("--spread", type=float, default=0.5, help="th0 ~ U(+-spread) (1.5: the stress workload)")
    ap.add_argument("--sync-every", type=int, default=4, help="host synchronisation cadence (bench.py's default)")
    ap.add_argument("--box", action="store_true", help="record SCLK / power over each solve (sysfs)")
    a = ap.parse_args()
    import torch
    from bench import load_refs, make_x0
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    x_ref, u_ref = load_refs()
    x0 = make_x0(a.batch, spread=a.spread)
    from gymnast_optimalcontrol_amd import _lib
    def split(spec):
        path, *opts = spec.split(":")
        sched = {"serial": False, "pipe": True, "run": "run"}
        return (os.path.abspath(path), next((sched[o] for o in opts if o in sched), None), "nou0z" not in opts,
                "ck" in opts, "noreorder" not in opts, "notime" in opts)
    eng = AcrobotEngine(lib_path=split(a.libs[0])[0])
    s = BatchedNewtonSolver(eng, x_ref, u_ref, a.batch, tol=1e-4, gamma_0=0.1).enable_timing()
    default_pipe = s.pipeline
    default_u0z = s.u0_zero
    xd = eng.t(x0)
    libs = {p: _lib.load(split(p)[0]) for p in a.libs}
    res = {p: {"bwd": [], "trial": [], "its": [], "sec": [], "sclk": [], "power": []} for p in a.libs}
    samp = None
    if a.box:   # sysfs clocks / power over each solve (tools/box_state.py)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from box_state import Sampler
        samp = Sampler(0, 0.05).start()
    for r in range(a.rounds + 1):
        for p in a.libs:
            eng.lib = libs[p]
            _, sched, u0z, ck, reorder, notime = split(p)
            s.reorder = reorder
            s.persistent = sched == "run"
            s.pipeline = default_pipe if sched in (None, "run") else sched
            s.u0_zero = default_u0z and u0z
            s.checkpoint = ck and not s.persistent
            s.batch.flags = (_lib.FLAG_U0_ZERO if s.u0_zero else 0) | (_lib.FLAG_X_CKPT if s.checkpoint else 0)
            s.reset_timing()
            s.batch.timing = None if notime else C.pointer(s.timing)
            if samp is not None:
                torch.cuda.synchronize()
                samp.mark()
            out = s.solve(xd, a.max_iters, sync_every=a.sync_every)
            if samp is not None:
                torch.cuda.synchronize()
                w = samp.window()
                res[p]["sclk"].append(w.get("dpm_sclk_mhz", [float("nan")])[0])
                res[p]["power"].append(w.get("power_ppt_in_w", [float("nan")])[0])
            kt = s.kernel_times()
            if notime:
                kt = {k: (0.0, 0) for k in kt}
            if r == 0:
                continue   # warm-up round
            if notime:
                res[p]["bwd"].append(0.0)
                res[p]["trial"].append(0.0)
            elif kt["run"][1]:     # persistent: the run launch(es) as "bwd", nothing as "trial"
                res[p]["bwd"].append(kt["run"][0] / kt["run"][1])
                res[p]["trial"].append(0.0)
            elif kt["backward"][1]:
                res[p]["bwd"].append(kt["backward"][0] / kt["backward"][1])
                res[p]["trial"].append(kt["trial"][0] / kt["trial"][1])
            else:   # pipelined: report the phase pair as "bwd" (odd) / "trial" (even)
                res[p]["bwd"].append(kt["phase_odd"][0] / max(1, kt["phase_odd"][1]))
                res[p]["trial"].append(kt["phase_even"][0] / max(1, kt["phase_even"][1]))
            res[p]["its"].append(out.lane_iterations / out.seconds)
            res[p]["sec"].append(out.seconds)
    for p in a.libs:
        d = res[p]
        print(json.dumps({"lib": os.path.basename(p), "bwd_ms": float(np.median(d["bwd"])),
                          "trial_ms": float(np.median(d["trial"])), "Mits": float(np.median(d["its"])) / 1e6,
                          "sclk_mhz": [round(v) for v in d["sclk"]], "power_w": [round(v) for v in d["power"]],
                          "bwd_all": [round(v, 4) for v in d["bwd"]], "trial_all": [round(v, 4) for v in d["trial"]]}),
              flush=True)


if __name__ == "__main__":
    main()
