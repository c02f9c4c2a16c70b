#!/usr/bin/env python3
"""Leg-order probe: does the headline leg run its phase kernel slower than later legs of the
same process, and why?

    python tools/leg_order.py --order cfg3:5:20,cfg4:1:2,general:1:2,cfg3:1:5 --out gpurun_out/r05/leg/a.jsonl

Each item is ``leg[:warmup:steps]``.  Legs: cfg3 (bench.py's headline leg), general (u0_zero off), cfg3nc (the
headline with the candidate scratch off), cfg3ck (the headline with state checkpointing), *ser (the serial schedule: sweep and trial launches apart), cfg4 (1,048,576 lanes), stress (spread 1.5), pad<GB> (allocate and hold
a buffer of that many GB: shifts where later legs' buffers land), unpad (release the pads), idle<s> (sleep).
Per solve one JSON line: leg, solve index, wall seconds, lane-iterations, the phase kernel's average ms (HIP events
on the solver's stream) and the GB/s it implies, and the box state over that solve (tools/box_state.py: DPM clocks,
power, temperatures, mean / min / max).  bench.NewtonLeg builds every leg exactly as bench.py does.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--sync-every", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    from box_state import Sampler, smi_counters, smi_delta
    from gymnast_optimalcontrol_amd import distributed as gd
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver
    gd.init_process_group()
    torch.cuda.set_device(0)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    fout = open(a.out, "w")
    samp = Sampler(0, 0.1).start()
    print("sysfs", samp.dev, sorted(samp.ch.files) if samp.ch else None, flush=True)
    fout.write(json.dumps({"sysfs_dir": samp.dev, "channels": sorted(samp.ch.files) if samp.ch else None,
                           "snapshot": samp.snapshot()}) + "\n")
    x_ref, u_ref = bench.load_refs()
    N = x_ref.shape[0]
    eng = AcrobotEngine()
    pads = []
    held = []

    def contig_arena(n):
        """n doubles of physically contiguous VRAM (hipExtMallocWithFlags(hipDeviceMallocContiguous)), as a torch
        tensor through __cuda_array_interface__ (kept allocated for the process)."""
        import ctypes as C
        lib = C.CDLL(os.path.join(ROOT, "tools", "libcontig_alloc.so"))
        p = C.c_void_p()
        rc = lib.ca_malloc(C.c_int64(8 * n), 4, C.byref(p))
        print("contiguous allocation of", 8 * n, "bytes: rc", rc, hex(p.value or 0), flush=True)
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags(contiguous) failed: {rc}")

        class Blob:
            __cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (p.value, False), "version": 2,
                                        "strides": None}
        t = torch.as_tensor(Blob(), device="cuda")
        assert t.data_ptr() == p.value
        held.append((lib, p))
        return t
    ns = argparse.Namespace(spread=0.5, schedule="auto", chunk=128, split_waves="on", tail_lanes=None,
                            compact="auto", max_iters=5000, sync_every=a.sync_every)
    for item in a.order.split(","):
        parts = item.split(":")
        name = parts[0]
        if name.startswith("pad"):
            gb = float(name[3:])
            pads.append(torch.empty(int(gb * 2**30 // 8), dtype=torch.float64, device="cuda"))
            print("pad", gb, "GB held", flush=True)
            continue
        if name == "unpad":
            pads.clear()
            torch.cuda.empty_cache()
            continue
        if name.startswith("idle"):
            samp.mark()
            time.sleep(float(name[4:]))
            rec = {"leg": name, "box": samp.window()}
            fout.write(json.dumps(rec) + "\n"); fout.flush()
            print(json.dumps(rec), flush=True)
            continue
        warm = int(parts[1]) if len(parts) > 1 else 1
        steps = int(parts[2]) if len(parts) > 2 else 3
        total = 1048576 if name == "cfg4" else 262144
        spread = 1.5 if name == "stress" else 0.5
        old = BatchedNewtonSolver.CAND_SLOTS
        if name == "cfg3nc":
            BatchedNewtonSolver.CAND_SLOTS = 0
        t_build = time.perf_counter()
        kw = {"checkpoint": True} if name == "cfg3ck" else {"arena": True} if name == "cfg3arena" else {}
        if name == "cfg3contig":
            kw = {"arena": contig_arena}
        if name == "cfg3sel":
            kw = {"placement_trials": 3}
        ns.schedule = "serial" if name.endswith("ser") else "auto"
        leg = bench.NewtonLeg(ns, gd, eng, x_ref, u_ref, total, True,
                              u0_zero=False if name.startswith("general") else None, spread=spread, **kw)
        BatchedNewtonSolver.CAND_SLOTS = old
        sv = leg.solver
        ptrs = {k: hex(t.data_ptr()) for k, t in (("x0", sv.x[0]), ("x1", sv.x[1]), ("u0", sv.u[0]), ("u1", sv.u[1]),
                                                   ("K1", sv.K1), ("cs", sv.cs))}
        if sv._cand_scratch is not None:
            ptrs["cand"] = hex(sv._cand_scratch.data_ptr())
        print(name, "buffers", ptrs, "built in", round(time.perf_counter() - t_build, 2), "s", "placement",
              sv.placement, flush=True)
        res = None
        t_smi = time.perf_counter()
        smi0 = smi_counters(bdf=os.path.basename(samp.dev) if samp.dev else None)
        t_smi = time.perf_counter() - t_smi
        t_leg = time.perf_counter()
        for i in range(warm + steps):
            res = None
            sv.reset_timing()
            torch.cuda.synchronize()
            samp.mark()
            t0 = time.perf_counter()
            res = sv.solve(leg.x0_dev, 5000, sync_every=a.sync_every)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            kt = sv.kernel_times()
            ph_ms = sum(kt[k][0] for k in ("phase_odd", "phase_even") if k in kt)
            ph_n = sum(kt[k][1] for k in ("phase_odd", "phase_even") if k in kt)
            its = res.lane_iterations - res.tail_lane_iterations - res.lowocc_lane_iterations
            ab = bench.algorithmic_bytes(N, sv.u0_zero)["iteration"]
            per_launch = its * ab / max(sv.launches["phase"], 1)
            avg = ph_ms / max(ph_n, 1)
            if not ph_n and kt.get("backward", (0, 0))[1]:   # serial schedule: the sweep and trial launches
                bw, tr = kt["backward"], kt["trial"]
                bb = bench.algorithmic_bytes(N, sv.u0_zero)
                per_b, per_t = its * bb["backward"] / bw[1], its * bb["trial"] / tr[1]
                avg = (bw[0] + tr[0]) / bw[1]          # one iteration's two launches
                ph_n = bw[1]
                per_launch = its * ab / bw[1]
                print(f"  serial: backward {bw[0] / bw[1]:.4f} ms ({per_b / (bw[0] / bw[1]) / 1e6:.0f} GB/s), trial "
                      f"{tr[0] / tr[1]:.4f} ms ({per_t / (tr[0] / tr[1]) / 1e6:.0f} GB/s)", flush=True)
            rec = {"leg": name, "i": i, "warmup": i < warm, "wall_s": dt, "lane_its": res.lane_iterations,
                   "it_per_s": res.lane_iterations / dt, "phase_avg_ms": avg, "phase_launches": ph_n,
                   "phase_GBs": per_launch / (avg * 1e-3) / 1e9 if ph_n else None,
                   "frac": per_launch / (avg * 1e-3) / 1e9 / 8000 if ph_n else None, "box": samp.window()}
            fout.write(json.dumps(rec) + "\n"); fout.flush()
            b = rec["box"]
            print(f"{name} {i} {'W' if i < warm else 'T'} {dt:.3f}s {rec['it_per_s'] / 1e6:.2f}M it/s phase "
                  f"{avg:.4f} ms frac {rec['frac'] or 0:.4f} | "
                  + " ".join(f"{k}={v[0]}" for k, v in b.items() if isinstance(v, list)), flush=True)
        smi = smi_delta(smi0, smi_counters(bdf=os.path.basename(samp.dev) if samp.dev else None))
        smi["seconds"] = round(time.perf_counter() - t_leg, 2)
        smi["smi_call_s"] = round(t_smi, 2)
        fout.write(json.dumps({"leg": name, "smi": smi}) + "\n"); fout.flush()
        print(name, "smi", smi, flush=True)
        res = None
        leg.free()
    samp.stop()
    fout.close()


if __name__ == "__main__":
    main()
