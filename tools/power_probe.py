#!/usr/bin/env python3
"""Energy per byte and per fp64 instruction on this MI355X, next to the phase kernel's (measurement tool).

    hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/power_probe.hip -o tools/libpower_probe.so
    python tools/power_probe.py --seconds 4 --out gpurun_out/r05/power/probe.json

For each load (tools/power_probe.hip: k_stream = the phase kernel's HBM streams with no arithmetic, k_valu = fp64
FMAs with no memory traffic; then the real headline solve through bench.NewtonLeg) it runs back to back for
--seconds while tools/box_state.py samples power and clocks, and reports the achieved rate, the mean power, SCLK,
the PPT-throttled share (amd-smi) and the energy per unit (power over rate, and the amd-smi energy counter over the
work).  Idle power is sampled first, so dynamic energy per unit = (power - idle) / rate.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "libpower_probe.so"))
    a = ap.parse_args()
    import torch
    from box_state import Sampler, smi_counters, smi_delta
    torch.cuda.set_device(0)
    lib = C.CDLL(a.lib)
    lib.pp_stream.argtypes = [C.c_void_p] * 4 + [C.c_int64, C.c_int, C.c_void_p]
    lib.pp_valu.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_double, C.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    samp = Sampler(0, 0.05).start()
    bdf = os.path.basename(samp.dev) if samp.dev else None
    B, T = 262144, 500
    out = {"lanes": B, "stages": T}

    def window(run, seconds):
        torch.cuda.synchronize()
        s0 = smi_counters(bdf=bdf)
        samp.mark()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < seconds:
            run()
            n += 1
            if n % 8 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        w = samp.window()
        d = smi_delta(s0, smi_counters(bdf=bdf))
        return n, dt, w, d

    samp.mark()
    time.sleep(2.0)
    idle = samp.window()
    out["idle"] = {"power_w": idle.get("power_ppt_in_w"), "sclk_mhz": idle.get("dpm_sclk_mhz")}
    p_idle = idle.get("power_ppt_in_w", [0.0])[0]
    print("idle", out["idle"], flush=True)

    in2 = torch.ones((T, 2, B, 2), dtype=torch.float64, device="cuda")
    in1 = torch.ones((T, B), dtype=torch.float64, device="cuda")
    out2, out1 = torch.empty_like(in2), torch.empty_like(in1)
    bytes_per_launch = B * T * 80
    for _ in range(3):
        lib.pp_stream(in2.data_ptr(), in1.data_ptr(), out2.data_ptr(), out1.data_ptr(), B, T, stream)
    n, dt, w, d = window(lambda: lib.pp_stream(in2.data_ptr(), in1.data_ptr(), out2.data_ptr(), out1.data_ptr(), B, T,
                                               stream), a.seconds)
    rate = n * bytes_per_launch / dt
    p = w.get("power_ppt_in_w", [0.0])[0]
    out["stream"] = {"GBs": rate / 1e9, "ms_per_launch": 1e3 * dt / n, "power_w": w.get("power_ppt_in_w"),
                     "sclk_mhz": w.get("dpm_sclk_mhz"), "temp_mem_c": w.get("temp_mem_c"), "smi": d,
                     "pj_per_byte": 1e12 * p / rate, "pj_per_byte_dynamic": 1e12 * (p - p_idle) / rate}
    print("stream", json.dumps(out["stream"]), flush=True)
    del in2, in1, out2, out1

    vo = torch.empty(B, dtype=torch.float64, device="cuda")
    n_iter = 2000
    instr_per_launch = (B // 64) * n_iter * 32         # fp64 FMA wave-instructions
    for _ in range(3):
        lib.pp_valu(vo.data_ptr(), B, n_iter, 0.999, stream)
    n, dt, w, d = window(lambda: lib.pp_valu(vo.data_ptr(), B, n_iter, 0.999, stream), a.seconds)
    rate = n * instr_per_launch / dt
    p = w.get("power_ppt_in_w", [0.0])[0]
    out["valu"] = {"fp64_wave_instr_per_s": rate, "ms_per_launch": 1e3 * dt / n, "power_w": w.get("power_ppt_in_w"),
                   "sclk_mhz": w.get("dpm_sclk_mhz"), "smi": d, "nj_per_wave_instr": 1e9 * p / rate,
                   "nj_per_wave_instr_dynamic": 1e9 * (p - p_idle) / rate,
                   "issue_cycles_per_instr_per_simd": (w.get("dpm_sclk_mhz", [0.0])[0] * 1e6 * 1024) / rate}
    print("valu", json.dumps(out["valu"]), flush=True)

    # the headline solve itself, as bench.py's main leg builds it
    import argparse as _ap
    import bench
    from gymnast_optimalcontrol_amd import distributed as gd
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine
    x_ref, u_ref = bench.load_refs()
    ns = _ap.Namespace(spread=0.5, schedule="auto", chunk=128, split_waves="on", tail_lanes=None, compact="auto",
                       max_iters=5000, sync_every=4)
    leg = bench.NewtonLeg(ns, gd, AcrobotEngine(), x_ref, u_ref, B, False)
    leg.solver.solve(leg.x0_dev, 5000, sync_every=4)
    its = [0]

    def solve():
        r = leg.solver.solve(leg.x0_dev, 5000, sync_every=4)
        its[0] += r.lane_iterations
    n, dt, w, d = window(solve, max(a.seconds, 3.5))
    rate = its[0] / dt
    p = w.get("power_ppt_in_w", [0.0])[0]
    out["headline"] = {"lane_it_per_s": rate, "power_w": w.get("power_ppt_in_w"), "sclk_mhz": w.get("dpm_sclk_mhz"),
                       "smi": d, "uj_per_lane_it": 1e6 * p / rate, "uj_per_lane_it_dynamic": 1e6 * (p - p_idle) / rate,
                       "bytes_per_lane_it": 80096, "valu_wave_instr_per_lane_it": 724082227.2 * 809 / 102862555}
    print("headline", json.dumps(out["headline"]), flush=True)
    leg.free()
    # the general path (tau1 planes streamed: 92,096 B per lane-iteration) on the same box
    legg = bench.NewtonLeg(ns, gd, AcrobotEngine(), x_ref, u_ref, B, False, u0_zero=False)
    legg.solver.solve(legg.x0_dev, 5000, sync_every=4)
    its[0] = 0

    def solve_g():
        r = legg.solver.solve(legg.x0_dev, 5000, sync_every=4)
        its[0] += r.lane_iterations
    n, dt, w, d = window(solve_g, max(a.seconds, 3.5))
    rate = its[0] / dt
    p = w.get("power_ppt_in_w", [0.0])[0]
    out["general"] = {"lane_it_per_s": rate, "power_w": w.get("power_ppt_in_w"), "sclk_mhz": w.get("dpm_sclk_mhz"),
                      "smi": d, "uj_per_lane_it": 1e6 * p / rate, "uj_per_lane_it_dynamic": 1e6 * (p - p_idle) / rate,
                      "bytes_per_lane_it": 92096}
    for k, b in (("headline", 80096), ("general", 92096)):     # whole-solve bytes/s (launch gaps included)
        out[k]["solve_GBs"] = out[k]["lane_it_per_s"] * b / 1e9
    print("general", json.dumps(out["general"]), flush=True)
    print("solve GB/s: stream probe %.0f, headline %.0f, general %.0f" % (out["stream"]["GBs"],
          out["headline"]["solve_GBs"], out["general"]["solve_GBs"]), flush=True)
    samp.stop()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
