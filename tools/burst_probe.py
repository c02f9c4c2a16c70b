#!/usr/bin/env python3
"""Energy per byte of the solver's stream pattern against a two-stage-block layout (measurement tool).

    hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/burst_probe.hip -o tools/libburst_probe.so
    python tools/burst_probe.py --seconds 4 --rounds 2 --out gpurun_out/r05/burst/probe.json

Runs tools/burst_probe.hip's k_sb1 (the phase kernel's per-stage wave blocks) and k_sb2 (two stages per block, both
loaded together) back to back for --seconds each, alternating, while tools/box_state.py samples power and clocks;
reports TB/s, mean power, SCLK and the energy per byte above the idle power sampled first.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "libburst_probe.so"))
    a = ap.parse_args()
    import torch
    from box_state import Sampler
    torch.cuda.set_device(0)
    lib = C.CDLL(a.lib)
    lib.bp_run.argtypes = [C.c_int] + [C.c_void_p] * 4 + [C.c_int64, C.c_int, C.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    samp = Sampler(0, 0.05).start()
    B, T = 262144, 500
    samp.mark()
    time.sleep(2.0)
    idle = samp.window().get("power_ppt_in_w", [0.0])[0]
    in2 = torch.ones((T, 2, B, 2), dtype=torch.float64, device="cuda")
    in1 = torch.ones((T, B), dtype=torch.float64, device="cuda")
    out2, out1 = torch.empty_like(in2), torch.empty_like(in1)
    nbytes = B * T * 80
    ptrs = (in2.data_ptr(), in1.data_ptr(), out2.data_ptr(), out1.data_ptr())
    res = {"idle_w": idle, "lanes": B, "stages": T, "runs": []}
    for v in (1, 2):
        for _ in range(3):
            assert lib.bp_run(v, *ptrs, B, T, stream) == 0
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for v in (1, 2):
            samp.mark()
            t0 = time.perf_counter()
            n = 0
            while time.perf_counter() - t0 < a.seconds:
                assert lib.bp_run(v, *ptrs, B, T, stream) == 0
                n += 1
                if n % 8 == 0:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            w = samp.window()
            rate = n * nbytes / dt
            p = w.get("power_ppt_in_w", [0.0])[0]
            rec = {"variant": f"k_sb{v}", "round": r, "TBs": rate / 1e12, "ms_per_launch": 1e3 * dt / n,
                   "power_w": w.get("power_ppt_in_w"), "sclk_mhz": w.get("dpm_sclk_mhz"),
                   "pj_per_byte": 1e12 * p / rate, "pj_per_byte_above_idle": 1e12 * (p - idle) / rate}
            res["runs"].append(rec)
            print(json.dumps(rec), flush=True)
    samp.stop()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
