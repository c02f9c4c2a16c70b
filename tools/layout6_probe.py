#!/usr/bin/env python3
"""Six separate streams against interleaved records, with the phase kernel's access pattern and no arithmetic
(measurement tool; tools/layout6_probe.hip, profiles/r06/README.md "layout6").

    hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/layout6_probe.hip -o tools/liblayout6_probe.so
    python tools/layout6_probe.py --sep-sets 4 --rec-sets 3 --seconds 1.5 --rounds 2 --out gpurun_out/r06/l6/l6.json

Allocates --sep-sets sets of the solver's six streams (262,144 lanes, T = 500) and --rec-sets record arrays, all
alive at once, and runs each back to back for --seconds per round (buffers alternating as the solver's iterations
do), rounds interleaved; reports TB/s of the 10.49 GB each launch moves (the phase kernel's algorithmic bytes), the
power and SCLK over the run and the energy per byte above idle (tools/box_state.py).
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
    ap.add_argument("--sep-sets", type=int, default=4)
    ap.add_argument("--rec-sets", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools", "liblayout6_probe.so"))
    a = ap.parse_args()
    import torch
    from box_state import Sampler
    torch.cuda.set_device(0)
    lib = C.CDLL(a.lib)
    lib.l6_run.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.c_int64, C.c_int, C.c_int, C.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    B, T = 262144, 500
    N = T + 1
    samp = Sampler(0, 0.05).start()
    samp.mark()
    time.sleep(1.5)
    idle = samp.window().get("power_ppt_in_w", [0.0])[0]
    f64 = dict(dtype=torch.float64, device="cuda")
    shapes = [(N, 2, B, 2), (N, 2, B, 2), (T, 2, B), (T, 2, B), (T, 2, B, 2), (T, 2, B)]
    sets = []
    for i in range(a.sep_sets):
        st = [torch.ones(sh, **f64) for sh in shapes]
        sets.append(("sep", i, st, (C.c_void_p * 6)(*[t.data_ptr() for t in st])))
    rec = int(lib.l6_rec_doubles())
    for i in range(a.rec_sets):
        r = torch.ones((N * (B // 64) * rec,), **f64)
        sets.append(("rec", i, [r], (C.c_void_p * 6)(r.data_ptr(), 0, 0, 0, 0, 0)))
    nbytes = B * T * 80
    for kind, _, _, p in sets:                    # warm-up
        for cb in (0, 1):
            assert lib.l6_run(0 if kind == "sep" else 1, p, B, T, cb, stream) == 0
    torch.cuda.synchronize()
    out = {"idle_w": idle, "lanes": B, "stages": T, "bytes_per_launch": nbytes, "runs": []}
    for r in range(a.rounds):
        order = sets if r % 2 == 0 else sets[::-1]
        for kind, i, _, p in order:
            samp.mark()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            t0 = time.perf_counter()
            n = 0
            while time.perf_counter() - t0 < a.seconds:
                assert lib.l6_run(0 if kind == "sep" else 1, p, B, T, n & 1, stream) == 0
                n += 1
                if n % 16 == 0:
                    torch.cuda.synchronize()
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / n
            w = samp.window()
            pw = w.get("power_ppt_in_w", [0.0])[0]
            rate = nbytes / (ms * 1e-3)
            rec_ = {"layout": kind, "set": i, "round": r, "ms_per_launch": ms, "TBs": rate / 1e12,
                    "power_w": w.get("power_ppt_in_w"), "sclk_mhz": w.get("dpm_sclk_mhz"),
                    "pj_per_byte_above_idle": 1e12 * (pw - idle) / rate}
            out["runs"].append(rec_)
            print(json.dumps(rec_), flush=True)
    samp.stop()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
