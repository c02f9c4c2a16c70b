#!/usr/bin/env python3
"""Can a combination of streams from several stream sets beat every whole set?  (measurement tool)

    python tools/greedy_streams.py --sets 8 --out gpurun_out/r06/greedy/g.json

Keeps --sets stream-buffer sets of the headline solver alive in one process, ranks them with the placement probe
(gym_placement_probe), then from the best set replaces one stream at a time by the same stream of another set
whenever the probe gets faster (coordinate descent over the six streams, two passes), and finally times the real
phase kernel (12-iteration blocks of the pipelined schedule, interleaved rounds) on the probe's best whole set, the
second best, and the best combination.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import ctypes as C
    import torch
    import bench
    from gymnast_optimalcontrol_amd.engine import AcrobotEngine, F64
    from gymnast_optimalcontrol_amd.solver import BatchedNewtonSolver, morton_order
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
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

    def probe(st, reps=2):
        sv._set_streams(st, zero=False)
        ts = []
        for r in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            assert eng.lib.gym_placement_probe(C.byref(sv.batch), r & 1, eng.stream) == 0
            ev[1].record()
            ev[1].synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        return min(ts)

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

    probe(sets[0]); kernel_ms(sets[0])
    pm = [min(probe(st), probe(st)) for st in sets]
    order = sorted(range(a.sets), key=lambda i: pm[i])
    best = list(sets[order[0]])
    src = [order[0]] * 6
    cur = probe(best)
    steps = []
    for _ in range(2):
        for j in range(6):
            for i in range(a.sets):
                if i == src[j]:
                    continue
                trial = list(best)
                trial[j] = sets[i][j]
                t = probe(trial)
                if t < cur * 0.998:
                    best, cur, src[j] = trial, t, i
                    steps.append({"stream": j, "from_set": i, "probe_ms": t})
    print(json.dumps({"probe_sets": pm, "best_set": order[0], "combo_src": src, "combo_probe_ms": cur,
                      "steps": steps}), flush=True)
    cands = {"best_set": sets[order[0]], "second_set": sets[order[1]], "combo": best}
    recs = {k: [] for k in cands}
    for r in range(a.rounds):
        for k in (list(cands) if r % 2 == 0 else list(cands)[::-1]):
            recs[k].append(kernel_ms(cands[k]))
    out = {"probe_sets": pm, "best_set": order[0], "combo_src": src, "combo_probe_ms": cur, "steps": steps,
           "kernel_phase_ms": recs, "kernel_min": {k: min(v) for k, v in recs.items()}}
    print(json.dumps({"kernel_min": out["kernel_min"], "probe_best_set": pm[order[0]], "combo_probe": cur}), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
