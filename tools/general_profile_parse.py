#!/usr/bin/env python3
"""Summarise tools/r04_general_profile.sh: the general (tau1-streaming) and the specialised (tau1-zero) phase kernels
of one process side by side (measurement tool).

    python tools/general_profile_parse.py gpurun_out/r04_general profiles/r04/general

Per instantiation (k_nt_phase<U0Z = true / false, ...>): rocprofv3's average duration over the traced launches,
FETCH_SIZE (x2, the gfx950 correction of MI355X_MICROARCH.md) + WRITE_SIZE per launch against the algorithmic bytes
(bench.algorithmic_bytes: 80,096 / 92,096 B per lane-iteration), the HBM rate both ways, and the SQ counters per
launch (VALU / VMEM / SALU instructions, wave cycles, busy cycles, waits).  Writes summary.json and summary.md.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def variant(name: str):
    """'general' / 'u0zero' for a k_nt_phase instantiation, else None."""
    if "k_nt_phase" not in name:
        return None
    targs = name.split("k_nt_phase<", 1)[1].split(">", 1)[0].replace(" ", "")
    return "u0zero" if targs.startswith("true") else "general"


def find(path, pattern):
    hits = glob.glob(os.path.join(path, "**", pattern), recursive=True)
    return hits[0] if hits else None


def steady_rows(rows, key):
    """Drop each variant's first dispatch of a solve (the prologue phase: one half's sweep only) -- approximated by
    dropping dispatches whose value is below half of the variant's median."""
    by = defaultdict(list)
    for r in rows:
        v = variant(r["Kernel_Name"])
        if v:
            by[v].append(r)
    out = {}
    for v, rs in by.items():
        vals = sorted(float(r[key]) for r in rs)
        med = vals[len(vals) // 2]
        out[v] = [r for r in rs if float(r[key]) >= 0.5 * med]
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    from bench import algorithmic_bytes
    B = 262144
    algo = {"u0zero": (B // 2) * algorithmic_bytes(501, True)["iteration"],
            "general": (B // 2) * algorithmic_bytes(501, False)["iteration"]}
    res = {v: {"algorithmic_bytes_per_launch": float(a)} for v, a in algo.items()}
    tr = find(os.path.join(src, "trace"), "*kernel_trace.csv")
    if tr:
        rows = list(csv.DictReader(open(tr)))
        with open(os.path.join(dst, "phase_launches.csv"), "w", newline="") as f:   # the phase kernels' rows only
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(r for r in rows if variant(r["Kernel_Name"]))
        for r in rows:
            r["dur"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for v, rs in steady_rows(rows, "dur").items():
            d = [r["dur"] for r in rs]
            res[v]["trace_avg_us"] = sum(d) / len(d) / 1e3
            res[v]["trace_launches"] = len(d)
            res[v]["algorithmic_GBs"] = algo[v] / (res[v]["trace_avg_us"] * 1e-6) / 1e9
            res[v]["frac_of_8TBs"] = res[v]["algorithmic_GBs"] / 8000.0
    st = find(os.path.join(src, "trace"), "*kernel_stats.csv")
    if st:
        shutil.copy(st, os.path.join(dst, "kernel_stats.csv"))
    for sub in ("fetch", "write", "sq"):
        cc = find(os.path.join(src, sub), "*counter_collection.csv")
        if not cc:
            continue
        shutil.copy(cc, os.path.join(dst, f"{sub}_counter_collection.csv"))
        rows = list(csv.DictReader(open(cc)))
        agg = defaultdict(lambda: defaultdict(list))
        for r in rows:
            v = variant(r["Kernel_Name"])
            if v:
                agg[v][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for v, cs in agg.items():
            for c, vals in cs.items():
                xs = sorted(x for _, x in vals)
                med = xs[len(xs) // 2]
                keep = [x for x in xs if x >= 0.5 * med]       # prologue phases out
                res[v][c] = sum(keep) / len(keep)
    for v, d in res.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
            d["traffic_over_algorithmic"] = d["hbm_bytes_per_launch"] / d["algorithmic_bytes_per_launch"]
            if "trace_avg_us" in d:
                d["measured_GBs"] = d["hbm_bytes_per_launch"] / (d["trace_avg_us"] * 1e-6) / 1e9
    json.dump(res, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    keys = ["trace_avg_us", "trace_launches", "algorithmic_bytes_per_launch", "algorithmic_GBs", "frac_of_8TBs",
            "hbm_bytes_per_launch", "traffic_over_algorithmic", "measured_GBs", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY",
            "GRBM_GUI_ACTIVE"]
    lines = ["| quantity | u0zero (specialised) | general | general / u0zero |", "|---|---|---|---|"]
    for k in keys:
        a, b = res.get("u0zero", {}).get(k), res.get("general", {}).get(k)
        if a is None and b is None:
            continue
        ratio = f"{b / a:.3f}" if a and b else ""
        fa = f"{a:.4g}" if isinstance(a, float) else str(a)
        fb = f"{b:.4g}" if isinstance(b, float) else str(b)
        lines.append(f"| {k} | {fa} | {fb} | {ratio} |")
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
