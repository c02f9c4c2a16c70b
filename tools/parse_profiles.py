#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of tools/profile.sh into profiles/ (measurement tool).

    python tools/parse_profiles.py gpurun_out/prof profiles r01

Writes:
  profiles/<tag>_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary of the bench run (copied)
  profiles/<tag>_pmc.json           -- per-kernel PMC averages (FETCH_SIZE, WRITE_SIZE, SQ_* ...)
  profiles/pmc_traffic.json         -- HBM bytes per launch of the solver kernels, read by bench.py:
                                       (2 * FETCH_SIZE + WRITE_SIZE) * 1024, gfx950 correction of
                                       MI355X_MICROARCH.md (FETCH_SIZE reports half of a wide streaming read)
  profiles/<tag>_summary.md         -- the table quoted in DESIGN.md
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0].split("::")[-1].strip()
    return n.split("<")[0]          # k_nt_phase<true> -> k_nt_phase


def load_pmc(path):
    agg = defaultdict(list)
    if not os.path.exists(path):
        return agg
    rows = list(csv.DictReader(open(path)))
    # keep the main leg's launches only: per kernel the most common grid size (bench.py's process warm-up runs a small
    # batch of the same kernels first)
    grids = defaultdict(lambda: defaultdict(int))
    for r in rows:
        grids[short(r["Kernel_Name"])][r.get("Grid_Size", "")] += 1
    mode = {k: max(g, key=g.get) for k, g in grids.items()}
    rows = [r for r in rows if r.get("Grid_Size", "") == mode[short(r["Kernel_Name"])]]
    first_phase = None
    for r in rows:
        k = short(r["Kernel_Name"])
        if k == "k_nt_phase":
            # the prologue phase (p = 0, backward of one half only) is not representative
            did = int(r["Dispatch_Id"])
            first_phase = did if first_phase is None else min(first_phase, did)
    for r in rows:
        k = short(r["Kernel_Name"])
        if k == "k_nt_phase" and int(r["Dispatch_Id"]) == first_phase:
            continue
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main():
    src, dst, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    os.makedirs(dst, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    kstats = []
    if os.path.exists(stats_csv):
        shutil.copy(stats_csv, os.path.join(dst, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats_csv)):
            kstats.append((short(r["Name"]), int(r["Calls"]), float(r["AverageNs"]), float(r["Percentage"])))
    pmc = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_valu", "pmc_stall"):
        for (k, c), v in load_pmc(os.path.join(src, sub, "run_counter_collection.csv")).items():
            pmc.setdefault(k, {})[c] = {"mean": sum(v) / len(v), "n": len(v)}
    json.dump(pmc, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    traffic = {}
    for k, d in pmc.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            fetch = d["FETCH_SIZE"]["mean"] * 1024.0
            write = d["WRITE_SIZE"]["mean"] * 1024.0
            traffic[k] = {"fetch_bytes_raw": fetch, "fetch_bytes_corrected": 2 * fetch, "write_bytes": write,
                          "hbm_bytes_per_launch": 2 * fetch + write}
    # algorithmic bytes per launch of the profiled run (tools/profile.sh: 262,144 lanes, 20 iterations, every
    # lane active): a steady-state phase = sweep of one half + trial of the other half
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import algorithmic_bytes
    ab = algorithmic_bytes(501)
    lanes = 262144
    algo = {"k_nt_phase": (lanes // 2) * ab["iteration"], "k_nt_backward": lanes * ab["backward"],
            "k_nt_trial": lanes * ab["trial"]}
    for k, v in traffic.items():
        if k in algo:
            v["algorithmic_bytes_per_launch"] = float(algo[k])
            v["traffic_over_algorithmic"] = v["hbm_bytes_per_launch"] / algo[k]
    # fp64 VALU issue estimate: SQ_INSTS_VALU wave-instructions x 4 cycles (a wave64 fp64 FMA on a 32-wide SIMD;
    # 32-bit VALU takes 2, so this is an upper estimate) over the SIMD-cycles of the launch; GRBM_GUI_ACTIVE is
    # summed over the 8 XCDs (3.2e7 for a ~1.7 ms launch at 2.4 GHz), 1024 SIMDs in all
    for k, d in pmc.items():
        if k in traffic and "SQ_INSTS_VALU" in d and "GRBM_GUI_ACTIVE" in d:
            valu, gui = d["SQ_INSTS_VALU"]["mean"], d["GRBM_GUI_ACTIVE"]["mean"]
            traffic[k]["sq_insts_valu_per_launch"] = valu
            traffic[k]["grbm_gui_active_per_launch"] = gui
            traffic[k]["valu_busy_upper_est"] = valu * 4.0 / (1024.0 * gui / 8.0)
    # bench.py names the dominant kernel "phase" (pipelined) or "backward" / "trial" (serial)
    alias = {"k_nt_phase": "phase", "k_nt_backward": "backward", "k_nt_trial": "trial"}
    out = {alias.get(k, k): v for k, v in traffic.items()}
    out["_note"] = ("per launch, from rocprofv3 --pmc passes of tools/profile.sh; FETCH_SIZE doubled per the gfx950 "
                    "calibration in MI355X_MICROARCH.md (HBM section); the prologue phase is excluded")
    json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    lines = [f"# rocprofv3 summary ({tag})", "", "Kernel trace (`--kernel-trace --stats`, one bench step + warmup):", "",
             "| kernel | calls | avg us | % time |", "|---|---|---|---|"]
    for k, n, avg, pct in kstats[:12]:
        lines.append(f"| {k} | {n} | {avg / 1e3:.1f} | {pct:.2f} |")
    lines += ["", "PMC per launch (separate passes, 20-iteration solve):", "",
              "| kernel | FETCH_SIZE x2 (GB) | WRITE_SIZE (GB) | SQ_INSTS_VALU | SQ_WAVES | GRBM_GUI_ACTIVE |",
              "|---|---|---|---|---|---|"]
    for k, d in sorted(pmc.items()):
        g = lambda c: d.get(c, {}).get("mean", float("nan"))  # noqa: E731
        lines.append(f"| {k} | {2 * g('FETCH_SIZE') * 1024 / 1e9:.3f} | {g('WRITE_SIZE') * 1024 / 1e9:.3f} | "
                     f"{g('SQ_INSTS_VALU'):.3e} | {g('SQ_WAVES'):.0f} | {g('GRBM_GUI_ACTIVE'):.3e} |")
    open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
