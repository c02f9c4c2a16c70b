#!/usr/bin/env python3
"""Assign the PMC records of a tools/placement_pmc.py run to its segments and compare fast and slow placements.

    python tools/placement_pmc_parse.py <rocprofv3 -d dir> <run.json> <summary.json>

Reads the k_nt_phase dispatches of the pass, from `run_counter_collection.csv` (counters summed over their hardware
instances) and, when the pass also wrote a rocpd database (`--output-format rocpd`), the per-instance values
(rocpd_pmc_event rows, one per hardware instance, in instance order within a dispatch).  Dispatches are matched to
the run's segments by order (each segment = one init + iterations on one stream set; the counts are in run.json).
Writes per segment the mean of every counter per dispatch and, per instance, the spread (max / mean, coefficient of
variation) of each counter over the instances, with the segment's phase time, so fast and slow sets compare side by
side.  Only the steady phases of a segment are used (its first, the prologue, is dropped).
"""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("::")[-1].strip().split("<")[0]


def csv_records(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(dict)
    for r in rows:
        if short(r["Kernel_Name"]) != "k_nt_phase":
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def db_records(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        return None, None
    con = sqlite3.connect(dbs[0])
    q = ("SELECT K.dispatch_id, S.display_name, I.name, E.id, E.value, E.extdata FROM rocpd_pmc_event E "
         "JOIN rocpd_info_pmc I ON I.id = E.pmc_id AND I.guid = E.guid "
         "JOIN rocpd_kernel_dispatch K ON K.event_id = E.event_id AND K.guid = E.guid "
         "JOIN rocpd_info_kernel_symbol S ON S.id = K.kernel_id AND S.guid = K.guid ORDER BY E.id")
    per = defaultdict(lambda: defaultdict(list))
    sample = []
    for did, kname, cname, eid, val, ext in con.execute(q):
        if short(kname) != "k_nt_phase":
            continue
        per[int(did)][cname].append(float(val))
        if len(sample) < 4:
            sample.append({"counter": cname, "value": val, "extdata": ext})
    return [per[k] for k in sorted(per)], sample


def main():
    pdir, run_json, out = sys.argv[1], sys.argv[2], sys.argv[3]
    run = json.load(open(run_json))
    segs = run["segments"]
    recs = csv_records(pdir)
    inst, sample = db_records(pdir)
    need = sum(s["phase_launches"] for s in segs)
    res = {"dispatches": len(recs), "expected": need, "probe_phase_ms": run["probe_phase_ms"], "fast": run["fast"],
           "slow": run["slow"], "swaps": run["swaps"], "torch_stream": run.get("torch_stream"),
           "db_sample": sample, "segments": []}
    if len(recs) != need:
        print(f"dispatch count {len(recs)} != expected {need}: no assignment", flush=True)
        json.dump(res, open(out, "w"), indent=1)
        return
    i = 0
    for s in segs:
        n = s["phase_launches"]
        part = recs[i + 1:i + n]                      # the prologue phase dropped
        ipart = inst[i + 1:i + n] if inst and len(inst) == need else None
        i += n
        mean = {}
        for c in part[0]:
            mean[c] = sum(p[c] for p in part) / len(part)
        rec = {"label": s["label"], "phase_ms": s["phase_ms"], "ms_per_iteration": s["ms_per_iteration"],
               "counters": mean}
        if ipart:
            spread = {}
            for c in ipart[0]:
                k = len(ipart[0][c])
                if k < 2:
                    continue
                avg = [sum(p[c][j] for p in ipart) / len(ipart) for j in range(k)]
                m = sum(avg) / k
                sd = (sum((v - m) ** 2 for v in avg) / k) ** 0.5
                spread[c] = {"instances": k, "mean": m, "max_over_mean": max(avg) / m if m else None,
                             "min_over_mean": min(avg) / m if m else None, "cov": sd / m if m else None,
                             "per_instance": avg}
            rec["per_instance"] = spread
        res["segments"].append(rec)
        print(json.dumps({"label": s["label"], "phase_ms": round(s["phase_ms"], 4),
                          **{c: round(v, 1) for c, v in mean.items()},
                          **({f"{c}_cov": round(v["cov"], 4) for c, v in rec.get("per_instance", {}).items()
                              if v["cov"] is not None})}), flush=True)
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
