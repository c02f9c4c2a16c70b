#!/usr/bin/env python3
"""Merge the PMC traffic of the latency-bound workloads' dominant kernels into profiles/pmc_traffic.json
(measurement tool; run after tools/r02_profile.sh fetch2 write2 fetchm writem).

    python tools/pmc_extra.py gpurun_out/r02

  run           : k_nt_run2 of a 20-iteration cfg 2 solve (4,096 lanes, all active: one launch of 20 iterations);
                  algorithmic bytes = 4,096 x 20 x 80,096 (sweep + trial per lane-iteration, U0Z)
  track_rollout : k_track_rollout_pair of the cfg 5 run (8,192 lanes); algorithmic bytes = the trajectories written
                  plus x0 read, B (32 N + 16 T + 32)
FETCH_SIZE is doubled (profiles/r02_probe/README.md: it reports half of the bytes of 16-B and 8-B-per-lane loads);
WRITE_SIZE is exact.  Units: KiB."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(path, kernel_sub, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals), len(vals)


def main():
    src = sys.argv[1]
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    out = json.load(open(out_path))
    N, T = 501, 500
    jobs = {"run": ("cfg2", "k_nt_run2", 4096 * 20 * 80096),
            "track_rollout": ("mpc", "k_track_rollout_pair", 8192 * (32 * N + 16 * T + 32))}
    for key, (tag, kern, algo) in jobs.items():
        f, nf = mean_counter(os.path.join(src, f"pmc_fetch_{tag}", "run_counter_collection.csv"), kern, "FETCH_SIZE")
        w, nw = mean_counter(os.path.join(src, f"pmc_write_{tag}", "run_counter_collection.csv"), kern, "WRITE_SIZE")
        hbm = 2 * f * 1024.0 + w * 1024.0
        out[key] = {"fetch_bytes_raw": f * 1024.0, "fetch_bytes_corrected": 2 * f * 1024.0, "write_bytes": w * 1024.0,
                    "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": float(algo),
                    "traffic_over_algorithmic": hbm / algo, "launches_measured": [nf, nw]}
        print(key, json.dumps(out[key]))
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
