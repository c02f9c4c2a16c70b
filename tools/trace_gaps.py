#!/usr/bin/env python3
"""Where does a solve's time go between the phase kernels?  (measurement tool)

    python tools/trace_gaps.py <rocprofv3 -d dir> [--solves 3]

Reads the kernel trace (run_kernel_trace.csv) of `bench.py --steps K --warmup W --extra-legs ""` and splits the last
``--solves`` solves (each starts at a k_init dispatch) into: phase-kernel time, every other kernel's time by name, and
the idle gaps between dispatches, the gaps classified by the kernel that precedes them (a gap after k_stats_final is
where the host loop reads the statistics: sync_every iterations).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0].split("::")[-1].strip().split("<")[0]
    return n[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--solves", type=int, default=3)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    starts = [i for i, e in enumerate(ev) if e[0] == "k_init"]
    # the main leg's solves are the last k_init dispatches of the process (bench: process warm-up, then the leg)
    seg_starts = starts[-a.solves:]
    for si, s0 in enumerate(seg_starts):
        s1 = seg_starts[si + 1] if si + 1 < len(seg_starts) else len(ev)
        seg = ev[s0:s1]
        # the solve ends at its last unpack / finalize kernel
        last = max(i for i, e in enumerate(seg) if e[0].startswith("k_unpack") or e[0] == "k_finalize_status")
        seg = seg[:last + 1]
        busy = defaultdict(float)
        gaps = defaultdict(float)
        gapn = defaultdict(int)
        for i, (n, t0, t1) in enumerate(seg):
            busy[n] += (t1 - t0) / 1e6
            if i + 1 < len(seg):
                g = max(0, seg[i + 1][1] - t1) / 1e6
                gaps[n] += g
                gapn[n] += 1
        wall = (seg[-1][2] - seg[0][1]) / 1e6
        print(f"solve {si}: wall {wall:.2f} ms, dispatches {len(seg)}, kernel busy {sum(busy.values()):.2f} ms, "
              f"gaps {sum(gaps.values()):.2f} ms")
        for n, v in sorted(busy.items(), key=lambda kv: -kv[1])[:12]:
            print(f"   busy {n:40s} {v:9.2f} ms  ({sum(1 for e in seg if e[0] == n)} dispatches)")
        for n, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:8]:
            print(f"   gap after {n:35s} {v:9.2f} ms over {gapn[n]} gaps")


if __name__ == "__main__":
    main()
