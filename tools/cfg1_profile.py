#!/usr/bin/env python3
"""Where BASELINE cfg 1's drop-in call spends its time (measurement tool).

    python tools/cfg1_profile.py [--cprofile OUT.txt]

Runs bench.cfg1_line() (main.task_2's newton_Algorithm call through the drop-in module, one warm-up call and one
timed call) and prints its record; with --cprofile, the timed call's Python profile (cumulative time, top 40)."""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cprofile", default=None)
    a = ap.parse_args()
    import bench
    bench.cfg1_line(repeats=1)                     # warm-up (module loads, first launches)
    pr = cProfile.Profile() if a.cprofile else None
    if pr:
        pr.enable()
    rec = bench.cfg1_line(repeats=1)
    if pr:
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(40)
        s2 = io.StringIO()
        pstats.Stats(pr, stream=s2).sort_stats("tottime").print_stats(25)
        os.makedirs(os.path.dirname(os.path.abspath(a.cprofile)), exist_ok=True)
        open(a.cprofile, "w").write(s.getvalue() + "\n\n" + s2.getvalue())
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
