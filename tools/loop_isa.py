#!/usr/bin/env python3
"""Per-loop instruction mix of a kernel in a gfx950 assembly listing (measurement tool).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I gymnast_optimalcontrol_amd/csrc --cuda-device-only \
        -S gymnast_optimalcontrol_amd/csrc/acrobot_kernels.hip -o /tmp/k.s
    python tools/loop_isa.py /tmp/k.s k_nt_runILb1E k_nt_phaseILb1ELb0E

For every backward branch (a loop back edge) prints the loop's line span, its instruction count, VALU
count, scratch (VGPR spill) accesses, v_readlane / v_writelane (SGPR spills), and s_waitcnt count.
"""
import re
import sys


def kernels(lines):
    starts = [(i, l[:-1]) for i, l in enumerate(lines) if re.match(r"^_Z\S+:(\s|$)", l) or re.match(r"^_Z\S+:\s*;", l)]
    for j, (i, name) in enumerate(starts):
        end = starts[j + 1][0] if j + 1 < len(starts) else len(lines)
        yield name.split(":")[0], i, end


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    lines = open(path).read().splitlines()
    for name, lo, hi in kernels(lines):
        if not any(p in name for p in pats):
            continue
        print(f"== {name[:90]}")
        body = lines[lo:hi]
        labels = {}
        for i, l in enumerate(body):
            m = re.match(r"^(\.LBB\S+):", l)
            if m:
                labels[m.group(1)] = i
        for i, l in enumerate(body):
            m = re.search(r"\bs_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
            if m and m.group(2) in labels and labels[m.group(2)] < i:
                a = labels[m.group(2)]
                seg = [x.strip() for x in body[a:i + 1] if x.strip() and not x.strip().startswith((";", "."))]
                ins = [x for x in seg if not x.endswith(":")]
                valu = sum(1 for x in ins if x.startswith("v_"))
                scr = sum(1 for x in ins if x.startswith("scratch_") or "buffer_store_dword" in x and "off, s[0:3]" in x)
                rl = sum(1 for x in ins if x.startswith("v_readlane"))
                wl = sum(1 for x in ins if x.startswith("v_writelane"))
                wc = sum(1 for x in ins if x.startswith("s_waitcnt"))
                vm = sum(1 for x in ins if x.startswith(("buffer_load", "global_load")))
                vs = sum(1 for x in ins if x.startswith(("buffer_store", "global_store")))
                print(f"  loop lines {lo + a}-{lo + i}: {len(ins):5d} instr  VALU {valu:5d}  scratch {scr:3d}  "
                      f"readlane {rl:3d}  writelane {wl:3d}  waitcnt {wc:3d}  vload {vm:3d}  vstore {vs:3d}")


if __name__ == "__main__":
    main()
