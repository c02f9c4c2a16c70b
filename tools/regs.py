#!/usr/bin/env python3
"""Register / spill summary of the solver kernels (gfx950), from the compiler's resource-usage remarks."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", f"{ROOT}/include", "-I",
       f"{ROOT}/gymnast_optimalcontrol_amd/csrc", "-c", f"{ROOT}/gymnast_optimalcontrol_amd/csrc/acrobot_kernels.hip",
       "-o", "/tmp/regs_probe.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"\(.*", "", cur.replace("(anonymous namespace)::", ""))
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^]]*\])?: (\S+)", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if "k_nt_" in k or "k_track" in k:
        print(f"{k:42s} VGPR {v.get('VGPRs', '?'):>4}  spillV {v.get('VGPRs Spill', '?'):>3}  "
              f"spillS {v.get('SGPRs Spill', '?'):>3}  occ {v.get('Occupancy', '?')}")
