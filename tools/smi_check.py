import sys, os, json, subprocess
sys.path.insert(0, "tools")
out = subprocess.run(["amd-smi", "list", "--json"], capture_output=True, text=True, timeout=30).stdout
print("LIST", out[:600])
import box_state, torch
d = box_state.pci_dir(0)
print("pci", d)
print("index", box_state.smi_index(os.path.basename(d)))
print("counters", box_state.smi_counters(bdf=os.path.basename(d)))
