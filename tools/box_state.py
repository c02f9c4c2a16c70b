"""Box state of the GPU a process runs on, read from sysfs (measurement infrastructure; bench.py's ``box`` field).

The GPU's PCI function is found from torch's device properties (domain / bus / device) and its sysfs directory read:
  * pp_dpm_sclk / pp_dpm_mclk / pp_dpm_fclk / pp_dpm_socclk: the DPM level marked current ('*'), in MHz;
  * hwmon: power (power1_average or power1_input, W), temperatures (temp*_input with their labels: edge, hotspot /
    junction, mem; degC) and clocks (freq*_input with labels, MHz).
``Sampler`` reads them on a background thread (default every 0.1 s) and reports per-window mean / min / max, so a
timed leg can say what clocks, power and temperatures it ran at.  Nothing here touches the GPU: plain file reads.
Missing files (containers that hide sysfs) give an empty record, never an error.
"""
from __future__ import annotations

import glob
import os
import re
import threading
import time


def pci_dir(device_index: int = 0) -> str | None:
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        d = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        return d if os.path.isdir(d) else None
    except Exception:
        return None


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read()
    except Exception:
        return None


def _dpm_current(text: str | None) -> float | None:
    if not text:
        return None
    for line in text.splitlines():
        if line.rstrip().endswith("*"):
            m = re.search(r"([\d.]+)\s*[Mm]hz", line)
            if m:
                return float(m.group(1))
    return None


class _Channels:
    def __init__(self, dev: str):
        self.files = {}
        for name in ("sclk", "mclk", "fclk", "socclk"):
            p = os.path.join(dev, f"pp_dpm_{name}")
            if os.path.exists(p):
                self.files[f"dpm_{name}_mhz"] = (p, "dpm")
        for hw in sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*"))):
            for kind, scale, unit in (("power", 1e-6, "w"), ("temp", 1e-3, "c"), ("freq", 1e-6, "mhz")):
                for p in sorted(glob.glob(os.path.join(hw, f"{kind}*_input")) +
                                glob.glob(os.path.join(hw, f"{kind}*_average"))):
                    base = os.path.basename(p).rsplit("_", 1)[0]
                    label = (_read(os.path.join(hw, base + "_label")) or base).strip().lower().replace(" ", "_")
                    suffix = "avg" if p.endswith("_average") else "in"
                    key = f"{kind}_{label}_{suffix}_{unit}" if kind == "power" else f"{kind}_{label}_{unit}"
                    self.files.setdefault(key, (p, scale))
            p = os.path.join(hw, "power1_cap")
            if os.path.exists(p):
                self.files.setdefault("power_cap_w", (p, 1e-6))

    def read(self) -> dict:
        out = {}
        for key, (p, how) in self.files.items():
            t = _read(p)
            if how == "dpm":
                v = _dpm_current(t)
            else:
                try:
                    v = float(t.strip()) * how
                except Exception:
                    v = None
            if v is not None:
                out[key] = v
        return out


def _smi_json(args, timeout):
    import json
    import subprocess
    out = subprocess.run(["amd-smi", *args, "--json"], capture_output=True, text=True, timeout=timeout).stdout
    i = min(k for k in (out.find("{"), out.find("[")) if k >= 0)
    return json.loads(out[i:])


_SMI_INDEX = {}


def smi_index(bdf: str | None, timeout: float = 30.0) -> int | None:
    """amd-smi's index of the GPU at PCI address ``bdf`` (e.g. 0000:0d:00.0, from pci_dir), from ``amd-smi list``;
    with one GPU listed, that one; None if it cannot be told."""
    if bdf in _SMI_INDEX:
        return _SMI_INDEX[bdf]
    idx = None
    try:
        lst = _smi_json(["list"], timeout)
        lst = lst if isinstance(lst, list) else lst.get("gpu_list", lst.get("gpus", []))
        for e in lst:
            if bdf and str(e.get("bdf", "")).lower() == bdf.lower():
                idx = int(e["gpu"])
        if idx is None and len(lst) == 1:
            idx = int(lst[0].get("gpu", 0))
    except Exception:
        idx = None
    _SMI_INDEX[bdf] = idx
    return idx


def smi_counters(timeout: float = 30.0, bdf: str | None = None) -> dict:
    """amd-smi's accumulated throttle and energy counters of the GPU at ``bdf`` (the one GPU listed, if bdf is None),
    or {}: ``acc`` (the SMU's accumulation ticks), ``ppt`` / ``socket_thermal`` / ``hbm_thermal`` / ``prochot``
    (ticks spent under that limit) and ``energy_j``.  Two snapshots give the share of a window spent at the power
    cap and the energy it used."""
    try:
        idx = smi_index(bdf, timeout)
        if idx is None:
            return {}
        data = _smi_json(["metric", "-g", str(idx)], timeout)
        gl = data["gpu_data"] if isinstance(data, dict) else data
        g = next((e for e in gl if int(e.get("gpu", idx)) == idx), None) if len(gl) != 1 else gl[0]
        if g is None:
            return {}
        th = g.get("throttle", {})
        rec = {"acc": th.get("accumulation_counter"), "ppt": th.get("ppt_accumulated"),
               "socket_thermal": th.get("socket_thermal_accumulated"), "hbm_thermal": th.get("hbm_thermal_accumulated"),
               "prochot": th.get("prochot_accumulated"),
               "energy_j": g.get("energy", {}).get("total_energy_consumption", {}).get("value")}
        return {k: v for k, v in rec.items() if isinstance(v, (int, float))}
    except Exception:
        return {}


def smi_delta(a: dict, b: dict) -> dict:
    """Shares of the window between two smi_counters() snapshots spent under each limit, and its energy."""
    out = {}
    if a.get("acc") is not None and b.get("acc") is not None and b["acc"] > a["acc"]:
        n = b["acc"] - a["acc"]
        for k in ("ppt", "socket_thermal", "hbm_thermal", "prochot"):
            if k in a and k in b:
                out[f"{k}_share"] = round((b[k] - a[k]) / n, 4)
    if "energy_j" in a and "energy_j" in b:
        out["energy_j"] = round(b["energy_j"] - a["energy_j"], 1)
    return out


class Sampler:
    """Background sysfs sampler.  ``mark()`` starts a window; ``window()`` returns {channel: [mean, min, max]} over the
    samples since the last mark (plus the sample count and the window's seconds)."""

    def __init__(self, device_index: int = 0, period: float = 0.1, dev: str | None = None):
        dev = dev or pci_dir(device_index)
        self.dev = dev
        self.ch = _Channels(dev) if dev else None
        self.period = period
        self.samples = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._t = None
        self._mark = 0
        self._t_mark = time.perf_counter()

    @property
    def available(self) -> bool:
        return bool(self.ch and self.ch.files)

    def start(self):
        if self.available and self._t is None:
            self._t = threading.Thread(target=self._loop, daemon=True)
            self._t.start()
        return self

    def _loop(self):
        while not self._stop.is_set():
            s = self.ch.read()
            with self._lock:
                self.samples.append((time.perf_counter(), s))
            self._stop.wait(self.period)

    def snapshot(self) -> dict:
        return self.ch.read() if self.available else {}

    def mark(self):
        with self._lock:
            self._mark = len(self.samples)
        self._t_mark = time.perf_counter()

    def window(self) -> dict:
        with self._lock:
            win = self.samples[self._mark:]
        out = {"samples": len(win), "seconds": time.perf_counter() - self._t_mark}
        keys = sorted({k for _, s in win for k in s})
        for k in keys:
            v = [s[k] for _, s in win if k in s]
            out[k] = [round(sum(v) / len(v), 2), round(min(v), 2), round(max(v), 2)]
        return out

    def stop(self):
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2)
