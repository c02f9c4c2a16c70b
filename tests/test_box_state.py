"""The bench line's box record (tools/box_state.py, bench.BoxMonitor / stress_tail_record) on a synthetic sysfs tree
and a stand-in leg: no GPU, no amd-smi."""
import os
import sys
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _fake_sysfs(tmp_path, sclk_level=1):
    dev = tmp_path / "0000:0d:00.0"
    hw = dev / "hwmon" / "hwmon3"
    hw.mkdir(parents=True)
    levels = ["0: 500Mhz", "1: 1700Mhz", "2: 2400Mhz"]
    (dev / "pp_dpm_sclk").write_text("\n".join(l + (" *" if i == sclk_level else "") for i, l in enumerate(levels)) + "\n")
    (dev / "pp_dpm_mclk").write_text("0: 2000Mhz *\n")
    (hw / "power1_input").write_text("1388000000\n")
    (hw / "power1_label").write_text("PPT\n")
    (hw / "power1_cap").write_text("1400000000\n")
    (hw / "temp2_input").write_text("54000\n")
    (hw / "temp2_label").write_text("junction\n")
    (hw / "temp3_input").write_text("66500\n")
    (hw / "temp3_label").write_text("mem\n")
    return str(dev)


def test_sysfs_channels_and_windows(tmp_path):
    import box_state
    dev = _fake_sysfs(tmp_path)
    s = box_state.Sampler(period=0.01, dev=dev)
    assert s.available
    snap = s.snapshot()
    assert snap == {"dpm_sclk_mhz": 1700.0, "dpm_mclk_mhz": 2000.0, "power_ppt_in_w": 1388.0, "power_cap_w": 1400.0,
                    "temp_junction_c": 54.0, "temp_mem_c": 66.5}
    s.start()
    s.mark()
    time.sleep(0.1)
    (tmp_path / "0000:0d:00.0" / "pp_dpm_sclk").write_text("0: 500Mhz\n1: 1700Mhz\n2: 2400Mhz *\n")
    time.sleep(0.1)
    w = s.window()
    s.stop()
    assert w["samples"] >= 5 and w["dpm_sclk_mhz"][1] == 1700.0 and w["dpm_sclk_mhz"][2] == 2400.0
    assert 1700.0 < w["dpm_sclk_mhz"][0] < 2400.0


def test_missing_sysfs_gives_an_empty_record(tmp_path):
    import box_state
    s = box_state.Sampler(dev=str(tmp_path / "absent")).start()
    assert not s.available and s.snapshot() == {} and s.window()["samples"] == 0
    s.stop()


def test_smi_delta_shares_and_energy():
    import box_state
    a = {"acc": 1000, "ppt": 10, "socket_thermal": 0, "hbm_thermal": 0, "prochot": 0, "energy_j": 100.0}
    b = {"acc": 1200, "ppt": 190, "socket_thermal": 0, "hbm_thermal": 20, "prochot": 0, "energy_j": 2100.5}
    d = box_state.smi_delta(a, b)
    assert d == {"ppt_share": 0.9, "socket_thermal_share": 0.0, "hbm_thermal_share": 0.1, "prochot_share": 0.0,
                 "energy_j": 2000.5}
    assert box_state.smi_delta({}, b) == {}


def test_stress_tail_record_critical_path():
    """The stress leg's straggler-tail bound: the tail's seconds over the outer iterations it ran is one lane-iteration's
    latency; the longest lane's iterations times that latency is the critical path."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    res = types.SimpleNamespace(n_iter=torch.tensor([400, 5000, 380]), tail_from_iteration=772)
    leg = types.SimpleNamespace(steps=2, solver=types.SimpleNamespace(launches={"tail": 68}), tail_lane_its=2 * 4400,
                                lane_its=2 * 105_000_000, tail_iters_max=4228, res=res, elapsed=2 * 4.4,
                                box={"sclk_mhz": [2100.0, 1650.0, 2400.0]})
    ks = {"tail": {"avg_ms": 2 * 2285.0 / 68, "launches": 68}}
    r = bench.stress_tail_record(leg, ks, 500)
    lat = 2.285 / 4228
    assert np.isclose(r["seconds_per_step"], 2.285) and np.isclose(r["lane_iteration_latency_ms"], 1e3 * lat)
    assert r["max_lane_iterations"] == 5000 and np.isclose(r["critical_path_s"], 5000 * lat)
    assert np.isclose(r["frac_of_critical_path"], 5000 * lat / 4.4) and np.isclose(r["share_of_solve"], 2.285 / 4.4)
    assert np.isclose(r["cycles_per_stage_at_sclk"]["max"], lat * 2400e6 / 500)
    # no tail: the record keeps its keys without a bound
    leg.tail_iters_max = 0
    assert bench.stress_tail_record(leg, {}, 500)["seconds_per_step"] is None


def test_persistent_chain_record():
    """The cfg 2 leg's bound: the persistent kernel's seconds per solve over the longest lane's iterations is one
    lane-iteration's chain latency; at the leg's SCLK that is the chain's cycles per stage."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    res = types.SimpleNamespace(n_iter=torch.tensor([390, 404, 12]))
    leg = types.SimpleNamespace(steps=5, res=res, elapsed=5 * 0.2017, box={"sclk_mhz": [2390.0, 2380.0, 2400.0]})
    ks = {"run": {"avg_ms": 49.7, "launches": 20}}
    r = bench.persistent_chain_record(leg, ks, 500)
    run_s = 49.7 * 20 / 1e3 / 5
    assert np.isclose(r["run_seconds_per_step"], run_s) and r["max_lane_iterations"] == 404
    assert np.isclose(r["lane_iteration_latency_ms"], 1e3 * run_s / 404)
    assert np.isclose(r["share_of_solve"], run_s / 0.2017)
    assert np.isclose(r["cycles_per_stage_at_sclk"]["mean"], run_s / 404 * 2390e6 / 500)
    assert bench.persistent_chain_record(leg, {}, 500) == {}
