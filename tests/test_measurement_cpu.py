"""Measurement helpers on CPU (no GPU): tools/pmc_summary.py pools rocprofv3 counter CSVs per kernel
group (lean instantiations only) and bench.aggregate_roofline pools the window-filter + CC kernels'
bytes, time and counted traffic the way DESIGN.md §6 states."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _write(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_pmc_summary_groups_and_lean_filter(tmp_path):
    from tools.pmc_summary import summarise
    lean = "void rgpu::k_cc_step_pk<false, false, true, 6>(int, long)"
    prof = "void rgpu::k_cc_step_pk<false, true, false, 1>(int, long)"
    k2 = "void rgpu::k_cc_slots<false, true, false, 6>(long)"
    hub = "rgpu::k_heavy_gather<6>(int)"
    other = "void rocprim::trampoline_kernel<x>(y)"
    f = [dict(Kernel_Name=lean, Counter_Name="FETCH_SIZE", Counter_Value=100.0),
         dict(Kernel_Name=lean, Counter_Name="FETCH_SIZE", Counter_Value=300.0),
         dict(Kernel_Name=prof, Counter_Name="FETCH_SIZE", Counter_Value=9e9),
         dict(Kernel_Name=k2, Counter_Name="FETCH_SIZE", Counter_Value=50.0),
         dict(Kernel_Name=hub, Counter_Name="FETCH_SIZE", Counter_Value=10.0),
         dict(Kernel_Name=other, Counter_Name="FETCH_SIZE", Counter_Value=7.0)]
    w = [dict(Kernel_Name=lean, Counter_Name="WRITE_SIZE", Counter_Value=20.0),
         dict(Kernel_Name=lean, Counter_Name="WRITE_SIZE", Counter_Value=40.0),
         dict(Kernel_Name=prof, Counter_Name="WRITE_SIZE", Counter_Value=9e9),
         dict(Kernel_Name=k2, Counter_Name="WRITE_SIZE", Counter_Value=5.0),
         dict(Kernel_Name=hub, Counter_Name="WRITE_SIZE", Counter_Value=1.0)]
    _write(str(tmp_path / "fetch" / "x" / "run_counter_collection.csv"), f)
    _write(str(tmp_path / "write" / "x" / "run_counter_collection.csv"), w)
    out = summarise(str(tmp_path / "fetch"), str(tmp_path / "write"))
    g = out["by_group"]
    assert set(g) == {"cc_step", "cc_slots", "heavy"}  # (the profiling instantiation and rocprim are left out)
    assert g["cc_step"]["dispatches"] == 2
    assert g["cc_step"]["traffic_bytes_per_launch"] == (2 * 400 * 1024 + 60 * 1024) / 2
    assert out["traffic_bytes_per_launch"]["value"] == g["cc_step"]["traffic_bytes_per_launch"]
    assert out["FETCH_SIZE"]["mean_kb_per_dispatch"] == 200.0


def test_aggregate_roofline_pools_bytes_time_and_traffic(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    pmc = {"by_group": {"cc_step": {"dispatches": 2, "traffic_bytes_per_launch": 3e9},
                        "cc_slots": {"dispatches": 1, "traffic_bytes_per_launch": 2e9},
                        "window_mask": {"dispatches": 1, "traffic_bytes_per_launch": 1e9}}}
    (prof / "latest_pmc_c4.json").write_text(json.dumps(pmc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    kraw = {"cc_step": {"launches": 2, "ms": 2.0, "bytes": 2e9},
            "cc_slots": {"launches": 1, "ms": 1.0, "bytes": 1e9},
            "window_mask": {"launches": 1, "ms": 1.0, "bytes": 1e9},
            "cc_hist": {"launches": 1, "ms": 9.0, "bytes": 9e9}}  # (not a window-filter + CC kernel)
    a = bench.aggregate_roofline(kraw, "C4")
    assert a["ms"] == 4.0 and a["algorithmic_bytes"] == 4e9
    assert abs(a["achieved"] - 1000.0) < 1e-6  # 4 GB / 4 ms
    assert a["traffic"] == round(3e9 * 2 + 2e9 + 1e9)
    assert a["traffic_over_algorithmic"] == round(9e9 / 4e9, 2)
    assert set(a["by_kernel"]) == {"cc_step", "cc_slots", "window_mask"}
    # a group without a PMC record: no aggregate traffic claimed
    kraw["heavy"] = {"launches": 3, "ms": 1.0, "bytes": 1e9}
    b = bench.aggregate_roofline(kraw, "C4")
    assert b["traffic"] is None and b["traffic_over_algorithmic"] is None
