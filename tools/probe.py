#!/usr/bin/env python3
"""Performance probe (GPU box): time the C2 batched-window CC query under several library
configurations and summarise the per-step trace.  Usage:
  python tools/probe.py "RGPU_STEP_VARIANT=0" "RGPU_STEP_VARIANT=1,RGPU_SLOTS=1" ...
Each argument is a comma-separated env assignment list applied before rgpu_open."""
import csv
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, T0_README, gen_uniform, range_hops  # noqa: E402

KN = ["window_mask", "cc_slots", "cc_step", "cc_hist", "cc_summary", "pr_step", "degree"]


def run(cfg: str, s, hops, reps: int, trace_dir: str):
    env = dict(kv.split("=") for kv in cfg.split(",") if kv)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    tpath = os.path.join(trace_dir, "trace_" + cfg.replace("=", "").replace(",", "_") + ".csv")
    os.environ["RGPU_TRACE"] = tpath
    g = TemporalGraph()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    g.ingest_stream(s)
    g.seal()
    g.run("cc", hops, BATCH_WINDOWS)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        g.run("cc", hops, BATCH_WINDOWS)
        ts.append((time.perf_counter() - t0) * 1e3)
    ref = g.cc_summaries()
    g.run("cc", hops, BATCH_WINDOWS, profile=True)
    st = g.stats()
    assert np.array_equal(ref, g.cc_summaries())
    g.close()
    print(f"\n## {cfg or 'default'}: query ms = {' '.join(f'{t:.1f}' for t in ts)}  (best {min(ts):.1f})")
    print("   profiled pass wall ms %.1f" % st["ms_total"])
    for k, v in st["kernels"].items():
        if v["launches"]:
            print(f"   {k:12s} launches {v['launches']:6d}  ms {v['ms']:8.2f}  avg_us {v['ms'] * 1e3 / v['launches']:7.2f}"
                  f"  GB/s {v['bytes'] / max(v['ms'], 1e-9) / 1e6:8.1f}")
    # per-step summary
    lt = defaultdict(list)
    sw = defaultdict(lambda: [0, 0, 0, 0])
    with open(tpath) as f:
        for row in csv.DictReader(f):
            if row["kind"] == "L" and int(row["kernel"]) == 2:
                lt[int(row["step"])].append(float(row["ms"]))
            elif row["kind"] == "S":
                a = sw[int(row["step"])]
                a[0] += 1
                a[1] += int(row["pv"] or 0)
                a[2] += int(row["ps"] or 0)
                a[3] += int(row["changed"] or 0)
    print("   step  launches  avg_us   batches  avg_visited  avg_slots  avg_changed")
    for r in sorted(set(lt) | set(sw)):
        t = lt.get(r, [])
        a = sw.get(r, [0, 0, 0, 0])
        nb = max(a[0], 1)
        print(f"   {r:4d}  {len(t):8d}  {np.mean(t) * 1e3 if t else 0:7.1f}  {a[0]:7d}  {a[1] / nb:11.0f}  {a[2] / nb:9.0f}  {a[3] / nb:11.0f}")
    return min(ts)


def main():
    s = gen_uniform(1, 100_000, 1_000_000)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, HOUR)
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    cfgs = sys.argv[1:] or [""]
    res = {c: run(c, s, hops, 2, out) for c in cfgs}
    print("\nsummary:", {k or "default": round(v, 1) for k, v in res.items()})


if __name__ == "__main__":
    main()
