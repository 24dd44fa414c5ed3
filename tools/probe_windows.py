#!/usr/bin/env python3
"""Probe (GPU box): cost of the C2 query by window.  Runs the 8,041-hop CC Range query with all
five batched windows, then with each window alone (64 hops per batch), and prints wall time and
the serial per-kernel breakdown of each, to decide how views should be grouped into batches."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, T0_README, gen_uniform, range_hops  # noqa: E402


def main():
    s = gen_uniform(1, 100_000, 1_000_000)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, HOUR)
    g = TemporalGraph()
    g.ingest_stream(s)
    g.seal()
    sets = [("all5", BATCH_WINDOWS)] + [(f"w{w // HOUR}h", [w]) for w in BATCH_WINDOWS]
    tot = 0.0
    for name, wins in sets:
        g.run("cc", hops, wins)
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            g.run("cc", hops, wins)
            ts.append((time.perf_counter() - t0) * 1e3)
        g.run("cc", hops, wins, profile=True, serial=True)
        st = g.stats()
        ks = "  ".join(f"{k}={v['ms']:.1f}/{v['launches']}" for k, v in st["kernels"].items() if v["launches"])
        print(f"{name:8s} wall {min(ts):7.1f} ms  batches {st['batches']}  supersteps/batch "
              f"{st['supersteps'] / max(st['batches'], 1):.1f}  serial: {ks}", flush=True)
        if name != "all5":
            tot += min(ts)
    print(f"sum of single-window walls: {tot:.1f} ms")
    g.close()


if __name__ == "__main__":
    main()
