"""Per-superstep trace of the C4 query on one GPU (RGPU_TRACE): for every batch and superstep the
visited vertices, slots, gathered labels and changes, and every launch's event time.  Writes
the CSV to --out and prints a per-batch digest (steps, cc_step ms, visited / slots / gathers)."""
import argparse
import collections
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range, range_hops  # noqa: E402

KID = {0: "window_mask", 1: "cc_slots", 2: "cc_step", 3: "cc_hist", 4: "cc_summary", 7: "cc_tail", 8: "heavy"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=20_000_000)
    ap.add_argument("--interactions", type=int, default=333_333_334)
    ap.add_argument("--out", default="gpurun_out/c4_trace.csv")
    ap.add_argument("--lean", action="store_true", help="time the lean kernels (RGPU_PROF_LEAN): launch times only")
    a = ap.parse_args()
    inter_full = 333_333_334
    t0 = time.time()
    os.environ["RGPU_TRACE"] = a.out  # read when the context is created; written after each run
    g = TemporalGraph()
    for first in range(0, a.interactions, 20_000_000):
        s = gen_gab_range(4, a.users, inter_full, first, min(20_000_000, a.interactions - first))
        g.ingest_stream(s)
        end = int(s.t[-1])
        del s
    g.seal()
    print(f"built in {time.time() - t0:.1f} s: {g.stats()['vertices']} vertices, {g.stats()['edges']} edges",
          flush=True)
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    g.run("cc", hops, BATCH_WINDOWS)
    if a.lean:
        os.environ["RGPU_PROF_LEAN"] = "1"
    g.run("cc", hops, BATCH_WINDOWS, profile=True, serial=True)
    st = g.stats()
    print({k: round(v["ms"], 2) for k, v in st["kernels"].items()}, flush=True)
    g.close()
    digest(a.out)


def digest(path):
    steps = collections.defaultdict(list)
    ms = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        b = int(r["batch"])
        if r["kind"] == "S":
            steps[b].append((int(r["step"]), int(r["pv"]), int(r["ps"]), int(r["changed"]), int(r["pg"] or 0)))
        else:
            ms[(b, KID.get(int(r["kernel"]), r["kernel"]))] += float(r["ms"])
    # cc_step ms by (window group, superstep) over the batches (window-major: batch % 5 = window)
    by = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["kind"] != "S" and KID.get(int(r["kernel"])) == "cc_step":
            by[(int(r["batch"]) % 5, int(r["step"]))] += float(r["ms"])
    for w in range(5):
        row = [(k[1], round(v, 1)) for k, v in sorted(by.items()) if k[0] == w]
        print(f"window {w}: cc_step {sum(v for _, v in row):7.1f} ms; by step {row}")
    for b in sorted(steps):
        st = steps[b]
        pv = sum(x[1] for x in st)
        ps = sum(x[2] for x in st)
        pg = sum(x[4] for x in st)
        print(f"batch {b:3d}: steps {len(st):3d} step_ms {ms[(b, 'cc_step')]:8.2f} slots_ms {ms[(b, 'cc_slots')]:7.2f}"
              f" visited {pv / 1e6:8.2f}M slots {ps / 1e6:9.2f}M gathers {pg / 1e6:9.2f}M "
              f"per-step visited(M) {[round(x[1] / 1e6, 2) for x in st[:12]]} "
              f"slots(M) {[round(x[2] / 1e6, 1) for x in st[:12]]}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--digest":
        digest(sys.argv[2])
    else:
        main()
