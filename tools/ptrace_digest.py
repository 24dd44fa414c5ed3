#!/usr/bin/env python3
"""Digest of a partitioned rehearsal's per-launch trace (tools/part_sim.py --trace DIR): per kernel,
launches, total ms, and the share spent in launches under a floor threshold (idle late supersteps),
for one partition file (trace_P<P>.csv.p<k>) or a one-partition trace.

  python tools/ptrace_digest.py gpurun_out/ptrace/trace_P8.csv.p0 [--floor-us 40]
"""
import argparse
import collections
import csv

KID = ["window_mask", "cc_slots", "cc_step", "cc_hist", "cc_summary", "pr_step", "degree", "cc_tail", "heavy",
       "diffusion", "vp_step", "edge_mask", "xchg", "xchg_pack", "xchg_unpack", "xchg_mark"]  # rgpu.cpp KernelId


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--floor-us", type=float, default=40.0, help="launches shorter than this count as floor")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: [0, 0.0, 0, 0.0])  # launches, ms, short launches, short ms
    by_step = collections.defaultdict(float)
    for row in csv.DictReader(open(a.trace)):
        if row["kind"] != "L":
            continue
        k, ms = KID[int(row["kernel"])], float(row["ms"])
        p = per[k]
        p[0] += 1
        p[1] += ms
        if ms * 1e3 < a.floor_us:
            p[2] += 1
            p[3] += ms
        by_step[int(row["step"])] += ms
    tot = sum(p[1] for p in per.values())
    print(f"{a.trace}: {tot:.2f} ms in launches")
    for k, (n, ms, ns, mss) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:12s} {n:5d} launches {ms:8.2f} ms  avg {1e3 * ms / max(n, 1):7.1f} us   "
              f"< {a.floor_us:.0f} us: {ns:4d} launches {mss:7.2f} ms")
    print("  by superstep (ms):", ", ".join(f"{s}:{v:.2f}" for s, v in sorted(by_step.items())))


if __name__ == "__main__":
    main()
