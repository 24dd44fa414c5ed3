"""One-GPU rehearsal of the C4 query on R full graph replicas (SURVEY.md §8(e) "Graph replicas ...
with hop batches split across GPUs need zero exchange. Report both"): the 1B stream (or a prefix)
is sealed once, and every replica's share of the 168 hops x 5 windows runs alone on the GPU, timed
with the library's synchronous run call around it; the slowest replica is what R GPUs would take (no
exchange: a replica's results are final for its views, and the summaries are concatenated).

Two splits of the query's views:
  hops    replica r takes a contiguous range of ceil(168 / R) hops x all 5 windows (one call);
  batches the query's (64-hop block, window) batches — the units the library runs — are dealt to
          the replicas longest-first by a static cost weight per window (a year batch costs about
          ten hour batches); a replica's batches of one block run as one call (their windows in
          the query's descending order, so shrinkWindow keeps vertex window = edge window).
Both check that the concatenated per-view summaries equal the whole query's.  Prints one JSON line
per (split, R).

usage: python tools/replica_sim.py [--interactions N] [--replicas 2,4,8] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range, range_hops  # noqa: E402

# relative cost of one 64-hop batch per window (C4 1B serial profile, profiles/r04: year ~45 ms,
# month ~20, week ~10, day ~6, hour ~4 per block)
WEIGHT = {0: 11.0, 1: 5.0, 2: 2.5, 3: 1.5, 4: 1.0}


def timed(g, calls):
    """Run the calls [(hops, windows)] back to back; (ms of the runs, [summaries per call]).
    A run returns when its results are on the host (rgpu_run_view_batch is synchronous); the
    summaries are read outside the timing."""
    ms = 0.0
    out = []
    for hops, wins in calls:
        t = time.perf_counter()
        g.run("cc", hops, wins)
        ms += (time.perf_counter() - t) * 1e3
        out.append(g.cc_summaries()[..., :7].copy())
    return ms, out


def split_hops(hops, R):
    """[(first hop index, hop count, window indices)] per replica"""
    k = -(-len(hops) // R)
    return [[(r * k, min(k, len(hops) - r * k), list(range(len(BATCH_WINDOWS))))] for r in range(R) if r * k < len(hops)]


def split_batches(hops, R):
    blocks = [(b, min(64, len(hops) - b)) for b in range(0, len(hops), 64)]
    units = [(WEIGHT[w] * blocks[b][1] / 64.0, b, w) for b in range(len(blocks)) for w in range(len(BATCH_WINDOWS))]
    units.sort(key=lambda u: -u[0])
    load = [0.0] * R
    own = [[] for _ in range(R)]
    for wgt, b, w in units:
        r = min(range(R), key=lambda i: load[i])
        load[r] += wgt
        own[r].append((b, w))
    plans = []
    for r in range(R):
        by_block = {}
        for b, w in own[r]:
            by_block.setdefault(b, []).append(w)
        plans.append([(blocks[b][0], blocks[b][1], sorted(ws)) for b, ws in sorted(by_block.items())])
    return [p for p in plans if p]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--interactions", type=int, default=333_333_334)
    ap.add_argument("--users", type=int, default=20_000_000)
    ap.add_argument("--replicas", default="2,4,8")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    g = TemporalGraph()
    t0 = time.time()
    for first in range(0, a.interactions, 20_000_000):
        s = gen_gab_range(4, a.users, 333_333_334, first, min(20_000_000, a.interactions - first))
        g.ingest_stream(s)
        end = int(s.t[-1])
        del s
    g.seal()
    print(f"sealed in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    W = len(BATCH_WINDOWS)
    n_edges = g.stats()["edges"]
    g.run("cc", hops, BATCH_WINDOWS)  # warm
    whole = None
    for _ in range(a.rounds):
        ms, (summ,) = timed(g, [(hops, BATCH_WINDOWS)])
        whole = ms if whole is None else min(whole, ms)
    ref = summ  # [hops, windows, fields 0..6] (supersteps depend on the batch grouping)
    print(json.dumps({"split": "none", "R": 1, "query_ms": round(whole, 2),
                      "edge_windows_per_s": n_edges * W * len(hops) / (whole / 1e3)}), flush=True)
    for R in [int(x) for x in a.replicas.split(",")]:
        for name, plans in (("hops", split_hops(hops, R)), ("batches", split_batches(hops, R))):
            per = []
            ok = True
            for plan in plans:
                best = None
                for _ in range(a.rounds):
                    ms, outs = timed(g, [(hops[i0:i0 + n], [BATCH_WINDOWS[w] for w in ws]) for i0, n, ws in plan])
                    best = ms if best is None else min(best, ms)
                for (i0, n, ws), o in zip(plan, outs):
                    ok &= bool(np.array_equal(o, ref[i0:i0 + n][:, ws]))
                per.append(round(best, 2))
            slow = max(per)
            print(json.dumps({
                "split": name, "R": R, "replica_ms": per, "slowest_replica_ms": slow,
                "speedup_vs_whole": round(whole / slow, 2),
                "modelled_edge_windows_per_s_at_R_gpus": n_edges * W * len(hops) / (slow / 1e3),
                "summaries_equal_whole_query": ok,
                "plan": [[[i0, n, ws] for i0, n, ws in p] for p in plans]}), flush=True)
    g.close()


if __name__ == "__main__":
    main()
