"""TEST INFRASTRUCTURE: golden per-view results of the C4 query (BASELINE configs[3]) on prefixes of
the 1B-update GAB-shaped stream, computed by the CPU oracle (oracle/, lazy edge mode) in this
container and committed as tests/golden/c4_prefix_goldens.json, so that the GPU suite compares
the HIP path with the oracle on prefixes far larger than it could replay inside its own budget
(the oracle needs ~13 GB and ~2 min per 100M updates to build, and ~2 min per hop for the five
windows).  The full 1B stream does not fit this container's memory in the oracle (~130 GB);
the 1B query itself is checked on the GPU by its summary invariants and batch-composition
cross-checks (tests/test_gpu_configs.py).

Per prefix and sampled hop (of the last 168 hourly hops), per window of {y, m, w, d, h}:
ConnectedComponents summary fields (ConnectedComponents.scala:137-145), the hop's superstep count
(AnalysisTask.endStep), the member count, and an order-independent checksum of the (id, label)
pairs of every member (label_checksum below) — per-vertex label parity without storing labels.

usage: python tools/make_c4_goldens.py [--prefixes 33333334:8,100000000:4] [--threads 8]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import Oracle, label_counts  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range, range_hops  # noqa: E402
from tests.goldens import label_checksum  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "c4_prefix_goldens.json")
USERS, INTER = 20_000_000, 333_333_334


def view_record(ids, labels):
    c = label_counts(labels)
    counts = np.fromiter(c.values(), np.int64) if c else np.zeros(0, np.int64)
    big = counts[counts > 1]
    return {"members": int(len(ids)), "biggest": int(counts.max()) if counts.size else 0, "total": int(counts.size),
            "total_without_islands": int(big.size), "clusters_gt2": int((counts > 2).sum()),
            "sum_all": int(counts.sum()), "sum_without_islands": int(big.sum()),
            "label_checksum": label_checksum(ids, labels)}


def picks(n_hops, k):
    return sorted(set(np.linspace(0, n_hops - 1, k).round().astype(int).tolist()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefixes", default="33333334:8,100000000:4",
                    help="interactions (x3 updates) : sampled hops, comma separated")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    data = json.load(open(OUT)) if os.path.exists(OUT) else {"note": __doc__.split("\n\n")[0], "prefixes": {}}
    for spec in a.prefixes.split(","):
        inter, k = (int(x) for x in spec.split(":"))
        t0 = time.time()
        s = gen_gab_range(4, USERS, INTER, 0, inter)
        end = int(s.t[-1])
        hops = range_hops(end - 167 * HOUR, end, HOUR)
        o = Oracle.from_stream(s, True)
        n_upd = len(s)
        del s
        print(f"prefix {inter}: {n_upd} updates, oracle built in {time.time() - t0:.0f} s "
              f"({o.nv} vertices, {o.ne} edges)", flush=True)
        sel = picks(len(hops), k)

        def one(h):
            res, steps = o.cc(int(hops[h]), BATCH_WINDOWS, mode=1)
            return h, steps, [view_record(ids, lab) for ids, lab in res]

        views = {}
        with ThreadPoolExecutor(a.threads) as ex:
            for h, steps, recs in ex.map(one, sel):
                views[str(h)] = {"t": int(hops[h]), "supersteps": int(steps), "windows": recs}
                print(f"  hop {h}: {steps} supersteps, {time.time() - t0:.0f} s", flush=True)
        data["prefixes"][str(inter)] = {"interactions": inter, "updates": n_upd, "hop0": int(hops[0]),
                                        "n_hops": int(len(hops)), "windows": list(BATCH_WINDOWS),
                                        "vertices": int(o.nv), "edges": int(o.ne), "hops": views}
        o.close()
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print(f"prefix {inter} done in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
