"""Same-process A/B of superstep launch knobs on one sealed C4 graph (the knobs rgpu re-reads
per run: RGPU_STEP_GRID, RGPU_TAIL_STEP, RGPU_TAIL_GRID, RGPU_CHUNK0,
RGPU_CHUNK).  Variants are "name:K=V,K=V" (empty = defaults); each is timed twice, interleaved,
with a serial profile pass for its per-kernel times; the summaries must agree across variants.
One JSON line per variant and round."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range, range_hops  # noqa: E402

KNOBS = ("RGPU_FINAL", "RGPU_HUB_PIPE", "RGPU_STEP_CH", "RGPU_TSG", "RGPU_IEM", "RGPU_DENSE1", "RGPU_DEAL_SLOTS", "RGPU_DEAL_STEP", "RGPU_DENSE", "RGPU_CHGBITS", "RGPU_STEP_GRID", "RGPU_TAIL_STEP", "RGPU_TAIL_GRID", "RGPU_CHUNK0", "RGPU_CHUNK")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=20_000_000)
    ap.add_argument("--interactions", type=int, default=333_333_334)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--heavy", default="", help="comma list of RGPU_HEAVY values: one sealed graph each")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    for hv in (a.heavy.split(",") if a.heavy else [None]):
        if hv is not None:
            os.environ["RGPU_HEAVY"] = hv
        one_graph(a, hv)


def one_graph(a, hv):
    t0 = time.time()
    g = TemporalGraph()
    for first in range(0, a.interactions, 20_000_000):
        s = gen_gab_range(4, a.users, 333_333_334, first, min(20_000_000, a.interactions - first))
        g.ingest_stream(s)
        end = int(s.t[-1])
        del s
    g.seal()
    print(f"built in {time.time() - t0:.1f} s", flush=True)
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    ref = None
    for rnd in range(2):
        for spec in a.variants:
            name, _, kv = spec.partition(":")
            for k in KNOBS:
                os.environ.pop(k, None)
            for item in filter(None, kv.split(",")):
                k, v = item.split("=")
                os.environ[k] = v
            g.run("cc", hops, BATCH_WINDOWS)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(a.steps):
                g.run("cc", hops, BATCH_WINDOWS)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t1) * 1e3 / a.steps
            summ = g.cc_summaries()
            chk = [int(summ[..., 0].sum()), int(summ[..., 1].sum()), int(summ[..., 5].sum())]
            ref = ref or chk
            g.run("cc", hops, BATCH_WINDOWS, profile=True, serial=True)
            ks = {k: [v["launches"], round(v["ms"], 2)] for k, v in g.stats()["kernels"].items() if v["launches"]}
            print(json.dumps({"variant": name, "heavy": hv, "round": rnd, "ms": round(ms, 2), "same": chk == ref, "kernels": ks}),
                  flush=True)
    g.close()


if __name__ == "__main__":
    main()
