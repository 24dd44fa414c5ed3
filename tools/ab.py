"""Same-process A/B timing on one sealed graph (measurement tool, not part of the product): the
C4 stream (or a prefix) is generated and sealed once, then the CC query runs under each setting
of one environment variable that the library reads per launch, in interleaved rounds.  Prints
one JSON line per (round, setting): wall ms of the query and, with --profile, the serial
per-kernel ms of a lean profile pass (RGPU_PROF_LEAN).

usage: python tools/ab.py --var RGPU_AB --values 0,1 [--interactions N] [--rounds 2] [--profile]
       python tools/ab.py --settings "base,RGPU_A=1,RGPU_A=2+RGPU_B=1" ...  (several variables: each
       setting sets its K=V pairs and unsets the others' keys; "base" sets nothing)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range, range_hops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", default="")
    ap.add_argument("--values", default="")
    ap.add_argument("--settings", default="")
    ap.add_argument("--interactions", type=int, default=333_333_334)
    ap.add_argument("--users", type=int, default=20_000_000)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--config", default="c4", choices=["c4", "c2"], help="c2: the 8,041-hop C2 query instead")
    a = ap.parse_args()
    g = TemporalGraph()
    t0 = time.time()
    if a.config == "c2":  # bench.py run_c2's stream and hops
        from raphtory_amd.synth import DAY, T0_README, gen_uniform
        g.ingest_stream(gen_uniform(1, 100_000, 1_000_000))
        hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, HOUR)
    else:
        for first in range(0, a.interactions, 20_000_000):
            s = gen_gab_range(4, a.users, 333_333_334, first, min(20_000_000, a.interactions - first))
            g.ingest_stream(s)
            end = int(s.t[-1])
            del s
        hops = range_hops(end - 167 * HOUR, end, HOUR)
    g.seal()
    print(f"sealed in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    if a.settings:
        settings = [dict(kv.split("=", 1) for kv in st.split("+") if kv != "base") for st in a.settings.split(",")]
    else:
        settings = [{a.var: v} for v in a.values.split(",")]
    keys = sorted({k for st in settings for k in st})
    ref = None
    for rnd in range(a.rounds):
        for st in settings:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(st)
            val = "+".join(f"{k}={v}" for k, v in st.items()) or "base"
            g.run("cc", hops, BATCH_WINDOWS)  # warm
            t = time.perf_counter()
            g.run("cc", hops, BATCH_WINDOWS)
            ms = (time.perf_counter() - t) * 1e3
            summ = g.cc_summaries()[..., :8]
            same = ref is None or bool((summ == ref).all())
            ref = summ if ref is None else ref
            out = {"round": rnd, (a.var or "setting"): (st.get(a.var) if a.var else val), "query_ms": round(ms, 2),
                   "summaries_equal": same}
            if a.profile:
                os.environ["RGPU_PROF_LEAN"] = "1"
                g.run("cc", hops, BATCH_WINDOWS, profile=True, serial=True)
                os.environ.pop("RGPU_PROF_LEAN")
                out["serial_ms"] = {k: round(v["ms"], 1) for k, v in g.stats()["kernels"].items() if v["launches"]}
            print(json.dumps(out), flush=True)
    g.close()


if __name__ == "__main__":
    main()
