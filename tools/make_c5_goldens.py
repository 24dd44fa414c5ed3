"""TEST INFRASTRUCTURE: oracle goldens for C5 at size (BASELINE configs[4], bench.py --config c5):
the 100M-update GAB base (seed 4, 20M users) followed by 6 hour ticks of 10M updates (seeds
100..105, id_key 4, each drawn for (now, now + 1 h]), committed as tests/golden/c5_goldens.json.

The whole C5 stream is add-only.  Its ticks overlap in time (a tick drawn for (now, now + 1 h]
runs ~1.6 h past now: the generator's diurnal shape), but an add-only history is the set of its
add times whatever the arrival order (every put is an add; equal times collapse to an add), so the
stream sorted by time has the same views, and the add-only restatement of the oracle (oracle.h
orc_addonly_*, checked against the literal replay in tests/test_oracle_addonly.py) replays all
stream as ingested up to a tick (base + ticks 0..i; 160M updates at the last) and gives
ConnectedComponents over
{year, month, week, day, hour} at the live time after a tick: per window the summary fields
(ConnectedComponents.scala:137-145), member count and (id, label) checksum, and the hop's superstep
count.  The live time after tick i is the newest update time so far (LiveAnalysisTask.setLiveTime,
one partition).  tests/test_gpu_configs.py test_c5_live_at_size_vs_oracle merges the ticks into the
resident graph one by one (the live path) and compares.  PageRank(20, hour) at the last tick is
checked there against the literal replay of the last hour's updates (exact for an add-only view).

usage: python tools/make_c5_goldens.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import AddOnlyOracle  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range  # noqa: E402
from tools.make_c4_goldens import view_record  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "c5_goldens.json")
USERS, BASE, TICK, TICKS = 20_000_000, 33_333_334, 3_333_334, 6
CHECK_TICKS = (0, TICKS - 1)


def c5_stream():
    """(base, [tick streams]) exactly as bench.py run_c5 draws them at N = 1"""
    base = gen_gab_range(4, USERS, BASE, 0, BASE)
    now = int(base.t[-1])
    ticks = []
    for i in range(TICKS):
        ticks.append(gen_gab_range(100 + i, USERS, TICK, 0, TICK, t0=now + 1, t1=now + HOUR, id_key=4))
        now += HOUR
    return base, ticks


def main():
    t0 = time.time()
    base, ticks = c5_stream()
    lives = np.maximum.accumulate([int(x.t.max()) for x in ticks]).tolist()  # newest time after tick i
    n_base = len(base)
    out = {"note": __doc__.split("\n\n")[0], "users": USERS, "base_interactions": BASE, "base_updates": n_base,
           "tick_interactions": TICK, "ticks": TICKS, "windows": list(BATCH_WINDOWS), "at": {}}
    for i in CHECK_TICKS:
        # the stream as ingested up to tick i (the next ticks overlap tick i's times: they are not in yet)
        cols = [np.concatenate([getattr(base, f)] + [getattr(x, f) for x in ticks[:i + 1]])
                for f in ("t", "kind", "src", "dst")]
        order = np.argsort(cols[0], kind="stable")
        o = AddOnlyOracle(*(c[order] for c in cols))
        del cols, order
        res, steps = o.cc(lives[i], BATCH_WINDOWS)
        out["at"][str(i)] = {"live": lives[i], "supersteps": int(steps),
                             "windows": [view_record(ids, lab) for ids, lab in res]}
        print(f"tick {i}: live {lives[i]}, {steps} supersteps, members "
              f"{[r['members'] for r in out['at'][str(i)]['windows']]} ({time.time() - t0:.0f} s)", flush=True)
        o.close()
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"-> {OUT}", flush=True)


if __name__ == "__main__":
    main()
