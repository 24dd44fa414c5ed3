"""TEST INFRASTRUCTURE: oracle goldens for the views of the REAL 1B-update C4 headline query
(BASELINE configs[3]: 168 hourly hops x {year, month, week, day, hour}), computed from a time
slice of the stream, committed as tests/golden/c4_sliced_goldens.json.

Why a slice is exact (Entity.scala:173-201):
  * C4 is add-only (GabUserGraphRouter.scala:31-33: VertexAdd src, VertexAdd dst, EdgeAdd at one
    t), so every history point is an add and no vertex ever dies (no killList entries).
  * aliveAtWithWindow(t, w) = floor(t) is an add and t - floor(t).time <= w.  For an add-only
    history that holds iff the entity has a point in [t - w, t], and then floor(t) is the newest
    such point — which the slice holds as well.  Points older than t - w decide nothing.
  * The batched vertex set of window i uses min(w_0..w_i) (shrinkWindow); for the descending
    {y, m, w, d, h} that is w_i itself, so dropping the year window changes no other window's
    vertex set, and each window's edges use w_i alone (WindowLens.scala:54-65).
  * CC labels after R rounds are min{id(u): dist_w(u, v) <= R} with R = min(100, the hop's
    superstep count).  A hop whose month/week/day/hour views converge before the year view only
    runs empty rounds for them, and a capped hop caps every window at 100 either way: the
    per-window labels do not depend on whether the year view rides along.  (The hop's
    superstep count does — it is not recorded here.)
So the views (t, w) for t in [hop0, hop167], w <= month, depend only on the interactions with
time >= hop0 - month: ~37 days, ~56M of the 1B updates, which the oracle replays in ~8 GB.
The year window (a year of the stream) stays out: ~550M updates do not fit the oracle here.

tests/test_c4_slice.py checks the argument on the 100M-update prefix, whose views the oracle
replayed in full (tests/golden/c4_prefix_goldens.json): the sliced replay must give the same
summary, member count and label checksum in every window it covers.

The slice's first interaction is found by bisection on the generator itself (gen_gab_range
draws any interaction range; times are monotone in the index, synth.c rg_gen_gab_range).

Round 5, --year: the year views too.  A year of the stream (~550M updates) does not fit the
literal replay here (~200 B per update), so the add-only restatement (oracle.h orc_addonly_*, the
view read off the time-sorted stream; checked against the literal replay in
tests/test_oracle_addonly.py and on the 100M / 300M prefix goldens) replays the year slice and
gives all five windows and the hop's superstep count.  Its month / week / day / hour records must
equal the literal-replay records already in the file (the run stops otherwise); the year records
and the superstep counts are added.

usage: python tools/make_c4_sliced_goldens.py [--hops 8] [--threads 8] [--year]
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

from oracle import Oracle  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, MONTH, gen_gab_range, range_hops  # noqa: E402
from tools.make_c4_goldens import picks, view_record  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "c4_sliced_goldens.json")
SEED, USERS, INTER = 4, 20_000_000, 333_333_334


def t_of(i: int, inter: int = INTER) -> int:
    """time of interaction i of the `inter`-interaction C4 stream"""
    return int(gen_gab_range(SEED, USERS, inter, i, 1).t[0])


def first_at(t_from: int, n: int, inter: int = INTER) -> int:
    """first interaction index in [0, n) with time >= t_from (n if none)"""
    lo, hi = 0, n
    while lo < hi:
        mid = (lo + hi) // 2
        if t_of(mid, inter) >= t_from:
            hi = mid
        else:
            lo = mid + 1
    return lo


def headline_hops(n: int, inter: int = INTER) -> np.ndarray:
    """the C4 query's 168 hourly hops ending at the newest update of the first n interactions"""
    end = t_of(n - 1, inter)
    return range_hops(end - 167 * HOUR, end, HOUR)


def sliced_stream(n: int, t_from: int, inter: int = INTER, chunk: int = 20_000_000):
    """interactions [first_at(t_from), n) as one stream, and that first index"""
    first = first_at(t_from, n, inter)
    parts = [gen_gab_range(SEED, USERS, inter, a, min(chunk, n - a)) for a in range(first, n, chunk)]
    from raphtory_amd.synth import Stream
    cat = Stream(*(np.concatenate([getattr(p, f) for p in parts]) for f in ("t", "kind", "src", "dst")))
    return cat, first


def sliced_views(n: int, windows, sel, threads: int, inter: int = INTER, log=print):
    """oracle per-window records at the sampled hop indices `sel` of the query over the first n
    interactions, replaying only the interactions that can be alive in the widest window given"""
    t0 = time.time()
    hops = headline_hops(n, inter)
    s, first = sliced_stream(n, int(hops[0]) - max(windows), inter)
    o = Oracle.from_stream(s, True)
    meta = {"first_interaction": int(first), "slice_updates": int(len(s)), "slice_t0": int(s.t[0]),
            "vertices": int(o.nv), "edges": int(o.ne), "hop0": int(hops[0]), "n_hops": int(len(hops))}
    del s
    log(f"slice of {n} interactions from {first}: {meta['slice_updates']} updates, oracle built in "
        f"{time.time() - t0:.0f} s ({o.nv} vertices, {o.ne} edges)")

    def one(h):
        res, _ = o.cc(int(hops[h]), windows, mode=1)
        return h, [view_record(ids, lab) for ids, lab in res]

    views = {}
    with ThreadPoolExecutor(threads) as ex:
        for h, recs in ex.map(one, sel):
            views[str(h)] = {"t": int(hops[h]), "windows": recs}
            log(f"  hop {h}: {time.time() - t0:.0f} s")
    o.close()
    return meta, views


def verify_prefix(threads: int, out_path: str) -> bool:
    """the slice argument on the 100M-update prefix, month window included: the sliced replay
    against the full-prefix replay committed in tests/golden/c4_prefix_goldens.json"""
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_prefix_goldens.json")))["prefixes"]
    lines = []

    def log(m):
        print(m, flush=True)
        lines.append(m)

    ok = True
    for key in sorted(gold, key=int):
        P = gold[key]
        n = int(key)
        sel = sorted(int(h) for h in P["hops"])
        meta, views = sliced_views(n, BATCH_WINDOWS[1:], sel, threads, log=log)
        for h in sel:
            for k, rec in enumerate(views[str(h)]["windows"]):
                same = rec == P["hops"][str(h)]["windows"][1 + k]
                ok &= same
                log(f"prefix {n} interactions, hop {h}, window {BATCH_WINDOWS[1 + k]}: "
                    f"members {rec['members']}, checksum {rec['label_checksum']} "
                    f"{'== full replay' if same else '!= FULL REPLAY'}")
    log("slice equivalence: " + ("all views equal" if ok else "MISMATCH"))
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return ok


def sliced_arrays(n: int, t_from: int, inter: int = INTER, chunk: int = 20_000_000):
    """interactions [first_at(t_from), n) generated straight into preallocated columns (no
    concatenated copy: a year slice is ~550M updates), and that first index"""
    first = first_at(t_from, n, inter)
    m = 3 * (n - first)
    t, k, s, d = (np.empty(m, np.int64), np.empty(m, np.uint8), np.empty(m, np.int64), np.empty(m, np.int64))
    o = 0
    for a in range(first, n, chunk):
        p = gen_gab_range(SEED, USERS, inter, a, min(chunk, n - a))
        q = len(p)
        t[o:o + q], k[o:o + q], s[o:o + q], d[o:o + q] = p.t, p.kind, p.src, p.dst
        o += q
        del p
    assert o == m
    return (t, k, s, d), first


def year_views(n: int, sel, threads: int, inter: int = INTER, log=print):
    """all five windows and the hop's superstep count at the sampled hops, by the add-only
    restatement over the year slice"""
    from oracle import AddOnlyOracle
    from raphtory_amd.synth import YEAR
    t0 = time.time()
    hops = headline_hops(n, inter)
    (t, k, s, d), first = sliced_arrays(n, int(hops[0]) - YEAR, inter)
    log(f"year slice from interaction {first}: {len(t)} updates generated in {time.time() - t0:.0f} s")
    o = AddOnlyOracle(t, k, s, d)
    meta = {"year_first_interaction": int(first), "year_slice_updates": int(len(t)), "year_slice_t0": int(t[0]),
            "year_slice_vertices": int(o.nv)}
    del k, s, d
    log(f"add-only oracle built in {time.time() - t0:.0f} s ({o.nv} vertices)")

    def one(h):
        res, steps = o.cc(int(hops[h]), BATCH_WINDOWS)
        return h, steps, [view_record(ids, lab) for ids, lab in res]

    views = {}
    with ThreadPoolExecutor(threads) as ex:
        for h, steps, recs in ex.map(one, sel):
            views[str(h)] = {"t": int(hops[h]), "supersteps": int(steps), "windows": recs}
            log(f"  hop {h}: {steps} supersteps, {time.time() - t0:.0f} s")
    o.close()
    return meta, views


def add_year(threads: int):
    data = json.load(open(OUT))
    assert data["windows"] == BATCH_WINDOWS[1:] and data["window_index_in_query"] == [1, 2, 3, 4]
    sel = sorted(int(h) for h in data["hops"])
    meta, views = year_views(INTER, sel, threads, log=lambda m: print(m, flush=True))
    for h in sel:
        old = data["hops"][str(h)]
        new = views[str(h)]
        assert new["t"] == old["t"], h
        # the literal replay's month..hour records (already committed) must be reproduced exactly
        for j in range(4):
            if new["windows"][1 + j] != old["windows"][j]:
                raise SystemExit(f"hop {h} window {BATCH_WINDOWS[1 + j]}: add-only {new['windows'][1 + j]} != "
                                 f"literal {old['windows'][j]}")
        print(f"hop {h}: month..hour == literal replay; year members {new['windows'][0]['members']}, "
              f"{new['supersteps']} supersteps", flush=True)
        data["hops"][str(h)] = {"t": new["t"], "supersteps": new["supersteps"], "windows": new["windows"]}
    data["windows"] = list(BATCH_WINDOWS)
    data["window_index_in_query"] = [0, 1, 2, 3, 4]
    data["year_oracle"] = ("add-only restatement (oracle.h orc_addonly_cc) over the year slice; month..hour "
                           "equal to the literal replay over the 37-day slice")
    data.update(meta)
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"-> {OUT}", flush=True)


def extend(k: int, threads: int):
    """Round 6 (40 of the 840 views were oracle-checked): k more hops, the ones of
    picks(168, k) not in the file yet.  Their month..hour records come from the literal replay over the
    37-day slice and their year record and superstep count from the add-only restatement over the year
    slice; the add-only month..hour records must equal the literal replay's (the run stops otherwise), as
    for the first eight."""
    data = json.load(open(OUT))
    assert data["windows"] == list(BATCH_WINDOWS)
    have = {int(h) for h in data["hops"]}
    sel = [h for h in picks(168, k) if h not in have]
    log = lambda m: print(m, flush=True)  # noqa: E731
    log(f"extending {sorted(have)} by {sel}")
    _, lit = sliced_views(INTER, BATCH_WINDOWS[1:], sel, threads, log=log)
    _, yv = year_views(INTER, sel, threads, log=log)
    for h in sel:
        new, old = yv[str(h)], lit[str(h)]
        assert new["t"] == old["t"], h
        for j in range(4):
            if new["windows"][1 + j] != old["windows"][j]:
                raise SystemExit(f"hop {h} window {BATCH_WINDOWS[1 + j]}: add-only {new['windows'][1 + j]} != "
                                 f"literal {old['windows'][j]}")
        log(f"hop {h}: month..hour == literal replay; year members {new['windows'][0]['members']}, "
            f"{new['supersteps']} supersteps")
        data["hops"][str(h)] = {"t": new["t"], "supersteps": new["supersteps"], "windows": new["windows"]}
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    log(f"-> {OUT} ({len(data['hops'])} hops)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--extend", type=int, default=0,
                    help="add the hops of picks(168, N) not in the file yet (all five windows, both oracles)")
    ap.add_argument("--hops", type=int, default=8, help="hops sampled over the 168")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--verify-prefix", action="store_true",
                    help="check the slice argument against the full-prefix goldens (month..hour)")
    ap.add_argument("--year", action="store_true",
                    help="add the year views and superstep counts (add-only oracle over the year slice)")
    a = ap.parse_args()
    if a.extend:
        return extend(a.extend, a.threads)
    if a.year:
        return add_year(a.threads)
    if a.verify_prefix:
        sys.exit(0 if verify_prefix(a.threads, os.path.join(ROOT, "profiles", "r04", "c4_slice_equivalence.txt"))
                 else 1)
    windows = BATCH_WINDOWS[1:]  # month, week, day, hour
    assert windows[0] == MONTH
    t0 = time.time()
    sel = picks(168, a.hops)
    meta, views = sliced_views(INTER, windows, sel, a.threads, log=lambda m: print(m, flush=True))
    data = {"note": __doc__.split("\n\n")[0], "interactions": INTER, "updates": 3 * INTER,
            "windows": list(windows), "window_index_in_query": [1, 2, 3, 4], **meta, "hops": views}
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"done in {time.time() - t0:.0f} s -> {OUT}", flush=True)


if __name__ == "__main__":
    main()
