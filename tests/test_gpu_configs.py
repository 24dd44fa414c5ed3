"""Every BASELINE.json config at (or near) full size, HIP path against the CPU oracle.

  C1  100k vertices / 1M updates, ViewLens CC at t_end            per-vertex labels, whole view
  C2  same stream, 8,041 hourly hops x {y,m,w,d,h}                full query summaries at 64 hops
                                                                  spread over the range + per-vertex
                                                                  labels of those 320 views
  C3  10M vertices / 100M power-law updates, 61 daily hops x      degree totals of every view
      {month, week, day}, DegreeBasic + PageRank(20)              (properties) + per-vertex degrees
                                                                  and PR (L1 <= 1e-6) at sampled hops
  C4  prefixes of the 1B GAB stream (20M users; 100M and 300M    summaries of all 840 views
      updates), 168 hourly hops x {y,m,w,d,h}, CC                 (properties); at 8 / 4 hops spread
                                                                  over the 168, every window: summary,
                                                                  supersteps and a checksum of every
                                                                  member's label vs the oracle's
                                                                  committed goldens
      the whole 1B stream                                         summary invariants on all 840 views;
                                                                  at 8 hops every window (year too)
                                                                  and the hop's supersteps vs the
                                                                  sliced oracle's goldens; another
                                                                  batch composition of those hops
  C5  30M-update GAB base + one 10M-update hour tick merged       labels / PR / counts equal to a
      into the resident graph, CC + PR(20) on the newest hour     one-shot seal of the same stream
      the bench's C5: 100M-update base + 6 ticks of 10M updates,  every window after ticks 0 and 5 vs
      each merged live, CC {y,m,w,d,h} at the live time           the add-only oracle's goldens; PR(20,
                                                                  hour) at tick 5 vs the oracle (L1)

The oracle at C3/C4 size is the lazy-edge replay (oracle.h ORC_LAZY_EDGES, checked against the
literal replay in tests/test_oracle_scale.py); it is built in a background thread while the GPU
path ingests and seals (ctypes releases the GIL), and per-view queries run in a thread pool.
Reference semantics: ConnectedComponents.scala:10-42,137-145; DegreeBasic.scala:16-28;
SURVEY.md App. A.5 (PageRank spec).
"""
import json
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import (BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, YEAR, gen_gab, gen_gab_range,
                                gen_powerlaw, gen_uniform, range_hops)
from tests.goldens import label_checksum

pytestmark = [pytest.mark.gpu, pytest.mark.fullsize]

PR_L1_TOL = 1e-6  # BASELINE.json north_star: PageRank within 1e-6 L1 per view
POOL = 8          # oracle query threads (the GPU box gives this job 16 host cores)


def _graph(s, order="locality"):
    g = TemporalGraph(vertex_order=order)
    g.ingest_stream(s)
    g.seal()
    return g


def _summary_props(summ):
    """Invariants of processBatchWindowResults fields (ConnectedComponents.scala:137-145) on every
    view: [hops, windows, 8] = biggest, total, >1, islands, >2, sum, sum(>1), supersteps."""
    big, tot, nis, isl, gt2, sall, snis = (summ[..., i] for i in range(7))
    assert np.all(tot == nis + isl) and np.all(gt2 <= nis) and np.all(big <= sall)
    assert np.all(snis <= sall) and np.all((tot == 0) == (sall == 0))
    assert np.all(sall - snis == isl)  # every island is one vertex
    assert np.all((big > 0) == (sall > 0))
    assert np.all(np.diff(sall, axis=1) <= 0)  # descending windows: nested vertex sets (shrinkWindow)


def _check_labels(g, h, w, ids, lab, where):
    gids, glab = g.cc_vertex_labels(h, w)
    assert np.array_equal(gids, ids), where
    assert np.array_equal(glab, lab), where


# ------------------------------------------------------------------ C1
def test_c1_view_cc_at_t_end():
    s = gen_uniform(1, 100_000, 1_000_000)
    t_end = int(s.t[-1])
    with ThreadPoolExecutor(1) as ex:
        fo = ex.submit(Oracle.from_stream, s)
        g = _graph(s)
        g.run("cc", [t_end], [], retain=True)  # ViewLens: no window
        o = fo.result()
    ((ids, lab),), steps = o.cc(t_end, [], mode=1)
    assert len(ids) > 50_000
    _check_labels(g, 0, 0, ids, lab, "C1")
    exp = label_counts(lab)
    assert g.cc_result(0, 0) == exp
    assert cc_fields_from_summary(g.cc_summary(0, 0)) == cc_fields(exp)
    g.close()


# ------------------------------------------------------------------ C2
def test_c2_range_64_spread_hops_per_vertex():
    s = gen_uniform(1, 100_000, 1_000_000)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, HOUR)
    assert len(hops) == 8041
    pick = np.linspace(0, len(hops) - 1, 64).round().astype(int)
    with ThreadPoolExecutor(POOL) as ex:
        fo = ex.submit(Oracle.from_stream, s)
        g = _graph(s)
        g.run("cc", hops, BATCH_WINDOWS)  # the benchmark query: 630 window-major batches
        full = g.cc_summaries()
        _summary_props(full)
        g.run("cc", hops[pick], BATCH_WINDOWS, retain=True)  # other batch composition, same views
        part = g.cc_summaries()
        o = fo.result()
        res = list(ex.map(lambda t: o.cc(int(t), BATCH_WINDOWS, mode=1), hops[pick]))
    for k, h in enumerate(pick):
        assert full[h, 0, 7] == part[k, 0, 7] == res[k][1], (h, full[h, 0, 7], res[k][1])  # supersteps
        for w in range(5):
            ids, lab = res[k][0][w]
            _check_labels(g, k, w, ids, lab, ("C2", int(hops[h]), w))
            exp = cc_fields(label_counts(lab))
            assert cc_fields_from_summary(g.cc_summary(k, w)) == exp, (h, w)
            assert full[h, w, :7].tolist() == part[k, w, :7].tolist(), (h, w)
    g.close()


# ------------------------------------------------------------------ C3
def test_c3_powerlaw_degree_and_pagerank():
    end = T0_README + 2 * YEAR
    s = gen_powerlaw(3, 10_000_000, 100_000_000, t0=T0_README, t1=end)
    hops = range_hops(end - 60 * DAY, end, DAY)
    windows = [MONTH, WEEK, DAY]
    assert len(hops) == 61
    with ThreadPoolExecutor(POOL) as ex:
        fo = ex.submit(Oracle.from_stream, s, True)
        g = _graph(s)
        st = g.stats()
        assert st["vertices"] > 9_000_000 and st["edges"] > 70_000_000
        g.run("degree", hops, windows)
        tot = np.array([[g.degree_result(h, w)[:3] for w in range(3)] for h in range(len(hops))])
        assert np.all(np.diff(tot[..., 0], axis=1) <= 0)  # nested vertex sets
        assert np.all(tot[..., 1] >= 0) and np.all(tot[..., 2] >= 0)
        g.run("pagerank", hops, windows, pr_iters=20)  # the benchmark query runs clean
        sample = [0, 30, 60]
        g.run("degree", hops[sample], windows, retain=True)
        gdeg = {(k, w): g.degree_vertex(k, w) for k in range(len(sample)) for w in range(3)}
        gtot = {(k, w): g.degree_result(k, w)[:3] for k in range(len(sample)) for w in range(3)}
        gtop = {(k, w): g.degree_result(k, w)[3] for k in range(len(sample)) for w in range(3)}
        g.run("pagerank", hops[sample], windows, pr_iters=20, retain=True)
        gpr = {(k, w): g.pr_result(k, w) for k in range(len(sample)) for w in range(3)}
        g.close()
        o = fo.result()
        # per window alone: with descending windows the running-min vertex set is the window's own
        deg = {(k, w): ex.submit(lambda t, w: o.degree(int(t), [windows[w]])[0], hops[h], w)
               for k, h in enumerate(sample) for w in range(3)}
        pr = {(k, w): ex.submit(lambda t, w: o.pagerank(int(t), [windows[w]], iters=20)[0], hops[h], w)
              for k, h in enumerate(sample) for w in range(3)}
        for (k, w), f in deg.items():
            ids, od, idg = f.result()
            gids, god, gid = gdeg[(k, w)]
            assert np.array_equal(gids, ids) and np.array_equal(god, od) and np.array_equal(gid, idg), (k, w)
            assert gtot[(k, w)] == (len(ids), int(od.sum()), int(idg.sum()))
            assert tuple(tot[sample[k], w]) == gtot[(k, w)]  # the 61-hop run agrees
            top = np.lexsort((ids, -idg.astype(np.int64)))[:20]  # DegreeRanking: in-degree desc, ties by id
            assert gtop[(k, w)] == [(int(ids[i]), int(od[i]), int(idg[i])) for i in top], (k, w)
        for (k, w), f in pr.items():  # PageRank at three hops, every window
            ids, p = f.result()
            gids, gp = gpr[(k, w)]
            assert np.array_equal(gids, ids)
            assert np.abs(gp - p).sum() <= PR_L1_TOL, (k, w, np.abs(gp - p).sum())
    o.close()


# ------------------------------------------------------------------ C4
_GOLD_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c4_prefix_goldens.json")
_GOLD = json.load(open(_GOLD_PATH))["prefixes"] if os.path.exists(_GOLD_PATH) else {}


@pytest.mark.parametrize("inter", sorted(_GOLD, key=int))
def test_c4_prefix_vs_oracle_goldens(inter):
    """C4 on prefixes of the 1B stream against the oracle's results committed by
    tools/make_c4_goldens.py: the whole 168-hop x 5-window query, and at every sampled hop (spread
    over the 168) every window (year, month, week, day, hour): summary fields, the hop's superstep
    count, member count and the checksum of every member's (id, label)."""
    P = _GOLD[inter]
    n = int(inter)
    g = TemporalGraph()
    for first in range(0, n, 20_000_000):
        s = gen_gab_range(4, 20_000_000, 333_333_334, first, min(20_000_000, n - first))
        g.ingest_stream(s)
        end = int(s.t[-1])
        del s
    g.seal()
    assert g.stats()["vertices"] == P["vertices"]
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    assert len(hops) == P["n_hops"] and int(hops[0]) == P["hop0"]
    g.run("cc", hops, BATCH_WINDOWS)
    full = g.cc_summaries()
    _summary_props(full)
    pick = sorted(int(h) for h in P["hops"])
    g.run("cc", hops[pick], BATCH_WINDOWS, retain=True)
    for k, h in enumerate(pick):
        rec = P["hops"][str(h)]
        assert int(hops[h]) == rec["t"]
        assert full[h, 0, 7] == rec["supersteps"], (h, full[h, 0, 7], rec["supersteps"])
        for w in range(5):
            exp = rec["windows"][w]
            got = dict(zip(("biggest", "total", "total_without_islands", "total_islands", "clusters_gt2", "sum_all",
                            "sum_without_islands"), full[h, w, :7].tolist()))
            for f in ("biggest", "total", "total_without_islands", "clusters_gt2", "sum_all", "sum_without_islands"):
                assert got[f] == exp[f], (h, w, f, got[f], exp[f])
            ids, lab = g.cc_vertex_labels(k, w)
            assert len(ids) == exp["members"], (h, w)
            assert label_checksum(ids, lab) == exp["label_checksum"], (h, w)
    g.close()


_SLICED_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c4_sliced_goldens.json")
_SLICED = json.load(open(_SLICED_PATH)) if os.path.exists(_SLICED_PATH) else None
_FIELDS = ("biggest", "total", "total_without_islands", "total_islands", "clusters_gt2", "sum_all",
           "sum_without_islands")


def _check_view(full_row, ids, lab, exp, where):
    got = dict(zip(_FIELDS, full_row[:7].tolist()))
    for f in ("biggest", "total", "total_without_islands", "clusters_gt2", "sum_all", "sum_without_islands"):
        assert got[f] == exp[f], (where, f, got[f], exp[f])
    assert len(ids) == exp["members"], where
    assert label_checksum(ids, lab) == exp["label_checksum"], where


def test_c4_full_1b_vs_sliced_oracle_goldens():
    """The headline query itself: the whole 1B-update C4 stream, 168 hourly hops x {y,m,w,d,h}.
    Summary invariants on all 840 views; at the 30 hops of tests/golden/c4_sliced_goldens.json
    (spread over the 168; 8 in round 5, 22 more in round 6), the month, week, day and hour views against the oracle — summary
    fields, member count and the checksum of every member's (id, label).  The oracle replays the
    stream's last 37 days, which is exact for these windows on an add-only stream
    (tools/make_c4_sliced_goldens.py; tests/test_c4_slice.py checks it on the 100M prefix).
    The year views (round 5): the add-only restatement of the oracle over the year slice
    (tools/make_c4_sliced_goldens.py --year; it reproduces the literal replay's month..hour records
    at every sampled hop) gives their records and the hops' superstep counts too.  The sampled hops
    re-run as one hop-major batch (other superstep interleaving, other heavy / uniform-word paths)
    must also give the window-major query's summaries."""
    users, inter = 20_000_000, 333_333_334
    g = TemporalGraph()
    for first in range(0, inter, 20_000_000):
        s = gen_gab_range(4, users, inter, first, min(20_000_000, inter - first))
        g.ingest_stream(s)
        end = int(s.t[-1])
        del s
    g.seal()
    st = g.stats()
    assert st["vertices"] > 19_000_000 and st["edges"] > 280_000_000
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    g.run("cc", hops, BATCH_WINDOWS)
    full = g.cc_summaries()
    _summary_props(full)
    assert np.all(full[..., 5] > 0)
    pick = sorted(int(h) for h in _SLICED["hops"]) if _SLICED else [0, 83, 167]
    g.run("cc", hops[pick], BATCH_WINDOWS, retain=_SLICED is not None)
    part = g.cc_summaries()
    for k, h in enumerate(pick):
        assert full[h, :, :7].tolist() == part[k, :, :7].tolist(), h
    if _SLICED is not None:
        assert int(hops[0]) == _SLICED["hop0"] and len(hops) == _SLICED["n_hops"]
        for k, h in enumerate(pick):
            rec = _SLICED["hops"][str(h)]
            assert int(hops[h]) == rec["t"]
            if "supersteps" in rec:  # (the year views are in: the hop's count, over its five views, is the oracle's)
                got = int(full[h, :, 7].max())
                assert got == rec["supersteps"], (h, full[h, :, 7].tolist(), rec["supersteps"])
            for j, w in enumerate(_SLICED["window_index_in_query"]):
                ids, lab = g.cc_vertex_labels(k, w)
                _check_view(full[h, w], ids, lab, rec["windows"][j], ("1B", h, w))
    g.close()


@pytest.mark.skipif("33333334" not in _GOLD, reason="no 100M-prefix goldens")
def test_c4_prefix_partitioned_p8_vs_oracle_goldens():
    """The vertex-partitioned path at C4 size: the 100M-update prefix as 8 loopback partitions
    (Utils.getPartition placement, ghost copies, the per-superstep record exchange, routed
    component counts) on one GPU, the whole 168-hop x 5-window query, against the oracle's
    goldens at 8 hops: every window's merged summary, the hop's superstep count, member count and
    the checksum of every member's (id, label)."""
    from raphtory_amd.partitioned import LoopbackPartitions
    P = _GOLD["33333334"]
    n = 33_333_334
    lp = LoopbackPartitions(8)
    for first in range(0, n, 10_000_000):
        s = gen_gab_range(4, 20_000_000, 333_333_334, first, min(10_000_000, n - first))
        lp.ingest_stream(s)
        end = int(s.t[-1])
        del s
    lp.seal()
    assert sum(st["vertices"] for st in lp.stats()) == P["vertices"]
    assert sum(st["edges_owned"] for st in lp.stats()) == P["edges"]
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    assert int(hops[0]) == P["hop0"]
    lp.run("cc", hops, BATCH_WINDOWS)
    full = lp.parts[0].cc_summaries()
    _summary_props(full)
    for g in lp.parts[1:]:  # every partition holds the merged summaries
        assert np.array_equal(g.cc_summaries(), full)
    pick = sorted(int(h) for h in P["hops"])
    lp.run("cc", hops[pick], BATCH_WINDOWS, retain=True)
    for k, h in enumerate(pick):
        rec = P["hops"][str(h)]
        assert full[h, 0, 7] == rec["supersteps"], (h, full[h, 0, 7], rec["supersteps"])
        for w in range(5):
            ids, lab = lp.cc_vertex_labels(k, w)
            _check_view(full[h, w], ids, lab, rec["windows"][w], ("P8", h, w))
    lp.close()


def cc_fields_from_summary_row(row):
    from raphtory_amd._native import CCSummary
    s = CCSummary()
    for (f, _), v in zip(CCSummary._fields_, row.tolist()):
        setattr(s, f, v)
    return cc_fields_from_summary(s)


# ------------------------------------------------------------------ C5
def test_c5_ten_million_update_tick_equals_one_shot_seal():
    users = 20_000_000
    base = gen_gab(4, users, 10_000_000)
    now = int(base.t[-1])
    tick = gen_gab(100, users, 3_333_334, t0=now + 1, t1=now + HOUR, id_key=4)
    assert len(tick) == 10_000_002
    now = int(tick.t[-1])
    live = _graph(base, "id")
    live.ingest_stream(tick)
    live.seal()  # merged into the resident graph (merge.hip)
    assert live.stats()["seal_incremental"] == 1 and live.stats()["seal_delta_updates"] == len(tick)
    one = TemporalGraph()
    one.ingest_stream(base)
    one.ingest_stream(tick)
    one.seal()
    a, b = live.stats(), one.stats()
    for k in ("vertices", "edges", "vertex_events", "edge_events", "deaths"):
        assert a[k] == b[k], k
    for g in (live, one):
        g.run("cc", [now], BATCH_WINDOWS, retain=True)
    for w in range(5):
        ia, la = live.cc_vertex_labels(0, w)
        ib, lb = one.cc_vertex_labels(0, w)
        assert np.array_equal(ia, ib) and np.array_equal(la, lb), w
        assert live.cc_summaries()[0, w].tolist() == one.cc_summaries()[0, w].tolist()
    for g in (live, one):
        g.run("pagerank", [now], [HOUR], pr_iters=20, retain=True)
    ia, pa = live.pr_result(0, 0)
    ib, pb = one.pr_result(0, 0)
    assert np.array_equal(ia, ib) and np.abs(pa - pb).sum() <= PR_L1_TOL
    live.close()
    one.close()


_C5_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c5_goldens.json")


@pytest.mark.skipif(not os.path.exists(_C5_PATH), reason="no C5 goldens")
def test_c5_live_at_size_vs_oracle():
    """BASELINE configs[4] as bench.py --config c5 runs it at N = 1: the 100M-update base sealed, then
    6 hour ticks of 10M updates each ingested and merged into the resident graph (the live path:
    device delta packer + merge; after the first run every merged graph is parked and swapped in by
    the next run).  After ticks 0 and 5, CC over {y,m,w,d,h} at the live time (the newest update,
    LiveAnalysisTask.setLiveTime) against the oracle's goldens (tools/make_c5_goldens.py: the
    add-only restatement over the whole C5 stream): every window's summary fields, member count and
    (id, label) checksum, and the hop's superstep count.  After tick 5, PageRank(20, hour) against
    the literal oracle replaying the updates of the last hour (an add-only view depends on nothing
    older), L1 <= 1e-6."""
    from tools.make_c5_goldens import c5_stream
    G = json.load(open(_C5_PATH))
    base, ticks = c5_stream()
    g = _graph(base, "id")
    del base
    for i, tick in enumerate(ticks):
        g.ingest_stream(tick)
        g.seal()
        assert g.stats()["seal_incremental"] == 1
        live = g.newest_time()
        rec = G["at"].get(str(i))
        g.run("cc", [live], BATCH_WINDOWS, retain=rec is not None)
        if rec is None:
            continue
        assert live == rec["live"]
        full = g.cc_summaries()
        assert full[0, 0, 7] == rec["supersteps"], (i, full[0, 0, 7], rec["supersteps"])
        for w in range(5):
            ids, lab = g.cc_vertex_labels(0, w)
            _check_view(full[0, w], ids, lab, rec["windows"][w], ("C5 tick", i, w))
    # PageRank(20) over the newest hour, against the literal replay of the updates of the last hour
    # (from every tick: ticks overlap in time; the base ends hours before)
    g.run("pagerank", [live], [HOUR], pr_iters=20, retain=True)
    keep = [x.t >= live - HOUR for x in ticks]
    o = Oracle(*(np.concatenate([getattr(x, f)[k] for x, k in zip(ticks, keep)]) for f in ("t", "kind", "src", "dst")))
    (ids, pr), = o.pagerank(live, [HOUR], iters=20)
    gids, gpr = g.pr_result(0, 0)
    assert np.array_equal(gids, ids)
    assert np.abs(gpr - pr).sum() <= PR_L1_TOL
    o.close()
    g.close()
