"""Host mirrors of the reference's analysis plugin surface on the GPU path, against the CPU oracle:

* DegreeRanking (DegreeRanking.scala:14-26): the top 20 by in-degree of every view comes from
  the device (k_deg_top_merge) without RGPU_RUN_RETAIN; ties by ascending id.  Checked exactly
  against the oracle's degrees, and its result lines ("bestusers") against lines built from them.
* LiveAnalysisTask / WindowedLiveAnalysisTask / BWindowedLiveAnalysisTask
  (LiveTasks/LiveAnalysisTask.scala:13-107): timestamps = the minimum newest time over the
  partitions, event-time restarts at liveTime + repeatTime (waiting for ingest), processing-time
  restarts at the then-current minimum; the windowed live tasks run un-windowed.
  Each job's line equals ConnectedComponents' line for the oracle's view at that timestamp.
"""
import re

import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import (BWindowedLiveAnalysisTask, BWindowedRangeAnalysisTask, ConnectedComponents,
                                   DegreeRanking, LiveAnalysisTask, WindowedLiveAnalysisTask, cc_fields)
from raphtory_amd.partitioned import LoopbackPartitions
from raphtory_amd.synth import BATCH_WINDOWS, DAY, MONTH, T0_README, WEEK, YEAR, Stream, gen_gab, gen_powerlaw, \
    gen_uniform, range_hops

pytestmark = pytest.mark.gpu


def expected_top(o, t, windows):
    """oracle degrees -> per window [(id, out, in)] of the 20 largest in-degrees, ties by id"""
    out = []
    for ids, od, idg in o.degree(t, windows):
        order = np.lexsort((ids, -idg.astype(np.int64)))[:20]
        out.append([(int(ids[i]), int(od[i]), int(idg[i])) for i in order])
    return out


@pytest.mark.parametrize("heavy", ["2048", "40"])
def test_degree_ranking_top20_without_retain(heavy, monkeypatch):
    monkeypatch.setenv("RGPU_HEAVY", heavy)  # 40: hubs' in-degrees come from k_heavy_degree
    s = gen_powerlaw(13, 4000, 120_000, t0=0, t1=2 * YEAR)
    o = Oracle.from_stream(s)
    hops = range_hops(YEAR, 2 * YEAR, 20 * DAY)
    wins = [YEAR, MONTH, WEEK]
    with TemporalGraph() as g:
        g.ingest_stream(s)
        g.seal()
        g.run("degree", hops, wins)  # no retain
        for h, t in enumerate(hops.tolist()):
            exp = expected_top(o, t, wins)
            for w in range(len(wins)):
                tv, to, ti, top = g.degree_result(h, w)
                assert top == exp[w], (t, w)
        # the result lines of a batched-window range job
        a = DegreeRanking()
        # (the range ends at the newest ingested time: a later end waits for ingestion)
        task = BWindowedRangeAnalysisTask([g], a, int(hops[0]), int(s.t.max()), 20 * DAY, wins, retain_results=False)
        lines = task.run()
        want = []
        for t in task.hops().tolist():
            for w, (ids, od, idg) in zip(wins, o.degree(t, wins)):
                tv, te = len(ids), int(idg.sum())
                top = expected_top(o, t, [w])[0]
                best = "[" + ",".join(f'{{"id":{i},"indegree":{d},"outdegree":{u}}}' for i, u, d in top) + "]"
                deg = DegreeRanking._body([(tv, int(od.sum()), te, top)])
                assert deg.endswith(f'"bestusers":{best}')
                want.append(f'{{"time":{t},"windowsize":{w},{deg},')
        strip = [re.sub(r'"viewTime":-?\d+,"concatTime":0},$', "", x) for x in lines]
        assert strip == want


def test_degree_ranking_partitioned_shards():
    """per-partition top lists (the per-shard returnResults); merged like the reference's lines"""
    s = gen_powerlaw(14, 3000, 60_000, t0=0, t1=YEAR)
    o = Oracle.from_stream(s)
    lp = LoopbackPartitions(3)
    lp.ingest_stream(s)
    lp.seal()
    hops = range_hops(YEAR // 2, YEAR, 30 * DAY)
    lp.run("degree", hops, [MONTH, WEEK])
    for h, t in enumerate(hops.tolist()):
        exp = expected_top(o, t, [MONTH, WEEK])
        for w in range(2):
            tops = [p.degree_result(h, w)[3] for p in lp.parts]
            merged = sorted((u for tp in tops for u in tp), key=lambda u: (-u[2], u[0]))[:20]
            assert merged == exp[w], (t, w)
    lp.close()


def _cc_line(o, t):
    res, _ = o.cc(t, [])
    f = cc_fields(label_counts(res[0][1]))
    return ConnectedComponents._line(t, None, f, 0) if f is not None else f"No activity for  view at {t}"


def _strip(lines):
    return [re.sub(r'"viewTime":-?\d+', '"viewTime":0', x) for x in lines]


@pytest.mark.parametrize("cls", ["live", "windowed", "bwindowed"])
def test_live_tasks_event_time(cls):
    s = gen_uniform(17, 600, 30_000, t0=T0_README, dt=1_051_200)
    arrs = [s.t, s.kind, s.src, s.dst]
    cuts = [10_000, 14_000, 21_000, 30_000]
    R = 40 * DAY
    with TemporalGraph(vertex_order="id") as g:
        a = ConnectedComponents()
        task = {"live": lambda: LiveAnalysisTask([g], a, R, True),
                "windowed": lambda: WindowedLiveAnalysisTask([g], a, R, True, MONTH),
                "bwindowed": lambda: BWindowedLiveAnalysisTask([g], a, R, True, BATCH_WINDOWS)}[cls]()
        lo, got, want = 0, [], []
        live_time = None
        for hi in cuts:
            g.ingest(*[x[lo:hi] for x in arrs])
            g.seal()
            lo = hi
            newest = int(s.t[hi - 1])
            while True:
                ts = task.timestamp()
                out = task.tick()
                if out is None:  # not ingested yet: the job waits
                    assert ts > newest
                    break
                ts = task.last_job_time
                if live_time is None:
                    assert ts == newest  # the first job: the minimum newest time
                else:
                    assert ts == live_time + R  # event time: liveTime of the previous check + repeatTime
                live_time = newest
                got += out
                want.append(_cc_line(Oracle(*[x[:hi] for x in arrs]), ts))
        assert len(got) >= 4
        assert _strip(got) == _strip(want)


def test_live_task_processing_time_and_partitions():
    """processing time: every job at the then-current minimum newest time; on 3 loopback
    partitions (each partition's newest time from its own ingest) against the oracle"""
    s = gen_gab(18, 2000, 20_000)
    arrs = [s.t, s.kind, s.src, s.dst]
    lp = LoopbackPartitions(3)
    a = ConnectedComponents()
    task = LiveAnalysisTask(lp.parts, a, 1, False)
    lo = 0
    for hi in (20_000, 35_000, 60_000):
        lp.ingest_stream(Stream(*[x[lo:hi] for x in arrs]))
        lp.seal()
        lo = hi
        ts_exp = min(p.newest_time() for p in lp.parts)
        out = task.tick()
        assert out is not None and task.last_job_time == ts_exp
        assert _strip(out) == _strip([_cc_line(Oracle(*[x[:hi] for x in arrs]), ts_exp)])
    lp.close()
