"""Live ingest: updates appended after a seal are merged into the
HBM-resident graph by the incremental seal (merge.hip) instead of a full re-pack.

Parity: after every seal the HIP path must answer exactly as the CPU oracle replaying the
whole stream so far (labels, component maps, degrees bit-exact; PageRank L1 <= 1e-6), and
exactly as a graph sealed once from the same full stream.  The later chunk counts as later
in stream order (the reference applies updates in arrival order, EntityStorage.scala:73-453),
so ties between a sealed point and a new one resolve to the new one — the cut points below
split groups of equal timestamps on purpose.
"""
import numpy as np
import pytest

from oracle import Oracle
from raphtory_amd import RGPUError, TemporalGraph
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, WEEK, YEAR, gen_gab, gen_powerlaw, gen_uniform
from tests.test_gpu_parity import check_cc, check_degree, check_pr

pytestmark = pytest.mark.gpu


def _growing_tie_stream(seed, n, nv_max=200):
    """Equal timestamps in groups of 4 and ids that keep appearing (new vertices per chunk)."""
    rng = np.random.default_rng(seed)
    t = (np.arange(n) // 4).astype(np.int64) * 10
    kind = rng.choice(4, size=n, p=[0.25, 0.45, 0.12, 0.18]).astype(np.uint8)
    hi = np.minimum(nv_max, 8 + np.arange(n) // 12)
    src = (rng.random(n) * hi).astype(np.int64)
    dst = np.where(kind >= 2, (rng.random(n) * hi).astype(np.int64), -1).astype(np.int64)
    return t, kind, src, dst


def _cut(arrs, lo, hi):
    return [a[lo:hi] for a in arrs]


def _live(arrs, cuts, check):
    """Ingest arrs in the chunks given by `cuts`, sealing after each; check(g, prefix) each time."""
    g = TemporalGraph(vertex_order="id")  # later seals merge into it (rgpu_set_vertex_order)
    bounds = [0] + list(cuts) + [len(arrs[0])]
    for k in range(len(bounds) - 1):
        g.ingest(*_cut(arrs, bounds[k], bounds[k + 1]))
        g.seal()
        st = g.stats()
        assert st["seal_incremental"] == (1 if k else 0)
        assert st["seal_delta_updates"] == (bounds[k + 1] - bounds[k] if k else 0)
        check(g, _cut(arrs, 0, bounds[k + 1]))
    return g


def _same_as_full(g, arrs, algo, hops, windows):
    f = TemporalGraph()
    f.ingest(*arrs)
    f.seal()
    a, b = g.stats(), f.stats()
    for k in ("vertices", "edges", "vertex_events", "edge_events", "deaths"):
        assert a[k] == b[k], (k, a[k], b[k])
    f.run(algo, hops, windows)
    g.run(algo, hops, windows)
    if algo == "cc":
        assert np.array_equal(g.cc_summaries(), f.cc_summaries())
    f.close()


def test_live_ties_new_vertices_each_seal():
    arrs = _growing_tie_stream(7, 8000)
    wins = [5000, 1000, 200, 40]

    def check(g, pre):
        o = Oracle(*pre)
        end = int(pre[0][-1])
        hops = np.arange(0, end + 20, max(37, end // 12), dtype=np.int64)
        check_cc(g, o, hops, wins)
        check_degree(g, o, hops[::2], wins)

    # cut points inside groups of equal timestamps (t = i // 4)
    g = _live(arrs, [1001, 2002, 2003, 4507, 6001], check)
    hops = np.arange(0, int(arrs[0][-1]) + 20, 97, dtype=np.int64)
    _same_as_full(g, arrs, "cc", hops, wins)
    g.close()


def test_live_out_of_order_deltas():
    # later chunks carry times all over the sealed range (late events and endpoint deaths
    # landing on sealed edge points)
    s = gen_uniform(3, 90, 4000, t0=0, dt=1000)
    rng = np.random.default_rng(2)
    p = rng.permutation(len(s))
    arrs = [s.t[p], s.kind[p], s.src[p], s.dst[p]]
    wins = [2_000_000, 500_000, 100_000]
    hops = np.arange(100_000, 4_000_000, 190_000, dtype=np.int64)

    def check(g, pre):
        o = Oracle(*pre)
        check_cc(g, o, hops, wins)
        check_pr(g, o, hops[::4], wins)

    g = _live(arrs, [1500, 2600, 3900], check)
    _same_as_full(g, arrs, "cc", hops, wins)
    g.close()


def test_live_deaths_tie_sealed_edge_points():
    # hand-made: a sealed edge point and a later VertexDelete of an endpoint at the same t
    # (the kill is the later put: EntityStorage.vertexRemoval :189-228), a re-add after it,
    # and a new edge created at the time of an earlier (sealed) death (killList, :262,277)
    base = ([10, 20, 30, 40], [2, 2, 2, 1], [1, 2, 3, 5], [2, 3, 4, -1])
    d1 = ([20, 30, 40], [1, 3, 2], [3, 3, 5], [-1, 4, 6])
    d2 = ([30, 50, 20], [2, 0, 2], [3, 2, 2], [4, -1, 3])
    arrs = [np.asarray(np.concatenate([b, x, y]), dt)
            for b, x, y, dt in zip(base, d1, d2, (np.int64, np.uint8, np.int64, np.int64))]
    hops = np.arange(0, 80, 5, dtype=np.int64)
    wins = [100, 25, 10, 0]

    def check(g, pre):
        o = Oracle(*pre)
        check_cc(g, o, hops, wins)
        check_degree(g, o, hops, wins)

    g = _live(arrs, [4, 7], check)
    g.close()


def test_live_powerlaw_heavy_vertices_and_gab():
    # hubs above the heavy-vertex threshold change their segment lists between seals
    s = gen_powerlaw(3, 2000, 24_000, t0=0, t1=2 * YEAR)
    arrs = [s.t, s.kind, s.src, s.dst]
    hops = np.linspace(2 * YEAR - 60 * DAY, 2 * YEAR, 5).astype(np.int64)
    wins = [MONTH, WEEK, DAY]

    def check(g, pre):
        o = Oracle(*pre)
        check_cc(g, o, hops, wins)
        check_degree(g, o, hops, wins)
        check_pr(g, o, hops[-2:], wins)

    import os
    old = os.environ.get("RGPU_HEAVY")
    os.environ["RGPU_HEAVY"] = "64"  # small graph: make hubs heavy
    try:
        g = _live(arrs, [16_000, 20_000], check)
        _same_as_full(g, arrs, "cc", hops, wins)
    finally:
        if old is None:
            os.environ.pop("RGPU_HEAVY", None)
        else:
            os.environ["RGPU_HEAVY"] = old
    g.close()
    s = gen_gab(4, 3000, 6000)
    arrs = [s.t, s.kind, s.src, s.dst]
    end = int(s.t[-1])
    hops = np.arange(end - 48 * HOUR, end + 1, 8 * HOUR, dtype=np.int64)

    def check2(g, pre):
        check_cc(g, Oracle(*pre), hops, BATCH_WINDOWS)

    g = _live(arrs, [9000, 15000], check2)
    g.close()


def test_live_seal_errors_and_noop():
    g = TemporalGraph(vertex_order="id")
    g.ingest([1, 2], [2, 2], [1, 2], [2, 3])
    g.seal()
    g.seal()  # nothing new: no-op
    assert g.stats()["seal_incremental"] == 0
    g.ingest([3], [2], [1], [1 << 40])  # id out of range in the delta
    with pytest.raises(RGPUError):
        g.seal()
    g.close()


def _packer_graph(monkeypatch, mode):
    monkeypatch.setenv("RGPU_DELTA", mode)  # read when the context is created
    g = TemporalGraph(vertex_order="id")
    monkeypatch.delenv("RGPU_DELTA")
    return g


@pytest.mark.parametrize("stream", ["ties", "shuffled", "deaths_powerlaw"])
def test_live_device_packer_equals_host_packer(stream, monkeypatch):
    """The device delta packer (gdelta.hip, the default) and the host one (packer.cpp pack_delta /
    finish_delta, RGPU_DELTA=2) merge the same ticks into the same graph: stats, and every CC
    label and degree of a spread of views after each seal (both also match the oracle above)."""
    if stream == "ties":
        arrs = list(_growing_tie_stream(11, 12_000, nv_max=600))
        cuts = [3001, 3002, 7777, 9000]
        wins = [5000, 1000, 200]
    elif stream == "shuffled":  # out of order: the device packer's time sort
        s = gen_uniform(5, 300, 9000, t0=0, dt=1000)
        p = np.random.default_rng(5).permutation(len(s))
        arrs = [s.t[p], s.kind[p], s.src[p], s.dst[p]]
        cuts = [3000, 6000, 8000]
        wins = [2_000_000, 300_000]
    else:
        s = gen_powerlaw(9, 3000, 30_000, t0=0, t1=YEAR)
        arrs = [s.t, s.kind, s.src, s.dst]
        cuts = [10_000, 10_001, 22_000]
        wins = [MONTH, WEEK]
    end = int(np.max(arrs[0]))
    hops = np.linspace(end // 3, end, 6).astype(np.int64)
    gd, gh = _packer_graph(monkeypatch, "1"), _packer_graph(monkeypatch, "2")
    bounds = [0] + cuts + [len(arrs[0])]
    for k in range(len(bounds) - 1):
        for g in (gd, gh):
            g.ingest(*_cut(arrs, bounds[k], bounds[k + 1]))
            g.seal()
        a, b = gd.stats(), gh.stats()
        for key in ("vertices", "edges", "vertex_events", "edge_events", "deaths", "seal_incremental"):
            assert a[key] == b[key], (k, key, a[key], b[key])
        for g in (gd, gh):
            g.run("cc", hops, wins, retain=True)
        for h in range(len(hops)):
            for w in range(len(wins)):
                x, y = gd.cc_vertex_labels(h, w), gh.cc_vertex_labels(h, w)
                assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]), (k, h, w)
        for g in (gd, gh):
            g.run("degree", hops[::2], wins, retain=True)
        for h in range(len(hops[::2])):
            for w in range(len(wins)):
                x, y = gd.degree_vertex(h, w), gh.degree_vertex(h, w)
                assert all(np.array_equal(u, v) for u, v in zip(x, y)), (k, h, w)
    gd.close()
    gh.close()


def test_live_device_packer_invalid_update_messages(monkeypatch):
    """the device packer reports the first invalid update of the tick as the host one does,
    and the resident graph stays as it was"""
    for mode in ("1", "2"):
        g = _packer_graph(monkeypatch, mode)
        g.ingest([1, 2], [2, 2], [1, 2], [2, 3])
        g.seal()
        g.ingest([3, -4, 5], [2, 2, 2], [1, 1, 1], [2, 2, 1 << 40])  # a bad time first, then a bad id
        with pytest.raises(RGPUError, match="time out of range"):
            g.seal()
        assert g.stats()["vertices"] == 3
        g.close()


@pytest.mark.parametrize("P", [2, 4])
def test_live_partitioned_loopback_ticks(P):
    """Live ticks into vertex partitions (the C5 shape at P ranks, here as loopback partitions on one
    GPU): every seal after the first merges on the device (ghosts appear as edges reach them, a
    ghost's earlier deaths follow it in).  After each tick the partitioned CC equals the oracle over
    the whole prefix, and every partition's graph equals a one-shot seal of the same prefix."""
    from raphtory_amd.partitioned import LoopbackPartitions
    from tests.test_gpu_parity import check_cc
    arrs = list(_growing_tie_stream(13, 9000, nv_max=400))
    cuts = [2001, 2002, 5003, 7000]
    wins = [5000, 1000, 200]
    lp = LoopbackPartitions(P, vertex_order="id")
    bounds = [0] + cuts + [len(arrs[0])]
    for k in range(len(bounds) - 1):
        chunk = _cut(arrs, bounds[k], bounds[k + 1])
        lp.ingest(*chunk)
        lp.seal()
        for p, st in enumerate(lp.stats()):
            # a partition that kept nothing of the chunk (rgpu_ingest's filter) has nothing to merge
            own = lambda ids: (np.abs(ids) % (10 * P)) // 10 == p  # noqa: E731 (Utils.getPartition)
            kept = (chunk[1] == 1) | own(chunk[2]) | ((chunk[1] >= 2) & own(chunk[3]))
            if k == 0 or kept.any():
                assert st["seal_incremental"] == (1 if k else 0), (k, p)
        pre = _cut(arrs, 0, bounds[k + 1])
        end = int(pre[0][-1])
        hops = np.arange(0, end + 20, max(41, end // 10), dtype=np.int64)
        check_cc(lp, Oracle(*pre), hops, wins)
        one = LoopbackPartitions(P, vertex_order="id")
        one.ingest(*pre)
        one.seal()
        for a, b in zip(lp.stats(), one.stats()):
            for key in ("vertices", "edges", "edges_owned", "vertex_events", "edge_events", "deaths"):
                assert a[key] == b[key], (k, key, a[key], b[key])
        one.close()
    lp.close()


def test_live_ingest_and_merge_concurrent_with_runs():
    """Live analysis under concurrent ingest (IngestionWorker keeps applying updates while
    LiveAnalysisTask runs, IngestionWorker.scala:31-61, LiveAnalysisTask.scala:55-105): while the
    main thread runs CC on the resident graph at tick i's live time, a second thread ingests tick
    i+1 and seals it (the merged graph is built beside the resident one and swapped in between
    runs).  Every run equals the oracle over the stream through tick i at that time (later points
    are invisible to a view at the live time), and after the last tick the merged graph equals a
    one-shot seal.  The sealed prefix of the log is dropped on the host as the ticks go (the
    whole-stream check below re-ingests from the arrays)."""
    import threading
    users = 4000
    base = gen_gab(4, users, 20_000)
    now = int(base.t[-1])
    ticks = []
    for i in range(5):
        ticks.append(gen_gab(100 + i, users, 4000, t0=now + 1, t1=now + HOUR, id_key=4))
        now = int(ticks[-1].t[-1])
    g = TemporalGraph(vertex_order="id")
    g.ingest_stream(base)
    g.seal()
    err = []

    def ingest_merge(s):
        try:
            g.ingest_stream(s)
            g.seal()
        except BaseException as e:  # noqa: BLE001
            err.append(e)

    prefix = [base]
    ingest_merge(ticks[0])
    prefix.append(ticks[0])
    wins = [MONTH, DAY, HOUR]
    for i in range(len(ticks)):
        assert not err, err
        live = int(prefix[-1].t[-1])
        th = threading.Thread(target=ingest_merge, args=(ticks[i + 1],)) if i + 1 < len(ticks) else None
        if th:
            th.start()
        g.run("cc", [live, live - HOUR // 2], wins, retain=True)
        if th:
            th.join()
        cat = [np.concatenate([getattr(s, f) for s in prefix]) for f in ("t", "kind", "src", "dst")]
        o = Oracle(*cat)
        for h, t in enumerate([live, live - HOUR // 2]):
            res, steps = o.cc(t, wins, mode=1)
            for w in range(len(wins)):
                ids, lab = res[w]
                gids, glab = g.cc_vertex_labels(h, w)
                assert np.array_equal(gids, ids) and np.array_equal(glab, lab), (i, t, w)
                assert g.cc_summary(h, w).supersteps == steps
        o.close()
        if i + 1 < len(ticks):
            prefix.append(ticks[i + 1])
    assert not err, err
    one = TemporalGraph()
    for s in prefix:
        one.ingest_stream(s)
    one.seal()
    a, b = g.stats(), one.stats()
    for k in ("vertices", "edges", "vertex_events", "edge_events"):
        assert a[k] == b[k], k
    g.close()
    one.close()
