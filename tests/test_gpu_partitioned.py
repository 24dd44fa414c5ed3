"""Vertex-partitioned mode on one GPU: P partitions in one process over the
library's loopback exchange (same superstep protocol as RCCL), against the CPU oracle on
the whole stream.  Bit-exact CC labels / merged component maps / merged summaries /
degrees; PageRank within the north-star L1 tolerance."""
import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.partitioned import LoopbackPartitions
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, YEAR, gen_gab, gen_powerlaw, gen_uniform, range_hops

pytestmark = pytest.mark.gpu

PR_L1_TOL = 1e-6


def _parts(s, P, env=None):
    import os
    env = env or {}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        lp = LoopbackPartitions(P)  # rgpu_open reads the RGPU_* knobs
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    lp.ingest_stream(s)
    lp.seal()
    return lp


def check_cc(lp, o, hops, windows, max_steps=100):
    lp.run("cc", hops, windows, max_steps=max_steps, retain=True)
    for h, t in enumerate(np.asarray(hops).tolist()):
        res, steps = o.cc(t, windows, max_steps=max_steps, mode=1)
        for w in range(max(1, len(windows))):
            ids, lab = res[w]
            for g in lp.parts:
                assert g.cc_summary(h, w).supersteps == steps, (t, w)
            gids, glab = lp.cc_vertex_labels(h, w)
            assert np.array_equal(gids, ids), (t, w)
            assert np.array_equal(glab, lab), (t, w)
            exp = label_counts(lab)
            assert lp.cc_result(h, w) == exp, (t, w)
            for g in lp.parts:  # every partition holds the merged summary
                assert cc_fields_from_summary(g.cc_summary(h, w)) == cc_fields(exp), (t, w)


def check_degree(lp, o, hops, windows):
    lp.run("degree", hops, windows, retain=True)
    for h, t in enumerate(np.asarray(hops).tolist()):
        res = o.degree(t, windows)
        for w in range(max(1, len(windows))):
            ids, od, idg = res[w]
            gids, god, gid = lp.degree_vertex(h, w)
            assert np.array_equal(gids, ids) and np.array_equal(god, od) and np.array_equal(gid, idg)
            assert lp.degree_totals(h, w) == (len(ids), int(od.sum()), int(idg.sum()))


def check_pr(lp, o, hops, windows, iters=20):
    lp.run("pagerank", hops, windows, pr_iters=iters, retain=True)
    for h, t in enumerate(np.asarray(hops).tolist()):
        res = o.pagerank(t, windows, iters=iters)
        for w in range(max(1, len(windows))):
            ids, pr = res[w]
            gids, gpr = lp.pr_result(h, w)
            assert np.array_equal(gids, ids)
            assert np.abs(gpr - pr).sum() <= PR_L1_TOL


@pytest.mark.parametrize("P", [2, 3])
def test_partitioned_uniform(P):
    s = gen_uniform(11, 500, 10_000, t0=T0_README, dt=3_153_600)
    o = Oracle.from_stream(s)
    lp = _parts(s, P)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 4 * DAY)
    check_cc(lp, o, hops, BATCH_WINDOWS)
    check_cc(lp, o, hops[:5], [])  # ViewLens
    check_degree(lp, o, hops[::7], BATCH_WINDOWS)
    check_pr(lp, o, hops[::20], [MONTH, WEEK])
    lp.close()


def test_partitioned_superstep_cap():
    s = gen_uniform(5, 300, 6000, t0=T0_README, dt=3_153_600)
    o = Oracle.from_stream(s)
    lp = _parts(s, 4)
    hops = range_hops(T0_README + 200 * DAY, T0_README + 260 * DAY, 10 * DAY)
    for cap in (1, 2, 3):
        check_cc(lp, o, hops, [YEAR, MONTH], max_steps=cap)
    lp.close()


def test_partitioned_powerlaw_and_gab():
    s = gen_powerlaw(3, 2000, 20_000, t0=0, t1=2 * YEAR)
    o = Oracle.from_stream(s)
    lp = _parts(s, 2)
    hops = range_hops(2 * YEAR - 60 * DAY, 2 * YEAR, 10 * DAY)
    check_cc(lp, o, hops, [MONTH, WEEK, DAY])
    check_degree(lp, o, hops, [MONTH, WEEK, DAY])
    check_pr(lp, o, hops[:3], [MONTH, WEEK, DAY])
    lp.close()
    s = gen_gab(4, 3000, 5000)
    o = Oracle.from_stream(s)
    lp = _parts(s, 3)
    end = int(s.t[-1])
    check_cc(lp, o, range_hops(end - 48 * HOUR, end, 6 * HOUR), BATCH_WINDOWS)
    lp.close()


@pytest.mark.parametrize("P", [5, 8])
def test_partitioned_many_partitions_window_major(P):
    """P up to 8 (one node's GPUs) on one GPU: window-major batches (64 hops x one window),
    three batches in flight on their own channels; record buffers forced to start tiny so
    that every growth path (send, receive with records still awaiting their clear, component
    counts) runs."""
    s = gen_uniform(13, 600, 12_000, t0=T0_README, dt=2_628_000)
    o = Oracle.from_stream(s)
    lp = _parts(s, P, {"RGPU_XREC_TINY": "1"})
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 2 * DAY)  # 168 hops x 5
    check_cc(lp, o, hops, BATCH_WINDOWS)
    lp.close()


@pytest.mark.parametrize("heavy", ["300", "0"])
def test_partitioned_heavy_hubs(heavy):
    """Star hubs with thousands of leaves split into 512-slot segments on the partition that
    owns them and as ghosts elsewhere (RGPU_HEAVY=300: every vertex above 300 static slots)."""
    from tests.test_gpu_heavy import hubs_stream
    s = hubs_stream()
    o = Oracle.from_stream(s)
    lp = _parts(s, 3, {"RGPU_HEAVY": heavy})
    hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, DAY)
    check_cc(lp, o, hops, [MONTH, WEEK, DAY])
    check_degree(lp, o, hops[::9], [MONTH, WEEK, DAY])
    check_pr(lp, o, hops[::20], [MONTH, WEEK])
    lp.close()


def test_partitioned_filtered_ingest_equals_whole_stream():
    """Each partition handed only its part of the stream (what rgpu_ingest keeps anyway) answers
    exactly as when handed the whole stream."""
    from raphtory_amd.partition import get_partition
    s = gen_powerlaw(7, 1500, 15_000, t0=0, t1=YEAR)
    o = Oracle.from_stream(s)
    P = 3
    lp = LoopbackPartitions(P)
    for p, g in enumerate(lp.parts):
        own_s = get_partition(s.src, P) == p
        own_d = (s.dst >= 0) & (get_partition(np.maximum(s.dst, 0), P) == p)
        keep = (s.kind == 1) | own_s | ((s.kind >= 2) & own_d)
        g.ingest(s.t[keep], s.kind[keep], s.src[keep], s.dst[keep])
    lp.seal()
    check_cc(lp, o, range_hops(YEAR - 40 * DAY, YEAR, 8 * DAY), [MONTH, WEEK, DAY])
    lp.close()


def test_loopback_rejects_mixed_devices():
    with pytest.raises(ValueError):
        LoopbackPartitions(2, device=[0, 1])


def test_partitioned_path_one_partition_scattered_ids():
    """The partitioned path with P = 1 (RGPU_PARTITIONED=1, no peers): labels are vertex ids and
    the component counts go to the label's owned rank — on power-law ids scattered over
    [0, 2^31) (ranks differ from ids) with heavy hubs."""
    s = gen_powerlaw(9, 3000, 40_000, t0=0, t1=YEAR)
    o = Oracle.from_stream(s)
    lp = _parts(s, 1, {"RGPU_PARTITIONED": "1", "RGPU_HEAVY": "200"})
    check_cc(lp, o, range_hops(YEAR - 50 * DAY, YEAR, 5 * DAY), [MONTH, WEEK, DAY])
    lp.close()


@pytest.mark.parametrize("P", [2, 3])
def test_partitioned_partition_without_edges(P):
    """A partition that owns only vertex adds (no edge has an endpoint it owns) has no time-ordered
    slots; the ghost-membership decision (ghost_vm_free) must still be the same on every partition
    (ensure_tab agrees on it), or that partition enters an exchange its peers skip."""
    from raphtory_amd.partition import get_partition
    from raphtory_amd.synth import Stream
    s = gen_gab(21, 2000, 6000)
    e = s.kind == 2
    keep = ~e | ((get_partition(s.src, P) == 0) & (get_partition(np.maximum(s.dst, 0), P) == 0))
    s = Stream(s.t[keep], s.kind[keep], s.src[keep], s.dst[keep])
    assert np.any(get_partition(s.src[s.kind == 0], P) == P - 1)  # the edgeless partition owns vertices
    o = Oracle.from_stream(s)
    lp = _parts(s, P)
    end = int(s.t[-1])
    check_cc(lp, o, range_hops(end - 30 * DAY, end, 2 * DAY), BATCH_WINDOWS)
    lp.close()


@pytest.mark.parametrize("P,letters", [(1, "mwdh"), (2, "dh"), (3, "wdh")])
def test_window_hybrid_equals_one_graph(P, letters):
    """bench.py's N > 1 window-class hybrid (raphtory_amd/partitioned.py): the partitions answer the
    long windows, each rank its block of the hops for the short windows on a replica of the stream's
    time slice [hop0 - the longest short window, end].  On the add-only GAB stream every view's
    summary — the hop's superstep count included — equals the one-graph batched query's (itself
    oracle-checked on the C4 goldens), and a sampled view's labels equal the oracle's."""
    from raphtory_amd import TemporalGraph
    from raphtory_amd.partitioned import combine_window_groups, hop_blocks
    from raphtory_amd.synth import Stream
    s = gen_gab(4, 30_000, 1_000_000)
    end = int(s.t[-1])
    hops = range_hops(end - 99 * HOUR, end, HOUR)  # 100 hops: two batches per window
    g = TemporalGraph()
    g.ingest_stream(s)
    g.seal()
    g.run("cc", hops, BATCH_WINDOWS)
    ref = g.cc_summaries()
    g.close()
    short_i = [i for i, c in enumerate("ymwdh") if c in letters]
    long_i = [i for i in range(len(BATCH_WINDOWS)) if i not in short_i]
    sw = [BATCH_WINDOWS[i] for i in short_i]
    if P == 1:  # bench.py's N = 1 default: the long windows on the graph itself
        g = TemporalGraph()
        g.ingest_stream(s)
        g.seal()
        g.run("cc", hops, [BATCH_WINDOWS[i] for i in long_i])
        ls = g.cc_summaries()
        g.close()
    else:
        lp = _parts(s, P)
        lp.run("cc", hops, [BATCH_WINDOWS[i] for i in long_i])
        ls = lp.parts[0].cc_summaries()
        lp.close()
    keep = s.t >= int(hops[0]) - max(sw)
    assert 0 < keep.sum() < len(s) // 10  # a real slice
    sl = Stream(s.t[keep], s.kind[keep], s.src[keep], s.dst[keep])
    rep = TemporalGraph()
    rep.ingest_stream(sl)
    rep.seal()
    blocks = []
    for lo, hi in hop_blocks(len(hops), P):
        rep.run("cc", hops[lo:hi], sw, retain=lo == 0)
        blocks.append((lo, hi, rep.cc_summaries()))
        if lo == 0:  # the first hop of rank 0's block, the shortest window: labels vs the oracle on the slice
            res, _ = Oracle.from_stream(sl).cc(int(hops[0]), [sw[-1]], mode=1)
            gids, glab = rep.cc_vertex_labels(0, len(sw) - 1)
            assert np.array_equal(gids, res[0][0]) and np.array_equal(glab, res[0][1])
    rep.close()
    got = combine_window_groups(len(BATCH_WINDOWS), long_i, ls, short_i, blocks)
    assert np.array_equal(got, ref)
