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


def _parts(s, P):
    lp = LoopbackPartitions(P)
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
