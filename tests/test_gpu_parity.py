"""HIP path (through the C ABI, librgpu.so) against the CPU oracle on identical streams.

Bit-exact: CC labels per vertex, component-size maps and summaries, per-vertex degrees.
PageRank: L1 <= 1e-6 per view (BASELINE.json north_star), fp64 on both sides.
"""
import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import RGPUError, TemporalGraph
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import (BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, YEAR, gen_gab,
                                gen_powerlaw, gen_uniform, range_hops)
from tests.kat import arrays, cc_expect, load_cases

pytestmark = pytest.mark.gpu

PR_L1_TOL = 1e-6  # BASELINE.json north_star: PageRank within 1e-6 L1


def gpu_graph(t, kind, src, dst):
    g = TemporalGraph()
    g.ingest(t, kind, src, dst)
    g.seal()
    return g


def check_cc(g, o, hops, windows, max_steps=100):
    g.run("cc", hops, windows, max_steps=max_steps, retain=True)
    nw = max(1, len(windows))
    for h, t in enumerate(np.asarray(hops).tolist()):
        res, steps = o.cc(t, windows, max_steps=max_steps, mode=1)
        for w in range(nw):
            # the hop's job superstep count (AnalysisTask.endStep), whatever batches held its views
            assert g.cc_summary(h, w).supersteps == steps, (t, w, g.cc_summary(h, w).supersteps, steps)
            ids, lab = res[w]
            gids, glab = g.cc_vertex_labels(h, w)
            assert np.array_equal(gids, ids), (t, w)
            assert np.array_equal(glab, lab), (t, w)
            exp = label_counts(lab)
            assert g.cc_result(h, w) == exp, (t, w)
            f_exp = cc_fields(exp)
            f_got = cc_fields_from_summary(g.cc_summary(h, w))
            assert f_got == f_exp, (t, w, f_got, f_exp)


def check_degree(g, o, hops, windows):
    g.run("degree", hops, windows, retain=True)
    nw = max(1, len(windows))
    for h, t in enumerate(np.asarray(hops).tolist()):
        res = o.degree(t, windows)
        for w in range(nw):
            ids, od, idg = res[w]
            gids, god, gid = g.degree_vertex(h, w)
            assert np.array_equal(gids, ids) and np.array_equal(god, od) and np.array_equal(gid, idg), (t, w)
            tv, to, ti, top = g.degree_result(h, w)
            assert (tv, to, ti) == (len(ids), int(od.sum()), int(idg.sum()))
            # top-20 by in-degree: compare the in-degree multiset (tie order is unordered in the reference)
            assert sorted([x[2] for x in top], reverse=True) == sorted(idg.tolist(), reverse=True)[:20]


def check_pr(g, o, hops, windows, iters=20):
    g.run("pagerank", hops, windows, pr_iters=iters, retain=True)
    nw = max(1, len(windows))
    for h, t in enumerate(np.asarray(hops).tolist()):
        res = o.pagerank(t, windows, iters=iters)
        for w in range(nw):
            ids, pr = res[w]
            gids, gpr = g.pr_result(h, w)
            assert np.array_equal(gids, ids)
            assert np.abs(gpr - pr).sum() <= PR_L1_TOL, (t, w, np.abs(gpr - pr).sum())


# ------------------------------------------------------------------ known answers
CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_kat_gpu(case):
    g = gpu_graph(*arrays(case))
    for q in case.get("cc", []):
        g.run("cc", [q["t"]], q["windows"], retain=True)
        for w, m in enumerate(q["expect"]):
            ids, lab = g.cc_vertex_labels(0, w)
            assert dict(zip(ids.tolist(), lab.tolist())) == cc_expect(m), (q, w)
    for q in case.get("degree", []):
        g.run("degree", [q["t"]], q["windows"], retain=True)
        for w, rows in enumerate(q["expect"]):
            ids, od, idg = g.degree_vertex(0, w)
            assert [[int(a), int(b), int(c)] for a, b, c in zip(ids, od, idg)] == rows, (q, w)
    g.close()


def _path(n):
    t = np.arange(1, n, dtype=np.int64)
    return t, np.full(n - 1, 2, np.uint8), np.arange(0, n - 1, dtype=np.int64), np.arange(1, n, dtype=np.int64)


def test_superstep_cap_gpu():
    g = gpu_graph(*_path(150))
    g.run("cc", [1000], [], max_steps=100, retain=True)
    ids, lab = g.cc_vertex_labels(0, 0)
    assert np.array_equal(lab, np.maximum(ids - 100, 0))
    assert g.cc_summary(0, 0).supersteps == 100
    g.run("cc", [1000], [], max_steps=120, retain=True)
    ids, lab = g.cc_vertex_labels(0, 0)
    assert np.array_equal(lab, np.maximum(ids - 120, 0))
    g.close()


# ------------------------------------------------------------------ seeded streams
@pytest.fixture(scope="module")
def uniform_small():
    # C1/C2 shape at 1/100 scale: 10k events over one year, 500 vertices
    s = gen_uniform(11, 500, 10_000, t0=T0_README, dt=3_153_600)
    return s, Oracle.from_stream(s), gpu_graph(s.t, s.kind, s.src, s.dst)


def test_cc_batched_range_uniform(uniform_small):
    s, o, g = uniform_small
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, DAY)  # 336 hops, 28 batches
    check_cc(g, o, hops, BATCH_WINDOWS)


def test_cc_view_and_single_window(uniform_small):
    s, o, g = uniform_small
    hops = range_hops(T0_README + 100 * DAY, T0_README + 120 * DAY, 2 * DAY)
    check_cc(g, o, hops, [])
    check_cc(g, o, hops, [WEEK])


def test_cc_ascending_windows_quirk(uniform_small):
    s, o, g = uniform_small
    hops = range_hops(T0_README + 200 * DAY, T0_README + 210 * DAY, DAY)
    check_cc(g, o, hops, [DAY, WEEK, MONTH])


def test_cc_partial_last_batch_and_many_windows(uniform_small):
    s, o, g = uniform_small
    hops = range_hops(T0_README + 40 * DAY, T0_README + 68 * DAY, DAY)  # 29 hops
    check_cc(g, o, hops, BATCH_WINDOWS)
    wins = [YEAR - i * WEEK for i in range(13)]  # W=13 -> K=4
    check_cc(g, o, hops[:9], wins)


def test_cc_hops_before_and_after_stream(uniform_small):
    s, o, g = uniform_small
    hops = [0, T0_README - 1, T0_README, int(s.t[-1]) + YEAR * 3]
    check_cc(g, o, hops, BATCH_WINDOWS)
    g.run("cc", [0], BATCH_WINDOWS)
    assert cc_fields_from_summary(g.cc_summary(0, 0)) is None  # "No activity"


def test_degree_uniform(uniform_small):
    s, o, g = uniform_small
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 7 * DAY)
    check_degree(g, o, hops, BATCH_WINDOWS)
    check_degree(g, o, hops[:5], [])


def test_pagerank_uniform(uniform_small):
    s, o, g = uniform_small
    hops = range_hops(T0_README + 60 * DAY, T0_README + 365 * DAY, 30 * DAY)
    check_pr(g, o, hops, [MONTH, WEEK, DAY])
    check_pr(g, o, hops[:3], [])


def test_ties_random_stream():
    # many updates share a timestamp (t = i // 4): exercises the put-order tie rules
    rng = np.random.default_rng(5)
    n = 6000
    t = (np.arange(n) // 4).astype(np.int64) * 10
    kind = rng.choice(4, size=n, p=[0.25, 0.45, 0.12, 0.18]).astype(np.uint8)
    src = rng.integers(0, 60, n).astype(np.int64)
    dst = np.where(kind >= 2, rng.integers(0, 60, n), -1).astype(np.int64)
    o = Oracle(t, kind, src, dst)
    g = gpu_graph(t, kind, src, dst)
    hops = np.arange(0, int(t[-1]) + 20, 370, dtype=np.int64)
    check_cc(g, o, hops, [5000, 1000, 200, 40])
    check_degree(g, o, hops, [5000, 1000, 200, 40])
    g.close()


def test_out_of_order_stream():
    s = gen_uniform(3, 80, 3000, t0=0, dt=1000)
    rng = np.random.default_rng(1)
    p = rng.permutation(len(s))
    t, k, a, b = s.t[p], s.kind[p], s.src[p], s.dst[p]
    o = Oracle(t, k, a, b)
    g = gpu_graph(t, k, a, b)
    hops = np.arange(100_000, 3_000_000, 150_000, dtype=np.int64)
    check_cc(g, o, hops, [2_000_000, 500_000, 100_000])
    g.close()


def test_powerlaw_and_gab_small():
    s = gen_powerlaw(3, 2000, 20_000, t0=0, t1=2 * YEAR)
    o = Oracle.from_stream(s)
    g = gpu_graph(s.t, s.kind, s.src, s.dst)
    hops = range_hops(2 * YEAR - 60 * DAY, 2 * YEAR, 10 * DAY)
    check_cc(g, o, hops, [MONTH, WEEK, DAY])
    check_degree(g, o, hops, [MONTH, WEEK, DAY])
    check_pr(g, o, hops[:3], [MONTH, WEEK, DAY])
    g.close()
    s = gen_gab(4, 3000, 5000)
    o = Oracle.from_stream(s)
    g = gpu_graph(s.t, s.kind, s.src, s.dst)
    end = int(s.t[-1])
    hops = range_hops(end - 48 * HOUR, end, 6 * HOUR)
    check_cc(g, o, hops, BATCH_WINDOWS)
    g.close()


# ------------------------------------------------------------------ errors
def test_error_behaviour():
    g = TemporalGraph()
    with pytest.raises(RGPUError) as e:
        g.run("cc", [1], [])
    assert "before rgpu_seal" in str(e.value)
    g.ingest([1], [2], [1], [1 << 40])
    with pytest.raises(RGPUError):
        g.seal()
    g.close()
    g = gpu_graph(*_path(5))
    with pytest.raises(RGPUError):
        g.run("cc", [3], [DAY, DAY])  # duplicate windows share state in the reference
    with pytest.raises(RGPUError):
        g.cc_summary(0, 0)  # nothing run yet
    g.close()


# ------------------------------------------------------------------ full size (BASELINE C2)
def test_c2_full_size_properties_and_sampled_parity():
    s = gen_uniform(1, 100_000, 1_000_000)
    g = gpu_graph(s.t, s.kind, s.src, s.dst)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, HOUR)
    assert len(hops) == 8041
    g.run("cc", hops, BATCH_WINDOWS)
    summ = g.cc_summaries()  # [hops, 5, 8]
    big, tot, nis, isl, gt2, sall, snis = (summ[..., i] for i in range(7))
    assert np.all(tot == nis + isl) and np.all(big <= sall) and np.all(gt2 <= nis)
    assert np.all(np.diff(sall, axis=1) <= 0)  # descending windows: nested vertex sets
    assert np.all(snis <= sall) and np.all((tot == 0) == (sall == 0))
    o = Oracle.from_stream(s)
    for h in (0, 4000, 8040):
        res, _ = o.cc(int(hops[h]), BATCH_WINDOWS, mode=1)
        for w in range(5):
            exp = cc_fields(label_counts(res[w][1]))
            assert cc_fields_from_summary(g.cc_summary(h, w)) == exp, (h, w)
    g.close()


def test_alive_edge_counts_vs_oracle(uniform_small):
    """|E_{t,w}| per view (RGPU_RUN_EDGE_COUNTS, the SURVEY §8(d) byte model's edge count) equals
    the number of edge entities the oracle finds alive (Entity.aliveAtWithWindow)."""
    s, o, g = uniform_small
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 29 * DAY)
    g.run("cc", hops, BATCH_WINDOWS, edge_counts=True)
    summ = g.cc_summaries()
    pairs = sorted({(int(a), int(b)) for a, b, k in zip(s.src, s.dst, s.kind) if k >= 2})
    for h, t in enumerate(hops.tolist()):
        for w, win in enumerate(BATCH_WINDOWS):
            exp = sum(o.alive(True, a, b, t, win) for a, b in pairs)
            assert summ[h, w, 8] == exp, (t, win, summ[h, w, 8], exp)
    assert g.stats()["alive_edge_windows"] == int(summ[..., 8].sum())
    g.run("cc", hops, BATCH_WINDOWS)
    assert np.all(g.cc_summaries()[..., 8] == -1) and g.stats()["alive_edge_windows"] == -1
