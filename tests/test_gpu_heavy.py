"""Heavy vertices (power-law hubs): slots cut into segments, each compacted / gathered / marked
by its own wave (k_heavy_slots, k_heavy_gather, k_heavy_mark), the hub's own superstep in the
full-grid kernel.  Against the CPU oracle and against the undivided path (RGPU_HEAVY=0):
bit-exact CC labels, component maps and summaries (ConnectedComponents.scala:10-42,137-145)."""
import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, YEAR, Stream, gen_gab, gen_powerlaw, range_hops
from tests.test_gpu_batch_modes import graph_env

pytestmark = pytest.mark.gpu


def hubs_stream(seed=3, hubs=(1, 2, 3), leaves=2600, other=5000, n_rand=20_000):
    """Three star hubs with ~2.6k leaves each (several 512-slot segments), edges added and
    deleted over two months, leaf deletions, plus a uniform random stream among the leaves:
    hubs change label in many views and their neighbourhoods overlap."""
    rng = np.random.default_rng(seed)
    t, k, s, d = [], [], [], []
    span = 60 * DAY
    for h in hubs:
        for leaf in rng.choice(np.arange(100, 100 + other), leaves, replace=False):
            ta = int(rng.integers(0, span))
            t.append(ta); k.append(2)
            if rng.random() < 0.5:
                s.append(int(h)); d.append(int(leaf))
            else:
                s.append(int(leaf)); d.append(int(h))
            if rng.random() < 0.2:  # edge delete later
                t.append(ta + int(rng.integers(1, span))); k.append(3); s.append(s[-1]); d.append(d[-1])
    for _ in range(300):  # leaf deaths
        t.append(int(rng.integers(0, span))); k.append(1); s.append(int(rng.integers(100, 100 + other))); d.append(-1)
    for _ in range(n_rand):
        a, b = rng.integers(100, 100 + other, 2)
        t.append(int(rng.integers(0, span))); k.append(2 if rng.random() < 0.8 else 3); s.append(int(a)); d.append(int(b))
    t = np.asarray(t, np.int64) + T0_README
    o = np.argsort(t, kind="stable")
    return Stream(t[o], np.asarray(k, np.uint8)[o], np.asarray(s, np.int64)[o], np.asarray(d, np.int64)[o])


def check_vs_oracle(g, o, hops, wins, max_steps=100):
    g.run("cc", hops, wins, max_steps=max_steps, retain=True)
    for h, t in enumerate(np.asarray(hops).tolist()):
        res, _ = o.cc(t, wins, max_steps=max_steps, mode=1)
        for w in range(max(1, len(wins))):
            ids, lab = res[w]
            gids, glab = g.cc_vertex_labels(h, w)
            assert np.array_equal(gids, ids) and np.array_equal(glab, lab), (t, w)
            exp = label_counts(lab)
            assert g.cc_result(h, w) == exp
            assert cc_fields_from_summary(g.cc_summary(h, w)) == cc_fields(exp)


@pytest.mark.parametrize("heavy", ["0", "8", "300"])
def test_hubs_vs_oracle(heavy):
    st = hubs_stream()
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_HEAVY": heavy})
    hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, 3 * DAY)
    check_vs_oracle(g, o, hops, [MONTH, WEEK, DAY])
    check_vs_oracle(g, o, hops[:6], [])       # ViewLens
    check_vs_oracle(g, o, hops[:6], [WEEK], max_steps=2)
    g.close()


@pytest.mark.parametrize("heavy", ["16", "100"])
def test_powerlaw_and_gab_heavy_vs_oracle(heavy):
    st = gen_powerlaw(9, 3000, 60_000, t0=0, t1=YEAR)
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_HEAVY": heavy})
    check_vs_oracle(g, o, range_hops(YEAR - 40 * DAY, YEAR, 4 * DAY), [MONTH, WEEK, DAY])
    g.close()
    st = gen_gab(6, 4000, 30_000)
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_HEAVY": heavy})
    end = int(st.t[-1])
    check_vs_oracle(g, o, range_hops(end - 96 * HOUR, end, 8 * HOUR), BATCH_WINDOWS)
    g.close()


def test_heavy_split_matches_undivided_on_gab_range():
    """GAB-shaped stream (C4 shape at small scale), 200 hourly hops x 5 windows: the split and
    undivided paths give identical summaries for every view (supersteps included)."""
    st = gen_gab(8, 20_000, 300_000)
    end = int(st.t[-1])
    hops = range_hops(end - 199 * HOUR, end, HOUR)
    out = []
    for heavy in ("0", "64", "2048"):
        g = graph_env(st, {"RGPU_HEAVY": heavy})
        g.run("cc", hops, BATCH_WINDOWS, retain=True)
        out.append((g.cc_summaries(), [g.cc_vertex_labels(h, w)[1] for h in (0, 199) for w in range(5)]))
        g.close()
    for summ, labs in out[1:]:
        assert np.array_equal(summ, out[0][0])
        assert all(np.array_equal(a, b) for a, b in zip(labs, out[0][1]))


PR_L1_TOL = 1e-6


@pytest.mark.parametrize("heavy", ["0", "8", "300"])
def test_hubs_degree_and_pagerank_vs_oracle(heavy):
    """DegreeBasic per-vertex degrees (DegreeBasic.scala:16-28) exact, PageRank (App. A.5) within
    L1 <= 1e-6, with the hubs' slots counted / pulled per segment (k_heavy_degree, k_heavy_pr)."""
    st = hubs_stream(seed=5)
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_HEAVY": heavy})
    hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, 5 * DAY)
    wins = [MONTH, WEEK, DAY]
    g.run("degree", hops, wins, retain=True)
    for h, t in enumerate(hops.tolist()):
        res = o.degree(t, wins)
        for w in range(3):
            ids, od, idg = res[w]
            gids, god, gid = g.degree_vertex(h, w)
            assert np.array_equal(gids, ids) and np.array_equal(god, od) and np.array_equal(gid, idg), (heavy, t, w)
            assert g.degree_result(h, w)[:3] == (len(ids), int(od.sum()), int(idg.sum()))
    g.run("pagerank", hops[::3], wins, pr_iters=20, retain=True)
    for h, t in enumerate(hops[::3].tolist()):
        res = o.pagerank(t, wins, iters=20)
        for w in range(3):
            ids, pr = res[w]
            gids, gpr = g.pr_result(h, w)
            assert np.array_equal(gids, ids)
            assert np.abs(gpr - pr).sum() <= PR_L1_TOL, (heavy, t, w, np.abs(gpr - pr).sum())
    g.close()
