"""Batch compositions and superstep paths of the CC query against the CPU oracle: window-major
batches (64 hops of one window, the default), hop-major batches (all windows of a hop in one
row, RGPU_WMAJOR=0), one batch in flight (RGPU_RUN_SERIAL), dense supersteps forced on almost
every step (RGPU_DENSE), and the final-label skip (a vertex holding its view's minimum member
label gathers nothing) on hub graphs and partial batches.  Every mode must give the same
bit-exact CC labels / component maps / summaries and per-hop superstep counts
(ConnectedComponents.scala:10-42,137-145; AnalysisTask.scala:208-225)."""
import contextlib
import os

import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, YEAR, Stream, gen_uniform, range_hops

pytestmark = pytest.mark.gpu

# (rgpu_open env, run kwargs)
MODES = [
    ({}, {}),                                   # defaults (window-major, three batches in flight)
    ({"RGPU_WMAJOR": "0"}, {}),                  # hop-major batches (all windows per row)
    ({"RGPU_WMAJOR": "0"}, {"serial": True}),    # hop-major, one batch in flight
    ({"RGPU_DENSE": "1000"}, {}),                # dense supersteps nearly everywhere
]
MODE_IDS = ["default", "hopmajor", "hopmajor-serial", "dense"]


@contextlib.contextmanager
def envset(env):
    """the RGPU_* knobs of a mode, for rgpu_open and for every run inside (RGPU_DENSE is read per run)"""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def graph_env(stream, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        g = TemporalGraph()  # rgpu_open reads the RGPU_* knobs
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    g.ingest_stream(stream)
    g.seal()
    return g


def chains_stream(lengths, seed=7, noise=3000, nverts=4000):
    """Disjoint paths of the given lengths (edges added in random order over a month), plus a
    uniform add/delete stream on other ids: long chains keep a few vertices changing for up to
    the 100-superstep cap (the tail kernel's workload)."""
    rng = np.random.default_rng(seed)
    t, k, s, d = [], [], [], []
    base = 1_000_000
    for L in lengths:
        ids = base + rng.permutation(L + 1)  # random labels along the chain
        base += L + 1
        for i in rng.permutation(L):
            t.append(int(T0_README + rng.integers(0, 30 * DAY)))
            k.append(2)
            s.append(int(ids[i]))
            d.append(int(ids[i + 1]))
    u = gen_uniform(seed, nverts, noise, t0=T0_README, dt=30 * DAY // noise)
    t = np.concatenate([np.asarray(t, np.int64), u.t])
    o = np.argsort(t, kind="stable")
    cat = lambda a, b: np.concatenate([np.asarray(a, np.int64), b.astype(np.int64)])[o]
    return Stream(t[o], np.concatenate([np.asarray(k, np.uint8), u.kind])[o], cat(s, u.src), cat(d, u.dst))


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_chains_vs_oracle(mode, monkeypatch):
    env, kw = mode
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    st = chains_stream([1, 4, 31, 64, 98, 99, 100, 101, 140])
    o = Oracle.from_stream(st)
    g = graph_env(st, env)
    hops = range_hops(T0_README + 10 * DAY, T0_README + 40 * DAY, 2 * DAY)
    for cap in (100, 37):
        g.run("cc", hops, [YEAR, MONTH, WEEK], max_steps=cap, retain=True, **kw)
        for h, t in enumerate(hops.tolist()):
            res, steps = o.cc(t, [YEAR, MONTH, WEEK], max_steps=cap, mode=1)
            for w in range(3):
                assert g.cc_summary(h, w).supersteps == steps, (mode, cap, t, w)
                ids, lab = res[w]
                gids, glab = g.cc_vertex_labels(h, w)
                assert np.array_equal(gids, ids) and np.array_equal(glab, lab), (mode, cap, t, w)
                exp = label_counts(lab)
                assert g.cc_result(h, w) == exp
                assert cc_fields_from_summary(g.cc_summary(h, w)) == cc_fields(exp)
    g.close()


@pytest.mark.parametrize("heavy", ["300", "2048"])
@pytest.mark.parametrize("n_hops", [1, 5, 40])
def test_final_label_skip_hubs_partial_batches(heavy, n_hops):
    """The final-label skip (kernels.hip holds_final: a uniform vertex whose word equals its views'
    minimum member label on every member lane gathers nothing, in the superstep kernel and the
    hub gather) on star hubs cut into segments (RGPU_HEAVY=300) or kept whole, with batches of
    fewer than 64 views (1 and 5 hops x 3 windows: lanes without members) and full ones."""
    from tests.test_gpu_heavy import hubs_stream
    st = hubs_stream(seed=5)
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_HEAVY": heavy})
    hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, DAY)[:n_hops]
    wins = [MONTH, WEEK, DAY]
    g.run("cc", hops, wins, retain=True)
    for h, t in enumerate(hops.tolist()):
        res, steps = o.cc(t, wins, mode=1)
        for w in range(3):
            assert g.cc_summary(h, w).supersteps == steps, (heavy, t, w)
            ids, lab = res[w]
            gids, glab = g.cc_vertex_labels(h, w)
            assert np.array_equal(gids, ids) and np.array_equal(glab, lab), (heavy, t, w)
    g.close()


def test_modes_agree_on_c2_slice():
    """C2 stream, 1,200 hourly hops: every mode gives identical summaries for all 6,000 views
    (superstep counts included: they are per hop, whatever batches held the views), and identical
    per-vertex labels on sampled hops."""
    s = gen_uniform(1, 100_000, 1_000_000)
    hops = range_hops(T0_README + 200 * DAY, T0_README + 250 * DAY, HOUR)[:1200]
    ref_summ, ref_lab = None, None
    for env, kw in MODES:
        with envset(env):
            g = graph_env(s, env)
            g.run("cc", hops, BATCH_WINDOWS, retain=True, **kw)
        summ = g.cc_summaries()
        labs = [g.cc_vertex_labels(h, w)[1] for h in (0, 599, 1199) for w in range(5)]
        g.close()
        if ref_summ is None:
            ref_summ, ref_lab = summ[..., :8], labs
            continue
        assert np.array_equal(summ[..., :8], ref_summ), env
        assert all(np.array_equal(a, b) for a, b in zip(labs, ref_lab)), env


@pytest.mark.parametrize("ivmax", ["-1", "0", "3", "96"])
def test_window_mask_forms_vs_oracle(ivmax):
    """K1 computes a hop block's masks per history point (interval form) for entities with at
    most RGPU_IVMAX points in the block's range, per hop otherwise; both forms, and every mix
    of them, give the oracle's per-vertex degrees (DegreeBasic.scala:16-28: vertex set and edge
    liveness straight from the masks) and CC labels.  Power-law stream: hubs with long
    histories and many deaths; out-of-order hops take the per-hop form."""
    from raphtory_amd.synth import gen_powerlaw
    st = gen_powerlaw(5, 3000, 40_000, t0=0, t1=YEAR)
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_IVMAX": ivmax})
    hops = range_hops(YEAR - 70 * DAY, YEAR + DAY, DAY)
    wins = [MONTH, WEEK, DAY]
    for hs in (hops, hops[::-1][:20]):
        g.run("degree", hs, wins, retain=True)
        for h, t in enumerate(np.asarray(hs).tolist()):
            res = o.degree(t, wins)
            for w in range(3):
                ids, od, idg = res[w]
                gids, god, gid = g.degree_vertex(h, w)
                assert np.array_equal(gids, ids) and np.array_equal(god, od) and np.array_equal(gid, idg), (ivmax, t, w)
    g.run("cc", hops[:40], wins, retain=True)
    for h, t in enumerate(hops[:40].tolist()):
        res, _ = o.cc(t, wins, mode=1)
        for w in range(3):
            assert np.array_equal(g.cc_vertex_labels(h, w)[1], res[w][1]), (ivmax, t, w)
    g.close()


@pytest.mark.parametrize("wmajor", ["1", "0"])
def test_k1_floor_carry_equals_from_scratch(wmajor):
    """§8(f) row 2, K1 part (BatchParams::carry): each hop block's window masks start from the floor
    indices the previous block left at its last hop instead of searching every history afresh.
    Against the from-scratch path (RGPU_K1_CARRY=0) and the oracle: a uniform stream with vertex
    and edge deletions (interval form and endpoint death lists), power-law hubs whose histories take
    the per-hop form, many blocks of hourly hops, hops that go backwards between blocks (the carry
    must not be read there), and degree / PageRank runs (their K1 carries too)."""
    from raphtory_amd.synth import gen_powerlaw
    uni = gen_uniform(17, 700, 40_000, t0=T0_README, dt=788_400)
    pl = gen_powerlaw(4, 1500, 30_000, t0=0, t1=YEAR)
    cases = [(uni, range_hops(T0_README + 20 * DAY, T0_README + 300 * DAY, 14 * HOUR)),
             (pl, range_hops(YEAR - 120 * DAY, YEAR, 9 * HOUR))]
    for s, hops in cases:
        back = np.concatenate([hops[200:264], hops[:64], hops[64:140]])  # block 2 starts before block 1 ends
        o = Oracle.from_stream(s)
        for hs in (hops, back):
            res = {}
            for carry in ("1", "0"):
                with envset({"RGPU_K1_CARRY": carry, "RGPU_WMAJOR": wmajor}):
                    g = graph_env(s, {"RGPU_WMAJOR": wmajor})
                    g.run("cc", hs, BATCH_WINDOWS, retain=True)
                    summ = g.cc_summaries().copy()
                    labs = [g.cc_vertex_labels(h, w) for h in range(0, len(hs), 23) for w in range(5)]
                    g.run("degree", hs[::11], [MONTH, DAY], retain=True)
                    deg = [g.degree_vertex(h, w) for h in range(len(hs[::11])) for w in range(2)]
                    g.run("pagerank", hs[::40], [WEEK], retain=True, pr_iters=10)
                    pr = [g.pr_result(h, 0) for h in range(len(hs[::40]))]
                    g.close()
                res[carry] = (summ, labs, deg, pr)
            a, b = res["1"], res["0"]
            assert np.array_equal(a[0], b[0])
            for (i1, l1), (i2, l2) in zip(a[1], b[1]):
                assert np.array_equal(i1, i2) and np.array_equal(l1, l2)
            for x, y in zip(a[2], b[2]):
                assert all(np.array_equal(p, q) for p, q in zip(x, y))
            for (i1, p1), (i2, p2) in zip(a[3], b[3]):
                assert np.array_equal(i1, i2) and np.array_equal(p1, p2)
            for k, h in enumerate(range(0, len(hs), 23)):
                r, _ = o.cc(int(hs[h]), BATCH_WINDOWS, mode=1)
                for w in range(5):
                    gi, gl = a[1][k * 5 + w]
                    assert np.array_equal(gi, r[w][0]) and np.array_equal(gl, r[w][1]), (h, w)


def test_k1_floor_carry_backward_blocks_overlap():
    """a K1 that only writes the floor carry (its first hop is before the previous
    block's last) runs on another slot's stream than the previous carry K1, and must still be
    ordered after it (rgpu.cpp k1_ev_live), or a later block reads floors left at a later hop.
    A 4M-update power-law graph makes each K1 last long enough for the blocks to overlap; the hop
    list alternates late and early 64-hop blocks.  Carry on and off must agree on every summary."""
    from raphtory_amd.synth import gen_powerlaw
    s = gen_powerlaw(5, 200_000, 4_000_000, t0=0, t1=YEAR)
    hops = range_hops(YEAR - 60 * DAY, YEAR, HOUR)
    blocks = []
    for i in range(3):
        blocks += [hops[800 + 64 * i:864 + 64 * i], hops[64 * i:64 * i + 64]]
    hs = np.concatenate(blocks)
    out = {}
    for carry in ("1", "0"):
        with envset({"RGPU_K1_CARRY": carry}):
            g = graph_env(s, {})
            g.run("cc", hs, BATCH_WINDOWS)
            out[carry] = g.cc_summaries().copy()
            g.close()
    assert np.array_equal(out["1"], out["0"])
