"""Late supersteps in the one-workgroup tail kernel (k_cc_tail) against the full-grid superstep
kernel and the CPU oracle.  The two kernels share buffers and hand over at any superstep, so
every combination of where the tail starts (RGPU_CHUNK0) and how narrow a frontier it takes
(RGPU_TAIL_CAP: small caps force hand-backs to the full-grid kernel mid-batch) must give the
same bit-exact CC labels / component maps / summaries (ConnectedComponents.scala:10-42,137-145)."""
import os

import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, YEAR, Stream, gen_uniform, range_hops

pytestmark = pytest.mark.gpu

MODES = [
    {},                                                    # defaults (window-major, full-grid steps)
    {"RGPU_TAIL": "1"},                                    # tail kernel after the first chunk
    {"RGPU_TAIL": "1", "RGPU_CHUNK0": "1", "RGPU_TAIL_CAP": "3"},  # tail from step 3, hands back often
    {"RGPU_TAIL": "1", "RGPU_CHUNK0": "2", "RGPU_CHUNK": "1", "RGPU_TAIL_CAP": "40", "RGPU_POLL": "0"},
    {"RGPU_WMAJOR": "0", "RGPU_TAIL": "1"},                # hop-major batches (all windows per row)
    {"RGPU_WMAJOR": "0", "RGPU_SLOTS": "1"},
]
MODE_IDS = ["default", "tail", "tail-cap3", "tail-cap40-blocking", "hopmajor-tail", "hopmajor-serial"]


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
def test_tail_chains_vs_oracle(mode):
    st = chains_stream([1, 4, 31, 64, 98, 99, 100, 101, 140])
    o = Oracle.from_stream(st)
    g = graph_env(st, mode)
    hops = range_hops(T0_README + 10 * DAY, T0_README + 40 * DAY, 2 * DAY)
    for cap in (100, 37):
        g.run("cc", hops, [YEAR, MONTH, WEEK], max_steps=cap, retain=True)
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


@pytest.mark.parametrize("ch", ["2", "4"])
def test_superstep_chunk_sizes_vs_oracle(ch, monkeypatch):
    """The superstep kernel with 2-vertex (default) and 4-vertex chunks (RGPU_STEP_CH, read per
    run) against the oracle: chains up to past the cap, and a hub-free uniform stream."""
    monkeypatch.setenv("RGPU_STEP_CH", ch)
    st = chains_stream([1, 4, 31, 64, 98, 99, 100, 101, 140], seed=11)
    o = Oracle.from_stream(st)
    g = graph_env(st, {})
    hops = range_hops(T0_README + 10 * DAY, T0_README + 40 * DAY, 3 * DAY)
    for cap in (100, 37):
        g.run("cc", hops, [YEAR, MONTH, WEEK], max_steps=cap, retain=True)
        for h, t in enumerate(hops.tolist()):
            res, steps = o.cc(t, [YEAR, MONTH, WEEK], max_steps=cap, mode=1)
            for w in range(3):
                assert g.cc_summary(h, w).supersteps == steps, (ch, cap, t, w)
                ids, lab = res[w]
                gids, glab = g.cc_vertex_labels(h, w)
                assert np.array_equal(gids, ids) and np.array_equal(glab, lab), (ch, cap, t, w)
    g.close()


def test_tail_modes_agree_on_c2_slice():
    """C2 stream, 1,200 hourly hops: every mode gives identical summaries for all 6,000 views
    (superstep counts included: they are per hop, whatever batches held the views), and identical
    per-vertex labels on sampled hops."""
    s = gen_uniform(1, 100_000, 1_000_000)
    hops = range_hops(T0_README + 200 * DAY, T0_README + 250 * DAY, HOUR)[:1200]
    ref_summ, ref_lab = None, None
    for mode in MODES:
        g = graph_env(s, mode)
        g.run("cc", hops, BATCH_WINDOWS, retain=True)
        summ = g.cc_summaries()
        labs = [g.cc_vertex_labels(h, w)[1] for h in (0, 599, 1199) for w in range(5)]
        g.close()
        if ref_summ is None:
            ref_summ, ref_lab = summ[..., :8], labs
            continue
        assert np.array_equal(summ[..., :8], ref_summ), mode
        assert all(np.array_equal(a, b) for a, b in zip(labs, ref_lab)), mode


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
