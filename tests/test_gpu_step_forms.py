"""The superstep kernel's forms and options against the CPU oracle.

The long-window form (lane-parallel final-label members, full folds as segmented mins, lane-parallel
simple members) runs only for batches whose windows span >= RGPU_LONG_RATIO x their hop span, and only
in its early supersteps; the short form is the round-4 kernel.  Each setting below forces one mix of
them on the same graph — long everywhere, short everywhere, each option alone — and every one must
give the oracle's labels, component maps, summaries and superstep counts (bit-exact), on an add-only
GAB-shaped stream with power-law hubs (hub segments, uniform and mixed label words) over C4-shaped
hourly hops and the five batched windows.
"""
import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab

pytestmark = pytest.mark.gpu

SETTINGS = [
    {},                                                  # the default mix
    {"RGPU_LONG_RATIO": "0"},                            # long form in every batch (early supersteps)
    {"RGPU_LONG_RATIO": "0", "RGPU_LONG_STEPS": "100"},  # long form in every superstep
    {"RGPU_LONG_RATIO": "-1"},                           # short form everywhere
    {"RGPU_LONG_RATIO": "0", "RGPU_STEP_OPTS": "1"},     # final-label members only
    {"RGPU_LONG_RATIO": "0", "RGPU_STEP_OPTS": "3"},     # + full folds, no simple members
    {"RGPU_HUB_PRO": "1"},                               # one hub segment per wave and round
]


@pytest.fixture(scope="module")
def gab():
    s = gen_gab(7, 20_000, 120_000)
    g = TemporalGraph()
    g.ingest_stream(s)
    g.seal()
    end = int(s.t[-1])
    hops = np.arange(end - 69 * HOUR, end + 1, HOUR, dtype=np.int64)  # 70 hourly hops: two batches
    o = Oracle.from_stream(s)
    pick = [0, 1, 31, 63, 64, 69]
    exp = {h: o.cc(int(hops[h]), BATCH_WINDOWS, max_steps=100, mode=1) for h in pick}
    yield g, hops, exp
    g.close()


@pytest.mark.parametrize("env", SETTINGS, ids=lambda e: "+".join(f"{k}={v}" for k, v in e.items()) or "default")
def test_step_forms_vs_oracle(gab, env, monkeypatch):
    g, hops, exp = gab
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g.run("cc", hops, BATCH_WINDOWS, max_steps=100, retain=True)
    for h, (res, steps) in exp.items():
        for w in range(len(BATCH_WINDOWS)):
            assert g.cc_summary(h, w).supersteps == steps, (env, h, w)
            ids, lab = res[w]
            gids, glab = g.cc_vertex_labels(h, w)
            assert np.array_equal(gids, ids), (env, h, w)
            assert np.array_equal(glab, lab), (env, h, w)
            cnt = label_counts(lab)
            assert g.cc_result(h, w) == cnt, (env, h, w)
            assert cc_fields_from_summary(g.cc_summary(h, w)) == cc_fields(cnt), (env, h, w)
