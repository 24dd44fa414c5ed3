"""A run that fails mid-way must leave the context usable: the next run on the same sealed graph
gives the oracle's results (a throw between batches used to leave slots in phase 1-3,
count rows, island / lane-change shards and hub minima dirty, so the next run harvested a stale
slot and added leftover counts into its summaries).  The failure is injected with
RGPU_INJECT_FAIL=n (the n-th batch start of a run throws, after earlier batches ran)."""
import os

import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import RGPUError, TemporalGraph
from raphtory_amd.analysis import cc_fields, cc_fields_from_summary
from raphtory_amd.synth import BATCH_WINDOWS, DAY, T0_README, gen_powerlaw, gen_uniform, range_hops, YEAR

pytestmark = pytest.mark.gpu


def _check(g, o, hops, windows):
    for h, t in enumerate(np.asarray(hops).tolist()):
        res, steps = o.cc(t, windows, mode=1)
        for w in range(len(windows)):
            ids, lab = res[w]
            gids, glab = g.cc_vertex_labels(h, w)
            assert np.array_equal(gids, ids) and np.array_equal(glab, lab), (t, w)
            assert g.cc_result(h, w) == label_counts(lab), (t, w)
            assert cc_fields_from_summary(g.cc_summary(h, w)) == cc_fields(label_counts(lab)), (t, w)
            assert g.cc_summary(h, w).supersteps == steps, (t, w)


@pytest.mark.parametrize("which", ["uniform", "hubs"])
def test_run_after_injected_failure(which, monkeypatch):
    if which == "uniform":
        s = gen_uniform(7, 800, 20_000, t0=T0_README, dt=1_576_800)
        hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 2 * DAY)
    else:  # power-law hubs: the heavy-vertex minima (hbest) must be clean again too
        s = gen_powerlaw(5, 3000, 60_000, t0=0, t1=YEAR)
        hops = range_hops(60 * DAY, 360 * DAY, 3 * DAY)
        monkeypatch.setenv("RGPU_HEAVY", "64")
    o = Oracle.from_stream(s)
    with TemporalGraph() as g:
        g.ingest_stream(s)
        g.seal()
        for n_fail in (4, 2):  # a failure with batches of earlier windows / blocks in flight
            monkeypatch.setenv("RGPU_INJECT_FAIL", str(n_fail))
            with pytest.raises(RGPUError, match="INJECT"):
                g.run("cc", hops, BATCH_WINDOWS, retain=True)
            monkeypatch.delenv("RGPU_INJECT_FAIL")
            g.run("cc", hops, BATCH_WINDOWS, retain=True)
            _check(g, o, hops, BATCH_WINDOWS)
        # the summary-only path (no retained rows) after a failure
        monkeypatch.setenv("RGPU_INJECT_FAIL", "3")
        with pytest.raises(RGPUError):
            g.run("cc", hops, BATCH_WINDOWS)
        monkeypatch.delenv("RGPU_INJECT_FAIL")
        g.run("cc", hops, BATCH_WINDOWS)
        for h, t in enumerate(hops.tolist()[::5]):
            res, _ = o.cc(t, BATCH_WINDOWS, mode=1)
            for w in range(len(BATCH_WINDOWS)):
                assert cc_fields_from_summary(g.cc_summary(h * 5, w)) == cc_fields(label_counts(res[w][1]))


def test_corrupt_label_record_is_reported(monkeypatch):
    """Partitioned mode: a received label record that names no boundary vertex of its sender (a
    bug upstream, injected with RGPU_INJECT_FAIL=rec) is counted on the device, skipped instead of
    becoming an out-of-bounds store, and the run fails with RGPU_EHIP naming the count; the next
    run on the same partitions gives the oracle's results (include/rgpu.h error contract)."""
    from raphtory_amd.partitioned import LoopbackPartitions
    from tests.test_gpu_partitioned import check_cc
    s = gen_uniform(7, 800, 20_000, t0=T0_README, dt=1_576_800)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 6 * DAY)
    o = Oracle.from_stream(s)
    lp = LoopbackPartitions(3)
    lp.ingest_stream(s)
    lp.seal()
    monkeypatch.setenv("RGPU_INJECT_FAIL", "rec")
    with pytest.raises(RGPUError, match="outside the receive plan"):
        lp.run("cc", hops, BATCH_WINDOWS)
    monkeypatch.delenv("RGPU_INJECT_FAIL")
    check_cc(lp, o, hops, BATCH_WINDOWS)
    lp.close()


def test_corrupt_count_record_is_reported(monkeypatch):
    """Partitioned mode: a received component-count record whose label getPartition routes here but
    no owned vertex holds (injected with RGPU_INJECT_FAIL=cnt) is counted on the device
    (xchg.hip label_row) instead of being dropped, and the run fails with RGPU_EHIP naming the
    count; the next run on the same partitions gives the oracle's results."""
    from raphtory_amd.partitioned import LoopbackPartitions
    from tests.test_gpu_partitioned import check_cc
    s = gen_uniform(7, 800, 20_000, t0=T0_README, dt=1_576_800)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 6 * DAY)
    o = Oracle.from_stream(s)
    lp = LoopbackPartitions(3)
    lp.ingest_stream(s)
    lp.seal()
    monkeypatch.setenv("RGPU_INJECT_FAIL", "cnt")
    with pytest.raises(RGPUError, match="found no owned vertex"):
        lp.run("cc", hops, BATCH_WINDOWS)
    monkeypatch.delenv("RGPU_INJECT_FAIL")
    check_cc(lp, o, hops, BATCH_WINDOWS)
    lp.close()
