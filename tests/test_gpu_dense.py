"""Dense supersteps (kernels.hip dense_rule): when step r-1 changed at least
nv / RGPU_DENSE vertices, step r writes no frontier flags and step r+1 visits every member; the
hub gather / hub mark / boundary-record pack treat such a step as visiting all.  The default rule
only fires above 2M vertices (the full-size C4 tests run it); here RGPU_DENSE forces it on small
graphs, so nearly every step is dense, and the results must stay bit-exact against the CPU
oracle: labels, component maps and summaries (ConnectedComponents.scala:10-42,137-145)."""
import contextlib
import os

import numpy as np
import pytest

from oracle import Oracle
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, gen_gab, range_hops
from tests.test_gpu_heavy import check_vs_oracle, hubs_stream
from tests.test_gpu_partitioned import _parts, check_cc
from tests.test_gpu_batch_modes import graph_env

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def dense(div):
    """RGPU_DENSE is read at every rgpu_run_view_batch"""
    old = os.environ.get("RGPU_DENSE")
    os.environ["RGPU_DENSE"] = str(div)
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("RGPU_DENSE", None)
        else:
            os.environ["RGPU_DENSE"] = old


@pytest.mark.parametrize("div", [1000, 3])
def test_dense_steps_hubs_vs_oracle(div):
    st = hubs_stream()
    o = Oracle.from_stream(st)
    g = graph_env(st, {"RGPU_HEAVY": "8"})  # hubs split into segments: gather / mark paths
    hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, 3 * DAY)
    with dense(div):
        check_vs_oracle(g, o, hops, [MONTH, WEEK, DAY])
        check_vs_oracle(g, o, hops[:6], [WEEK], max_steps=3)  # the cap inside dense runs
    g.close()
    o.close()


def test_dense_steps_partitioned_vs_oracle():
    st = hubs_stream()
    o = Oracle.from_stream(st)
    lp = _parts(st, 3, {"RGPU_HEAVY": "300"})
    hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, 2 * DAY)
    with dense(1000):
        check_cc(lp, o, hops, [MONTH, WEEK, DAY])
    lp.close()
    o.close()


def test_dense_steps_gab_window_major_equal_flagged():
    """A GAB-shaped stream under window-major batches: dense-forced and flag-driven runs give
    identical summaries on every view, and per-vertex labels equal the oracle at sampled hops."""
    st = gen_gab(4, 20_000, 150_000)
    end = int(st.t[-1])
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    o = Oracle.from_stream(st)
    g = graph_env(st, {})
    with dense(0):
        g.run("cc", hops, BATCH_WINDOWS)
        flagged = g.cc_summaries()
    with dense(1000):
        g.run("cc", hops, BATCH_WINDOWS)
        forced = g.cc_summaries()
        assert np.array_equal(flagged, forced)
        check_vs_oracle(g, o, hops[[0, 80, 167]], BATCH_WINDOWS)
    g.close()
    o.close()
