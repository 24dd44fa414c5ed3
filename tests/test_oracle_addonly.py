"""The add-only restatement of the oracle (oracle.h orc_addonly_*, TEST INFRASTRUCTURE): on streams
of VertexAdds and EdgeAdds in time order it must answer ConnectedComponents exactly as the literal
EntityStorage replay does (oracle.h orc_cc) — members, labels and the hop's superstep count — for
descending and ascending window lists, ViewLens and superstep caps; and reproduce the literal
replay's goldens of the 100M-update C4 prefix.  It is what pins the 1B headline's year views
(tools/make_c4_sliced_goldens.py --year), which the literal replay cannot hold in memory."""
import json
import os

import numpy as np
import pytest

from oracle import AddOnlyOracle, Oracle
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, Stream, gen_gab, range_hops


def _same(o, a, t, windows, cap):
    r1, s1 = o.cc(t, windows, max_steps=cap, mode=1)
    r2, s2 = a.cc(t, windows, max_steps=cap)
    assert s1 == s2, (t, windows, cap, s1, s2)
    for w, ((i1, l1), (i2, l2)) in enumerate(zip(r1, r2)):
        assert np.array_equal(i1, i2) and np.array_equal(l1, l2), (t, windows, cap, w)


@pytest.mark.parametrize("seed", [5, 6])
def test_addonly_equals_literal_replay_on_gab_streams(seed):
    s = gen_gab(seed, 3000, 20_000)
    o, a = Oracle.from_stream(s), AddOnlyOracle.from_stream(s)
    assert a.nv == o.nv
    end = int(s.t[-1])
    for t in range_hops(end - 400 * DAY, end, 53 * DAY).tolist():
        for ws in (BATCH_WINDOWS, BATCH_WINDOWS[::-1], [], [3 * DAY, 5 * HOUR]):
            for cap in (1, 2, 3, 100):
                _same(o, a, t, ws, cap)
    o.close()
    a.close()


def test_addonly_chains_self_loops_duplicates_isolated():
    """A 150-vertex path (runs into the 100-step cap), self-loops, repeated EdgeAdds of one pair
    and both directions, vertices with VertexAdds only, ties of equal times."""
    t, k, src, dst = [], [], [], []

    def add(tt, kk, s, d=-1):
        t.append(tt), k.append(kk), src.append(s), dst.append(d)
    for i in range(150):  # path 1000 - 1001 - ... with the minimum at the far end
        add(10 + i, 2, 1149 - i, 1148 - i)
    for i in range(20):
        add(200 + i // 3, 2, 50 + i % 4, 50 + i % 4 if i % 5 == 0 else 51 + i % 3)
    for i in range(10):
        add(230 + i, 0, 3000 + i)
    add(240, 2, 7, 9), add(240, 2, 9, 7), add(241, 2, 7, 9)
    s = Stream(*(np.asarray(x, dtype) for x, dtype in ((t, np.int64), (k, np.uint8), (src, np.int64),
                                                        (dst, np.int64))))
    o, a = Oracle.from_stream(s), AddOnlyOracle.from_stream(s)
    for tq in (5, 50, 160, 205, 235, 240, 300):
        for ws in ([], [1000, 100, 30, 5], [5, 30, 100], [0]):
            for cap in (1, 2, 50, 100, 150):
                _same(o, a, tq, ws, cap)


def test_addonly_rejects_other_streams():
    s = gen_gab(3, 100, 300)
    with pytest.raises(ValueError):  # a VertexDelete
        AddOnlyOracle(s.t, np.where(np.arange(len(s)) == 7, 1, s.kind).astype(np.uint8), s.src, s.dst)
    with pytest.raises(ValueError):  # time out of order
        AddOnlyOracle(s.t[::-1].copy(), s.kind, s.src, s.dst)


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c4_prefix_goldens.json")


@pytest.mark.skipif(not os.path.exists(GOLD), reason="no prefix goldens")
def test_addonly_reproduces_literal_c4_prefix_goldens():
    """The 100M-update C4 prefix (literal replay, tools/make_c4_goldens.py): one sampled hop, all
    five windows' summary fields, member count and (id, label) checksum, and the hop's supersteps."""
    from raphtory_amd.synth import gen_gab_range
    from tools.make_c4_goldens import view_record
    P = json.load(open(GOLD))["prefixes"]["33333334"]
    s = gen_gab_range(4, 20_000_000, 333_333_334, 0, 33_333_334)
    end = int(s.t[-1])
    a = AddOnlyOracle.from_stream(s)
    del s
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    assert int(hops[0]) == P["hop0"]
    h = sorted(int(x) for x in P["hops"])[-1]
    res, steps = a.cc(int(hops[h]), BATCH_WINDOWS)
    assert steps == P["hops"][str(h)]["supersteps"]
    assert [view_record(i, l) for i, l in res] == P["hops"][str(h)]["windows"]
    a.close()
