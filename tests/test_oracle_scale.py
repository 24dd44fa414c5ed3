"""The oracle's lazy-edge build (oracle.h ORC_LAZY_EDGES, used for the full-size C3/C4 parity
tests) against its literal EntityStorage replay: every edge history, liveness, CC, degree and
PageRank must be identical.  Streams with deletes, ties, out-of-order times, self-loops and
deaths before edges exist (the killList-at-creation rule, Edge.scala:36-44)."""
import numpy as np
import pytest

from oracle import Oracle
from raphtory_amd.synth import DAY, MONTH, WEEK, YEAR, gen_gab, gen_powerlaw, gen_uniform


def _tied(seed, n=4000, nv=40):
    rng = np.random.default_rng(seed)
    t = (np.arange(n) // 3).astype(np.int64) * 7
    kind = rng.choice(4, size=n, p=[0.2, 0.4, 0.2, 0.2]).astype(np.uint8)
    src = rng.integers(0, nv, n).astype(np.int64)
    dst = np.where(kind >= 2, rng.integers(0, nv, n), -1).astype(np.int64)
    return t, kind, src, dst


def _shuffled(seed):
    s = gen_uniform(seed, 60, 3000, t0=0, dt=1000)
    p = np.random.default_rng(seed).permutation(len(s))
    return s.t[p], s.kind[p], s.src[p], s.dst[p]


def _streams():
    s = gen_uniform(5, 200, 5000, t0=0, dt=1000)
    yield "uniform", (s.t, s.kind, s.src, s.dst)
    s = gen_powerlaw(3, 300, 8000, t0=0, t1=YEAR)
    yield "powerlaw", (s.t, s.kind, s.src, s.dst)
    s = gen_gab(4, 300, 2000)
    yield "gab", (s.t, s.kind, s.src, s.dst)
    for k in range(3):
        yield f"ties{k}", _tied(k)
    yield "shuffled", _shuffled(9)


STREAMS = list(_streams())


@pytest.mark.parametrize("name,arrs", STREAMS, ids=[n for n, _ in STREAMS])
def test_lazy_edges_match_literal_replay(name, arrs):
    t, kind, src, dst = arrs
    a, b = Oracle(t, kind, src, dst), Oracle(t, kind, src, dst, lazy=True)
    assert (a.nv, a.ne) == (b.nv, b.ne)
    pairs = sorted({(int(x), int(y)) for x, y, k in zip(src, dst, kind) if k >= 2})
    for x, y in pairs:
        assert a.history(True, x, y) == b.history(True, x, y), (x, y)
    lo, hi = int(t.min()), int(t.max())
    probes = np.linspace(lo - 5, hi + 5, 9).astype(np.int64).tolist()
    span = max(1, hi - lo)
    windows = [span, span // 4, span // 30]
    for x, y in pairs[::7]:
        for tt in probes:
            for w in (-1, *windows):
                assert a.alive(True, x, y, tt, w) == b.alive(True, x, y, tt, w), (x, y, tt, w)
    for tt in probes[1:-1:2]:
        ra, sa = a.cc(tt, windows)
        rb, sb = b.cc(tt, windows)
        assert sa == sb
        for (i1, l1), (i2, l2) in zip(ra, rb):
            assert np.array_equal(i1, i2) and np.array_equal(l1, l2)
        for (i1, o1, n1), (i2, o2, n2) in zip(a.degree(tt, windows), b.degree(tt, windows)):
            assert np.array_equal(i1, i2) and np.array_equal(o1, o2) and np.array_equal(n1, n2)
        for (i1, p1), (i2, p2) in zip(a.pagerank(tt, windows[:2]), b.pagerank(tt, windows[:2])):
            assert np.array_equal(i1, i2) and np.array_equal(p1, p2)
    a.close()
    b.close()
