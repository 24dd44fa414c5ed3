"""The product's host packer (raphtory_amd/csrc/packer.cpp), built on the CPU with g++ into a
test harness, against the oracle's literal EntityStorage replay: every vertex and edge
liveness decision (aliveAt / aliveAtWithWindow) at many times and windows, on tie-heavy and
out-of-order streams, single- and multi-threaded packing."""
import numpy as np
import pytest

from oracle import Oracle

from harness import P64, PU8, load_packer_harness, pack


@pytest.fixture(scope="module")
def ph():
    return load_packer_harness()


def _pack(L, t, k, s, d):
    return pack(L, t, k, s, d)


def _stream(seed, n, nv, tie, shuffle=False):
    rng = np.random.default_rng(seed)
    t = (np.arange(n) // tie).astype(np.int64) * 7
    k = rng.choice(4, size=n, p=[0.25, 0.45, 0.12, 0.18]).astype(np.uint8)
    s = rng.integers(0, nv, n).astype(np.int64)
    d = np.where(k >= 2, rng.integers(0, nv, n), -1).astype(np.int64)
    if shuffle:
        q = rng.permutation(n)
        t, k, s, d = t[q], k[q], s[q], d[q]
    return t, k, s, d


@pytest.mark.parametrize("seed,tie,shuffle,threads", [(1, 1, False, "1"), (2, 4, False, "1"), (3, 3, True, "1"),
                                                      (4, 5, False, "8"), (5, 2, True, "8")])
def test_packed_liveness_matches_oracle(ph, seed, tie, shuffle, threads, monkeypatch):
    monkeypatch.setenv("RGPU_THREADS", threads)
    t, k, s, d = _stream(seed, 5000, 40, tie, shuffle)
    o = Oracle(t, k, s, d)
    h = _pack(ph, t, k, s, d)
    assert ph.ph_num(h, 0) == o.nv and ph.ph_num(h, 1) == o.ne
    rng = np.random.default_rng(seed + 100)
    times = np.unique(np.concatenate([t, t + 1, t - 1, rng.integers(0, int(t.max()) + 50, 200)]))
    times = times[times >= 0][:: max(1, len(times) // 300)]
    pairs = sorted({(int(a), int(b)) for a, b, kk in zip(s, d, k) if kk >= 2})
    bad = 0
    for tt in times.tolist():
        for w in (-1, 0, 14, 200, 5000):
            for v in range(40):
                bad += ph.ph_alive(h, 0, v, -1, tt, w) != o.alive(False, v, -1, tt, w)
            for a, b in pairs[:: max(1, len(pairs) // 150)]:
                bad += ph.ph_alive(h, 1, a, b, tt, w) != o.alive(True, a, b, tt, w)
    ph.ph_free(h)
    assert bad == 0


def test_parallel_pack_is_deterministic(ph, monkeypatch):
    t, k, s, d = _stream(9, 200_000, 5000, 2)
    monkeypatch.setenv("RGPU_THREADS", "1")
    h1 = _pack(ph, t, k, s, d)
    monkeypatch.setenv("RGPU_THREADS", "8")
    h8 = _pack(ph, t, k, s, d)
    for w in range(4):
        assert ph.ph_num(h1, w) == ph.ph_num(h8, w)
    for tt in (1000, 100_000, 300_000):
        for v in range(0, 5000, 97):
            assert ph.ph_alive(h1, 0, v, -1, tt, 3000) == ph.ph_alive(h8, 0, v, -1, tt, 3000)
    ph.ph_free(h1)
    ph.ph_free(h8)


@pytest.mark.parametrize("seed,tie,shuffle,threads,frac,n", [(11, 1, False, "1", 0.5, 40_000),
                                                             (12, 4, False, "8", 0.7, 40_000),
                                                             (13, 3, True, "8", 0.4, 40_000),
                                                             (14, 2, True, "1", 0.9, 40_000),
                                                             (15, 2, False, "8", 0.3, 200_000)])
def test_live_delta_host_half_matches_one_shot_pack(ph, seed, tie, shuffle, threads, frac, n, monkeypatch):
    """pack_delta + finish_delta (live ingest) vs pack_events of the whole stream:
    ids, rank maps, offsets, death lists, edge set and merged vertex histories.  Cuts fall
    inside groups of equal times; the shuffled streams exercise the non-monotone fallback,
    the ordered ones the radix path (8 threads: multi-chunk parallel code; 200k updates: the
    multi-threaded radix passes)."""
    monkeypatch.setenv("RGPU_THREADS", threads)
    t, k, s, d = _stream(seed, n, 3_000 if n < 100_000 else 20_000, tie, shuffle)
    rc = ph.ph_delta_check(t.ctypes.data_as(P64), k.ctypes.data_as(PU8), s.ctypes.data_as(P64),
                           d.ctypes.data_as(P64), len(t), int(len(t) * frac))
    assert rc == 0, f"check {rc} failed"


def _records(ph, h, what):
    """plist records (kind 9 edges / 10 vertices) -> {first id(s): the rest}"""
    from harness import plist
    x = plist(ph, h, what).tolist()
    out, i = {}, 0
    while i < len(x):
        if what == 9:
            key, n = (x[i], x[i + 1]), x[i + 2]
            out[key] = tuple(x[i + 3:i + 3 + n])
            i += 3 + n
        else:
            vid, n = x[i], x[i + 1]
            hist = tuple(x[i + 2:i + 2 + n])
            m = x[i + 2 + n]
            out[vid] = (hist, tuple(x[i + 3 + n:i + 3 + n + m]))
            i += 3 + n + m
    return out


@pytest.mark.parametrize("seed,tie,shuffle,threads,nv", [(21, 1, False, "1", 40), (22, 3, True, "8", 40),
                                                         (23, 2, False, "8", 3000)])
def test_locality_order_is_the_same_graph(ph, seed, tie, shuffle, threads, nv, monkeypatch):
    """RGPU_ORDER_LOCALITY (packer.cpp locality_order) only renumbers the local ranks: per id the
    same vertex history and death list, per (src id, dst id) the same edge history (ties
    resolved the same way), labels still the id ranks, by_id ascending, CSR and in-edge order
    intact; and the liveness decisions equal the oracle's."""
    from harness import plist
    monkeypatch.setenv("RGPU_THREADS", threads)
    t, k, s, d = _stream(seed, 20_000, nv, tie, shuffle)
    ph.ph_set_locality(0)
    h0 = _pack(ph, t, k, s, d)
    ph.ph_set_locality(1)
    try:
        h1 = _pack(ph, t, k, s, d)
    finally:
        ph.ph_set_locality(0)
    assert plist(ph, h1, 11).tolist() == [0]
    assert _records(ph, h0, 9) == _records(ph, h1, 9)
    assert _records(ph, h0, 10) == _records(ph, h1, 10)
    ids1 = plist(ph, h1, 7)
    assert np.array_equal(ids1, plist(ph, h0, 0))          # by_id lists the ids ascending
    assert np.array_equal(plist(ph, h1, 8), plist(ph, h1, 0))  # every rank's label is its own id
    if nv >= 3000:  # the ranks really moved: most active first within a group
        assert not np.array_equal(plist(ph, h1, 0), plist(ph, h0, 0))
    o = Oracle(t, k, s, d)
    bad = 0
    for tt in np.unique(t)[:: max(1, len(np.unique(t)) // 25)].tolist():
        for w in (-1, 30, 5000):
            for v in range(0, nv, max(1, nv // 40)):
                bad += ph.ph_alive(h1, 0, v, -1, tt, w) != o.alive(False, v, -1, tt, w)
    assert bad == 0
    ph.ph_free(h0)
    ph.ph_free(h1)
