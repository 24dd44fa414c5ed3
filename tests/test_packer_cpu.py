"""The product's host packer (raphtory_amd/csrc/packer.cpp), built on the CPU with g++ into a
test harness, against the oracle's literal EntityStorage replay: every vertex and edge
liveness decision (aliveAt / aliveAtWithWindow) at many times and windows, on tie-heavy and
out-of-order streams, single- and multi-threaded packing."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "_build", "libpacker_harness.so")


@pytest.fixture(scope="module")
def ph():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = [os.path.join(ROOT, "tests", "packer_harness.cpp"), os.path.join(ROOT, "raphtory_amd", "csrc", "packer.cpp")]
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in src):
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread",
                        "-I", os.path.join(ROOT, "raphtory_amd", "csrc"), "-o", SO] + src, check=True)
    L = C.CDLL(SO)
    P64, PU8 = C.POINTER(C.c_int64), C.POINTER(C.c_uint8)
    L.ph_pack.restype = C.c_void_p
    L.ph_pack.argtypes = [P64, PU8, P64, P64, C.c_size_t]
    L.ph_alive.restype = C.c_int
    L.ph_alive.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64]
    L.ph_free.argtypes = [C.c_void_p]
    L.ph_num.restype = C.c_int64
    L.ph_num.argtypes = [C.c_void_p, C.c_int]
    return L


def _pack(L, t, k, s, d):
    p = lambda a, ty: a.ctypes.data_as(C.POINTER(ty))
    h = L.ph_pack(p(t, C.c_int64), p(k, C.c_uint8), p(s, C.c_int64), p(d, C.c_int64), len(t))
    assert h
    return h


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
