"""The partitioned exchange's region arithmetic (raphtory_amd/csrc/xregions.hpp, used by rgpu.cpp
part_after_counts), built on the CPU with g++: per-peer record counts from the exchanged counts
words, every peer's send / receive region offsets, and the check that each transfer lies inside its
region and each region inside its buffer.  The round-4 P = 8 rehearsal died with a host SIGSEGV
inside a loopback copy; these are the ranges that copy is handed."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "_build", "libxregions_harness.so")
P64 = C.POINTER(C.c_int64)


@pytest.fixture(scope="module")
def xr():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = [os.path.join(ROOT, "tests", "xregions_harness.cpp"), os.path.join(ROOT, "raphtory_amd", "csrc", "xregions.hpp")]
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in src):
        tmp = SO + f".{os.getpid()}"
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Werror",
                        "-I", os.path.join(ROOT, "raphtory_amd", "csrc"), "-o", tmp, src[0]], check=True)
        os.replace(tmp, SO)
    L = C.CDLL(SO)
    L.xr_plan.restype = C.c_int
    L.xr_plan.argtypes = [C.c_int, C.c_int, P64, P64, P64, C.c_int64, C.c_int64, P64, C.c_int64, C.c_int64,
                          C.c_int64, C.c_int64, P64]
    L.xr_error.restype = C.c_char_p
    return L


def _p(a):
    return a.ctypes.data_as(P64)


def plan(L, P, me, xa, xb, nbq, su_cap, smcap, rmcap, allocs=None):
    nbq = np.asarray(nbq, np.int64)
    rmcap = np.asarray(rmcap, np.int64)
    if allocs is None:
        allocs = (su_cap * P, smcap * P, int(nbq.sum()), int(rmcap.sum()))
    out = np.zeros(8 * P + 2, np.int64)
    rc = L.xr_plan(P, me, _p(np.asarray(xa, np.int64)), _p(np.asarray(xb, np.int64)), _p(nbq), su_cap, smcap,
                   _p(rmcap), *allocs, _p(out))
    return rc, L.xr_error().decode(), out


def words(P, me, u, m, vote):
    """counts words as k_xbc_counts writes them: [4q] U, [4q+1] M, [4q+2] vote, 0 for q = me"""
    w = np.zeros(4 * P, np.int64)
    for q in range(P):
        if q != me:
            w[4 * q], w[4 * q + 1] = u[q], m[q]
        w[4 * q + 2] = vote
    return w


@pytest.mark.parametrize("P", [2, 3, 8])
def test_random_counts_within_caps_lay_out_disjoint_in_bounds(xr, P):
    rng = np.random.default_rng(P)
    for it in range(200):
        me = int(rng.integers(0, P))
        nbq = rng.integers(0, 50, P)
        nbq[me] = 0
        su_cap = int(rng.integers(1, 60))
        sent_u = rng.integers(0, su_cap + 1, P)
        sent_m = rng.integers(0, 40, P)
        recv_u = np.minimum(rng.integers(0, 60, P), nbq)
        recv_m = rng.integers(0, 40, P)
        smcap = int(max(sent_m.max(), 1))
        rmcap = np.maximum(recv_m, rng.integers(0, 5, P))
        xa = words(P, me, sent_u, sent_m, 0)
        xb = words(P, me, recv_u, recv_m, int(it % 3 == 0))
        rc, err, out = plan(xr, P, me, xa, xb, nbq, su_cap, smcap, rmcap)
        assert rc == 0, err
        o = out[4 * P:8 * P].reshape(P, 4)
        cnt = out[:4 * P].reshape(P, 4)
        assert out[8 * P + 1] == int(it % 3 == 0)
        assert out[8 * P] == max(int(sent_m[q]) for q in range(P) if q != me) if P > 1 else 0
        # U / M receive regions: consecutive, in peer order, each of its own capacity
        assert np.array_equal(o[:, 2], np.concatenate([[0], np.cumsum(nbq)[:-1]]))
        assert np.array_equal(o[:, 3], np.concatenate([[0], np.cumsum(rmcap)[:-1]]))
        assert np.array_equal(o[:, 0], np.arange(P) * su_cap) and np.array_equal(o[:, 1], np.arange(P) * smcap)
        for q in range(P):
            if q == me:
                assert not cnt[q].any()
                continue
            # every transfer inside its own region, and so inside its buffer and clear of the next peer's
            assert o[q, 0] + cnt[q, 0] <= (q + 1) * su_cap <= su_cap * P
            assert o[q, 1] + cnt[q, 1] <= (q + 1) * smcap <= smcap * P
            assert o[q, 2] + cnt[q, 2] <= o[q, 2] + nbq[q] <= nbq.sum()
            assert o[q, 3] + cnt[q, 3] <= o[q, 3] + rmcap[q] <= rmcap.sum()


def test_overflows_are_named(xr):
    P, me = 4, 1
    nbq = [5, 0, 7, 3]
    ok = dict(su_cap=10, smcap=6, rmcap=[4, 0, 4, 4])
    xa = words(P, me, [2, 0, 2, 2], [1, 0, 6, 1], 1)
    xb = words(P, me, [5, 0, 7, 3], [4, 0, 4, 4], 1)
    assert plan(xr, P, me, xa, xb, nbq, **ok)[0] == 0
    # a peer announcing more U records than its boundary vertices: phase 1
    rc, err, _ = plan(xr, P, me, xa, words(P, me, [6, 0, 7, 3], [4, 0, 4, 4], 1), nbq, **ok)
    assert rc == 1 and "peer 0 announced 6 U records for 5 boundary vertices" in err
    # an M list larger than the send regions (the caller must grow them first): phase 2 names it
    rc, err, out = plan(xr, P, me, xa, xb, nbq, su_cap=10, smcap=5, rmcap=[4, 0, 4, 4])
    assert rc == 2 and "M send for peer 2" in err and out[8 * P] == 6
    # a received M list past its region
    rc, err, _ = plan(xr, P, me, xa, xb, nbq, su_cap=10, smcap=6, rmcap=[4, 0, 3, 4])
    assert rc == 2 and "M receive for peer 2: 4 records, region of 3" in err
    # U records past their send region
    rc, err, _ = plan(xr, P, me, words(P, me, [2, 0, 11, 2], [1, 0, 6, 1], 1), xb, nbq, **ok)
    assert rc == 2 and "U send for peer 2" in err
    # regions past their buffers (a buffer allocated for fewer peers or smaller caps)
    for i, what in enumerate(["U send regions", "M send regions", "U receive regions", "M receive regions"]):
        allocs = [40, 24, 15, 12]
        allocs[i] -= 1
        rc, err, _ = plan(xr, P, me, xa, xb, nbq, allocs=tuple(allocs), **ok)
        assert rc == 2 and what in err, (what, err)
    # negative counts never reach a copy
    rc, err, _ = plan(xr, P, me, words(P, me, [2, 0, -1, 2], [1, 0, 6, 1], 1), xb, nbq, **ok)
    assert rc == 1 and "negative" in err


def test_bad_partition_arguments(xr):
    z = np.zeros(40, np.int64)
    assert plan(xr, 9, 0, z, z, np.zeros(9), 1, 1, np.zeros(9))[0] == 1
    assert plan(xr, 2, 2, z, z, np.zeros(2), 1, 1, np.zeros(2))[0] == 1
