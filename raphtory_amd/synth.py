"""Seeded synthetic update streams — numpy front-end of libsynth.so.

The stream is the SoA the C ABI ingests: ``t`` int64 ms, ``kind`` uint8 (VADD 0, VDEL 1,
EADD 2, EDEL 3), ``src``/``dst`` int64 (dst = -1 for vertex updates).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _native as N

# README.md:66 range start (2016-08-10 00:00 +01:00), and the GAB span (README.md:21)
T0_README = 1470783600000
GAB_T0 = 1470787200000   # 2016-08-10T00:00Z
GAB_T1 = 1527724800000   # 2018-05-31T00:00Z
HOUR = 3_600_000
DAY = 86_400_000
WEEK = 604_800_000
MONTH = 2_592_000_000
YEAR = 31_536_000_000
BATCH_WINDOWS = [YEAR, MONTH, WEEK, DAY, HOUR]


@dataclass
class Stream:
    t: np.ndarray
    kind: np.ndarray
    src: np.ndarray
    dst: np.ndarray

    def __len__(self) -> int:
        return int(self.t.shape[0])

    def slice(self, n: int) -> "Stream":
        return Stream(self.t[:n], self.kind[:n], self.src[:n], self.dst[:n])


def _alloc(n: int):
    return (np.empty(n, np.int64), np.empty(n, np.uint8), np.empty(n, np.int64), np.empty(n, np.int64))


def gen_uniform(seed: int, nverts: int, n: int, t0: int = T0_README, dt: int = 31_536,
                mix=(0.3, 0.4, 0.1)) -> Stream:
    """C1/C2 shape: VADD/EADD/VDEL/EDEL = 30/40/10/20 % (paper mix), uniform ids."""
    t, k, s, d = _alloc(n)
    N.synth().rg_gen_uniform(seed, nverts, n, t0, dt, mix[0], mix[1], mix[2],
                             N.ptr(t, N.C.c_int64), N.ptr(k, N.C.c_uint8),
                             N.ptr(s, N.C.c_int64), N.ptr(d, N.C.c_int64))
    return Stream(t, k, s, d)


def gen_powerlaw(seed: int, nverts: int, n: int, gamma: float = 2.1,
                 t0: int = T0_README, t1: int = T0_README + 2 * YEAR) -> Stream:
    """C3 shape: Chung-Lu power-law endpoints, 8/85/5/2 % VADD/EADD/EDEL/VDEL."""
    t, k, s, d = _alloc(n)
    N.synth().rg_gen_powerlaw(seed, nverts, n, gamma, t0, t1,
                              N.ptr(t, N.C.c_int64), N.ptr(k, N.C.c_uint8),
                              N.ptr(s, N.C.c_int64), N.ptr(d, N.C.c_int64))
    return Stream(t, k, s, d)


def gen_gab(seed: int, users: int, interactions: int, t0: int = GAB_T0, t1: int = GAB_T1,
            id_key: int = None) -> Stream:
    """C4 shape: add-only (VADD s, VADD d, EADD s->d) triples at one t (GabUserGraphRouter).
    id_key (default: seed) scatters user ranks over ids; keep it fixed to draw later ticks of
    one live stream (same users) with other seeds."""
    n = 3 * interactions
    t, k, s, d = _alloc(n)
    N.synth().rg_gen_gab_keyed(seed, seed if id_key is None else id_key, users, interactions, t0, t1,
                               N.ptr(t, N.C.c_int64), N.ptr(k, N.C.c_uint8),
                               N.ptr(s, N.C.c_int64), N.ptr(d, N.C.c_int64))
    return Stream(t, k, s, d)


def gen_gab_range(seed: int, users: int, interactions: int, first: int, count: int, part: int = 0,
                  nparts: int = 1, t0: int = GAB_T0, t1: int = GAB_T1, id_key: int = None) -> Stream:
    """Interactions [first, first+count) of gen_gab(seed, users, interactions): a prefix is a
    slice of the full C4 stream, and chunks concatenate to it.  nparts > 1 keeps only what
    partition `part` ingests (the VertexAdds of its vertices and every EdgeAdd with an endpoint
    it owns, Utils.getPartition), so a rank holds O(stream / P) updates."""
    count = max(0, min(count, interactions - first))
    t, k, s, d = _alloc(3 * count)
    n = N.synth().rg_gen_gab_range(seed, seed if id_key is None else id_key, users, interactions, first, count,
                                   part, nparts, t0, t1, N.ptr(t, N.C.c_int64), N.ptr(k, N.C.c_uint8),
                                   N.ptr(s, N.C.c_int64), N.ptr(d, N.C.c_int64))
    return Stream(t[:n], k[:n], s[:n], d[:n])


def gab_first_at(seed: int, users: int, interactions: int, t_from: int) -> int:
    """The first interaction index of the gen_gab stream with time >= t_from (`interactions` if
    none): bisection on the generator itself, whose times are monotone in the index."""
    lo, hi = 0, interactions
    while lo < hi:
        mid = (lo + hi) // 2
        if int(gen_gab_range(seed, users, interactions, mid, 1).t[0]) >= t_from:
            hi = mid
        else:
            lo = mid + 1
    return lo


def range_hops(start: int, end: int, jump: int) -> np.ndarray:
    """Hop timestamps of a Range job: RangeAnalysisTask.restart (RangeAnalysisTask.scala:18-35)
    starts at `start`, adds `jump`, clamps to `end`, and stops once it has run `end`."""
    if jump <= 0:
        raise ValueError("jump must be positive")
    if start > end:  # restart(): start != end, start + jump > end is clamped to end
        return np.asarray([start, end], np.int64)
    hops = np.arange(start, end, jump, dtype=np.int64)
    return np.append(hops, np.int64(end))
