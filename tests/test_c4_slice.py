"""The time-slice argument behind tests/golden/c4_sliced_goldens.json (tools/make_c4_sliced_goldens.py):
on the add-only C4 stream a view (t, w) depends only on the updates with time in [t - w, t]
(Entity.scala:193-201 aliveAtWithWindow), so the oracle replaying only the
updates newer than hop0 - w must reproduce, window for window, what it computed replaying the
whole 100M-update prefix (tests/golden/c4_prefix_goldens.json, tools/make_c4_goldens.py):
summary fields, member count and the checksum of every member's (id, label).

CPU only (the oracle; test infrastructure).  The slice for week/day/hour is ~14 days of the
stream (~21M updates); the month window is checked at generation time by the same function
(profiles/r04/c4_slice_equivalence.txt) because its 37-day slice costs minutes here."""
import json
import os

import pytest

from raphtory_amd.synth import BATCH_WINDOWS

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c4_prefix_goldens.json")
PREFIX = "33333334"  # interactions (100,000,002 updates)


def test_first_at_bisection_on_the_generator():
    from tools.make_c4_sliced_goldens import first_at, t_of
    n = 1_000_000
    t_mid = t_of(n // 2)
    i = first_at(t_mid, n)
    assert t_of(i) >= t_mid and (i == 0 or t_of(i - 1) < t_mid)
    assert first_at(t_of(0), n) == 0
    assert first_at(t_of(n - 1) + 1, n) == n


@pytest.mark.skipif(not os.path.exists(GOLD), reason="no prefix goldens")
def test_sliced_oracle_equals_full_prefix_oracle():
    from tools.make_c4_sliced_goldens import headline_hops, sliced_views
    P = json.load(open(GOLD))["prefixes"][PREFIX]
    n = int(PREFIX)
    assert int(headline_hops(n)[0]) == P["hop0"]
    windows = BATCH_WINDOWS[2:]  # week, day, hour (indices 2..4 of the query)
    sel = sorted(int(h) for h in P["hops"])[::2]
    meta, views = sliced_views(n, windows, sel, threads=8, log=lambda m: None)
    assert meta["slice_updates"] < P["updates"] // 3  # a real slice, not the prefix
    for h in sel:
        full = P["hops"][str(h)]
        assert views[str(h)]["t"] == full["t"]
        for k, rec in enumerate(views[str(h)]["windows"]):
            assert rec == full["windows"][2 + k], (h, windows[k])
