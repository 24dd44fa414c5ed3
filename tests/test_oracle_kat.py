"""The CPU oracle against the hand-derived known answers (tests/golden/kat_semantics.json)
and against closed-form cases (superstep cap, path graphs).  No GPU."""
import numpy as np
import pytest

from oracle import Oracle
from tests.kat import arrays, cc_expect, load_cases

CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_kat(case):
    o = Oracle(*arrays(case))
    for h in case.get("history", []):
        got = o.history(h["edge"], h["src"], h["dst"])
        exp = None if h["expect"] is None else [tuple(x) for x in h["expect"]]
        assert got == exp, (h, got)
    for a in case.get("alive", []):
        assert o.alive(a["edge"], a["src"], a["dst"], a["t"], a["w"]) == a["expect"], a
    for q in case.get("cc", []):
        for mode in (0, 1):
            res, _ = o.cc(q["t"], q["windows"], mode=mode)
            got = [dict(zip(ids.tolist(), lab.tolist())) for ids, lab in res]
            assert got == [cc_expect(m) for m in q["expect"]], (q, mode, got)
    for q in case.get("degree", []):
        res = o.degree(q["t"], q["windows"])
        got = [[[int(i), int(a), int(b)] for i, a, b in zip(*r)] for r in res]
        assert got == q["expect"], (q, got)


def _path(n):
    t = np.arange(1, n, dtype=np.int64)
    return t, np.full(n - 1, 2, np.uint8), np.arange(0, n - 1, dtype=np.int64), np.arange(1, n, dtype=np.int64)


def test_superstep_cap_limits_label_radius():
    # ConnectedComponents.defineMaxSteps = 100 (:160), AnalysisTask.endStep (:214): after 100
    # supersteps label(v) = min id within distance 100
    o = Oracle(*_path(150))
    (res,), steps = o.cc(1000, [], max_steps=100)
    ids, lab = res
    assert steps == 100
    assert np.array_equal(lab, np.maximum(ids - 100, 0))
    (res,), steps = o.cc(1000, [], max_steps=200)
    assert steps == 150  # last improvement at step 149, step 150 votes to halt
    assert np.all(res[1] == 0)


def test_refsim_and_cached_modes_agree_on_random_stream():
    from raphtory_amd.synth import gen_uniform, BATCH_WINDOWS
    s = gen_uniform(7, 300, 3000, t0=0, dt=1_000_000)
    o = Oracle.from_stream(s)
    for t in (500_000_000, 1_500_000_000, 2_999_000_000):
        a, sa = o.cc(t, [2_000_000_000, 400_000_000, 50_000_000], mode=0)
        b, sb = o.cc(t, [2_000_000_000, 400_000_000, 50_000_000], mode=1)
        assert sa == sb
        for (i1, l1), (i2, l2) in zip(a, b):
            assert np.array_equal(i1, i2) and np.array_equal(l1, l2)


def test_pagerank_spec_on_cycle():
    # 3-cycle, everything alive: PR stays 1.0 (0.15 + 0.85 * 1)
    t = np.array([1, 2, 3], np.int64)
    o = Oracle(t, np.full(3, 2, np.uint8), np.array([0, 1, 2], np.int64), np.array([1, 2, 0], np.int64))
    ((ids, pr),) = o.pagerank(10, [], iters=20)
    assert ids.tolist() == [0, 1, 2]
    assert np.allclose(pr, 1.0, atol=1e-15)
    # star into 0 from 1,2 (0 has no out-edge, dangling mass dropped): PR(0)=0.15+0.85*2*0.15
    o = Oracle(np.array([1, 2], np.int64), np.full(2, 2, np.uint8), np.array([1, 2], np.int64),
               np.array([0, 0], np.int64))
    ((ids, pr),) = o.pagerank(10, [], iters=20)
    assert pr.tolist() == pytest.approx([0.15 + 0.85 * 0.3, 0.15, 0.15])
