"""BinaryDefusion on the GPU (raphtory_amd/csrc/diffusion.hip) against the oracle
(oracle/oracle.c:orc_diffusion), bit-exact: per view the infected ids and their infection
supersteps, and the infected count.  Both sides use the hash coin of include/rgpu.h."""
import numpy as np
import pytest

from oracle import Oracle
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import BinaryDefusion, BWindowedRangeAnalysisTask
from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, gen_powerlaw, gen_uniform, range_hops

pytestmark = pytest.mark.gpu


def gpu_graph(t, kind, src, dst):
    g = TemporalGraph()
    g.ingest(t, kind, src, dst)
    g.seal()
    return g


def check_diff(g, o, hops, windows, seed=31, coin_seed=0, coin=True, max_steps=100):
    g.set_diffusion(seed, coin_seed, coin)
    g.run("diffusion", hops, windows, max_steps=max_steps, retain=True)
    nw = max(1, len(windows))
    g_hop_major = len(hops) * nw <= 64 or nw == 1
    total = 0
    for h, t in enumerate(np.asarray(hops).tolist()):
        res, steps = o.diffusion(t, windows, max_steps=max_steps, seed_id=seed, coin_seed=coin_seed, coin=coin)
        for w in range(nw):
            ids, st = res[w]
            gids, gst = g.diffusion_vertex(h, w)
            assert np.array_equal(gids, ids), (t, w, len(gids), len(ids))
            assert np.array_equal(gst, st), (t, w)
            n, gsteps = g.diffusion_result(h, w)
            assert n == len(ids)
            # supersteps are the batch's (a reference job halts with its slowest window; a
            # window-major batch holds one window of 64 hops), so only hop-major batches bound it
            if g_hop_major:
                assert gsteps >= steps or max_steps <= 1
            total += n
    return total


@pytest.fixture(scope="module")
def uniform():
    s = gen_uniform(1, 2000, 40000, dt=31_536 * 25)
    o = Oracle.from_stream(s)
    g = gpu_graph(s.t, s.kind, s.src, s.dst)
    yield s, o, g
    g.close()


def test_taint_uniform_hop_major(uniform):
    s, o, g = uniform
    hops = range_hops(T0_README + 60 * DAY, T0_README + 365 * DAY, 30 * DAY)[:10]
    assert check_diff(g, o, hops, BATCH_WINDOWS, coin=False) > 0


def test_coin_uniform_window_major(uniform):
    s, o, g = uniform
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 7 * DAY)[:30]  # 150 views: window-major
    for cs in (0, 99):
        assert check_diff(g, o, hops, [MONTH, WEEK, DAY], coin_seed=cs) > 0
    check_diff(g, o, hops[:3], [], coin_seed=7)  # ViewLens
    # without retain: no per-vertex rows, the infected counts come from the step kernels alone
    g.set_diffusion(31, 99, True)
    g.run("diffusion", hops, [MONTH, WEEK, DAY], retain=True)
    kept = [g.diffusion_result(h, w) for h in range(len(hops)) for w in range(3)]
    g.run("diffusion", hops, [MONTH, WEEK, DAY], retain=False)
    assert [g.diffusion_result(h, w) for h in range(len(hops)) for w in range(3)] == kept
    g.run("diffusion", hops, [MONTH, WEEK, DAY], profile=True, serial=True)  # event-timed pass
    k = g.stats()["kernels"]["diffusion"]
    assert k["launches"] > 0 and k["ms"] > 0 and k["bytes"] > 0


def test_caps_and_absent_seed(uniform):
    s, o, g = uniform
    hops = range_hops(T0_README + 100 * DAY, T0_README + 200 * DAY, 20 * DAY)
    assert check_diff(g, o, hops, [MONTH, WEEK], coin=False, max_steps=1) == 0
    check_diff(g, o, hops, [MONTH, WEEK], coin=False, max_steps=2)
    check_diff(g, o, hops, [MONTH], seed=10**9, coin=False)


def test_chain_hits_superstep_cap():
    n = 150
    t = np.ones(n, np.int64)
    kind = np.full(n, 2, np.uint8)
    src = np.array([31] + [1000 + i for i in range(1, n)], np.int64)
    dst = np.array([1000 + i + 1 for i in range(n)], np.int64)
    o = Oracle(t, kind, src, dst)
    g = gpu_graph(t, kind, src, dst)
    check_diff(g, o, [5, 6], [], coin=False)
    g.run("diffusion", [5], [], max_steps=100, retain=True)
    assert g.diffusion_result(0, 0) == (101, 100)
    g.close()


def test_powerlaw_hub_seed():
    s = gen_powerlaw(3, 20000, 150000)
    o = Oracle.from_stream(s)
    g = gpu_graph(s.t, s.kind, s.src, s.dst)
    ids, cnt = np.unique(s.src[s.kind == 2], return_counts=True)
    hub = int(ids[np.argmax(cnt)])
    hops = np.array([int(s.t[-1]) - 40 * DAY, int(s.t[-1])], np.int64)
    assert check_diff(g, o, hops, [MONTH, WEEK, DAY, HOUR], seed=hub, coin_seed=3) > 1
    check_diff(g, o, hops, [MONTH, WEEK], seed=hub, coin=False)
    g.close()


def test_analysis_task_lines(uniform):
    s, o, g = uniform
    hops = range_hops(T0_README + 200 * DAY, T0_README + 260 * DAY, 30 * DAY)
    a = BinaryDefusion(coin=False)
    lines = BWindowedRangeAnalysisTask([g], a, int(hops[0]), int(hops[-1]), 30 * DAY, [MONTH, WEEK]).run()
    assert len(lines) == len(hops) * 2
    res, _ = o.diffusion(int(hops[0]), [MONTH, WEEK], coin=False)
    import json
    first = json.loads(lines[0])
    assert first["size"] == len(res[0][0])


def test_diffusion_after_live_delta_seals():
    # ids first seen in later chunks shift every rank: the coins hash ids, so the device id
    # array must follow the merged graph (rgpu_seal's delta path)
    s = gen_uniform(5, 1500, 30000, dt=31_536 * 33)
    n = len(s.t)
    g = TemporalGraph(vertex_order="id")
    cuts = [0, n // 3, 2 * n // 3, n]
    for a, b in zip(cuts[:-1], cuts[1:]):
        g.ingest(s.t[a:b], s.kind[a:b], s.src[a:b], s.dst[a:b])
        g.seal()
        o = Oracle(s.t[:b], s.kind[:b], s.src[:b], s.dst[:b])
        t_end = int(s.t[b - 1])
        hops = np.array([t_end - 20 * DAY, t_end - 5 * DAY, t_end], np.int64)
        check_diff(g, o, hops, [MONTH, WEEK], coin_seed=4)
        check_diff(g, o, hops, [MONTH], coin=False)
    assert g.stats()["seal_incremental"] == 1
    g.close()
