"""Generic vertex programs on the GPU (rgpu_set_vertex_program, vp.hip):
the VertexVisitor messaging surface (messageAllOutgoingNeighbors / messageAllIngoingNeighbors /
messageAllNeighbours, VertexVisitor.scala:81-166) with a min / max fold of the message queue,
against the oracle's run of the same program through the reference's BSP structure
(oracle.h orc_vertex_program): every member's state and the hop's superstep count, bit-exact.
The CC program must also give ConnectedComponents' labels (orc_cc)."""
import numpy as np
import pytest

from oracle import Oracle
from raphtory_amd import TemporalGraph
from raphtory_amd.synth import BATCH_WINDOWS, DAY, MONTH, T0_README, WEEK, YEAR, gen_gab, gen_powerlaw, gen_uniform, \
    range_hops

pytestmark = pytest.mark.gpu
INF = 2**63 - 1

PROGRAMS = {
    "cc": dict(direction="all", reduce="min", init="id"),
    "max_id_out": dict(direction="out", reduce="max", init="id"),
    "min_id_in": dict(direction="in", reduce="min", init="id"),
    "hops_out": dict(direction="out", reduce="min", init="const", senders="seed", init_value=INF, seed_value=0,
                     step_add=1),
    "hops_in": dict(direction="in", reduce="min", init="const", senders="seed", init_value=INF, seed_value=0,
                    step_add=1),
    "hops_all_capped": dict(direction="all", reduce="min", init="const", senders="seed", init_value=INF,
                            seed_value=0, step_add=1),
}


def _oracle_kw(p):
    k = dict(p)
    k["init"] = "id" if k.get("init", "id") == "id" else "const"
    return k


def check(g, o, hops, windows, prog, max_steps=100):
    g.set_vertex_program(**{k: v for k, v in prog.items()})
    g.run("vp", hops, windows, max_steps=max_steps, retain=True)
    for h, t in enumerate(np.asarray(hops).tolist()):
        res, steps = o.vertex_program(t, windows, max_steps=max_steps, **_oracle_kw(prog))
        assert g.vp_supersteps(h) == steps, (t, g.vp_supersteps(h), steps)
        for w in range(max(1, len(windows))):
            ids, vals = res[w]
            gids, gvals = g.vp_result(h, w)
            assert np.array_equal(gids, ids), (t, w)
            assert np.array_equal(gvals, vals), (t, w, int((gvals != vals).sum()))


@pytest.mark.parametrize("name", sorted(PROGRAMS))
def test_vertex_programs_uniform(name):
    s = gen_uniform(21, 400, 12_000, t0=T0_README, dt=2_628_000)
    o = Oracle.from_stream(s)
    prog = dict(PROGRAMS[name])
    if prog.get("senders") == "seed":
        prog["seed_id"] = int(s.src[len(s) // 3])
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 5 * DAY)
    with TemporalGraph() as g:
        g.ingest_stream(s)
        g.seal()
        check(g, o, hops, BATCH_WINDOWS, prog, max_steps=4 if name.endswith("capped") else 100)
        check(g, o, hops[:6], [], prog)  # ViewLens
        check(g, o, hops[::9], [WEEK, YEAR], prog, max_steps=1)  # no setup: the initial states


def test_cc_program_equals_connected_components():
    s = gen_powerlaw(22, 2000, 40_000, t0=0, t1=YEAR)
    o = Oracle.from_stream(s)
    hops = range_hops(YEAR // 2, YEAR, 10 * DAY)
    with TemporalGraph() as g:
        g.ingest_stream(s)
        g.seal()
        g.set_vertex_program(direction="all", reduce="min", init="id")
        g.run("vp", hops, [MONTH, WEEK], retain=True)
        for h, t in enumerate(hops.tolist()):
            res, steps = o.cc(t, [MONTH, WEEK])
            assert g.vp_supersteps(h) == steps
            for w in range(2):
                gids, gv = g.vp_result(h, w)
                assert np.array_equal(gids, res[w][0]) and np.array_equal(gv, res[w][1]), (t, w)


def test_vertex_program_gab_hubs_and_vertex_order():
    s = gen_gab(23, 3000, 30_000)
    o = Oracle.from_stream(s)
    end = int(s.t[-1])
    hops = range_hops(end - 40 * DAY, end, 2 * DAY)
    prog = dict(PROGRAMS["hops_out"], seed_id=int(s.src[0]))
    for order in ("locality", "id"):
        with TemporalGraph(vertex_order=order) as g:
            g.ingest_stream(s)
            g.seal()
            check(g, o, hops, [YEAR, MONTH], prog)
            check(g, o, hops, [YEAR, MONTH], PROGRAMS["max_id_out"])


def test_hop_distance_analyser_task_lines():
    """the host mirror (analysis.HopDistance through BWindowedRangeAnalysisTask) prints the states
    of the reached members, equal to the oracle's"""
    import json

    from raphtory_amd.analysis import BWindowedRangeAnalysisTask, HopDistance
    s = gen_uniform(24, 300, 8000, t0=T0_README, dt=3_942_000)
    o = Oracle.from_stream(s)
    seed = int(s.src[2000])
    with TemporalGraph() as g:
        g.ingest_stream(s)
        g.seal()
        a = HopDistance(seed_id=seed)
        task = BWindowedRangeAnalysisTask([g], a, T0_README + 100 * DAY, T0_README + 300 * DAY, 25 * DAY, [YEAR, MONTH])
        lines = [json.loads(x) for x in task.run()]
        k = 0
        for t in task.hops().tolist():
            res, _ = o.vertex_program(t, [YEAR, MONTH], direction="out", reduce="min", init="value", senders="seed",
                                      init_value=INF, seed_id=seed, seed_value=0, step_add=1)
            for w, (ids, vals) in zip([YEAR, MONTH], res):
                exp = sorted((int(i), int(v)) for i, v in zip(ids, vals) if v != INF)
                assert lines[k]["time"] == t and lines[k]["windowsize"] == w
                assert [tuple(x) for x in lines[k]["states"]] == exp
                k += 1


FLOAT_PROGRAMS = {
    "pagerank_shape": dict(direction="out", per_degree=True, bias=0.15, mult=0.85, init="const", init_value=1.0),
    "in_sum": dict(direction="in", per_degree=False, bias=0.0, mult=0.5),
    "seed_out": dict(direction="out", per_degree=True, bias=0.0, mult=1.0, senders="seed", init="const",
                     init_value=0.0, seed_value=1000.0),
}


@pytest.mark.parametrize("name", sorted(FLOAT_PROGRAMS))
@pytest.mark.parametrize("stream", ["uniform", "gab"])
def test_float_vertex_programs(name, stream):
    """VertexMessageFloat summed (rgpu_set_vertex_program_f, ABI 10) against the oracle's
    orc_vertex_program_f: every member's float state within float32 rounding (rgpu.h: the sum is
    double in both, in slot order on the GPU and arrival order in the oracle), float32 values, and
    the hop's superstep count exactly; power-law hubs (segments do not apply: the program walks its
    own slots) and window-major batches of many hops."""
    if stream == "uniform":
        s = gen_uniform(23, 500, 15_000, t0=T0_README, dt=2_102_400)
        hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 4 * DAY)
    else:
        s = gen_gab(8, 4000, 12_000)
        end = int(s.t[-1])
        hops = range_hops(end - 90 * DAY, end, 2 * DAY)
    o = Oracle.from_stream(s)
    prog = dict(FLOAT_PROGRAMS[name])
    if prog.get("senders") == "seed":
        prog["seed_id"] = int(s.src[len(s) // 2])
    with TemporalGraph() as g:
        g.ingest_stream(s)
        g.seal()
        g.set_vertex_program_f(**prog)
        g.run("vp", hops, BATCH_WINDOWS, max_steps=12, retain=True)
        okw = dict(prog)
        okw["init"] = "id" if okw.get("init", "id") == "id" else "const"
        for h, t in enumerate(np.asarray(hops).tolist()[::3]):
            res, steps = o.vertex_program_f(t, BATCH_WINDOWS, max_steps=12, **okw)
            assert g.vp_supersteps(h * 3) == steps, (t, g.vp_supersteps(h * 3), steps)
            for w in range(5):
                ids, vals = res[w]
                gids, gvals = g.vp_result_f(h * 3, w)
                assert np.array_equal(gids, ids), (t, w)
                assert np.all(gvals == gvals.astype(np.float32).astype(np.float64))
                bad = np.abs(gvals - vals) > 1e-6 * np.maximum(1.0, np.abs(vals))
                assert not bad.any(), (t, w, int(bad.sum()), gvals[bad][:4], vals[bad][:4])
        # the result calls follow the kind of the program the retained run ran, not the one set
        # since: an int program set after the float run changes neither
        keep = g.vp_result_f(0, 0)
        g.set_vertex_program(reduce="min")
        again = g.vp_result_f(0, 0)
        assert np.array_equal(keep[0], again[0]) and np.array_equal(keep[1], again[1])
        with pytest.raises(Exception):
            g.vp_result(0, 0)


@pytest.mark.parametrize("P", [2, 3])
def test_vertex_programs_partitioned(P):
    """Vertex programs across loopback partitions (run_partitioned_vp: boundary records of state rows
    and change words after setup and every superstep, the global vote by all-reduce): the min / max
    int64 programs bit-exact against the oracle (states and the hop's superstep count), a seeded
    program whose seed is owned by one partition only, and a per_degree float program (degree rows
    of ghosts from their owners) within the float32 bound."""
    from raphtory_amd.partitioned import LoopbackPartitions
    s = gen_uniform(29, 500, 14_000, t0=T0_README, dt=2_252_571)
    o = Oracle.from_stream(s)
    hops = range_hops(T0_README + 40 * DAY, T0_README + 360 * DAY, 9 * DAY)
    lp = LoopbackPartitions(P)
    lp.ingest_stream(s)
    lp.seal()
    seed = int(s.src[len(s) // 3])
    for name in ("cc", "max_id_out", "hops_in", "hops_all_capped"):
        prog = dict(PROGRAMS[name])
        if prog.get("senders") == "seed":
            prog["seed_id"] = seed
        cap = 4 if name == "hops_all_capped" else 100
        lp.set_vertex_program(**prog)
        lp.run("vp", hops, BATCH_WINDOWS, max_steps=cap, retain=True)
        for h, t in enumerate(np.asarray(hops).tolist()[::4]):
            res, steps = o.vertex_program(t, BATCH_WINDOWS, max_steps=cap, **_oracle_kw(prog))
            assert lp.vp_supersteps(h * 4) == steps, (name, t)
            for w in range(5):
                gids, gvals = lp.vp_result(h * 4, w)
                assert np.array_equal(gids, res[w][0]) and np.array_equal(gvals, res[w][1]), (name, t, w)
    prog = dict(FLOAT_PROGRAMS["pagerank_shape"])
    lp.set_vertex_program_f(**prog)
    lp.run("vp", hops, BATCH_WINDOWS, max_steps=8, retain=True)
    okw = dict(prog)
    okw["init"] = "const"
    for h, t in enumerate(np.asarray(hops).tolist()[::5]):
        res, steps = o.vertex_program_f(t, BATCH_WINDOWS, max_steps=8, **okw)
        assert lp.vp_supersteps(h * 5) == steps
        for w in range(5):
            gids, gvals = lp.vp_result_f(h * 5, w)
            assert np.array_equal(gids, res[w][0])
            assert np.all(np.abs(gvals - res[w][1]) <= 1e-6 * np.maximum(1.0, np.abs(res[w][1]))), (t, w)
    lp.close()
