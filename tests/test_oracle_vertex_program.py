"""The oracle's generic vertex program (oracle.h orc_vertex_program: VertexVisitor messaging through
the reference's BSP structure) against independent restatements: with the CC program it is
ConnectedComponents (orc_cc, labels and superstep counts), and the hop-distance program is a
breadth-first search over the view's alive edges among its members, written here from the
liveness rule alone (o.alive = Entity.aliveAtWithWindow).  No GPU."""
from collections import deque

import numpy as np
import pytest

from oracle import Oracle
from raphtory_amd.synth import BATCH_WINDOWS, DAY, MONTH, T0_README, WEEK, YEAR, gen_uniform

INF = 2**63 - 1


@pytest.fixture(scope="module")
def world():
    s = gen_uniform(31, 120, 3000, t0=T0_README, dt=10_512_000)
    return s, Oracle.from_stream(s)


def test_cc_program_is_connected_components(world):
    s, o = world
    for t in (T0_README + 60 * DAY, T0_README + 200 * DAY, T0_README + 364 * DAY):
        for wins, cap in ((BATCH_WINDOWS, 100), ([], 100), ([MONTH, WEEK], 2)):
            a, sa = o.cc(t, wins, max_steps=cap)
            b, sb = o.vertex_program(t, wins, max_steps=cap, direction="all", reduce="min", init="id")
            assert sa == sb
            for (i1, l1), (i2, l2) in zip(a, b):
                assert np.array_equal(i1, i2) and np.array_equal(l1, l2)


def _bfs(s, o, t, w, seed, direction, cap):
    ids = np.unique(np.concatenate([s.src, s.dst[s.kind >= 2]]))
    members = {int(v) for v in ids if o.alive(False, int(v), -1, t, w)}
    pairs = {(int(a), int(b)) for a, b, k in zip(s.src, s.dst, s.kind) if k >= 2}
    adj = {v: set() for v in members}
    for a, b in pairs:
        if a in members and b in members and o.alive(True, a, b, t, w):
            if direction in ("out", "all"):
                adj[a].add(b)
            if direction in ("in", "all") and a != b:
                adj[b].add(a)
    dist = {v: INF for v in members}
    if seed not in members:
        return dist, 1
    dist[seed] = 0
    q = deque([seed])
    while q:
        u = q.popleft()
        for x in adj[u]:
            if dist[x] == INF:
                dist[x] = dist[u] + 1
                q.append(x)
    far = max(d for d in dist.values() if d != INF)
    # distance d is set at superstep d; with the cap only d <= cap are reached
    for v in dist:
        if dist[v] != INF and dist[v] > cap:
            dist[v] = INF
    return dist, min(cap, far + 1)


@pytest.mark.parametrize("direction", ["out", "in", "all"])
def test_hop_distance_program_is_bfs(world, direction):
    s, o = world
    seed = int(s.src[500])
    for t in (T0_README + 150 * DAY, T0_README + 364 * DAY):
        for w in (YEAR, MONTH):
            for cap in (100, 3):
                res, steps = o.vertex_program(t, [w], max_steps=cap, direction=direction, reduce="min", init="const",
                                              senders="seed", init_value=INF, seed_id=seed, seed_value=0, step_add=1)
                ids, vals = res[0]
                dist, esteps = _bfs(s, o, t, w, seed, direction, cap)
                assert dict(zip(ids.tolist(), vals.tolist())) == dist, (t, w, cap)
                assert steps == esteps, (t, w, cap, steps, esteps)


def _float_program(s, o, t, w, direction, per_degree, cap, bias, mult, senders_seed=None):
    """VertexMessageFloat summed (include/rgpu.h rgpu_vertex_program_f_t), restated here from the
    liveness rule alone: message targets = distinct neighbours in `direction` over edges alive in
    the view (members or not; only members process theirs), sums in double"""
    ids = np.unique(np.concatenate([s.src, s.dst[s.kind >= 2]]))
    members = {int(v) for v in ids if o.alive(False, int(v), -1, t, w)}
    pairs = {(int(a), int(b)) for a, b, k in zip(s.src, s.dst, s.kind) if k >= 2}
    tg = {v: set() for v in members}
    for a, b in pairs:
        if o.alive(True, a, b, t, w):
            if direction == "out" and a in members:
                tg[a].add(b)
            if direction == "in" and b in members and a != b:
                tg[b].add(a)
    f32 = lambda x: float(np.float32(x))  # noqa: E731
    st = {v: f32(v) for v in members}
    send = set(members) if senders_seed is None else ({senders_seed} & members)

    def msgs(frm):
        q = {}
        for u in frm:
            x = f32(st[u] / max(len(tg[u]), 1)) if per_degree else st[u]
            for v in tg[u]:
                if v in members:
                    q[v] = q.get(v, 0.0) + x
        return q
    q = msgs(send)
    steps = 0
    for r in range(1, cap + 1):
        steps = r
        for v, x in q.items():
            st[v] = f32(bias + mult * x)
        if not q or r == cap:
            break
        q = msgs(set(q))
    return st, steps


@pytest.mark.parametrize("direction,per_degree", [("out", True), ("in", False), ("out", False)])
def test_float_program_matches_restatement(world, direction, per_degree):
    s, o = world
    seed = int(s.src[700])
    for t in (T0_README + 150 * DAY, T0_README + 364 * DAY):
        for w in (YEAR, MONTH):
            for cap, seeded in ((20, False), (4, True)):
                res, steps = o.vertex_program_f(t, [w], max_steps=cap, direction=direction, per_degree=per_degree,
                                                senders="seed" if seeded else "all", seed_id=seed if seeded else -1,
                                                bias=0.15, mult=0.85)
                ids, vals = res[0]
                st, esteps = _float_program(s, o, t, w, direction, per_degree, cap, 0.15, 0.85, seed if seeded else None)
                assert steps == esteps, (t, w, cap)
                assert ids.tolist() == sorted(st)
                exp = np.array([st[v] for v in ids.tolist()])
                assert np.all(np.abs(vals - exp) <= 1e-6 * np.maximum(1.0, np.abs(exp))), (t, w, cap)
                assert np.all(vals == vals.astype(np.float32).astype(np.float64))  # float32 values
