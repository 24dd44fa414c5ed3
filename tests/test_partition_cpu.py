"""Vertex-partitioned packing on the CPU: the product's host packer built
with g++ (tests/harness.py), fed what rgpu_ingest keeps for the partition (partition_keeps:
owned vertices' updates, edge updates with an owned endpoint, every VertexDelete).  Checks,
per partition of P:
  * owned vertices are exactly Utils.getPartition(id, P) == p (Utils.scala:32-33) and ghosts
    exactly their non-owned neighbours; edges exactly those touching an owned vertex; labels
    are the ids and every rank knows its owner;
  * every owned vertex and every kept edge is alive at exactly the same (t, w) as in the
    one-partition pack (so owned histories and endpoint deaths are complete; a ghost's
    membership comes from its owner at run time);
  * the exchange plan is symmetric: partition p's send list for q equals q's receive list
    from p, entry by entry (this is what lets boundary rows travel as (index, row) records);
  * the same plan agreement across two real processes (gloo, world size 2)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from harness import load_packer_harness, pack, plist
from raphtory_amd.partition import get_partition


@pytest.fixture(scope="module")
def ph():
    return load_packer_harness()


def _stream(seed, n, nv, tie=2):
    rng = np.random.default_rng(seed)
    t = (np.arange(n) // tie).astype(np.int64) * 5
    k = rng.choice(4, size=n, p=[0.25, 0.45, 0.12, 0.18]).astype(np.uint8)
    ids = rng.choice(np.arange(10 * nv), size=nv, replace=False).astype(np.int64)  # spread over partitions
    s = ids[rng.integers(0, nv, n)]
    d = np.where(k >= 2, ids[rng.integers(0, nv, n)], -1).astype(np.int64)
    return t, k, s, d


@pytest.mark.parametrize("P", [2, 3, 5])
def test_roles_edges_and_plan(ph, P):
    t, k, s, d = _stream(P, 6000, 300)
    all_ids = np.unique(np.concatenate([s, d[k >= 2]]))
    e = k >= 2
    pairs = {(int(a), int(b)) for a, b in zip(s[e], d[e])}
    handles = [pack(ph, t, k, s, d, p, P) for p in range(P)]
    owned_union = []
    for p, h in enumerate(handles):
        vid = plist(ph, h, 0)
        n_own = ph.ph_num(h, 4)
        own, ghost = vid[:n_own], vid[n_own:]
        assert np.all(np.diff(own) > 0) and np.all(np.diff(ghost) > 0)
        assert np.array_equal(own, all_ids[get_partition(all_ids, P) == p])
        owned_union.append(own)
        own_set = set(own.tolist())
        nbrs = {b for a, b in pairs if a in own_set and a != b} | {a for a, b in pairs if b in own_set and a != b}
        assert set(ghost.tolist()) == nbrs - own_set
        # CC labels are the ids; owners per Utils.getPartition
        assert np.array_equal(plist(ph, h, 1), vid)
        assert np.array_equal(plist(ph, h, 6), get_partition(vid, P))
        kept = set(zip(plist(ph, h, 4).tolist(), plist(ph, h, 5).tolist()))
        assert kept == {(a, b) for a, b in pairs if a in own_set or b in own_set}
    assert np.array_equal(np.sort(np.concatenate(owned_union)), all_ids)
    for p in range(P):
        assert len(plist(ph, handles[p], 2, p)) == 0 and len(plist(ph, handles[p], 3, p)) == 0
        for q in range(P):
            if q != p:
                assert np.array_equal(plist(ph, handles[p], 2, q), plist(ph, handles[q], 3, p))
    for h in handles:
        ph.ph_free(h)


@pytest.mark.parametrize("P", [2, 4])
def test_partition_liveness_matches_single(ph, P):
    t, k, s, d = _stream(10 + P, 5000, 120, tie=3)
    h1 = pack(ph, t, k, s, d)
    e = k >= 2
    pairs = sorted({(int(a), int(b)) for a, b in zip(s[e], d[e])})
    times = np.unique(np.concatenate([t[::37], t[::53] + 1]))[::3]
    bad = 0
    for p in range(P):
        hp = pack(ph, t, k, s, d, p, P)
        vid = plist(ph, hp, 0)
        n_own = ph.ph_num(hp, 4)
        kept = list(zip(plist(ph, hp, 4).tolist(), plist(ph, hp, 5).tolist()))
        for tt in times.tolist():
            for w in (-1, 0, 40, 2000):
                for v in vid[:n_own].tolist():
                    bad += ph.ph_alive(hp, 0, v, -1, tt, w) != ph.ph_alive(h1, 0, v, -1, tt, w)
                for a, b in kept[:: max(1, len(kept) // 60)]:
                    bad += ph.ph_alive(hp, 1, a, b, tt, w) != ph.ph_alive(h1, 1, a, b, tt, w)
        ph.ph_free(hp)
    ph.ph_free(h1)
    assert len(pairs) > 100 and bad == 0


# ---------------------------------------------------------------- two processes (gloo)
def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = load_packer_harness()
    t, k, s, d = _stream(77, 8000, 400)  # every rank is handed the whole stream (and keeps its part)
    h = pack(L, t, k, s, d, rank, world)
    mine = {"own": plist(L, h, 0)[:L.ph_num(h, 4)].tolist(),
            "send": {p: plist(L, h, 2, p).tolist() for p in range(world)},
            "recv": {p: plist(L, h, 3, p).tolist() for p in range(world)}}
    allp = [None] * world
    dist.all_gather_object(allp, mine)
    ok = all(allp[a]["send"][b] == allp[b]["recv"][a] for a in range(world) for b in range(world) if a != b)
    owned = sorted(sum((x["own"] for x in allp), []))
    ids = np.unique(np.concatenate([s, d[k >= 2]])).tolist()
    if rank == 0:
        q.put((ok, owned == ids, sum(len(x["send"][1 - i]) for i, x in enumerate(allp))))
    dist.barrier()
    dist.destroy_process_group()


def test_partition_plan_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, cover, nsend = q.get(timeout=180)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert ok and cover and nsend > 0


@pytest.mark.parametrize("P", [2, 3])
def test_locality_order_partitions(ph, P):
    """Partitioned packs in RGPU_ORDER_LOCALITY: owned and ghost ranks each reordered, yet the same
    owned / ghost id sets, labels = ids, the same kept edges, and exchange lists that still pair
    up by id between every two partitions (entry i of p's list for q is entry i of q's list)."""
    t, k, s, d = _stream(40 + P, 6000, 300)
    ph.ph_set_locality(1)
    try:
        hl = [pack(ph, t, k, s, d, p, P) for p in range(P)]
    finally:
        ph.ph_set_locality(0)
    hi = [pack(ph, t, k, s, d, p, P) for p in range(P)]
    for p in range(P):
        a, b = hl[p], hi[p]
        assert plist(ph, a, 11).tolist() == [0]
        na = ph.ph_num(a, 4)
        assert na == ph.ph_num(b, 4)
        va, vb = plist(ph, a, 0), plist(ph, b, 0)
        assert sorted(va[:na].tolist()) == vb[:na].tolist() and sorted(va[na:].tolist()) == vb[na:].tolist()
        assert np.array_equal(plist(ph, a, 7), vb[:na])
        assert np.array_equal(plist(ph, a, 1), va)  # labels are ids
        ka = sorted(zip(plist(ph, a, 4).tolist(), plist(ph, a, 5).tolist()))
        kb = sorted(zip(plist(ph, b, 4).tolist(), plist(ph, b, 5).tolist()))
        assert ka == kb
        for q in range(P):
            assert np.array_equal(plist(ph, a, 2, q), plist(ph, b, 2, q))
            assert np.array_equal(plist(ph, a, 3, q), plist(ph, b, 3, q))
    for p in range(P):
        for q in range(P):
            if q != p:
                assert np.array_equal(plist(ph, hl[p], 2, q), plist(ph, hl[q], 3, p))
    for h in hl + hi:
        ph.ph_free(h)


def test_window_hybrid_blocks_and_superstep_recombination():
    """bench.py's N > 1 window-class hybrid (raphtory_amd/partitioned.py): the hop blocks tile the
    range, and the combined summaries carry each hop's job superstep count over all its windows —
    the maximum of the two runs' counts (rgpu.cpp finish_supersteps reports min(maxSteps, 1 + the
    last changing step over the run's windows) on every view of the hop)."""
    from raphtory_amd.partitioned import combine_window_groups, hop_blocks
    for n, world in ((168, 8), (168, 3), (5, 8), (1, 2)):
        b = hop_blocks(n, world)
        assert len(b) == world and b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] and b[i][0] <= b[i][1] for i in range(world - 1))
        assert max(hi - lo for lo, hi in b) - min(hi - lo for lo, hi in b) <= 1
    rng = np.random.default_rng(0)
    H, W, long_i, short_i = 10, 5, [0, 1, 2], [3, 4]
    full = rng.integers(0, 1000, (H, W, 9))
    last = rng.integers(0, 120, (H, W))  # a view's last changing step
    cap = 100
    run_steps = lambda idx: np.minimum(cap, 1 + last[:, idx].max(axis=1))  # noqa: E731  (finish_supersteps)
    full[..., 7] = run_steps(list(range(W)))[:, None]
    ls = full[:, long_i].copy()
    ls[..., 7] = run_steps(long_i)[:, None]
    ss = full[:, short_i].copy()
    ss[..., 7] = run_steps(short_i)[:, None]
    blocks = [(lo, hi, ss[lo:hi]) for lo, hi in hop_blocks(H, 3)]
    assert np.array_equal(combine_window_groups(W, long_i, ls, short_i, blocks), full)
