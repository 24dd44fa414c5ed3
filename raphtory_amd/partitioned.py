"""Vertex-partitioned runs: one partition per GPU, boundary label rows
exchanged every superstep (RCCL), component sizes merged across partitions.

Two ways to hold the partitions:
  * one process per GPU (torch.distributed): :func:`open_rccl_partition` gives this rank's
    TemporalGraph, joined to an RCCL communicator whose id rank 0 broadcasts;
  * :class:`LoopbackPartitions`: all P partitions in one process and on ONE device (one host
    thread each) over the library's loopback exchange — the same protocol, used to test the
    partitioned path on one GPU (its copies and kernels read peers' buffers device-locally).

Each partition may be handed the whole update stream or only its part (include/rgpu.h: it
keeps its own vertices' updates, edge updates with an owned endpoint and every VertexDelete);
runs are collective (every partition calls run with the same arguments).
"""
from __future__ import annotations

import threading
from typing import Callable, List, Sequence

import numpy as np

from .graph import TemporalGraph


def open_rccl_partition(device: int, dist=None, vertex_order: str = "locality", kind: str = "rccl") -> TemporalGraph:
    """This rank's partition (partition = rank, P = world size), joined to the RCCL group
    (kind "shm": the shared-memory group of processes on one host instead).
    vertex_order "id": later seals merge into the resident partition (live ingest)."""
    if dist is None:
        import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    g = TemporalGraph(rank, world, device, vertex_order=vertex_order)
    box = [TemporalGraph.exchange_id(kind=kind) if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    g.exchange_init(box[0])  # collective: every rank joins the communicator here
    return g


class LoopbackPartitions:
    def __init__(self, nparts: int, device: int | Sequence[int] = 0, vertex_order: str = "locality"):
        devs = [device] * nparts if isinstance(device, int) else list(device)
        if len(set(devs)) != 1:
            raise ValueError("loopback partitions share one device (use one process per GPU and RCCL "
                             "across devices: open_rccl_partition)")
        self.parts: List[TemporalGraph] = [TemporalGraph(p, nparts, devs[p], vertex_order=vertex_order)
                                           for p in range(nparts)]
        xid = TemporalGraph.exchange_id(loopback=True)
        for g in self.parts:
            g.exchange_init(xid)

    def _all(self, fn: Callable[[TemporalGraph], object]) -> list:
        out, errs = [None] * len(self.parts), []

        def body(i):
            try:
                out[i] = fn(self.parts[i])
            except BaseException as e:  # noqa: BLE001 - re-raised below
                errs.append(e)

        th = [threading.Thread(target=body, args=(i,)) for i in range(len(self.parts))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return out

    def ingest_stream(self, s) -> None:
        for g in self.parts:
            g.ingest_stream(s)

    def ingest(self, t, kind, src, dst) -> None:
        for g in self.parts:
            g.ingest(t, kind, src, dst)

    def stats(self) -> list:
        return [g.stats() for g in self.parts]

    def seal(self) -> None:
        self._all(lambda g: g.seal())

    def run(self, *a, **kw) -> None:
        self._all(lambda g: g.run(*a, **kw))

    # merged results ------------------------------------------------------------
    def cc_summary(self, hop: int, win: int):
        return self.parts[0].cc_summary(hop, win)

    def cc_vertex_labels(self, hop: int, win: int):
        ids, lab = zip(*[g.cc_vertex_labels(hop, win) for g in self.parts])
        ids, lab = np.concatenate(ids), np.concatenate(lab)
        o = np.argsort(ids, kind="stable")
        return ids[o], lab[o]

    def cc_result(self, hop: int, win: int) -> dict:
        out: dict = {}
        for g in self.parts:  # processBatchWindowResults merge (ConnectedComponents.scala:49)
            for k, v in g.cc_result(hop, win).items():
                out[k] = out.get(k, 0) + v
        return out

    def degree_vertex(self, hop: int, win: int):
        cols = list(zip(*[g.degree_vertex(hop, win) for g in self.parts]))
        ids, od, idg = (np.concatenate(c) for c in cols)
        o = np.argsort(ids, kind="stable")
        return ids[o], od[o], idg[o]

    def degree_totals(self, hop: int, win: int):
        tot = np.zeros(3, np.int64)
        for g in self.parts:  # DegreeBasic.processWindowResults sums shard tuples (:35-36)
            tot += np.asarray(g.degree_result(hop, win)[:3])
        return tuple(int(x) for x in tot)

    def pr_result(self, hop: int, win: int):
        ids, pr = zip(*[g.pr_result(hop, win) for g in self.parts])
        ids, pr = np.concatenate(ids), np.concatenate(pr)
        o = np.argsort(ids, kind="stable")
        return ids[o], pr[o]

    # vertex programs (VertexVisitor messaging across partitions) ---------------------
    def set_vertex_program(self, **kw) -> None:
        for g in self.parts:
            g.set_vertex_program(**kw)

    def set_vertex_program_f(self, **kw) -> None:
        for g in self.parts:
            g.set_vertex_program_f(**kw)

    def _merged(self, fn, hop, win):
        ids, val = zip(*[fn(g, hop, win) for g in self.parts])
        ids, val = np.concatenate(ids), np.concatenate(val)
        o = np.argsort(ids, kind="stable")
        return ids[o], val[o]

    def vp_result(self, hop: int, win: int):
        return self._merged(lambda g, h, w: g.vp_result(h, w), hop, win)

    def vp_result_f(self, hop: int, win: int):
        return self._merged(lambda g, h, w: g.vp_result_f(h, w), hop, win)

    def vp_supersteps(self, hop: int) -> int:
        steps = {g.vp_supersteps(hop) for g in self.parts}
        assert len(steps) == 1, steps  # the job's superstep count is global
        return steps.pop()

    def close(self) -> None:
        for g in self.parts:
            g.close()


# ---------------------------------------------------------------- window-class hybrid (N > 1, C4)
# The short windows of a batched-window range query read only a recent time slice of the stream: on
# an add-only stream a view (t, w) depends only on the updates in [t - w, t] (aliveAtWithWindow,
# Entity.scala:173-201; tools/make_c4_sliced_goldens.py states the argument, tests/test_c4_slice.py
# checks it).  Partitioned, those windows do not scale (their batches are a few milliseconds of
# per-superstep floors on every partition), so with N ranks each rank answers them for
# its own contiguous block of the hops on a replica of that slice — no exchange — while the
# partitions answer the long windows.  Descending windows keep the batched lens exact under the split
# (each window's vertex set is the running minimum of the windows before it, i.e. its own, as
# WindowLens.shrinkWindow gives for {y, m, w, d, h}); the hop's superstep count is recombined below.

def hop_blocks(n_hops: int, world: int) -> list:
    """Rank r's contiguous block [lo, hi) of the hops."""
    return [(r * n_hops // world, (r + 1) * n_hops // world) for r in range(world)]


def combine_window_groups(n_windows: int, long_idx, long_summ: np.ndarray, short_idx, short_blocks) -> np.ndarray:
    """The query's [n_hops, n_windows, 9] cc_summaries from the partitions' long-window summaries
    and each rank's short-window block ((lo, hi, summaries) per rank).  Field 7 (supersteps) is the
    hop's job count over the windows of one run — min(maxSteps, 1 + the last changing step over
    them), rgpu.cpp finish_supersteps — so the hop's count over all its windows is the maximum of
    the two runs' counts (min and max commute with the monotone 1 + x)."""
    short_idx = list(short_idx)
    full = np.zeros((long_summ.shape[0], n_windows) + long_summ.shape[2:], long_summ.dtype)
    full[:, list(long_idx)] = long_summ
    for lo, hi, x in short_blocks:
        if hi > lo:
            full[lo:hi, short_idx] = x
    full[..., 7] = full[..., 7].max(axis=1, keepdims=True)
    return full
