"""World-size-2 gloo run of the replica logic bench.py uses (CPU, no GPU): hop grids of the
ranks are disjoint, interleave into the finer grid, and the timing reduction is a max."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from raphtory_amd.replicas import max_over_ranks, replica_hops
from raphtory_amd.synth import HOUR, range_hops


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base = range_hops(0, 100 * HOUR, HOUR)
    mine = replica_hops(base, HOUR, rank, world)
    import torch
    t = torch.from_numpy(mine)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    m = max_over_ranks(float(rank) * 1.5 + 1.0, dist)
    if rank == 0:
        q.put((np.concatenate([o.numpy() for o in out]), m))
    dist.barrier()
    dist.destroy_process_group()


def test_replica_hops_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    allhops, m = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert m == 2.5
    assert len(np.unique(allhops)) == len(allhops)  # disjoint
    fine = np.sort(allhops)
    assert np.all(np.diff(fine)[:-2] == HOUR // 2)  # interleaved half-hour grid (last hop clamps)
