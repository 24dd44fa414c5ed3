"""Vertex-partitioned CC over RCCL, one process per partition (python -m torch.distributed.run
--nproc-per-node P tools/rccl_partition_check.py; P = 1 runs the partitioned path with a one-rank
communicator — RCCL refuses two ranks on one GPU, so that is what a one-GPU box can check).  Rank 0 compares the merged
partition results with a one-partition run of the same stream.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.partitioned import open_rccl_partition  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, DAY, T0_README, gen_uniform, range_hops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true", help="every rank on cuda:0")
    ap.add_argument("--vertices", type=int, default=2000)
    ap.add_argument("--events", type=int, default=40_000)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")  # control plane only; the data path is the library's RCCL
    s = gen_uniform(21, a.vertices, a.events, t0=T0_README, dt=31_536_000_000 // a.events)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, 3 * DAY)
    if world == 1:  # exercise the partitioned path + RCCL calls with a one-rank communicator
        os.environ["RGPU_PARTITIONED"] = "1"
    g = open_rccl_partition(dev, dist)
    os.environ.pop("RGPU_PARTITIONED", None)
    g.ingest_stream(s)
    g.seal()
    t0 = time.perf_counter()
    g.run("cc", hops, BATCH_WINDOWS, retain=True)
    ms = (time.perf_counter() - t0) * 1e3
    mine = {"summ": g.cc_summaries().tolist(),
            "labels": [[a.tolist() for a in g.cc_vertex_labels(h, w)] for h in range(0, len(hops), 17) for w in range(5)]}
    g.run("degree", hops[::9], BATCH_WINDOWS, retain=True)
    mine["deg"] = [g.degree_result(h, w)[:3] for h in range(len(hops[::9])) for w in range(5)]
    allp = [None] * world
    dist.all_gather_object(allp, mine)
    if rank == 0:
        ref = TemporalGraph(0, 1, dev)
        ref.ingest_stream(s)
        ref.seal()
        ref.run("cc", hops, BATCH_WINDOWS, retain=True)
        summ_ok = all(np.array_equal(np.asarray(p["summ"]), ref.cc_summaries()) for p in allp)
        lab_ok = True
        k = 0
        for h in range(0, len(hops), 17):
            for w in range(5):
                ids = np.concatenate([np.asarray(p["labels"][k][0], np.int64) for p in allp])
                lab = np.concatenate([np.asarray(p["labels"][k][1], np.int64) for p in allp])
                o = np.argsort(ids)
                rid, rlab = ref.cc_vertex_labels(h, w)
                lab_ok &= bool(np.array_equal(ids[o], rid) and np.array_equal(lab[o], rlab))
                k += 1
        ref.run("degree", hops[::9], BATCH_WINDOWS)
        deg_ok = True
        k = 0
        for h in range(len(hops[::9])):
            for w in range(5):
                tot = np.sum([p["deg"][k] for p in allp], axis=0)
                deg_ok &= tuple(int(x) for x in tot) == ref.degree_result(h, w)[:3]
                k += 1
        print(json.dumps({"rccl_partitioned": world, "same_device": a.same_device, "cc_summaries_equal": summ_ok,
                          "cc_labels_equal": lab_ok, "degree_totals_equal": deg_ok, "cc_ms": round(ms, 1),
                          "pass": bool(summ_ok and lab_ok and deg_ok)}), flush=True)
        ref.close()
    dist.barrier()
    g.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
