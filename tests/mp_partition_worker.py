"""TEST INFRASTRUCTURE: one partition of a multi-process partitioned run (tests/test_gpu_multiprocess.py).

Started as its own process (subprocess, before it touches the GPU): opens partition `rank` of
`world` on device 0, joins the shared-memory exchange group named by the id blob on the command
line (include/rgpu.h RGPU_XCHG_SHM), ingests the whole stream (each partition keeps its part),
seals, runs the CC query and writes its own vertices' labels and the merged summaries to
<out>/rank<r>.npz.

usage: python tests/mp_partition_worker.py <rank> <world> <xid hex> <stream> <out dir>
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stream_and_query(name):
    from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, MONTH, T0_README, WEEK, gen_gab, range_hops
    if name == "hubs":
        from tests.test_gpu_heavy import hubs_stream
        return hubs_stream(), range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, DAY), [MONTH, WEEK, DAY]
    s = gen_gab(4, 3000, 6000)
    end = int(s.t[-1])
    return s, range_hops(end - 72 * HOUR, end, 2 * HOUR), BATCH_WINDOWS


def main():
    rank, world, xid, name, out = int(sys.argv[1]), int(sys.argv[2]), bytes.fromhex(sys.argv[3]), sys.argv[4], sys.argv[5]
    from raphtory_amd import TemporalGraph
    s, hops, windows = stream_and_query(name)
    g = TemporalGraph(rank, world, 0)
    g.exchange_init(xid)  # collective: every process joins here
    g.ingest_stream(s)
    g.seal()
    g.run("cc", hops, windows, retain=True)
    res = {}
    for h in range(len(hops)):
        for w in range(len(windows)):
            ids, lab = g.cc_vertex_labels(h, w)
            res[f"ids_{h}_{w}"] = ids
            res[f"lab_{h}_{w}"] = lab
    st = g.stats()
    np.savez(os.path.join(out, f"rank{rank}.npz"), summ=g.cc_summaries(), xchg=np.float64(st["xchg_bytes"]),
             vertices=np.int64(st["vertices"]), **res)
    g.close()


if __name__ == "__main__":
    main()
