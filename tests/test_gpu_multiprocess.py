"""The partitioned superstep protocol across PROCESSES (AnalysisTask.scala:208-283's
cross-PM barrier): two processes, one partition each (P = 2), sharing the one GPU of the box and
exchanging through the shared-memory group (include/rgpu.h RGPU_XCHG_SHM) — the same host
protocol as RCCL: three batch slots on forked channels served in a fixed round robin, the
per-superstep counts all-to-all carrying the halting vote, host-sized receive regions, the
broadcast label records, routed component counts and the summaries' all-reduce.  The processes
are started with subprocess before they touch the GPU; each writes its own vertices' labels,
which are merged here and compared bit-exactly with the CPU oracle on the whole stream
(ConnectedComponents.scala:10-42,137-145), on a GAB stream and on star hubs cut into segments,
with the record buffers forced to start tiny (every growth path runs)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import Oracle, label_counts
from raphtory_amd import TemporalGraph
from raphtory_amd.analysis import cc_fields

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("biggest", "total", "totalWithoutIslands", "totalIslands", "clustersGT2")  # summary row order


@pytest.mark.parametrize("name", ["gab", "hubs"])
def test_two_process_partitions_vs_oracle(name, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from mp_partition_worker import stream_and_query
    s, hops, windows = stream_and_query(name)
    world = 2
    xid = TemporalGraph.exchange_id(kind="shm").hex()  # (no device call)
    env = dict(os.environ, RGPU_XREC_TINY="1", RGPU_HEAVY="300", RGPU_CHECK="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_partition_worker.py"), str(r), str(world),
                               xid, name, str(tmp_path)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r}:\n{outs[r][-3000:]}"
    res = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    assert np.array_equal(res[0]["summ"], res[1]["summ"])  # both hold the merged summaries
    assert all(float(x["xchg"]) > 0 for x in res)  # the processes really exchanged
    o = Oracle.from_stream(s)
    for h, t in enumerate(np.asarray(hops).tolist()):
        exp, steps = o.cc(t, windows, mode=1)
        for w in range(len(windows)):
            ids = np.concatenate([x[f"ids_{h}_{w}"] for x in res])
            lab = np.concatenate([x[f"lab_{h}_{w}"] for x in res])
            k = np.argsort(ids, kind="stable")
            eids, elab = exp[w]
            assert np.array_equal(ids[k], eids) and np.array_equal(lab[k], elab), (name, t, w)
            summ = res[0]["summ"][h, w]
            assert int(summ[7]) == steps, (name, t, w)
            f = cc_fields(label_counts(elab))
            if f is None:  # empty view ("No activity")
                assert int(summ[1]) == 0, (name, t, w)
                continue
            for i, key in enumerate(FIELDS):
                assert int(summ[i]) == f[key], (name, t, w, key)
