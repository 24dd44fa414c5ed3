"""Debug: live-merged vs one-shot labels under RGPU_TSLOTS / RGPU_UW / RGPU_HEAVY."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_tail import graph_env
from raphtory_amd import TemporalGraph
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab

users, nb, nt = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
base = gen_gab(4, users, nb)
now = int(base.t[-1])
tick = gen_gab(100, users, nt, t0=now + 1, t1=now + HOUR, id_key=4)
now = int(tick.t[-1])
combos = [dict(kv.split("=") for kv in c.split(",")) for c in sys.argv[4:]]
for env in combos:
    live = graph_env(base, env)
    live.ingest_stream(tick)
    live.seal()
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    one = TemporalGraph()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    one.ingest_stream(base)
    one.ingest_stream(tick)
    one.seal()
    bad = []
    for g in (live, one):
        g.run("cc", [now], BATCH_WINDOWS, retain=True)
    for w in range(5):
        ia, la = live.cc_vertex_labels(0, w)
        ib, lb = one.cc_vertex_labels(0, w)
        if not (np.array_equal(ia, ib) and np.array_equal(la, lb)):
            bad.append((w, int((la != lb).sum()) if len(la) == len(lb) else ("len", len(ia), len(ib))))
    sa, sb = live.stats(), one.stats()
    print({k: (sa[k], sb[k]) for k in ("vertices", "edges", "vertex_events", "edge_events", "deaths")})
    print(env, "seal_incremental", live.stats()["seal_incremental"], "bad", bad, flush=True)
    live.close(); one.close()
