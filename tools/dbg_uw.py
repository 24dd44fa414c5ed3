"""Debug: summaries with and without the uniform-word count path on the hub stream."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_heavy import hubs_stream
from tests.test_gpu_tail import graph_env
from raphtory_amd.synth import BATCH_WINDOWS, DAY, MONTH, WEEK, T0_README, range_hops

st = hubs_stream()
hops = range_hops(T0_README + 5 * DAY, T0_README + 70 * DAY, 3 * DAY)
for name, hh, wins, ms in (("mwd", hops, [MONTH, WEEK, DAY], 100), ("viewlens", hops[:6], [], 100),
                           ("week2", hops[:6], [WEEK], 2)):
    for retain in (False, True):
        out = {}
        for uw in ("1", "0"):
            g = graph_env(st, {"RGPU_HEAVY": "0", "RGPU_UW": uw})
            g.run("cc", hh, wins, max_steps=ms, retain=retain)
            out[uw] = g.cc_summaries()
            g.close()
        a, b = out["1"], out["0"]
        bad = np.argwhere(np.any(a[..., :7] != b[..., :7], axis=-1))
        print(name, "retain", retain, "views", a.shape, "differing", len(bad))
        for h, w in bad[:4]:
            print("  ", h, w, a[h, w, :8].tolist(), b[h, w, :8].tolist())
