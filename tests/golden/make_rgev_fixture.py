"""Writes tests/golden/rgev_v1_small.{rgev,json}: a hand-written update list with its RGEV
encoding (block size 4, so the fixture holds several blocks, one of them split by a time
span past 2^32 - 1 ms).  The bytes are produced by the numpy restatement of the layout in
tests/test_rgev.py (not by the library), so the fixture pins the format itself."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.test_rgev import FIXTURE_UPDATES, np_encode  # noqa: E402

if __name__ == "__main__":
    t, k, s, d = (list(c) for c in zip(*FIXTURE_UPDATES))
    raw = np_encode(t, k, s, d, block=4)
    open(os.path.join(HERE, "rgev_v1_small.rgev"), "wb").write(raw)
    json.dump({"t": t, "kind": k, "src": s, "dst": [x if kk >= 2 else -1 for x, kk in zip(d, k)],
               "block": 4, "bytes": len(raw)}, open(os.path.join(HERE, "rgev_v1_small.json"), "w"), indent=1)
    print(len(raw), "bytes")
