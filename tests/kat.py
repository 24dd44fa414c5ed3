"""Loader for the hand-derived known-answer fixtures (tests/golden/kat_semantics.json)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases():
    with open(os.path.join(GOLDEN, "kat_semantics.json")) as f:
        return json.load(f)["cases"]


def arrays(case):
    ev = np.asarray(case["events"], dtype=np.int64).reshape(-1, 4)
    return ev[:, 0].copy(), ev[:, 1].astype(np.uint8), ev[:, 2].copy(), ev[:, 3].copy()


def cc_expect(m):
    return {int(k): int(v) for k, v in m.items()}
