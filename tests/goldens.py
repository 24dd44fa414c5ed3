"""TEST INFRASTRUCTURE: helpers shared by the golden-fixture generators (tools/make_*_goldens.py)
and the GPU tests that read the fixtures."""
import numpy as np


def label_checksum(ids, labels) -> str:
    """Order-independent checksum of a view's (id, label) pairs: the sum over members of
    splitmix64(id * 2^32 + label) mod 2^64, as 16 hex digits."""
    x = (np.asarray(ids, np.int64).astype(np.uint64) << np.uint64(32)) + np.asarray(labels, np.int64).astype(np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        return format(int(np.sum(x, dtype=np.uint64)), "016x")
