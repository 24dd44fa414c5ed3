"""Seeded synthetic spouts: chunked / partition-filtered C4 generation
equals the whole stream (no GPU)."""
import numpy as np

from raphtory_amd.partition import get_partition
from raphtory_amd.synth import gen_gab, gen_gab_range


def test_gab_chunks_concatenate_to_the_stream():
    whole = gen_gab(4, 2000, 9000)
    parts = [gen_gab_range(4, 2000, 9000, a, 2500) for a in range(0, 9000, 2500)]
    for f in ("t", "kind", "src", "dst"):
        assert np.array_equal(getattr(whole, f), np.concatenate([getattr(p, f) for p in parts])), f


def test_gab_partition_filter_keeps_exactly_the_owned_updates():
    whole = gen_gab(4, 2000, 6000)
    for P in (2, 5):
        for p in range(P):
            got = gen_gab_range(4, 2000, 6000, 0, 6000, p, P)
            own_s = np.array([get_partition(int(x), P) == p for x in whole.src])
            own_d = np.array([d >= 0 and get_partition(int(d), P) == p for d in whole.dst])
            keep = np.where(whole.kind == 0, own_s, own_s | own_d)
            for f in ("t", "kind", "src", "dst"):
                assert np.array_equal(getattr(got, f), getattr(whole, f)[keep]), (P, p, f)
