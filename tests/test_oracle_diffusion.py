"""Oracle BinaryDefusion (BinaryDefusion.scala:9-51) against closed forms (CPU, no GPU).

The reference's coin (Random.nextBoolean, :17/:32) is unseeded, so no reference run is
reproducible: the coin here is the hash of include/rgpu.h, restated independently below in
Python, and coin=False gives the deterministic taint form whose answer is the directed
BFS depth from infectedNode inside the view ("parity unpinned" against reference runs, as
for the rest of the oracle; the closed forms pin the BSP structure)."""
import numpy as np

from oracle import Oracle

M64 = (1 << 64) - 1


def mix(x):
    x &= M64
    x ^= x >> 30
    x = (x * 0xbf58476d1ce4e5b9) & M64
    x ^= x >> 27
    x = (x * 0x94d049bb133111eb) & M64
    x ^= x >> 31
    return x


def heads(coin_seed, t, w, u, v, r):
    salt = mix(coin_seed ^ mix((t & M64) ^ mix(w & M64)))
    a = mix((v + r) & M64)
    b = mix(((u * 0x9E3779B97F4A7C15) & M64) ^ a)
    return (mix(salt ^ b) >> 63) == 1


def stream(events):
    t = np.array([e[0] for e in events], np.int64)
    k = np.array([e[1] for e in events], np.uint8)
    s = np.array([e[2] for e in events], np.int64)
    d = np.array([e[3] if len(e) > 3 else -1 for e in events], np.int64)
    return t, k, s, d


VADD, VDEL, EADD, EDEL = 0, 1, 2, 3


def test_taint_is_directed_bfs_depth():
    ev = [(1, EADD, 31, 1), (1, EADD, 1, 2), (1, EADD, 2, 3), (1, EADD, 4, 31), (1, EADD, 31, 3),
          (2, EADD, 3, 5), (3, VADD, 6)]
    o = Oracle(*stream(ev))
    res, steps = o.diffusion(10, [], coin=False)
    ids, st = res[0]
    assert dict(zip(ids.tolist(), st.tolist())) == {31: 0, 1: 1, 3: 1, 2: 2, 5: 2}
    # step 1 infects {1, 3}; step 2 infects {2, 5}; step 3: 2 messages 3 (already infected): halt
    assert steps == 3


def test_taint_respects_windows_and_deaths():
    # 31->1 at t=1, 1->2 at t=50; vertex 1 deleted at t=60 (kills its edges)
    ev = [(1, EADD, 31, 1), (50, EADD, 1, 2), (60, VDEL, 1)]
    o = Oracle(*stream(ev))
    res, _ = o.diffusion(55, [100, 10], coin=False)
    assert dict(zip(*[a.tolist() for a in res[0]])) == {31: 0, 1: 1, 2: 2}
    assert dict(zip(*[a.tolist() for a in res[1]])) == {}  # 31 and 1 are outside the 10 ms window
    res, _ = o.diffusion(70, [], coin=False)
    assert dict(zip(*[a.tolist() for a in res[0]])) == {31: 0}  # 1 is dead at 70


def test_superstep_cap_and_no_setup():
    n = 150
    ev = [(1, EADD, 31 if i == 0 else 1000 + i, 1000 + i + 1) for i in range(n)]
    o = Oracle(*stream(ev))
    res, steps = o.diffusion(5, [], coin=False)
    got = dict(zip(*[a.tolist() for a in res[0]]))
    assert steps == 100 and len(got) == 101 and max(got.values()) == 100
    res, steps = o.diffusion(5, [], max_steps=1, coin=False)  # no Setup when maxSteps <= 1
    assert len(res[0][0]) == 0
    res, steps = o.diffusion(5, [], seed_id=7, coin=False)  # infectedNode absent
    assert len(res[0][0]) == 0 and steps == 1


def test_hash_coin_matches_spec_on_a_star():
    leaves = list(range(100, 1100))
    ev = [(1, EADD, 31, v) for v in leaves]
    o = Oracle(*stream(ev))
    for cs in (0, 12345):
        res, steps = o.diffusion(9, [8], coin_seed=cs)
        got = set(res[0][0].tolist()) - {31}
        exp = {v for v in leaves if heads(cs, 9, 8, 31, v, 0)}
        assert got == exp
        assert 400 < len(exp) < 600  # a fair coin
    res, _ = o.diffusion(9, [], coin_seed=5)  # ViewLens: window -1 in the salt
    assert set(res[0][0].tolist()) - {31} == {v for v in leaves if heads(5, 9, -1, 31, v, 0)}
