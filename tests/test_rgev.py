"""RGEV binary update log (layout in include/rgpu.h) — CPU tests.

The library codec (rgev.cpp) is checked against an independent numpy restatement of the
block layout (np_encode below), a committed fixture (tests/golden/rgev_v1_small.*), round
trips on the C1 stream, streaming reads with partial blocks, and corrupted/invalid input."""
import json
import os

import numpy as np
import pytest

from raphtory_amd import rgev
from raphtory_amd.synth import gen_uniform

HERE = os.path.dirname(os.path.abspath(__file__))

# (t, kind, src, dst): ties, out-of-order times, a 2^33 ms jump, every kind
FIXTURE_UPDATES = [
    (1470783600000, 0, 7, -1), (1470783600000, 2, 7, 9), (1470783599000, 3, 9, 7), (1470783600500, 1, 9, -1),
    (1470783600500, 2, 0, 2147483647), (1470783600501, 0, 2147483647, -1),
    (1470783600501 + (1 << 33), 2, 1, 2), (1470783600501 + (1 << 33), 3, 1, 2), (1470783600502, 0, 3, -1),
]


def _fletcher(words: np.ndarray) -> int:
    a = b = 0
    m = (1 << 64) - 1
    for w in words.tolist():
        a = (a + w) & m
        b = (b + a) & m
    return (a ^ (a >> 32) ^ b ^ (b >> 32)) & 0xFFFFFFFF


def np_encode(t, kind, src, dst, block=1 << 20) -> bytes:
    """Restatement of the RGEV v1 layout (include/rgpu.h), written independently of rgev.cpp."""
    t = np.asarray(t, np.int64)
    kind = np.asarray(kind, np.uint8)
    src = np.asarray(src, np.int64)
    dst = np.where(kind >= 2, np.asarray(dst, np.int64), -1)
    out = bytearray()
    i, n = 0, len(t)
    while i < n:
        j, lo, hi = i, t[i], t[i]
        while j < n and j - i < block:
            l2, h2 = min(lo, t[j]), max(hi, t[j])
            if h2 - l2 > 0xFFFFFFFF:
                break
            lo, hi, j = l2, h2, j + 1
        m = j - i
        pad = (-m) % 4
        payload = ((t[i:j] - lo).astype("<u4").tobytes() + kind[i:j].tobytes() + b"\0" * pad
                   + src[i:j].astype("<i4").tobytes() + dst[i:j].astype("<i4").tobytes())
        ck = _fletcher(np.frombuffer(payload, "<u4"))
        out += (np.array([0x56454752], "<u4").tobytes() + np.array([1, 0], "<u2").tobytes()
                + np.array([m, ck], "<u4").tobytes() + np.array([lo], "<i8").tobytes() + payload)
        i = j
    return bytes(out)


def _norm(t, k, s, d):
    k = np.asarray(k, np.uint8)
    return (np.asarray(t, np.int64), k, np.asarray(s, np.int64), np.where(k >= 2, np.asarray(d, np.int64), -1))


def _eq(a, b):
    for x, y in zip(_norm(*a), _norm(*b)):
        assert np.array_equal(x, y)


def test_fixture_bytes_and_decode():
    meta = json.load(open(os.path.join(HERE, "golden", "rgev_v1_small.json")))
    raw = open(os.path.join(HERE, "golden", "rgev_v1_small.rgev"), "rb").read()
    assert len(raw) == meta["bytes"]
    ups = (meta["t"], meta["kind"], meta["src"], meta["dst"])
    assert rgev.encode(*ups, block=meta["block"]) == raw
    got, used = rgev.decode(raw)
    assert used == len(raw)
    _eq(got, ups)


@pytest.mark.parametrize("block", [0, 1, 7, 4096])
def test_library_matches_restatement(block):
    s = gen_uniform(5, 1000, 20_000)
    t = s.t.copy()
    t[::997] += 1 << 32  # force span splits
    raw = rgev.encode(t, s.kind, s.src, s.dst, block=block)
    assert raw == np_encode(t, s.kind, s.src, s.dst, block=block or (1 << 20))


def test_round_trip_c1_stream():
    s = gen_uniform(1, 100_000, 1_000_000)
    raw = rgev.encode(s.t, s.kind, s.src, s.dst, block=65536)
    assert len(raw) == 13 * len(s.t) + 24 * -(-len(s.t) // 65536)
    got, used = rgev.decode(raw)
    assert used == len(raw)
    _eq(got, (s.t, s.kind, s.src, s.dst))


def test_streaming_partial_blocks():
    s = gen_uniform(2, 500, 5_000)
    raw = rgev.encode(s.t, s.kind, s.src, s.dst, block=333)
    rng = np.random.default_rng(0)
    cuts = np.sort(rng.integers(0, len(raw), 25))
    parts, pending = [], b""
    for a, b in zip(np.r_[0, cuts], np.r_[cuts, len(raw)]):
        pending += raw[a:b]
        got, used = rgev.decode(pending)
        parts.append(got)
        pending = pending[used:]
    assert pending == b""
    cat = tuple(np.concatenate([p[i] for p in parts]) for i in range(4))
    _eq(cat, (s.t, s.kind, s.src, s.dst))


def test_rejects_corrupt_and_invalid():
    s = gen_uniform(3, 100, 1000)
    raw = bytearray(rgev.encode(s.t, s.kind, s.src, s.dst, block=100))
    for pos, msg in ((0, "magic"), (4, "version"), (200, "checksum"), (24 + 400 + 5, "checksum")):
        bad = bytearray(raw)
        bad[pos] ^= 0x40
        with pytest.raises(rgev.RGEVError, match=msg):
            rgev.decode(bytes(bad))
    with pytest.raises(rgev.RGEVError, match="vertex id"):
        rgev.encode([1], [0], [-5], [-1])
    with pytest.raises(rgev.RGEVError, match="vertex id"):
        rgev.encode([1], [2], [1], [1 << 31])
    with pytest.raises(rgev.RGEVError, match="kind"):
        rgev.encode([1], [4], [1], [1])
    with pytest.raises(rgev.RGEVError, match="time"):
        rgev.encode([-1], [0], [1], [-1])
    (t, k, _, _), used = rgev.decode(b"")
    assert used == 0 and len(t) == 0
