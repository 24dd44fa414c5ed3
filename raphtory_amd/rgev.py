"""Binary GraphUpdate log ("RGEV") — host-side codec over the C ABI.

A Router packs its GraphUpdates (VertexAdd / VertexDelete / EdgeAdd / EdgeDelete,
raphtoryMessages.scala:38-55) into RGEV blocks instead of sending one actor message per
update (RouterWorker.sendGraphUpdate, RouterWorker.scala:88-116); a partition hands the bytes
to ``TemporalGraph.ingest_rgev`` (``rgpu_ingest_rgev``).  The block layout is specified in
include/rgpu.h.  Both directions run in librgpu.so (rgev.cpp) — no GPU needed.
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import numpy as np

from . import _native as N

MAX_BLOCK = 1 << 20
HEADER_BYTES = 24


class RGEVError(ValueError):
    pass


def _err(rc: int) -> RGEVError:
    return RGEVError(f"{N.ERROR_NAMES.get(rc, rc)}: {(N.rgpu().rgpu_rgev_last_error() or b'').decode()}")


def encode(t, kind, src, dst, block: int = 0) -> bytes:
    """Pack updates (stream order kept) into RGEV blocks of at most ``block`` updates."""
    t = np.ascontiguousarray(t, dtype=np.int64)
    kind = np.ascontiguousarray(kind, dtype=np.uint8)
    src = np.ascontiguousarray(src, dtype=np.int64)
    dst = np.ascontiguousarray(dst, dtype=np.int64)
    n = t.shape[0]
    if not (kind.shape[0] == src.shape[0] == dst.shape[0] == n):
        raise ValueError("update arrays must have equal length")
    lib = N.rgpu()
    args = (N.ptr(t, C.c_int64), N.ptr(kind, C.c_uint8), N.ptr(src, C.c_int64), N.ptr(dst, C.c_int64), n, block)
    need = C.c_size_t()
    rc = lib.rgpu_rgev_encode(*args, None, 0, C.byref(need))
    if rc != 0:
        raise _err(rc)
    out = np.empty(need.value, np.uint8)
    rc = lib.rgpu_rgev_encode(*args, N.ptr(out, C.c_uint8), need.value, C.byref(need))
    if rc != 0:
        raise _err(rc)
    return out.tobytes()


def decode(buf) -> Tuple[Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray], int]:
    """Expand the whole blocks in ``buf``: ((t, kind, src, dst), bytes consumed)."""
    b = np.frombuffer(buf, dtype=np.uint8)
    lib = N.rgpu()
    n, used = C.c_size_t(), C.c_size_t()
    bp = N.ptr(b, C.c_uint8) if b.shape[0] else None
    rc = lib.rgpu_rgev_decode(bp, b.shape[0], None, None, None, None, 0, C.byref(n), C.byref(used))
    if rc != 0:
        raise _err(rc)
    t, src, dst = (np.empty(n.value, np.int64) for _ in range(3))
    kind = np.empty(n.value, np.uint8)
    rc = lib.rgpu_rgev_decode(bp, used.value, N.ptr(t, C.c_int64), N.ptr(kind, C.c_uint8), N.ptr(src, C.c_int64),
                              N.ptr(dst, C.c_int64), n.value, C.byref(n), C.byref(used))
    if rc != 0:
        raise _err(rc)
    return (t, kind, src, dst), used.value
