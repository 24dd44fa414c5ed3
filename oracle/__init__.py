"""TEST INFRASTRUCTURE ONLY — ctypes front-end of oracle/_build/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package (as the checker / the timed CPU restatement).  See oracle.h for what it restates
and for its parity status ("parity unpinned" against reference-run outputs).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

_P64 = C.POINTER(C.c_int64)
_P32 = C.POINTER(C.c_int32)
_PU8 = C.POINTER(C.c_uint8)
_PD = C.POINTER(C.c_double)
_SZ = C.c_size_t
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.orc_build.restype = C.c_void_p
        L.orc_build.argtypes = [_P64, _PU8, _P64, _P64, _SZ]
        L.orc_build_ex.restype = C.c_void_p
        L.orc_build_ex.argtypes = [_P64, _PU8, _P64, _P64, _SZ, C.c_int]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_num_vertices.restype = _SZ
        L.orc_num_vertices.argtypes = [C.c_void_p]
        L.orc_num_edges.restype = _SZ
        L.orc_num_edges.argtypes = [C.c_void_p]
        L.orc_history.restype = C.c_long
        L.orc_history.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, _P64, _PU8, _SZ]
        L.orc_alive.restype = C.c_int
        L.orc_alive.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64]
        L.orc_cc.restype = C.c_int
        L.orc_cc.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, C.c_int, C.c_int, _P64, _P64, _SZ,
                             C.POINTER(_SZ), C.POINTER(C.c_int)]
        L.orc_degree.restype = C.c_int
        L.orc_degree.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, _P64, _P32, _P32, _SZ, C.POINTER(_SZ)]
        L.orc_pagerank.restype = C.c_int
        L.orc_pagerank.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, C.c_int, _P64, _PD, _SZ, C.POINTER(_SZ)]
        L.orc_vertex_program.restype = C.c_int
        L.orc_vertex_program.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64, _P64, _P64, _SZ,
                                         C.POINTER(_SZ), C.POINTER(C.c_int)]
        L.orc_vertex_program_f.restype = C.c_int
        L.orc_vertex_program_f.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_int, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double, _P64,
                                           _PD, _SZ, C.POINTER(_SZ), C.POINTER(C.c_int)]
        L.orc_diffusion.restype = C.c_int
        L.orc_diffusion.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, C.c_int, C.c_int64, C.c_uint64,
                                    C.c_int, _P64, _P32, _SZ, C.POINTER(_SZ), C.POINTER(C.c_int)]
        L.orc_addonly_build.restype = C.c_void_p
        L.orc_addonly_build.argtypes = [_P64, _PU8, _P64, _P64, _SZ]
        L.orc_addonly_free.argtypes = [C.c_void_p]
        L.orc_addonly_num_vertices.restype = _SZ
        L.orc_addonly_num_vertices.argtypes = [C.c_void_p]
        L.orc_addonly_cc.restype = C.c_int
        L.orc_addonly_cc.argtypes = [C.c_void_p, C.c_int64, _P64, C.c_int, C.c_int, _P64, _P64, _SZ,
                                     C.POINTER(_SZ), C.POINTER(C.c_int)]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


ORC_LAZY_EDGES = 1


class Oracle:
    """EntityStorage replay + reference-structured analysers on the CPU.

    lazy=True: the replay keeps endpoint deaths in the vertices' removeLists and reads them when
    an edge is evaluated, instead of copying them into every edge (oracle.h, ORC_LAZY_EDGES) —
    the same answers, without the O(degree x deaths) copies that make the literal replay
    intractable on power-law streams of 10^8 updates (configs C3/C4)."""

    def __init__(self, t, kind, src, dst, lazy: bool = False):
        L = lib()
        self.t = np.ascontiguousarray(t, np.int64)
        self.kind = np.ascontiguousarray(kind, np.uint8)
        self.src = np.ascontiguousarray(src, np.int64)
        self.dst = np.ascontiguousarray(dst, np.int64)
        self._g = L.orc_build_ex(_p(self.t, C.c_int64), _p(self.kind, C.c_uint8), _p(self.src, C.c_int64),
                                 _p(self.dst, C.c_int64), self.t.shape[0], ORC_LAZY_EDGES if lazy else 0)
        if not self._g:
            raise ValueError("oracle rejected the stream (negative time or id outside [0, 2^31))")
        self.nv = L.orc_num_vertices(self._g)
        self.ne = L.orc_num_edges(self._g)

    @classmethod
    def from_stream(cls, s, lazy: bool = False):
        return cls(s.t, s.kind, s.src, s.dst, lazy=lazy)

    def close(self):
        if self._g:
            lib().orc_free(self._g)
            self._g = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def history(self, is_edge: bool, src: int, dst: int = -1) -> Optional[List[Tuple[int, bool]]]:
        n = lib().orc_history(self._g, int(is_edge), src, dst, None, None, 0)
        if n < 0:
            return None
        ts = np.empty(max(n, 1), np.int64)
        fl = np.empty(max(n, 1), np.uint8)
        lib().orc_history(self._g, int(is_edge), src, dst, _p(ts, C.c_int64), _p(fl, C.c_uint8), n)
        return [(int(ts[i]), bool(fl[i])) for i in range(n)]

    def alive(self, is_edge: bool, src: int, dst: int, t: int, window: int = -1) -> bool:
        return bool(lib().orc_alive(self._g, int(is_edge), src, dst, t, window))

    def _win(self, windows: Sequence[int]):
        w = np.ascontiguousarray(list(windows), np.int64)
        return w, max(1, len(w))

    def cc(self, t: int, windows: Sequence[int] = (), max_steps: int = 100, mode: int = 1):
        """-> ([(ids, labels)] per window, supersteps)"""
        w, nw = self._win(windows)
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        labels = np.empty(nw * cap, np.int64)
        n = (C.c_size_t * nw)()
        steps = C.c_int()
        rc = lib().orc_cc(self._g, t, _p(w, C.c_int64) if len(w) else None, len(w), max_steps, mode,
                          _p(ids, C.c_int64), _p(labels, C.c_int64), cap, n, C.byref(steps))
        if rc != 0:
            raise RuntimeError("orc_cc failed")
        out = [(ids[i * cap:i * cap + n[i]].copy(), labels[i * cap:i * cap + n[i]].copy()) for i in range(nw)]
        return out, steps.value

    def degree(self, t: int, windows: Sequence[int] = ()):
        w, nw = self._win(windows)
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        od = np.empty(nw * cap, np.int32)
        idg = np.empty(nw * cap, np.int32)
        n = (C.c_size_t * nw)()
        rc = lib().orc_degree(self._g, t, _p(w, C.c_int64) if len(w) else None, len(w),
                              _p(ids, C.c_int64), _p(od, C.c_int32), _p(idg, C.c_int32), cap, n)
        if rc != 0:
            raise RuntimeError("orc_degree failed")
        return [(ids[i * cap:i * cap + n[i]].copy(), od[i * cap:i * cap + n[i]].copy(),
                 idg[i * cap:i * cap + n[i]].copy()) for i in range(nw)]

    def pagerank(self, t: int, windows: Sequence[int] = (), iters: int = 20):
        w, nw = self._win(windows)
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        pr = np.empty(nw * cap, np.float64)
        n = (C.c_size_t * nw)()
        rc = lib().orc_pagerank(self._g, t, _p(w, C.c_int64) if len(w) else None, len(w), iters,
                                _p(ids, C.c_int64), _p(pr, C.c_double), cap, n)
        if rc != 0:
            raise RuntimeError("orc_pagerank failed")
        return [(ids[i * cap:i * cap + n[i]].copy(), pr[i * cap:i * cap + n[i]].copy()) for i in range(nw)]

    VP_DIRS = {"out": 0, "in": 1, "all": 2}
    VP_REDUCE = {"min": 0, "max": 1}

    def vertex_program(self, t: int, windows: Sequence[int] = (), max_steps: int = 100, direction: str = "all",
                       reduce: str = "min", init: str = "id", senders: str = "all", init_value: int = 0,
                       seed_id: int = -1, seed_value: int = 0, step_add: int = 0):
        """generic VertexVisitor messaging (oracle.h orc_vertex_program) -> ([(ids, states)] per
        window, supersteps)"""
        w, nw = self._win(windows)
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        vals = np.empty(nw * cap, np.int64)
        n = (C.c_size_t * nw)()
        steps = C.c_int()
        rc = lib().orc_vertex_program(self._g, t, _p(w, C.c_int64) if len(w) else None, len(w), max_steps,
                                      self.VP_DIRS[direction], self.VP_REDUCE[reduce], 0 if init == "id" else 1,
                                      0 if senders == "all" else 1, init_value, seed_id, seed_value, step_add,
                                      _p(ids, C.c_int64), _p(vals, C.c_int64), cap, n, C.byref(steps))
        if rc != 0:
            raise RuntimeError("orc_vertex_program failed")
        return [(ids[i * cap:i * cap + n[i]].copy(), vals[i * cap:i * cap + n[i]].copy()) for i in range(nw)], steps.value

    def vertex_program_f(self, t: int, windows: Sequence[int] = (), max_steps: int = 100, direction: str = "out",
                         init: str = "id", senders: str = "all", per_degree: bool = False, seed_id: int = -1,
                         init_value: float = 0.0, seed_value: float = 0.0, bias: float = 0.0, mult: float = 1.0):
        """float vertex program, VertexMessageFloat summed (oracle.h orc_vertex_program_f) ->
        ([(ids, float states as float64)] per window, supersteps)"""
        w, nw = self._win(windows)
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        vals = np.empty(nw * cap, np.float64)
        n = (C.c_size_t * nw)()
        steps = C.c_int()
        rc = lib().orc_vertex_program_f(self._g, t, _p(w, C.c_int64) if len(w) else None, len(w), max_steps,
                                        self.VP_DIRS[direction], 0 if init == "id" else 1, 0 if senders == "all" else 1,
                                        int(per_degree), seed_id, init_value, seed_value, bias, mult,
                                        _p(ids, C.c_int64), _p(vals, C.c_double), cap, n, C.byref(steps))
        if rc != 0:
            raise RuntimeError("orc_vertex_program_f failed")
        return [(ids[i * cap:i * cap + n[i]].copy(), vals[i * cap:i * cap + n[i]].copy()) for i in range(nw)], steps.value

    def diffusion(self, t: int, windows: Sequence[int] = (), max_steps: int = 100, seed_id: int = 31,
                  coin_seed: int = 0, coin: bool = True):
        """BinaryDefusion -> ([(ids, infected_step)] per window, supersteps)"""
        w, nw = self._win(windows)
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        st = np.empty(nw * cap, np.int32)
        n = (C.c_size_t * nw)()
        steps = C.c_int()
        rc = lib().orc_diffusion(self._g, t, _p(w, C.c_int64) if len(w) else None, len(w), max_steps, seed_id,
                                 coin_seed & (2**64 - 1), int(coin), _p(ids, C.c_int64), _p(st, C.c_int32), cap,
                                 n, C.byref(steps))
        if rc != 0:
            raise RuntimeError("orc_diffusion failed")
        out = [(ids[i * cap:i * cap + n[i]].copy(), st[i * cap:i * cap + n[i]].copy()) for i in range(nw)]
        return out, steps.value


class AddOnlyOracle:
    """ConnectedComponents on an add-only stream (VertexAdds and EdgeAdds in time order, the
    GAB / C4 shape) read off the time-sorted stream itself (oracle.h orc_addonly_*): the same
    answers as Oracle.cc, in memory for a year of the 1B-update C4 stream.  Thread-safe cc()."""

    def __init__(self, t, kind, src, dst):
        self.t = np.ascontiguousarray(t, np.int64)  # kept alive: the C object reads it
        kind = np.ascontiguousarray(kind, np.uint8)
        src = np.ascontiguousarray(src, np.int64)
        dst = np.ascontiguousarray(dst, np.int64)
        self._a = lib().orc_addonly_build(_p(self.t, C.c_int64), _p(kind, C.c_uint8), _p(src, C.c_int64),
                                          _p(dst, C.c_int64), self.t.shape[0])
        if not self._a:
            raise ValueError("not an add-only stream in time order (or an id outside [0, 2^31))")
        self.nv = lib().orc_addonly_num_vertices(self._a)

    @classmethod
    def from_stream(cls, s):
        return cls(s.t, s.kind, s.src, s.dst)

    def close(self):
        if self._a:
            lib().orc_addonly_free(self._a)
            self._a = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def cc(self, t: int, windows: Sequence[int] = (), max_steps: int = 100):
        """-> ([(ids, labels)] per window, supersteps), as Oracle.cc"""
        w = np.ascontiguousarray(list(windows), np.int64)
        nw = max(1, len(w))
        cap = max(1, self.nv)
        ids = np.empty(nw * cap, np.int64)
        labels = np.empty(nw * cap, np.int64)
        n = (C.c_size_t * nw)()
        steps = C.c_int()
        rc = lib().orc_addonly_cc(self._a, t, _p(w, C.c_int64) if len(w) else None, len(w), max_steps,
                                  _p(ids, C.c_int64), _p(labels, C.c_int64), cap, n, C.byref(steps))
        if rc != 0:
            raise RuntimeError("orc_addonly_cc failed")
        out = [(ids[i * cap:i * cap + n[i]].copy(), labels[i * cap:i * cap + n[i]].copy()) for i in range(nw)]
        return out, steps.value


def label_counts(labels: np.ndarray) -> dict:
    u, c = np.unique(labels, return_counts=True)
    return {int(a): int(b) for a, b in zip(u, c)}
