"""TemporalGraph — one partition's GPU-resident temporal graph behind the C ABI (include/rgpu.h).

This is the host object a GpuReaderWorker would hold (one per Partition Manager / GPU):
ingest the update stream, seal it into HBM, then answer whole Range jobs per call.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N


class RGPUError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{N.ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


ALGOS = {"cc": N.RGPU_ALGO_CC, "degree": N.RGPU_ALGO_DEGREE, "pagerank": N.RGPU_ALGO_PR,
         "diffusion": N.RGPU_ALGO_DIFFUSION, "vp": N.RGPU_ALGO_VP}
VP_DIRS = {"out": 0, "in": 1, "all": 2}
VP_REDUCE = {"min": 0, "max": 1}


def _i64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


class TemporalGraph:
    def __init__(self, partition: int = 0, num_partitions: int = 1, device: int = 0, vertex_order: str = "locality"):
        """vertex_order: "locality" (default: hubs clustered for cache reuse) or "id" (ids ascending;
        live ingest needs it, so that later seals merge incrementally) — rgpu_set_vertex_order."""
        self._lib = N.rgpu()
        ctx = C.c_void_p()
        rc = self._lib.rgpu_open(partition, num_partitions, device, C.byref(ctx))
        if rc != 0:
            raise RGPUError(rc, f"rgpu_open(partition={partition}, num_partitions={num_partitions}, "
                                f"device={device}) failed")
        self._ctx = ctx
        if vertex_order != "locality":  # (the library's default)
            self.set_vertex_order(vertex_order)
        self._hops: Optional[np.ndarray] = None
        self._windows: List[int] = []

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc: int) -> None:
        if rc != 0:
            raise RGPUError(rc, (self._lib.rgpu_last_error(self._ctx) or b"").decode())

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.rgpu_close(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_vertex_order(self, order: str) -> None:
        code = {"locality": N.RGPU_ORDER_LOCALITY, "id": N.RGPU_ORDER_ID}[order]
        self._check(self._lib.rgpu_set_vertex_order(self._ctx, code))

    # ------------------------------------------------------------------ ingest
    def ingest(self, t, kind, src, dst) -> None:
        t, src, dst = _i64(t), _i64(src), _i64(dst)
        kind = np.ascontiguousarray(np.asarray(kind, dtype=np.uint8))
        n = t.shape[0]
        if not (kind.shape[0] == src.shape[0] == dst.shape[0] == n):
            raise ValueError("ingest arrays must have equal length")
        self._check(self._lib.rgpu_ingest(self._ctx, N.ptr(t, C.c_int64), N.ptr(kind, C.c_uint8),
                                          N.ptr(src, C.c_int64), N.ptr(dst, C.c_int64), n))

    def ingest_rgev(self, buf) -> int:
        """Ingest the whole RGEV blocks in ``buf`` (rgev.py); returns the bytes consumed (a
        trailing partial block is left for the caller's next call)."""
        b = np.frombuffer(buf, dtype=np.uint8)
        used = C.c_size_t()
        self._check(self._lib.rgpu_ingest_rgev(self._ctx, N.ptr(b, C.c_uint8) if b.shape[0] else None,
                                               b.shape[0], C.byref(used)))
        return used.value

    def ingest_stream(self, s) -> None:
        self.ingest(s.t, s.kind, s.src, s.dst)

    def seal(self) -> None:
        self._check(self._lib.rgpu_seal(self._ctx))

    # ------------------------------------------------------------------ partitions
    @staticmethod
    def exchange_id(loopback: bool = False, kind: str = None) -> bytes:
        """Id blob for rgpu_exchange_init (make it on one rank and broadcast it): kind "rccl" (an
        RCCL unique id: one process per GPU), "loopback" (partitions in one process) or "shm"
        (one process per partition on one host, staged through shared memory)."""
        kind = kind or ("loopback" if loopback else "rccl")
        code = {"rccl": N.RGPU_XCHG_RCCL, "loopback": N.RGPU_XCHG_LOOPBACK, "shm": N.RGPU_XCHG_SHM}[kind]
        buf = C.create_string_buffer(N.RGPU_XCHG_ID_BYTES)
        rc = N.rgpu().rgpu_exchange_id(code, buf)
        if rc != 0:
            raise RGPUError(rc, "rgpu_exchange_id failed")
        return buf.raw

    def exchange_init(self, xid: bytes) -> None:
        if len(xid) != N.RGPU_XCHG_ID_BYTES:
            raise ValueError("exchange id must be RGPU_XCHG_ID_BYTES long")
        self._check(self._lib.rgpu_exchange_init(self._ctx, xid))

    def exchange_probe(self, rounds: int = 200) -> dict:
        """rgpu_exchange_probe: the partitioned superstep's fixed cost on this context's channel
        (collective: every partition calls it) -> microseconds per round / per 64-word all-reduce"""
        us = (C.c_double * 4)()
        self._check(self._lib.rgpu_exchange_probe(self._ctx, int(rounds), us))
        return {"round_us_mean": us[0], "round_us_median": us[1], "allreduce_us_mean": us[2],
                "allreduce_us_median": us[3], "rounds": int(rounds)}

    def newest_time(self) -> int:
        out = C.c_int64()
        self._check(self._lib.rgpu_newest_time(self._ctx, C.byref(out)))
        return out.value

    # ------------------------------------------------------------------ run
    def run(self, algo: str, hops: Sequence[int], windows: Sequence[int] = (), max_steps: int = 100,
            pr_iters: int = 20, retain: bool = False, profile: bool = False, serial: bool = False,
            edge_counts: bool = False) -> None:
        hops = _i64(hops)
        w = _i64(list(windows))
        flags = ((N.RGPU_RUN_RETAIN if retain else 0) | (N.RGPU_RUN_PROFILE if profile else 0)
                 | (N.RGPU_RUN_SERIAL if serial else 0) | (N.RGPU_RUN_EDGE_COUNTS if edge_counts else 0))
        wptr = N.ptr(w, C.c_int64) if w.shape[0] else None
        self._check(self._lib.rgpu_run_view_batch(self._ctx, ALGOS[algo], N.ptr(hops, C.c_int64), hops.shape[0],
                                                  wptr, w.shape[0], max_steps, pr_iters, flags))
        self._hops = hops
        self._windows = list(w)

    @property
    def n_windows(self) -> int:
        return max(1, len(self._windows))

    def cc_summary(self, hop: int, win: int) -> N.CCSummary:
        out = N.CCSummary()
        self._check(self._lib.rgpu_cc_summary(self._ctx, hop, win, C.byref(out)))
        return out

    def cc_summaries(self) -> np.ndarray:
        """[n_hops, n_windows, 9] int64: the CCSummary fields of every view (biggest, total,
        total_without_islands, total_islands, clusters_gt2, sum_all, sum_without_islands,
        supersteps, alive_edges)."""
        nh, nw = len(self._hops), self.n_windows
        out = np.zeros((nh, nw, len(N.CCSummary._fields_)), np.int64)
        s = N.CCSummary()
        for h in range(nh):
            for w in range(nw):
                self._check(self._lib.rgpu_cc_summary(self._ctx, h, w, C.byref(s)))
                out[h, w] = [getattr(s, f) for f, _ in N.CCSummary._fields_]
        return out

    def _sized(self, fn, hop, win, arrays_factory):
        n = C.c_size_t()
        self._check(fn(self._ctx, hop, win, *[None for _ in range(arrays_factory(0)[1])], 0, C.byref(n)))
        arrs, _ = arrays_factory(n.value)
        ptrs = [N.ptr(a, t) for a, t in arrs]
        self._check(fn(self._ctx, hop, win, *ptrs, n.value, C.byref(n)))
        return [a for a, _ in arrs]

    def cc_vertex_labels(self, hop: int, win: int) -> Tuple[np.ndarray, np.ndarray]:
        ids, labels = self._sized(self._lib.rgpu_cc_vertex_labels, hop, win,
                                  lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.int64), C.c_int64)], 2))
        return ids, labels

    def cc_result(self, hop: int, win: int) -> Dict[int, int]:
        labels, counts = self._sized(self._lib.rgpu_cc_result, hop, win,
                                     lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.int32), C.c_int32)], 2))
        return {int(l): int(c) for l, c in zip(labels, counts)}

    def degree_vertex(self, hop: int, win: int):
        return self._sized(self._lib.rgpu_degree_vertex, hop, win,
                           lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.int32), C.c_int32),
                                       (np.empty(n, np.int32), C.c_int32)], 3))

    def degree_result(self, hop: int, win: int):
        tot = np.zeros(3, np.int64)
        ids = np.zeros(20, np.int64)
        od = np.zeros(20, np.int32)
        idg = np.zeros(20, np.int32)
        self._check(self._lib.rgpu_degree_result(self._ctx, hop, win, N.ptr(tot, C.c_int64), N.ptr(ids, C.c_int64),
                                                 N.ptr(od, C.c_int32), N.ptr(idg, C.c_int32)))
        top = [(int(i), int(o), int(d)) for i, o, d in zip(ids, od, idg) if i >= 0]
        return (int(tot[0]), int(tot[1]), int(tot[2]), top)

    def pr_result(self, hop: int, win: int):
        return self._sized(self._lib.rgpu_pr_result, hop, win,
                           lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.float64), C.c_double)], 2))

    def set_diffusion(self, seed_id: int = 31, coin_seed: int = 0, coin: bool = True) -> None:
        """BinaryDefusion parameters (infectedNode, hash-coin seed; coin=False sends every message)."""
        self._check(self._lib.rgpu_set_diffusion(self._ctx, seed_id, coin_seed & (2**64 - 1), int(coin)))

    def diffusion_result(self, hop: int, win: int) -> Tuple[int, int]:
        """-> (infected vertices, supersteps of the batch) of view (hop, win)"""
        n, st = C.c_int64(), C.c_int64()
        self._check(self._lib.rgpu_diffusion_result(self._ctx, hop, win, C.byref(n), C.byref(st)))
        return n.value, st.value

    def diffusion_vertex(self, hop: int, win: int) -> Tuple[np.ndarray, np.ndarray]:
        """BinaryDefusion.returnResults: (ids, infected superstep) ascending id (needs retain)."""
        ids, steps = self._sized(self._lib.rgpu_diffusion_vertex, hop, win,
                                 lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.int32), C.c_int32)], 2))
        return ids, steps

    def set_vertex_program(self, direction: str = "all", reduce: str = "min", init: str = "id", senders: str = "all",
                           init_value: int = 0, seed_id: int = -1, seed_value: int = 0, step_add: int = 0) -> None:
        """A generic vertex program for later run("vp", ...) calls (rgpu_set_vertex_program)."""
        p = N.VertexProgram(VP_DIRS[direction], VP_REDUCE[reduce], 0 if init == "id" else 1,
                            0 if senders == "all" else 1, init_value, seed_id, seed_value, step_add)
        self._check(self._lib.rgpu_set_vertex_program(self._ctx, C.byref(p)))

    def vp_result(self, hop: int, win: int) -> Tuple[np.ndarray, np.ndarray]:
        """(ids, final states) of the view's members, ascending id (needs retain)"""
        return self._sized(self._lib.rgpu_vp_result, hop, win,
                           lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.int64), C.c_int64)], 2))

    def set_vertex_program_f(self, direction: str = "out", init: str = "id", senders: str = "all",
                             per_degree: bool = False, seed_id: int = -1, init_value: float = 0.0,
                             seed_value: float = 0.0, bias: float = 0.0, mult: float = 1.0) -> None:
        """A float vertex program (VertexMessageFloat summed; rgpu_set_vertex_program_f) for later
        run("vp", ...) calls; read the states with vp_result_f"""
        if direction not in ("out", "in"):
            raise ValueError("float vertex programs message out- or in-neighbours")
        p = N.VertexProgramF(VP_DIRS[direction], 0 if init == "id" else 1, 0 if senders == "all" else 1,
                             int(bool(per_degree)), seed_id, init_value, seed_value, bias, mult)
        self._check(self._lib.rgpu_set_vertex_program_f(self._ctx, C.byref(p)))

    def vp_result_f(self, hop: int, win: int) -> Tuple[np.ndarray, np.ndarray]:
        """(ids, float states as float64) of the view's members, ascending id (needs retain)"""
        return self._sized(self._lib.rgpu_vp_result_f, hop, win,
                           lambda n: ([(np.empty(n, np.int64), C.c_int64), (np.empty(n, np.float64), C.c_double)], 2))

    def vp_supersteps(self, hop: int) -> int:
        out = C.c_int64()
        self._check(self._lib.rgpu_vp_supersteps(self._ctx, hop, C.byref(out)))
        return out.value

    def stats(self) -> dict:
        s = N.Stats()
        self._check(self._lib.rgpu_stats(self._ctx, C.byref(s)))
        d = {f: getattr(s, f) for f, _ in N.Stats._fields_
             if f not in ("kernel_launches", "kernel_ms", "kernel_bytes", "xchg_bytes_by")}
        d["xchg_bytes_by"] = {k: s.xchg_bytes_by[i] for i, k in enumerate(("membership", "records", "counts", "pagerank"))}
        d["kernels"] = {N.KERNEL_NAMES[i]: {"launches": s.kernel_launches[i], "ms": s.kernel_ms[i],
                                            "bytes": s.kernel_bytes[i]} for i in range(len(N.KERNEL_NAMES))}
        return d
