"""ctypes bindings of the in-tree native libraries.

``librgpu.so`` is the product: HIP kernels + host packer behind the C ABI declared in
``include/rgpu.h``.  There is no CPU fallback: if the library is missing or does not load,
every call raises :class:`NativeUnavailable`.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(_HERE, "_build")

# error codes / constants mirrored from include/rgpu.h
ABI_VERSION = 10
RGPU_OK = 0
RGPU_EINVAL, RGPU_ESTATE, RGPU_EHIP, RGPU_ENOMEM, RGPU_ENOTSUP = -1, -2, -3, -4, -5
RGPU_VADD, RGPU_VDEL, RGPU_EADD, RGPU_EDEL = 0, 1, 2, 3
RGPU_ALGO_CC, RGPU_ALGO_DEGREE, RGPU_ALGO_PR, RGPU_ALGO_DIFFUSION, RGPU_ALGO_VP = 0, 1, 2, 3, 4
RGPU_RUN_RETAIN, RGPU_RUN_PROFILE, RGPU_RUN_SERIAL, RGPU_RUN_EDGE_COUNTS = 1, 2, 4, 8
RGPU_XCHG_ID_BYTES, RGPU_XCHG_RCCL, RGPU_XCHG_LOOPBACK, RGPU_XCHG_SHM = 128, 0, 1, 2
RGPU_ORDER_LOCALITY, RGPU_ORDER_ID = 0, 1
ERROR_NAMES = {
    RGPU_EINVAL: "RGPU_EINVAL",
    RGPU_ESTATE: "RGPU_ESTATE",
    RGPU_EHIP: "RGPU_EHIP",
    RGPU_ENOMEM: "RGPU_ENOMEM",
    RGPU_ENOTSUP: "RGPU_ENOTSUP",
}
KERNEL_NAMES = ["window_mask", "cc_slots", "cc_step", "cc_hist", "cc_summary", "pr_step", "degree", "cc_tail",
                "heavy", "diffusion", "vp_step", "edge_mask", "xchg", "xchg_pack", "xchg_unpack", "xchg_mark"]

# exported symbols of librgpu.so, exactly the declarations of include/rgpu.h
EXPORTS = [
    "rgpu_abi_version", "rgpu_open", "rgpu_ingest", "rgpu_seal", "rgpu_newest_time",
    "rgpu_exchange_id", "rgpu_exchange_init", "rgpu_run_view_batch", "rgpu_cc_summary", "rgpu_cc_result",
    "rgpu_cc_vertex_labels", "rgpu_degree_result", "rgpu_degree_vertex", "rgpu_pr_result",
    "rgpu_stats", "rgpu_last_error", "rgpu_close",
    "rgpu_rgev_encode", "rgpu_rgev_decode", "rgpu_rgev_last_error", "rgpu_ingest_rgev",
    "rgpu_set_diffusion", "rgpu_diffusion_result", "rgpu_diffusion_vertex", "rgpu_set_vertex_order",
    "rgpu_set_vertex_program", "rgpu_vp_result", "rgpu_vp_supersteps", "rgpu_exchange_probe",
    "rgpu_set_vertex_program_f", "rgpu_vp_result_f",
]


class NativeUnavailable(RuntimeError):
    pass


class CCSummary(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "biggest", "total", "total_without_islands", "total_islands", "clusters_gt2",
        "sum_all", "sum_without_islands", "supersteps", "alive_edges")]


class VertexProgramF(C.Structure):
    _fields_ = [("direction", C.c_int32), ("init", C.c_int32), ("senders", C.c_int32), ("per_degree", C.c_int32),
                ("seed_id", C.c_int64), ("init_value", C.c_double), ("seed_value", C.c_double), ("bias", C.c_double),
                ("mult", C.c_double)]


class VertexProgram(C.Structure):
    _fields_ = [("direction", C.c_int32), ("reduce", C.c_int32), ("init", C.c_int32), ("senders", C.c_int32),
                ("init_value", C.c_int64), ("seed_id", C.c_int64), ("seed_value", C.c_int64), ("step_add", C.c_int64)]


class Stats(C.Structure):
    _fields_ = [
        ("vertices", C.c_int64), ("edges", C.c_int64),
        ("vertex_events", C.c_int64), ("edge_events", C.c_int64), ("deaths", C.c_int64),
        ("views", C.c_int64), ("batches", C.c_int64), ("supersteps", C.c_int64), ("launches", C.c_int64),
        ("ms_total", C.c_double),
        ("kernel_launches", C.c_int64 * 16), ("kernel_ms", C.c_double * 16), ("kernel_bytes", C.c_double * 16),
        ("seal_ms", C.c_double), ("seal_incremental", C.c_int64), ("seal_delta_updates", C.c_int64),
        ("alive_edge_windows", C.c_int64), ("edges_owned", C.c_int64), ("xchg_bytes", C.c_double),
        ("xchg_bytes_by", C.c_double * 4),
    ]


_P64 = C.POINTER(C.c_int64)
_P32 = C.POINTER(C.c_int32)
_PU8 = C.POINTER(C.c_uint8)
_PD = C.POINTER(C.c_double)
_SZ = C.c_size_t
_CTX = C.c_void_p

_SIGS = {
    "rgpu_abi_version": (C.c_int, []),
    "rgpu_open": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(_CTX)]),
    "rgpu_ingest": (C.c_int, [_CTX, _P64, _PU8, _P64, _P64, _SZ]),
    "rgpu_seal": (C.c_int, [_CTX]),
    "rgpu_newest_time": (C.c_int, [_CTX, _P64]),
    "rgpu_set_vertex_order": (C.c_int, [_CTX, C.c_int]),
    "rgpu_exchange_id": (C.c_int, [C.c_int, C.c_char_p]),
    "rgpu_exchange_init": (C.c_int, [_CTX, C.c_char_p]),
    "rgpu_exchange_probe": (C.c_int, [_CTX, C.c_int, _PD]),
    "rgpu_run_view_batch": (C.c_int, [_CTX, C.c_int, _P64, _SZ, _P64, _SZ, C.c_int, C.c_int, C.c_int]),
    "rgpu_cc_summary": (C.c_int, [_CTX, _SZ, _SZ, C.POINTER(CCSummary)]),
    "rgpu_cc_result": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P32, _SZ, C.POINTER(_SZ)]),
    "rgpu_cc_vertex_labels": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P64, _SZ, C.POINTER(_SZ)]),
    "rgpu_degree_result": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P64, _P32, _P32]),
    "rgpu_degree_vertex": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P32, _P32, _SZ, C.POINTER(_SZ)]),
    "rgpu_pr_result": (C.c_int, [_CTX, _SZ, _SZ, _P64, _PD, _SZ, C.POINTER(_SZ)]),
    "rgpu_set_diffusion": (C.c_int, [_CTX, C.c_int64, C.c_uint64, C.c_int]),
    "rgpu_set_vertex_program": (C.c_int, [_CTX, C.POINTER(VertexProgram)]),
    "rgpu_vp_result": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P64, _SZ, C.POINTER(_SZ)]),
    "rgpu_vp_supersteps": (C.c_int, [_CTX, _SZ, _P64]),
    "rgpu_set_vertex_program_f": (C.c_int, [_CTX, C.POINTER(VertexProgramF)]),
    "rgpu_vp_result_f": (C.c_int, [_CTX, _SZ, _SZ, _P64, _PD, _SZ, C.POINTER(_SZ)]),
    "rgpu_diffusion_result": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P64]),
    "rgpu_diffusion_vertex": (C.c_int, [_CTX, _SZ, _SZ, _P64, _P32, _SZ, C.POINTER(_SZ)]),
    "rgpu_stats": (C.c_int, [_CTX, C.POINTER(Stats)]),
    "rgpu_last_error": (C.c_char_p, [_CTX]),
    "rgpu_close": (None, [_CTX]),
    "rgpu_rgev_encode": (C.c_int, [_P64, _PU8, _P64, _P64, _SZ, _SZ, _PU8, _SZ, C.POINTER(_SZ)]),
    "rgpu_rgev_decode": (C.c_int, [_PU8, _SZ, _P64, _PU8, _P64, _P64, _SZ, C.POINTER(_SZ), C.POINTER(_SZ)]),
    "rgpu_rgev_last_error": (C.c_char_p, []),
    "rgpu_ingest_rgev": (C.c_int, [_CTX, _PU8, _SZ, C.POINTER(_SZ)]),
}

_lib = None
_synth = None


def lib_path(name: str = "librgpu.so") -> str:
    return os.path.join(BUILD_DIR, name)


def rgpu() -> C.CDLL:
    """The loaded librgpu.so (raises NativeUnavailable — never falls back)."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            lib = C.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeUnavailable(f"cannot load {path}: {e}") from e
        missing = [name for name in _SIGS if getattr(lib, name, None) is None]
        if missing:
            raise NativeUnavailable(f"{path} lacks entry points {missing}: rebuild it")
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        # the Stats / CCSummary layouts above are those of this ABI version (rgpu.h RGPU_ABI_VERSION)
        abi = lib.rgpu_abi_version()
        if abi != ABI_VERSION:
            raise NativeUnavailable(f"{path} speaks ABI {abi}, these bindings ABI {ABI_VERSION}: rebuild it")
        _lib = lib
    return _lib


def synth() -> C.CDLL:
    global _synth
    if _synth is None:
        path = lib_path("libsynth.so")
        if not os.path.exists(path):
            raise NativeUnavailable(f"{path} is missing")
        s = C.CDLL(path)
        s.rg_gen_uniform.restype = _SZ
        s.rg_gen_uniform.argtypes = [C.c_uint64, C.c_int64, _SZ, C.c_int64, C.c_int64,
                                     C.c_double, C.c_double, C.c_double, _P64, _PU8, _P64, _P64]
        s.rg_gen_powerlaw.restype = _SZ
        s.rg_gen_powerlaw.argtypes = [C.c_uint64, C.c_int64, _SZ, C.c_double, C.c_int64, C.c_int64,
                                      _P64, _PU8, _P64, _P64]
        s.rg_gen_gab.restype = _SZ
        s.rg_gen_gab.argtypes = [C.c_uint64, C.c_int64, _SZ, C.c_int64, C.c_int64, _P64, _PU8, _P64, _P64]
        s.rg_gen_gab_keyed.restype = _SZ
        s.rg_gen_gab_keyed.argtypes = [C.c_uint64, C.c_uint64, C.c_int64, _SZ, C.c_int64, C.c_int64, _P64, _PU8,
                                       _P64, _P64]
        s.rg_gen_gab_range.restype = _SZ
        s.rg_gen_gab_range.argtypes = [C.c_uint64, C.c_uint64, C.c_int64, _SZ, _SZ, _SZ, C.c_int, C.c_int,
                                       C.c_int64, C.c_int64, _P64, _PU8, _P64, _P64]
        _synth = s
    return _synth


def ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))
