"""TEST INFRASTRUCTURE: builds and loads tests/packer_harness.cpp + the product's host packer
(raphtory_amd/csrc/packer.cpp) with g++ — the packer runs on the CPU, no GPU needed."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "_build", "libpacker_harness.so")
P64, PU8 = C.POINTER(C.c_int64), C.POINTER(C.c_uint8)


def load_packer_harness():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = [os.path.join(ROOT, "tests", "packer_harness.cpp"), os.path.join(ROOT, "raphtory_amd", "csrc", "packer.cpp"),
           os.path.join(ROOT, "raphtory_amd", "csrc", "rgpu_internal.hpp")]
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in src):
        tmp = SO + f".{os.getpid()}"
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread",
                        "-I", os.path.join(ROOT, "raphtory_amd", "csrc"), "-o", tmp] + src[:2], check=True)
        os.replace(tmp, SO)
    L = C.CDLL(SO)
    L.ph_pack.restype = C.c_void_p
    L.ph_pack.argtypes = [P64, PU8, P64, P64, C.c_size_t]
    L.ph_pack_part.restype = C.c_void_p
    L.ph_pack_part.argtypes = [P64, PU8, P64, P64, C.c_size_t, C.c_int, C.c_int]
    L.ph_alive.restype = C.c_int
    L.ph_alive.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int64]
    L.ph_free.argtypes = [C.c_void_p]
    L.ph_num.restype = C.c_int64
    L.ph_num.argtypes = [C.c_void_p, C.c_int]
    L.ph_list.restype = C.c_int64
    L.ph_list.argtypes = [C.c_void_p, C.c_int, C.c_int, P64]
    L.ph_set_locality.argtypes = [C.c_int]
    L.ph_delta_check.restype = C.c_int
    L.ph_delta_check.argtypes = [P64, PU8, P64, P64, C.c_size_t, C.c_size_t]
    return L


def _p(a, ty):
    return a.ctypes.data_as(C.POINTER(ty))


def pack(L, t, k, s, d, part=None, nparts=1):
    if part is None:
        h = L.ph_pack(_p(t, C.c_int64), _p(k, C.c_uint8), _p(s, C.c_int64), _p(d, C.c_int64), len(t))
    else:
        h = L.ph_pack_part(_p(t, C.c_int64), _p(k, C.c_uint8), _p(s, C.c_int64), _p(d, C.c_int64), len(t),
                           part, nparts)
    assert h
    return h


def plist(L, h, what, q=0):
    n = L.ph_list(h, what, q, None)
    out = np.zeros(n, np.int64)
    L.ph_list(h, what, q, out.ctypes.data_as(P64))
    return out
