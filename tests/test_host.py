"""Host-side logic without a GPU: the C ABI library loads and exports every declared
symbol, the Analyser/Task mirror formats like the reference, range hops, partitioning."""
import ctypes
import os
import re

import numpy as np
import pytest

from raphtory_amd import _native as N
from raphtory_amd.analysis import ConnectedComponents, DegreeBasic, cc_fields, java_float_str
from raphtory_amd.partition import get_partition, get_worker
from raphtory_amd.synth import HOUR, T0_README, gen_gab, gen_powerlaw, gen_uniform, range_hops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "rgpu.h")).read()
    return sorted(set(re.findall(r"\b(rgpu_[a-z_0-9]+)\s*\(", src)))


def test_abi_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(N.lib_path())
    decl = declared_symbols()
    assert decl == sorted(N.EXPORTS)
    for name in decl:
        assert hasattr(lib, name), name
    lib.rgpu_abi_version.restype = ctypes.c_int
    assert lib.rgpu_abi_version() == 10
    # error path needs no device: null context
    lib.rgpu_last_error.restype = ctypes.c_char_p
    lib.rgpu_last_error.argtypes = [ctypes.c_void_p]
    assert lib.rgpu_last_error(None) == b"null context"


def test_lib_is_gfx950_code_object():
    blob = open(N.lib_path(), "rb").read()
    assert b"gfx950" in blob


def test_range_hops_follow_restart():
    # RangeAnalysisTask.restart: t += jump, clamp to end, stop after running end
    assert range_hops(0, 10, 3).tolist() == [0, 3, 6, 9, 10]
    assert range_hops(0, 9, 3).tolist() == [0, 3, 6, 9]
    assert range_hops(5, 5, 3).tolist() == [5]
    assert range_hops(7, 5, 3).tolist() == [7, 5]
    h = range_hops(T0_README + 30 * 86_400_000, T0_README + 365 * 86_400_000, HOUR)
    assert len(h) == 8041


def test_partition_function_matches_utils():
    ids = np.array([0, 9, 10, 19, 25, 79, 80, -25], np.int64)
    assert get_partition(ids, 8).tolist() == [0, 0, 1, 1, 2, 7, 0, 2]
    assert get_worker(ids, 8).tolist() == [0, 9, 0, 9, 5, 9, 0, 5]


def test_java_float_formatting():
    assert java_float_str(np.float32(3) / np.float32(7)) == "0.42857143"  # readmepics/results.png
    assert java_float_str(np.float32(1.0)) == "1.0"
    assert java_float_str(np.float32(np.inf)) == "Infinity"
    assert java_float_str(np.float32(0.0001)) == "1.0E-4"
    assert java_float_str(2.5, double=True) == "2.5"
    assert java_float_str(float("nan"), double=True) == "NaN"


def test_cc_summary_fields_and_lines():
    f = cc_fields({1: 3, 2: 1, 5: 2, 9: 1})
    assert f["biggest"] == 3 and f["total"] == 4 and f["totalWithoutIslands"] == 2
    assert f["totalIslands"] == 2 and f["clustersGT2"] == 1
    assert f["proportion"] == np.float32(3) / np.float32(7)
    assert f["proportionWithoutIslands"] == np.float32(3) / np.float32(5)
    a = ConnectedComponents()
    a.processBatchWindowResults([[{1: 3}, {2: 1}], [{}]], 123, [100, 10], 5)
    assert a.lines[0].startswith('{"time":123,"windowsize":100,"biggest":3,"total":2,')
    assert '"proportion":0.75,' in a.lines[0]
    assert a.lines[1] == "No activity for  view at 123 with window 10"
    d = DegreeBasic()
    d.processWindowResults([(3, 4, 4, []), (1, 0, 2, [])], 7, 99, 0)
    assert d.lines == ["7,99,4,6,1.5"]


def test_generators_are_seeded_and_shaped():
    a = gen_uniform(1, 100, 1000)
    b = gen_uniform(1, 100, 1000)
    assert np.array_equal(a.src, b.src) and np.all(np.diff(a.t) > 0)
    frac = np.bincount(a.kind, minlength=4) / 1000
    assert abs(frac[0] - 0.3) < 0.05 and abs(frac[2] - 0.4) < 0.05
    p = gen_powerlaw(3, 10_000, 20_000)
    assert np.all(np.diff(p.t) > 0) and p.src.max() < 2**31
    deg = np.bincount(np.unique(p.src, return_inverse=True)[1])
    assert deg.max() > 50 * np.median(deg)  # heavy tail
    g = gen_gab(4, 1000, 500)
    assert len(g) == 1500 and np.all(g.kind[2::3] == 2) and np.all(np.diff(g.t[::3]) >= 0)
