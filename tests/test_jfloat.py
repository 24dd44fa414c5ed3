"""Float.toString / Double.toString of the reference's JDK 12 (raphtory_amd/jfloat.py, the
FloatingDecimal algorithm restated; the strings ConnectedComponents.scala:143-148 and
DegreeBasic.scala:58-63 print).  No JDK exists in this image: the cases below are the JDK's
documented outputs (constant javadocs, the README's result line, the JDK-4511638 report of a
non-shortest output), cases derived by hand from the algorithm's rules, and round-trip properties
on random values (every string FloatingDecimal prints parses back to the same value)."""
import re
import struct

import numpy as np
import pytest

from raphtory_amd.jfloat import double_to_string as D
from raphtory_amd.jfloat import float_to_string as F


def f32(x):
    return float(np.float32(x))


def bits_f(b):
    return struct.unpack("<f", struct.pack("<I", b))[0]


def test_documented_float_outputs():
    assert F(bits_f(1)) == "1.4E-45"                    # Float.MIN_VALUE javadoc: 1.4e-45f
    assert F(bits_f(0x7F7FFFFF)) == "3.4028235E38"      # Float.MAX_VALUE javadoc: 3.4028235e+38f
    assert F(bits_f(0x00800000)) == "1.17549435E-38"    # Float.MIN_NORMAL javadoc: 1.17549435E-38f
    assert F(f32(3) / f32(7)) == "0.42857143"           # README results line ("proportion":0.42857143)
    assert F(f32(1) / f32(3)) == "0.33333334"
    assert F(float("inf")) == "Infinity" and F(float("-inf")) == "-Infinity" and F(float("nan")) == "NaN"
    assert F(0.0) == "0.0" and F(-0.0) == "-0.0"


def test_documented_double_outputs():
    assert D(5e-324) == "4.9E-324"                       # Double.MIN_VALUE javadoc: 4.9e-324
    assert D(1.7976931348623157e308) == "1.7976931348623157E308"  # Double.MAX_VALUE javadoc
    assert D(2.2250738585072014e-308) == "2.2250738585072014E-308"  # Double.MIN_NORMAL javadoc
    assert D(0.1 + 0.2) == "0.30000000000000004"
    assert D(1 / 3) == "0.3333333333333333" and D(2 / 3) == "0.6666666666666666"
    # JDK-4511638 (fixed only in JDK 19): not the shortest string — the integral fast path
    # (developLongDigits) prints the exact integer 282879384806159008
    assert D(2.82879384806159e17) == "2.82879384806159008E17"


def test_format_boundaries():
    """getChars: plain notation for 10^-3 <= |d| < 10^7, always a digit after the point"""
    assert F(0.001) == "0.001" and F(f32(0.001) * f32(0.999)) == "9.99E-4"
    assert F(9999999.0) == "9999999.0" and F(1e7) == "1.0E7" and F(1e10) == "1.0E10"
    assert F(100.0) == "100.0" and F(0.5) == "0.5" and F(-2.5) == "-2.5" and F(1e-5) == "1.0E-5"
    assert D(0.001) == "0.001" and D(1e7) == "1.0E7" and D(123456789.0) == "1.23456789E8"
    assert D(1.73) == "1.73" and D(100.0) == "100.0"


def test_derived_from_the_algorithm():
    """Hand-derived: the double nearest 1e23 is 99999999999999991611392 and 1e23 lies exactly on
    its upper rounding boundary (v + ulp/2).  The first digit (9) meets the stopping test there,
    but in E-form (decExp >= 8) dtoa never stops after the first digit, so the digits go on until
    the symmetric test stops them at 16 nines: not the shortest "1.0E23"."""
    assert D(1e23) == "9.999999999999999E22"
    # 2^n fast path: integral doubles below 2^63 print exactly (insignificant digits dropped only
    # above 2^54: 2^60 has 60 - 53 - 1 = 6 binary digits below precision -> 1 decimal digit)
    assert D(float(2 ** 53)) == "9.007199254740992E15"
    assert D(float(2 ** 60)) == "1.15292150460684698E18"


_FORMS = re.compile(r"^-?(\d+\.\d+|\d\.\d+E-?\d+)$")


@pytest.mark.parametrize("seed", [1, 2])
def test_round_trip_random_floats(seed):
    rng = np.random.default_rng(seed)
    xs = np.concatenate([rng.integers(1, 0x7F800000, 4000, dtype=np.uint64).astype(np.uint32).view(np.float32),
                         (rng.random(4000) * rng.choice([1e-6, 1e-3, 1, 1e3, 1e7], 4000)).astype(np.float32)])
    for x in xs.tolist():
        s = F(x)
        assert _FORMS.match(s), s
        assert np.float32(float(s.replace("E", "e"))) == np.float32(x), (x, s)
        v = abs(x)
        assert ("E" in s) == (not (1e-3 <= v < 1e7)), s


@pytest.mark.parametrize("seed", [3, 4])
def test_round_trip_random_doubles(seed):
    rng = np.random.default_rng(seed)
    xs = np.concatenate([rng.integers(1, 0x7FF0000000000000, 4000, dtype=np.uint64).view(np.float64),
                         rng.random(4000) * rng.choice([1e-6, 1e-3, 1, 1e3, 1e7, 1e17], 4000)])
    for x in xs.tolist():
        s = D(x)
        assert _FORMS.match(s), s
        assert float(s.replace("E", "e")) == x, (x, s)
