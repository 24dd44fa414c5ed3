"""java.lang.Float.toString / Double.toString as JDK 12 prints them (R/BUILD.md:5 pins JDK 12).

ConnectedComponents prints `proportion` / `proportionWithoutIslands` (Float, ConnectedComponents.scala
:143-148) and DegreeBasic prints `degree` (Double, DegreeBasic.scala:58-63) through string
interpolation, i.e. Float.toString / Double.toString.  Up to JDK 18 these are
jdk.internal.math.FloatingDecimal.toJavaFormatString: the BinaryToASCIIBuffer.dtoa digit generation
(Steele & White / dtoa-style, with fixed-width fast paths) followed by getChars.  Its output is NOT
always the shortest round-trip string (JDK-4511638, fixed by a new algorithm only in JDK 19): e.g.
2.82879384806159E17 prints as "2.82879384806159008E17", and Double.MIN_VALUE as "4.9E-324".  This
module restates that published algorithm step by step with exact integers:

  * unpacking (getBinaryToASCIIConverter): hidden bit, denormal normalisation, nSignificantBits
    (24 / 53 for normals); a float's fraction is shifted into the double's position and run through
    the same dtoa with isCompatibleFormat = true;
  * the integral fast path (dtoa: binExp in [-21, 62], no fraction bits): developLongDigits, which
    prints the exact integer, dropping insignificantDigitsForPow2(binExp - nSignificantBits - 1)
    low digits with rounding;
  * otherwise estimateDecExp, then B = d * 10^-decExp, S, M (half an ulp; halved again below an
    exact power of two: the "nFractBits == 1" hack) as 2^x 5^y products with the common power of
    two removed; digits by repeated division with the symmetric stopping test low = B < M,
    high = B + M > 10S; a zero first digit lowers decExp; in E-form (decExp < -3 or >= 8) the first
    digit never stops the loop (at least one digit after the point); the last digit is rounded up
    when high and not low, or on a tie (2B vs 10S) by digit parity, with the carry of roundup();
  * the three arithmetic widths dtoa picks by the estimated bit lengths (Bbits, tenSbits): int
    and long arithmetic wrap like Java's (the "m > 0" overflow guard included), and the
    FDBigInteger branch tests high as B + M >= 10S (tenSval.addAndCmp(Bval, Mval) <= 0);
  * getChars: plain notation for 10^-3 <= |d| < 10^7 (always a digit after the point), else
    d.dddE[-]n.

No JDK exists in this image, so the restatement is pinned by the JDK's documented outputs
(tests/test_jfloat.py) and by round-trip properties on random values.
"""
from __future__ import annotations

import math
import struct

_N_5_BITS = [0] + [(5 ** i).bit_length() for i in range(1, 27)]  # FloatingDecimal.N_5_BITS
_EXP_SHIFT = 52
_FRACT_HOB = 1 << _EXP_SHIFT
_MAX_SMALL_BIN_EXP = 62
_MIN_SMALL_BIN_EXP = -(63 // 3)


def _wrap(x: int, bits: int) -> int:
    m = 1 << bits
    x &= m - 1
    return x - m if x >= m >> 1 else x


def _insignificant_digits_for_pow2(p2: int) -> int:
    """insignificantDigitsForPow2: floor(p2 * log10(2)) for 1 < p2 < 64, else 0"""
    if 1 < p2 < 64:
        k = 0
        while 10 ** (k + 1) <= 1 << p2:
            k += 1
        return k
    return 0


def _estimate_dec_exp(fract_bits: int, bin_exp: int) -> int:
    """estimateDecExp: floor of a double-precision estimate of log10(d)"""
    d2 = struct.unpack("<d", struct.pack("<Q", 0x3FF0000000000000 | (fract_bits & (_FRACT_HOB - 1))))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + bin_exp * 0.301029995663981
    return math.floor(d)


def _develop_long_digits(lvalue: int, insignificant: int):
    dec_exp = 0
    if insignificant:
        pow10 = 10 ** insignificant
        residue = lvalue % pow10
        lvalue //= pow10
        dec_exp += insignificant
        if residue >= pow10 >> 1:
            lvalue += 1
    s = str(lvalue)
    stripped = s.rstrip("0")
    dec_exp += len(s) - len(stripped)
    dec_exp += len(stripped) - 1
    return list(stripped), dec_exp + 1


def _dtoa(bin_exp: int, fract_bits: int, n_sig: int):
    """BinaryToASCIIBuffer.dtoa(binExp, fractBits, nSignificantBits, isCompatibleFormat = true)
    -> (digits, decExponent)"""
    tail_zeros = (fract_bits & -fract_bits).bit_length() - 1
    n_fract_bits = _EXP_SHIFT + 1 - tail_zeros
    n_tiny_bits = max(0, n_fract_bits - bin_exp - 1)
    if _MIN_SMALL_BIN_EXP <= bin_exp <= _MAX_SMALL_BIN_EXP:
        if n_tiny_bits < 27 and n_fract_bits + _N_5_BITS[n_tiny_bits] < 64 and n_tiny_bits == 0:
            insig = _insignificant_digits_for_pow2(bin_exp - n_sig - 1) if bin_exp > n_sig else 0
            fb = fract_bits << (bin_exp - _EXP_SHIFT) if bin_exp >= _EXP_SHIFT else fract_bits >> (_EXP_SHIFT - bin_exp)
            return _develop_long_digits(fb, insig)
    dec_exp = _estimate_dec_exp(fract_bits, bin_exp)
    B5 = max(0, -dec_exp)
    B2 = B5 + n_tiny_bits + bin_exp
    S5 = max(0, dec_exp)
    S2 = S5 + n_tiny_bits
    M5 = B5
    M2 = B2 - n_sig
    fract_bits >>= tail_zeros
    B2 -= n_fract_bits - 1
    common2 = min(B2, S2)
    B2 -= common2
    S2 -= common2
    M2 -= common2
    if n_fract_bits == 1:  # exact power of two: the next lower value is half as far
        M2 -= 1
    if M2 < 0:
        B2 -= M2
        S2 -= M2
        M2 = 0
    b_bits = n_fract_bits + B2 + (_N_5_BITS[B5] if B5 < 27 else B5 * 3)
    ten_s_bits = S2 + 1 + (_N_5_BITS[S5 + 1] if S5 + 1 < 27 else (S5 + 1) * 3)
    digits = []
    if b_bits < 64 and ten_s_bits < 64:
        width = 32 if (b_bits < 32 and ten_s_bits < 32) else 64
        w = lambda x: _wrap(x, width)  # noqa: E731  (Java int / long arithmetic)
        b = w(w(fract_bits * 5 ** B5) << B2)
        s = w(5 ** S5 << S2)
        m = w(5 ** M5 << M2)
        tens = w(s * 10)
        q = b // s
        b = w(10 * (b % s))
        m = w(m * 10)
        low = b < m
        high = w(b + m) > tens
        if q == 0 and not high:
            dec_exp -= 1  # the estimate was one too high: drop the leading zero
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:  # E-form: at least two digits
            high = low = False
        while not low and not high:
            q = b // s
            b = w(10 * (b % s))
            m = w(m * 10)
            if m > 0:
                low = b < m
                high = w(b + m) > tens
            else:  # m overflowed: it is certainly > b, and b + m > tens
                low = high = True
            digits.append(q)
        low_diff = w(w(b << 1) - tens)  # (b << 1) - tens in int / long arithmetic: wraps before widening
    else:  # FDBigInteger
        S = 5 ** S5 << S2
        B = fract_bits * 5 ** B5 << B2
        M = 5 ** M5 << M2
        tenS = 10 * S
        q, B = divmod(B, S)
        B *= 10
        M *= 10
        low = B < M
        high = B + M >= tenS  # tenSval.addAndCmp(Bval, Mval) <= 0
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q, B = divmod(B, S)
            B *= 10
            M *= 10
            low = B < M
            high = B + M >= tenS
            digits.append(q)
        low_diff = (B << 1) - tenS if (high and low) else 0
    dec_exponent = dec_exp + 1
    digits = [chr(48 + x) for x in digits]
    if high:
        if low:
            if low_diff == 0:
                if (ord(digits[-1]) & 1) != 0:
                    dec_exponent = _roundup(digits, dec_exponent)
            elif low_diff > 0:
                dec_exponent = _roundup(digits, dec_exponent)
        else:
            dec_exponent = _roundup(digits, dec_exponent)
    return digits, dec_exponent


def _roundup(digits, dec_exponent):
    i = len(digits) - 1
    q = digits[i]
    if q == "9":
        while q == "9" and i > 0:
            digits[i] = "0"
            i -= 1
            q = digits[i]
        if q == "9":  # carry out: high-order 1, the rest 0s, a larger exponent
            digits[0] = "1"
            return dec_exponent + 1
    digits[i] = chr(ord(q) + 1)
    return dec_exponent


def _get_chars(neg: bool, digits, dec_exponent: int) -> str:
    """BinaryToASCIIBuffer.getChars (Java format)"""
    n = len(digits)
    out = "-" if neg else ""
    if 0 < dec_exponent < 8:
        k = min(n, dec_exponent)
        out += "".join(digits[:k])
        if k < dec_exponent:
            out += "0" * (dec_exponent - k) + ".0"
        else:
            out += "." + ("".join(digits[k:]) if k < n else "0")
    elif -3 < dec_exponent <= 0:
        out += "0." + "0" * (-dec_exponent) + "".join(digits)
    else:
        out += digits[0] + "." + ("".join(digits[1:]) if n > 1 else "0") + "E"
        e = dec_exponent - 1
        out += str(e) if e >= 0 else "-" + str(-e)
    return out


def _special(v: float, neg: bool):
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "-Infinity" if neg else "Infinity"
    if v == 0.0:
        return "-0.0" if neg else "0.0"
    return None


def float_to_string(x) -> str:
    """java.lang.Float.toString(x) (JDK 12) of the float32 value of x"""
    bits = struct.unpack("<I", struct.pack("<f", x))[0]
    neg = bool(bits >> 31)
    v = struct.unpack("<f", struct.pack("<I", bits))[0]
    sp = _special(v, neg)
    if sp is not None:
        return sp
    fract = bits & ((1 << 23) - 1)
    bin_exp = (bits >> 23) & 0xFF
    if bin_exp == 0:  # denormal: normalise (the top bit to the hidden position)
        lz = 32 - fract.bit_length()
        shift = lz - (31 - 23)
        fract <<= shift
        bin_exp = 1 - shift
        n_fract = 32 - lz
    else:
        fract |= 1 << 23
        n_fract = 24
    bin_exp -= 127
    digits, dexp = _dtoa(bin_exp, fract << (_EXP_SHIFT - 23), n_fract)
    return _get_chars(neg, digits, dexp)


def double_to_string(x) -> str:
    """java.lang.Double.toString(x) (JDK 12)"""
    bits = struct.unpack("<Q", struct.pack("<d", x))[0]
    neg = bool(bits >> 63)
    v = struct.unpack("<d", struct.pack("<Q", bits))[0]
    sp = _special(v, neg)
    if sp is not None:
        return sp
    fract = bits & (_FRACT_HOB - 1)
    bin_exp = (bits >> 52) & 0x7FF
    if bin_exp == 0:
        lz = 64 - fract.bit_length()
        shift = lz - (63 - 52)
        fract <<= shift
        bin_exp = 1 - shift
        n_fract = 64 - lz
    else:
        fract |= _FRACT_HOB
        n_fract = 53
    bin_exp -= 1023
    digits, dexp = _dtoa(bin_exp, fract, n_fract)
    return _get_chars(neg, digits, dexp)
