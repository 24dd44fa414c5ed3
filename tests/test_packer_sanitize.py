"""The multi-threaded host packer (raphtory_amd/csrc/packer.cpp: parallel radix sorts, per-thread
histograms, partition packing, live-ingest delta packing) under AddressSanitizer + UBSan and
under ThreadSanitizer, as a standalone driver (tests/packer_sanitize.cpp) on
streams with deletes, ties, out-of-order times, power-law hubs and GAB triples.  No GPU."""
import os
import subprocess

import numpy as np
import pytest

from raphtory_amd.synth import YEAR, gen_gab, gen_powerlaw, gen_uniform

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raphtory_amd", "csrc")
FLAGS = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
         "tsan": ["-fsanitize=thread"]}


def _build(kind, out):
    """Built fresh from the current sources into the test's temp dir on every run (never a cached
    binary whose sources or sanitizer runtime may differ)."""
    exe = os.path.join(str(out), f"packer_{kind}")
    srcs = [os.path.join(ROOT, "tests", "packer_sanitize.cpp"), os.path.join(CSRC, "packer.cpp")]
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", *FLAGS[kind], "-I", CSRC, "-o", exe, *srcs],
                   check=True)
    return exe


def _streams():
    s = gen_uniform(3, 500, 40_000, t0=0, dt=1000)
    yield "uniform", s.t, s.kind, s.src, s.dst
    rng = np.random.default_rng(1)
    p = rng.permutation(len(s))
    yield "shuffled", s.t[p], s.kind[p], s.src[p], s.dst[p]
    n = 30_000
    t = (np.arange(n) // 4).astype(np.int64) * 10
    k = rng.choice(4, size=n, p=[0.25, 0.45, 0.12, 0.18]).astype(np.uint8)
    a = rng.integers(0, 300, n).astype(np.int64)
    b = np.where(k >= 2, rng.integers(0, 300, n), -1).astype(np.int64)
    yield "ties", t, k, a, b
    s = gen_powerlaw(3, 3000, 120_000, t0=0, t1=YEAR)
    yield "powerlaw", s.t, s.kind, s.src, s.dst
    s = gen_gab(4, 5000, 40_000)
    yield "gab", s.t, s.kind, s.src, s.dst


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_packer_under_sanitizer(kind, tmp_path):
    exe = _build(kind, tmp_path)
    env = dict(os.environ, RGPU_THREADS="8", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    for name, t, k, s, d in _streams():
        f = tmp_path / f"{name}.bin"
        with open(f, "wb") as fh:
            fh.write(np.int64(len(t)).tobytes())
            for arr, dt in ((t, np.int64), (k, np.uint8), (s, np.int64), (d, np.int64)):
                fh.write(np.ascontiguousarray(arr, dt).tobytes())
        r = subprocess.run([exe, str(f)], env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0 and r.stdout.startswith("ok"), (kind, name, r.returncode, r.stderr[-3000:])
        assert "Sanitizer" not in r.stderr, (kind, name, r.stderr[-3000:])
