"""Every `Name.scala:N[-M][,N[-M]...]` citation in the oracle, the native sources, the host mirror,
the ABI header and the golden fixtures points inside the cited reference file (the
oracle cited WindowLens lines past the end of its 69-line file).  Reads the reference sources as
text only; skipped where /root/reference is absent (the GPU box)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
SCAN = ["oracle", "raphtory_amd", "include", "tests/golden", "INTEGRATION.md", "DESIGN.md"]
CITE = re.compile(r"\b([A-Z][A-Za-z0-9]*)\.scala:(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)")


def _ref_files():
    out = {}
    for d, _, fs in os.walk(REF):
        for f in fs:
            if f.endswith(".scala"):
                out.setdefault(f[:-6], []).append(os.path.join(d, f))
    return out


def _sources():
    for s in SCAN:
        p = os.path.join(ROOT, s)
        if os.path.isfile(p):
            yield p
            continue
        for d, _, fs in os.walk(p):
            if "_build" in d or "__pycache__" in d:
                continue
            for f in fs:
                if f.endswith((".c", ".h", ".cpp", ".hpp", ".hip", ".py", ".json", ".md")):
                    yield os.path.join(d, f)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent")
def test_scala_citations_in_range():
    files = _ref_files()
    nlines = {}
    bad, n = [], 0
    for src in _sources():
        text = open(src, encoding="utf-8", errors="replace").read()
        for m in CITE.finditer(text):
            name, spans = m.group(1), m.group(2)
            if name not in files:
                continue
            last = max(int(x) for x in re.split(r"[-,]", spans))
            # the longest file of that name (names repeat across example packages)
            size = max(nlines.setdefault(p, sum(1 for _ in open(p, errors="replace"))) for p in files[name])
            n += 1
            if last > size:
                bad.append(f"{os.path.relpath(src, ROOT)}: {name}.scala:{spans} (file has {size} lines)")
    assert n > 100, n
    assert not bad, "\n".join(bad)
