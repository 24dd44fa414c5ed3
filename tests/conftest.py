import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


def _ensure_built():
    # oracle (test infrastructure) and the product libraries; make is a no-op when fresh
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "raphtory_amd", "_build", "librgpu.so")) or \
            not os.path.exists(os.path.join(ROOT, "raphtory_amd", "_build", "libsynth.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raphtory_amd", "csrc")], check=True)


_ensure_built()
