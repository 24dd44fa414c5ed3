import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


_current = {"test": "", "t0": 0.0}


def pytest_runtest_logstart(nodeid, location):
    import time
    _current["test"], _current["t0"] = nodeid, time.time()


def _heartbeat(period=45.0):
    """A line on stderr every `period` s while a test runs: the full-size config tests run for
    minutes between two pytest outputs, and the GPU box takes a silent command for hung.  The
    thread writes to a duplicate of fd 2 taken before any capture starts, so it never touches
    pytest's (single-threaded) capture manager."""
    import threading
    import time

    try:
        fd = os.dup(2)
    except OSError:
        return

    def beat():
        while True:
            time.sleep(period)
            if _current["test"]:
                try:
                    os.write(fd, f"[heartbeat] {_current['test']} running {time.time() - _current['t0']:.0f} s\n".encode())
                except OSError:  # a heartbeat must never fail a test
                    pass

    threading.Thread(target=beat, daemon=True).start()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "fullsize: a BASELINE config at full size (minutes; deselect with "
                                       "-m 'gpu and not fullsize' for quick iterations)")
    _heartbeat(float(os.environ.get("RGPU_HEARTBEAT_S", "45")))


def _ensure_built():
    # oracle (test infrastructure) and the product libraries; make is a no-op when fresh
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "raphtory_amd", "_build", "librgpu.so")) or \
            not os.path.exists(os.path.join(ROOT, "raphtory_amd", "_build", "libsynth.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raphtory_amd", "csrc")], check=True)


_ensure_built()
