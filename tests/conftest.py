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


def _heartbeat(config, period=45.0):
    """A line on the terminal every `period` s while a test runs: the full-size config tests run
    for minutes between two pytest outputs, and the GPU box takes a silent command for hung."""
    import threading
    import time

    def beat():
        while True:
            time.sleep(period)
            tr = config.pluginmanager.get_plugin("terminalreporter")  # registered after this hook
            capman = config.pluginmanager.get_plugin("capturemanager")
            if _current["test"] and tr is not None and capman is not None:
                try:
                    with capman.global_and_fixture_disabled():  # past the test's output capture
                        tr.write_line(f"[heartbeat] {_current['test']} running {time.time() - _current['t0']:.0f} s")
                except Exception:  # noqa: BLE001 - a heartbeat must never fail a test
                    pass

    threading.Thread(target=beat, daemon=True).start()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "fullsize: a BASELINE config at full size (minutes; deselect with "
                                       "-m 'gpu and not fullsize' for quick iterations)")
    _heartbeat(config, float(os.environ.get("RGPU_HEARTBEAT_S", "45")))


def _ensure_built():
    # oracle (test infrastructure) and the product libraries; make is a no-op when fresh
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "raphtory_amd", "_build", "librgpu.so")) or \
            not os.path.exists(os.path.join(ROOT, "raphtory_amd", "_build", "libsynth.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raphtory_amd", "csrc")], check=True)


_ensure_built()
