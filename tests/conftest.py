import os
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "madipm.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(autouse=True)
def _heartbeat(request):
    """Long tests (full-size parity) print a line every 30 s on the real stderr, past pytest's capture,
    so a run that is busy is not mistaken for a hung one."""
    done = threading.Event()
    t0 = time.time()

    def beat():
        while not done.wait(30.0):
            sys.__stderr__.write(f"[heartbeat] {request.node.nodeid} running {time.time() - t0:.0f} s\n")
            sys.__stderr__.flush()

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    done.set()
