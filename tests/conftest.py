import os
import sys
import threading
import time

import pytest

# eager (MIOpen) reference convs: heuristic kernel choice instead of per-shape benchmarking, so the
# fp32 / bf16 oracles of the large parity cases do not spend minutes tuning on a fresh box
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


_CURRENT = {"name": None, "t0": 0.0}


def pytest_runtest_logstart(nodeid, location):
    _CURRENT["name"], _CURRENT["t0"] = nodeid, time.time()


def pytest_runtest_logfinish(nodeid, location):
    _CURRENT["name"] = None


def _heartbeat():
    # a line on the real stderr every 60 s while one test runs long (first MIOpen builds of a large
    # oracle, etc.): a silent GPU run is taken to be hung by the remote runner
    while True:
        time.sleep(60)
        name = _CURRENT["name"]
        if name is not None:
            sys.__stderr__.write(f"[heartbeat] {name} running {time.time() - _CURRENT['t0']:.0f} s\n")
            sys.__stderr__.flush()


threading.Thread(target=_heartbeat, daemon=True).start()
