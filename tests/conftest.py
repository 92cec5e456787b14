import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


def _heartbeat(path, period=30.0):
    """Append a timestamp to ``path`` every ``period`` s: long host-side oracle tests (minutes of
    CPU with no output) stay visibly alive to a runner that watches files for progress."""
    import threading
    import time

    def beat():
        while True:
            with open(path, "a") as f:
                f.write(f"{time.time():.0f}\n")
            time.sleep(period)
    threading.Thread(target=beat, daemon=True).start()


if os.environ.get("GANAMD_HEARTBEAT"):
    _heartbeat(os.environ["GANAMD_HEARTBEAT"])
